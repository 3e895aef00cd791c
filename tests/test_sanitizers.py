"""sanitizer builds of the host code (the reference has none).

  * the C restatement (oracle/) + a driver that walks all of it, built with AddressSanitizer and
    UndefinedBehaviorSanitizer (-fno-sanitize-recover: the first report fails the run);
  * the C++ mirror (backuwup_amd/host/backuwup.hpp) built with the same flags -- compiled here,
    run against the GPU library under -m gpu (host code only: the sanitizers never touch device
    code, and GPU AddressSanitizer is not used);
  * the HIP library's BW_DEBUG build (device bounds asserts) compiles for gfx950; it is run on the
    GPU by tools/debug_check.py (tools/gpu_r2.sh step `debug`).
"""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]


def test_oracle_under_asan_ubsan(tmp_path):
    exe = tmp_path / "oracle_selftest"
    src = [os.path.join(HERE, "cpp", "oracle_selftest.c")] + \
        [os.path.join(ROOT, "oracle", f) for f in ("bw_oracle.c", "bw_oracle_seal.c", "bw_oracle_simd.c")]
    subprocess.check_call(["gcc", "-std=c11", "-D_GNU_SOURCE", "-Wall"] + SAN + src + ["-lpthread", "-lm", "-o", str(exe)])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([str(exe)], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "oracle selftest ok" in r.stdout


def build_cpp_mirror_asan(tmp_path):
    exe = tmp_path / "host_parity_asan"
    libdir = os.path.join(ROOT, "backuwup_amd")
    subprocess.check_call(["g++", "-std=c++17", "-I", os.path.join(ROOT, "include")] + SAN +
                          [os.path.join(HERE, "cpp", "host_parity.cpp"), "-L", libdir, "-lbackuwup_amd",
                           "-Wl,-rpath," + libdir, "-o", str(exe)])
    return exe


def test_cpp_mirror_builds_with_sanitizers(tmp_path):
    assert build_cpp_mirror_asan(tmp_path).exists()


@pytest.mark.gpu
def test_cpp_mirror_runs_under_asan_ubsan(tmp_path):
    """The C++ mirror under ASan/UBSan, calling the real library on the GPU (host-side checks)."""
    exe = build_cpp_mirror_asan(tmp_path)
    # the HIP runtime keeps process-lifetime allocations: leak checking would only report those
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "gate 0 1 0 2" in r.stdout


def test_hip_debug_build_compiles():
    from backuwup_amd import build
    lib = build.build(debug=True)
    assert os.path.exists(lib) and lib.endswith("_debug.so")
