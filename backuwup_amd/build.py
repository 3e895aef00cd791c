"""Build libbackuwup_amd.so (HIP, gfx950) in-tree with hipcc.

The library is the product: every entry point in include/backuwup_gpu.h is implemented in
backuwup_amd/csrc/*.hip and runs on the GPU.  No torch extension, no JIT cache: the .so sits
next to this file so it travels with the repository snapshot to the GPU box.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libbackuwup_amd.so")
# BW_DEBUG build: the same sources with device bounds asserts (BW_ASSERT in csrc/bw_device.h); loaded
# only when BW_LIB points at it (tools/debug_check.py), never by the product path
LIB_DEBUG = os.path.join(HERE, "libbackuwup_amd_debug.so")
SOURCES = ["bw_capi.hip", "bw_cdc.hip", "bw_blake3.hip", "bw_dedup.hip", "bw_tree.hip", "bw_seal.hip", "bw_pack.hip", "bw_zstd.hip"]
ARCH = os.environ.get("BW_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def source_digest():
    """sha256 over the library's sources (csrc/* and the C ABI header): identifies the kernels a
    profile was taken with (profiles/pmc_traffic.json), so bench.py can tell stale evidence."""
    import hashlib
    h = hashlib.sha256()
    files = sorted(os.listdir(CSRC)) + ["../../include/backuwup_gpu.h"]
    for f in files:
        path = os.path.normpath(os.path.join(CSRC, f))
        if os.path.isfile(path) and not f.endswith((".tmp", ".o")):
            h.update(f.encode())
            h.update(open(path, "rb").read())
    return h.hexdigest()


def _stale(lib=LIB):
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    deps.append(os.path.join(HERE, "..", "include", "backuwup_gpu.h"))
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force=False, verbose=False, debug=False):
    lib = LIB_DEBUG if debug else LIB
    if not force and not _stale(lib):
        return lib
    cmd = [HIPCC, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wno-unused-value", "-Wno-unused-result", "-o", lib + ".tmp"]
    if debug:
        cmd += ["-DBW_DEBUG", "-g"]
    cmd += [os.path.join(CSRC, s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd, cwd=CSRC)
    os.replace(lib + ".tmp", lib)
    return lib


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, debug="--debug" in sys.argv))
