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
SOURCES = ["bw_capi.hip", "bw_cdc.hip", "bw_blake3.hip", "bw_dedup.hip", "bw_comm.hip", "bw_tree.hip", "bw_seal.hip",
           "bw_pack.hip", "bw_zstd.hip", "bw_dropin.hip", "bw_stream.hip", "bw_capi_pack.hip", "bw_b3_small.hip"]
HEADERS = ["backuwup_gpu.h", "backuwup_gpu_pack.h"]  # include/
ROCM_LIB = "/opt/rocm/lib"
ARCH = os.environ.get("BW_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


# sources that are not on the chunk -> hash -> dedup path the bench profiles (their kernels never
# run in the C2 command), so editing them does not make the committed PMC traffic stale; the write
# side's C ABI (bw_capi_pack.hip, include/backuwup_gpu_pack.h) and the drop-ins' small-message
# hashing (bw_b3_small.hip) are outside the digest too
OFF_PATH = ("bw_zstd.hip", "bw_seal.hip", "bw_pack.hip", "bw_tree.hip", "bw_comm.hip", "bw_dropin.hip", "bw_stream.hip",
            "bw_capi_pack.hip", "bw_b3_small.hip", "bw_b3_small.h")


def _code_only(text):
    """The source without its comments and blank space: documentation edits do not change what ran."""
    import re
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    text = re.sub(r"//[^\n]*", " ", text)
    return " ".join(text.split())


def source_digest():
    """sha256 over the code (comments stripped) of the hot path's sources (csrc/* minus OFF_PATH,
    and the hot path's C ABI header): identifies the kernels a profile was taken with
    (profiles/pmc_traffic.json), so bench.py can tell stale evidence."""
    import hashlib
    h = hashlib.sha256()
    files = [f for f in sorted(os.listdir(CSRC)) if f not in OFF_PATH] + ["../../include/backuwup_gpu.h"]
    for f in files:
        path = os.path.normpath(os.path.join(CSRC, f))
        if os.path.isfile(path) and not f.endswith((".tmp", ".o")):
            h.update(f.encode())
            h.update(_code_only(open(path, encoding="utf-8", errors="replace").read()).encode())
    return h.hexdigest()


def _stale(lib=LIB):
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    deps += [os.path.join(HERE, "..", "include", h) for h in HEADERS]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force=False, verbose=False, debug=False, jobs=8, variant=None, defines=()):
    """One object per source, compiled in parallel under build/ (an unchanged source whose object
    is newer than every header is not recompiled unless force), then one shared link.
    variant="name" with defines=("-DX", ...) builds a diagnostic library libbackuwup_amd_<name>.so
    (loaded only through BW_LIB by tools, never by the product path)."""
    from concurrent.futures import ThreadPoolExecutor
    lib = LIB_DEBUG if debug else (os.path.join(HERE, "libbackuwup_amd_%s.so" % variant) if variant else LIB)
    if not force and not _stale(lib):
        return lib
    odir = os.path.join(HERE, "..", "build", "debug" if debug else (variant or "release"))
    os.makedirs(odir, exist_ok=True)
    flags = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-Wno-unused-value", "-Wno-unused-result"]
    flags += list(defines)
    if debug:
        flags += ["-DBW_DEBUG", "-DBW_DIAG=1", "-g"]  # asserts + the diagnostic kernel variants
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".h", ".inc"))]
    headers += [os.path.join(HERE, "..", "include", h) for h in HEADERS]
    newest_hdr = max(os.path.getmtime(h) for h in headers)

    def compile_one(src):
        path = os.path.join(CSRC, src)
        obj = os.path.join(odir, src.replace(".hip", ".o"))
        if not force and os.path.exists(obj) and os.path.getmtime(obj) > max(os.path.getmtime(path), newest_hdr):
            return obj
        cmd = [HIPCC] + flags + ["-c", "-o", obj + ".tmp", path]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd, cwd=CSRC)
        os.replace(obj + ".tmp", obj)
        return obj

    with ThreadPoolExecutor(max_workers=max(1, min(jobs, len(SOURCES)))) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    # RCCL for the digest exchange (bw_comm.hip); under torch the process's already-loaded librccl.so.1
    # (same soname) is the one bound, so a process holds one RCCL
    cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", lib + ".tmp"] + objs + \
        ["-L" + ROCM_LIB, "-lrccl", "-Wl,-rpath," + ROCM_LIB]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd, cwd=CSRC)
    os.replace(lib + ".tmp", lib)
    return lib


if __name__ == "__main__":
    if "--clock" in sys.argv:  # clock stamps around scan tiles and leaf-pass waves (tools/clock_windows.py)
        print(build(force="--force" in sys.argv, verbose=True, variant="clock", defines=("-DBW_CLOCK_STAMPS=1",)))
    elif "--ztime" in sys.argv:  # zstd parse section timers (tools/zstd_bench.py --timing)
        print(build(force="--force" in sys.argv, verbose=True, variant="ztime", defines=("-DBW_ZSTD_TIMING",)))
    else:
        print(build(force="--force" in sys.argv, verbose=True, debug="--debug" in sys.argv))
