"""The C ABI boundary without a GPU: the library loads, exports every function that
include/*.h declares, and the ctypes/Python mirrors agree with the C struct layouts."""
import ctypes
import glob
import os
import re
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        txt = open(h).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?(?:int|void|char|uint\w+)\s*\*?\s*(bw_\w+)\s*\(", txt, re.M):
            names.add(m.group(1))
    return names


def test_header_declares_the_boundary():
    names = declared_functions()
    for required in ["bw_fastcdc_chunks", "bw_blake3_hash", "bw_blake3_hash_many", "bw_index_seed",
                     "bw_index_check_insert", "bw_process_files", "bw_process_files_device", "bw_results",
                     "bw_partition_by_owner", "bw_index_check_insert_device", "bw_scatter_verdicts"]:
        assert required in names


def test_library_exports_every_declared_symbol():
    from backuwup_amd import _lib
    lib = _lib.load()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    bound = {n for n, _, _ in _lib.SIGNATURES}
    assert declared_functions() == bound


def test_host_only_entry_points():
    from backuwup_amd import _lib
    lib = _lib.load()
    p = _lib.BwParams()
    lib.bw_params_default(ctypes.byref(p))
    assert (p.min_size, p.avg_size, p.max_size, p.small_file_threshold) == (262144, 1048576, 3145728, 1048576)
    assert lib.bw_strerror(-2) == b"output capacity too small"
    assert lib.bw_create(0, None) == _lib.BW_EINVAL


def test_struct_layout_matches_header(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "backuwup_gpu.h"\n'
                   'int main(void){printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(bw_blob), offsetof(bw_blob, digest),'
                   ' offsetof(bw_blob, is_dup), sizeof(bw_chunk), sizeof(bw_params),'
                   ' offsetof(bw_params, small_file_threshold)); return 0;}\n')
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    vals = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    from backuwup_amd import _lib
    from backuwup_amd.context import BLOB_DTYPE
    assert vals == [ctypes.sizeof(_lib.BwBlob), _lib.BwBlob.digest.offset, _lib.BwBlob.is_dup.offset,
                    ctypes.sizeof(_lib.BwChunk), ctypes.sizeof(_lib.BwParams), _lib.BwParams.small_file_threshold.offset]
    assert BLOB_DTYPE.itemsize == vals[0] and BLOB_DTYPE.fields["digest"][1] == vals[1]


def test_oracle_is_not_linked_by_the_product():
    """The product library must not reference the oracle (it is test infrastructure only)."""
    from backuwup_amd import _lib
    out = subprocess.check_output(["nm", "-D", _lib.LIB_PATH]).decode()
    assert "orc_" not in out
    for py in glob.glob(os.path.join(ROOT, "backuwup_amd", "*.py")):
        assert "oracle" not in open(py).read().replace("# oracle", ""), py


def test_missing_library_fails_loudly(monkeypatch):
    import importlib
    from backuwup_amd import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", "/nonexistent/libbackuwup_amd.so")
    with pytest.raises(RuntimeError):
        _lib.load()
    monkeypatch.undo()
    importlib.reload(_lib)


def test_blake3_module_validates_before_any_device_call():
    """backuwup_amd.blake3 (the blake3::hash mirror) rejects malformed batches on the host."""
    import numpy as np
    import pytest
    from backuwup_amd import blake3
    data = np.zeros(100, dtype=np.uint8)
    with pytest.raises(ValueError):
        blake3.hash_many(data, [0, 10], [5])
    with pytest.raises(ValueError):
        blake3.hash_many(data, [90], [11])
    with pytest.raises(TypeError):
        blake3.hash(np.zeros(4, dtype=np.uint32))



def test_fastcdc_mirror_validates_before_any_device_call():
    """backuwup_amd.fastcdc.FastCDC (the fastcdc::v2020 mirror) refuses sizes outside the crate's
    asserted ranges, and avg > max (the crate's cut() reads past max there), on the host."""
    import pytest
    from backuwup_amd.fastcdc import ChunkParameterError, FastCDC
    for bad in [(63, 256, 1024), (64, 255, 1024), (64, 256, 1023), (1 << 20 | 1, 4096, 8192), (64, 4096, 1024)]:
        with pytest.raises(ChunkParameterError):
            FastCDC(b"x" * 5000, *bad)
    assert issubclass(ChunkParameterError, ValueError)


_NULL_PROBE = """
import ctypes, sys
sys.path.insert(0, %r)
from backuwup_amd import _lib
L = _lib.load()
for name, res, argt in _lib.SIGNATURES:
    args = [t(0) if t in (ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_double) else None for t in argt]
    r = getattr(L, name)(*args)
    print(name, r if isinstance(r, (int, type(None))) else "ptr", flush=True)
print("@@done")
"""


def test_every_entry_point_survives_null_arguments():
    """The ABI never unwinds and never dereferences a missing argument: every exported function,
    called with null pointers and zero sizes (no GPU needed: the checks come first), returns
    BW_EINVAL or a harmless value instead of crashing."""
    import sys
    out = subprocess.run([sys.executable, "-c", _NULL_PROBE % ROOT], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and "@@done" in out.stdout, (out.stdout[-1500:], out.stderr[-1500:])
    from backuwup_amd import _lib
    rc = dict(l.split(" ", 1) for l in out.stdout.splitlines() if not l.startswith("@@"))
    benign = {"bw_zstd_store_size": "5", "bw_blake3_kept_hits": "0", "bw_blake3_coalesce_stats": "0",
              "bw_blake3_service_faults": "0"}  # a size, a counter, optional outputs
    for name, res, _ in _lib.SIGNATURES:
        if res is ctypes.c_int and name not in benign:
            assert rc[name] == str(_lib.BW_EINVAL), (name, rc[name])
        elif name in benign:
            assert rc[name] == benign[name], (name, rc[name])


def test_pool_device_list_from_environment(monkeypatch):
    """backuwup_amd.pool (the Rust crate's Pool policy): BACKUWUP_GPU_DEVICES lists devices (a device
    may repeat), the single BACKUWUP_GPU_DEVICE of earlier versions applies only when the list is
    unset; "all" / empty asks the library for the visible devices (bw_device_count: none here)."""
    import pytest
    from backuwup_amd.pool import devices_from_env
    monkeypatch.setenv("BACKUWUP_GPU_DEVICES", "0,0,3")
    monkeypatch.setenv("BACKUWUP_GPU_DEVICE", "5")
    assert devices_from_env() == [0, 0, 3]
    monkeypatch.delenv("BACKUWUP_GPU_DEVICES")
    assert devices_from_env() == [5]
    import ctypes
    from backuwup_amd import _lib
    n = ctypes.c_int()
    assert _lib.load().bw_device_count(ctypes.byref(n)) == 0
    for v in ("all", ""):
        monkeypatch.setenv("BACKUWUP_GPU_DEVICES", v)
        if n.value:
            assert devices_from_env() == list(range(n.value))
        else:
            with pytest.raises(RuntimeError):  # no GPU (the build container)
                devices_from_env()
