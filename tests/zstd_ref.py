"""The system libzstd through ctypes, configured as the reference's Compressor / Decompressor
(pack.rs:58-64: level 3, no checksum, no content size, no magic bytes; unpack.rs:66-68).
Test infrastructure only: it pins the zstd store frames of oracle/pack_oracle.py and decodes
the payloads of GPU-built packfiles.  The image has libzstd 1.4.8; the reference links zstd
1.5.5 (zstd-sys, Cargo.lock:2760).  Absent libzstd -> the tests that need it skip."""
import ctypes
import ctypes.util

ZSTD_c_compressionLevel, ZSTD_c_contentSizeFlag, ZSTD_c_checksumFlag = 100, 200, 201
ZSTD_c_format = 10      # ZSTD_c_experimentalParam2
ZSTD_d_format = 1000    # ZSTD_d_experimentalParam1
ZSTD_f_zstd1_magicless = 1

_lib = None


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(ctypes.util.find_library("zstd") or "libzstd.so.1")
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        L.ZSTD_createCCtx.restype = vp
        L.ZSTD_freeCCtx.argtypes = [vp]
        L.ZSTD_createDCtx.restype = vp
        L.ZSTD_freeDCtx.argtypes = [vp]
        L.ZSTD_CCtx_setParameter.argtypes = [vp, ctypes.c_int, ctypes.c_int]
        L.ZSTD_CCtx_setParameter.restype = sz
        L.ZSTD_DCtx_setParameter.argtypes = [vp, ctypes.c_int, ctypes.c_int]
        L.ZSTD_DCtx_setParameter.restype = sz
        L.ZSTD_compress2.argtypes = [vp, vp, sz, vp, sz]
        L.ZSTD_compress2.restype = sz
        L.ZSTD_decompressDCtx.argtypes = [vp, vp, sz, vp, sz]
        L.ZSTD_decompressDCtx.restype = sz
        L.ZSTD_compressBound.argtypes = [sz]
        L.ZSTD_compressBound.restype = sz
        L.ZSTD_isError.argtypes = [sz]
        L.ZSTD_isError.restype = ctypes.c_uint
        L.ZSTD_versionNumber.restype = ctypes.c_uint
        _lib = L
    return _lib


def available():
    try:
        lib()
        return True
    except OSError:
        return False


def version():
    return lib().ZSTD_versionNumber()


def compress(data, level=3):
    """zstd::bulk::Compressor::new(3) + include_checksum/contentsize/magicbytes(false)."""
    L = lib()
    c = L.ZSTD_createCCtx()
    try:
        for p, v in [(ZSTD_c_compressionLevel, level), (ZSTD_c_contentSizeFlag, 0), (ZSTD_c_checksumFlag, 0),
                     (ZSTD_c_format, ZSTD_f_zstd1_magicless)]:
            assert not L.ZSTD_isError(L.ZSTD_CCtx_setParameter(c, p, v))
        data = bytes(data)
        cap = L.ZSTD_compressBound(len(data))
        out = ctypes.create_string_buffer(cap)
        n = L.ZSTD_compress2(c, out, cap, data, len(data))
        assert not L.ZSTD_isError(n)
        return out.raw[:n]
    finally:
        L.ZSTD_freeCCtx(c)


def decompress(frame, capacity=3 * 1024 * 1024):
    """zstd::bulk::Decompressor with include_magicbytes(false), capacity BLOB_MAX_UNCOMPRESSED_SIZE."""
    L = lib()
    d = L.ZSTD_createDCtx()
    try:
        assert not L.ZSTD_isError(L.ZSTD_DCtx_setParameter(d, ZSTD_d_format, ZSTD_f_zstd1_magicless))
        frame = bytes(frame)
        out = ctypes.create_string_buffer(max(capacity, 1))
        n = L.ZSTD_decompressDCtx(d, out, capacity, frame, len(frame))
        if L.ZSTD_isError(n):
            raise ValueError("zstd error")
        return out.raw[:n]
    finally:
        L.ZSTD_freeDCtx(d)
