"""Independent AES-256-GCM for the seal parity tests: the system OpenSSL libcrypto (EVP API)
through ctypes.  Test infrastructure only; absent libcrypto -> tests that need it skip."""
import ctypes
import ctypes.util

_lib = None


def lib():
    global _lib
    if _lib is None:
        name = ctypes.util.find_library("crypto") or "libcrypto.so.3"
        L = ctypes.CDLL(name)
        vp, ip = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)
        L.EVP_CIPHER_CTX_new.restype = vp
        L.EVP_CIPHER_CTX_free.argtypes = [vp]
        L.EVP_aes_256_gcm.restype = vp
        L.EVP_EncryptInit_ex.argtypes = [vp, vp, vp, ctypes.c_char_p, ctypes.c_char_p]
        L.EVP_DecryptInit_ex.argtypes = [vp, vp, vp, ctypes.c_char_p, ctypes.c_char_p]
        L.EVP_EncryptUpdate.argtypes = [vp, ctypes.c_char_p, ip, ctypes.c_char_p, ctypes.c_int]
        L.EVP_DecryptUpdate.argtypes = [vp, ctypes.c_char_p, ip, ctypes.c_char_p, ctypes.c_int]
        L.EVP_EncryptFinal_ex.argtypes = [vp, ctypes.c_char_p, ip]
        L.EVP_DecryptFinal_ex.argtypes = [vp, ctypes.c_char_p, ip]
        L.EVP_CIPHER_CTX_ctrl.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp]
        _lib = L
    return _lib


EVP_CTRL_GCM_GET_TAG, EVP_CTRL_GCM_SET_TAG = 0x10, 0x11


def gcm_seal(key, nonce, pt):
    """AES-256-GCM, 96-bit nonce, empty AAD -> ciphertext || 16-byte tag."""
    L = lib()
    pt = bytes(pt)
    c = L.EVP_CIPHER_CTX_new()
    try:
        assert L.EVP_EncryptInit_ex(c, L.EVP_aes_256_gcm(), None, bytes(key), bytes(nonce)) == 1
        out = ctypes.create_string_buffer(len(pt) + 32)
        n = ctypes.c_int(0)
        if pt:
            assert L.EVP_EncryptUpdate(c, out, ctypes.byref(n), pt, len(pt)) == 1
        m = ctypes.c_int(0)
        assert L.EVP_EncryptFinal_ex(c, ctypes.cast(ctypes.byref(out, n.value), ctypes.c_char_p), ctypes.byref(m)) == 1
        tag = ctypes.create_string_buffer(16)
        assert L.EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_GET_TAG, 16, ctypes.cast(tag, ctypes.c_void_p)) == 1
        return out.raw[:n.value + m.value] + tag.raw
    finally:
        L.EVP_CIPHER_CTX_free(c)


def gcm_open(key, nonce, ct):
    """-> plaintext, or None if the tag does not verify."""
    L = lib()
    ct = bytes(ct)
    if len(ct) < 16:
        return None
    body, tag = ct[:-16], ct[-16:]
    c = L.EVP_CIPHER_CTX_new()
    try:
        assert L.EVP_DecryptInit_ex(c, L.EVP_aes_256_gcm(), None, bytes(key), bytes(nonce)) == 1
        out = ctypes.create_string_buffer(len(body) + 32)
        n = ctypes.c_int(0)
        if body:
            assert L.EVP_DecryptUpdate(c, out, ctypes.byref(n), body, len(body)) == 1
        tb = ctypes.create_string_buffer(tag, 16)
        L.EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_SET_TAG, 16, ctypes.cast(tb, ctypes.c_void_p))
        m = ctypes.c_int(0)
        ok = L.EVP_DecryptFinal_ex(c, ctypes.cast(ctypes.byref(out, n.value), ctypes.c_char_p), ctypes.byref(m))
        return out.raw[:n.value] if ok == 1 else None
    finally:
        L.EVP_CIPHER_CTX_free(c)
