"""Blob sealing: derive_backup_key (key_manager.rs:80-86, HKDF-SHA-256
expand of the blob hash) + Aes256Gcm::encrypt_in_place (pack.rs:70-80), and the inverse
(unpack.rs:58-63, blob_index.rs:185-191).

CPU tests pin the oracle (oracle/bw_oracle_seal.c) to published known answers and to two
independent implementations available offline: OpenSSL libcrypto (tests/openssl_ref.py) and
Python's hashlib/hmac.  GPU tests compare the HIP path (through the C ABI) with the oracle and
OpenSSL bit for bit: ciphertext and tag, across the piece / block / partial-block edges of the
kernels, many items per call, and tag verification on open.
"""
import hashlib
import hmac
import os

import numpy as np
import pytest

from backuwup_amd.synth import splitmix_bytes

PRK = bytes.fromhex("a5" * 32)

# ------------------------------------------------------------------ known answers (CPU)

# FIPS-197 Appendix C.3 (AES-256)
AES_KAT = ("000102030405060708090a0b0c0d0e0f101112131415161718191a1b1c1d1e1f",
           "00112233445566778899aabbccddeeff", "8ea2b7ca516745bfeafc49904b496089")
# GCM spec (McGrew & Viega) AES-256 test cases 13, 14, 15: (key, iv, plaintext, ciphertext||tag)
GCM_KAT = [
    ("00" * 32, "00" * 12, "", "530f8afbc74536b9a963b4f1c4cb738b"),
    ("00" * 32, "00" * 12, "00" * 16, "cea7403d4d606b6e074ec5d3baf39d18d0d1c8a799996bf0265b98b5d48ab919"),
    ("feffe9928665731c6d6a8f9467308308feffe9928665731c6d6a8f9467308308", "cafebabefacedbaddecaf888",
     "d9313225f88406e5a55909c5aff5269a86a7a9531534f7da2e4c303d8a318a721c3c0c95956809532fcf0e2449a6b525b16aedf5aa0de"
     "657ba637b391aafd255",
     "522dc1f099567d07f47f37a32a84427d643a8cdcbfe5c0c97598a2bd2555d1aa8cb08e48590dbb3da7b08b1056828838c5f61e6393ba7a0"
     "abcc9f662898015adb094dac5d93471bdec1a502270e3cc6c"),
]


def _ssl():
    try:
        import openssl_ref
        openssl_ref.lib()
        return openssl_ref
    except OSError:
        pytest.skip("OpenSSL libcrypto not available")


def test_sha256_hmac_match_hashlib(oracle):
    assert oracle.sha256(b"abc").hex() == "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"
    rng = np.random.default_rng(5)
    for n in (0, 1, 55, 56, 63, 64, 65, 1000):
        m = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert oracle.sha256(m) == hashlib.sha256(m).digest()
        for klen in (0, 32, 64, 65):
            k = bytes(range(klen))
            assert oracle.hmac_sha256(k, m) == hmac.new(k, m, hashlib.sha256).digest()


def test_hkdf_expand_rfc5869_case1(oracle):
    # RFC 5869 A.1: PRK = HMAC(salt, IKM); OKM[0:32] is what expand(info, [u8; 32]) returns
    prk = hmac.new(bytes(range(13)), b"\x0b" * 22, hashlib.sha256).digest()
    assert prk.hex() == "077709362c2e32df0ddc3f0dc47bba6390b6c73bb50f9c3122ec844ad7c2b3e5"
    okm = oracle.hkdf_expand32(prk, bytes(range(0xf0, 0xfa)))
    assert okm.hex() == "3cb25f25faacd57a90434f64d0362f2a2d2d0a90cf1a5a4c5db02d56ecc4c5bf"
    # T(1) = HMAC(prk, info || 0x01) for the infos the reference uses
    for info in (b"header", b"index", bytes(range(32))):
        assert oracle.hkdf_expand32(PRK, info) == hmac.new(PRK, info + b"\x01", hashlib.sha256).digest()


def test_aes_and_gcm_known_answers(oracle):
    k, p, c = AES_KAT
    assert oracle.aes256_block(bytes.fromhex(k), bytes.fromhex(p)).hex() == c
    for key, iv, pt, want in GCM_KAT:
        key, iv, pt = bytes.fromhex(key), bytes.fromhex(iv), bytes.fromhex(pt)
        assert oracle.gcm_seal(key, iv, pt).hex() == want
        assert oracle.gcm_open(key, iv, bytes.fromhex(want)) == pt


def test_gcm_oracle_matches_openssl(oracle):
    ssl = _ssl()
    rng = np.random.default_rng(7)
    for n in (0, 1, 15, 16, 17, 255, 4096, 65536 + 3):
        key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
        pt = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        ct = oracle.gcm_seal(key, iv, pt)
        assert ct == ssl.gcm_seal(key, iv, pt)
        assert ssl.gcm_open(key, iv, ct) == pt
        bad = bytearray(ct)
        bad[len(bad) // 2] ^= 0x40
        assert oracle.gcm_open(key, iv, bytes(bad)) is None and ssl.gcm_open(key, iv, bytes(bad)) is None


# ------------------------------------------------------------------ GPU parity

# 16-byte blocks per GPU wave task (bw_seal.hip PIECE_BLOCKS): sizes around its multiples
PIECE = 8192 * 16
EDGE_LENS = [0, 1, 15, 16, 17, 63, 64, 65, 1023, 1024, 1025, 16 * 63, 16 * 64, 16 * 64 + 1, PIECE - 1, PIECE,
             PIECE + 1, PIECE + 16, 2 * PIECE - 5, 3 * PIECE + 7, 262144, 1048576 + 13, 3145728]


def _items(lens, seed, info_len=32, gap=0):
    """Payload buffer with items back to back (optional gaps), hashes as infos, nonces."""
    lens = np.asarray(lens, dtype=np.uint64)
    off = np.zeros(len(lens), dtype=np.uint64)
    pos = 0
    for i, n in enumerate(lens):
        off[i] = pos
        pos += int(n) + gap
    data = splitmix_bytes(seed, max(pos, 1))
    rng = np.random.default_rng(seed)
    infos = rng.integers(0, 256, (len(lens), info_len), dtype=np.uint8)
    nonces = rng.integers(0, 256, (len(lens), 12), dtype=np.uint8)
    return data, off, lens, infos, nonces


def _sealed_layout(lens):
    dst_off = np.zeros(len(lens), dtype=np.uint64)
    pos = 0
    for i, n in enumerate(lens):
        dst_off[i] = pos
        pos += int(n) + 16
    return dst_off, pos


@pytest.mark.gpu
def test_seal_matches_oracle_edges(ctx, oracle):
    data, off, lens, infos, nonces = _items(EDGE_LENS, 11, gap=3)  # gaps: unaligned item starts
    dst_off, size = _sealed_layout(lens)
    out = ctx.seal(PRK, data, off, lens, infos, nonces, dst_off, size)
    for i in range(len(lens)):
        pt = data[int(off[i]):int(off[i] + lens[i])]
        want = oracle.seal_blob(PRK, bytes(infos[i]), bytes(nonces[i]), pt)
        got = out[int(dst_off[i]):int(dst_off[i]) + int(lens[i]) + 16].tobytes()
        assert got == want, (i, int(lens[i]))


@pytest.mark.gpu
def test_seal_matches_openssl_many_small(ctx, oracle):
    ssl = _ssl()
    rng = np.random.default_rng(3)
    lens = rng.integers(0, 70000, 300)
    data, off, lens, infos, nonces = _items(lens, 12)
    dst_off, size = _sealed_layout(lens)
    out = ctx.seal(PRK, data, off, lens, infos, nonces, dst_off, size)
    for i in range(len(lens)):
        pt = data[int(off[i]):int(off[i] + lens[i])].tobytes()
        key = oracle.hkdf_expand32(PRK, bytes(infos[i]))
        assert key == hmac.new(PRK, bytes(infos[i]) + b"\x01", hashlib.sha256).digest()
        got = out[int(dst_off[i]):int(dst_off[i]) + len(pt) + 16].tobytes()
        assert got == ssl.gcm_seal(key, bytes(nonces[i]), pt), i


@pytest.mark.gpu
def test_open_round_trip_and_tamper(ctx):
    lens = [0, 5, 16, 100000, PIECE + 1, 3 * PIECE]
    data, off, lens, infos, nonces = _items(lens, 13)
    dst_off, size = _sealed_layout(lens)
    sealed = ctx.seal(PRK, data, off, lens, infos, nonces, dst_off, size)
    slen = lens + 16
    plain, ok = ctx.seal(PRK, sealed, dst_off, slen, infos, nonces, off, int(off[-1] + lens[-1]), open_=True)
    assert ok.tolist() == [1] * len(lens)
    assert np.array_equal(plain, data[:len(plain)])
    # flip one bit in item 3's ciphertext and one in item 4's tag; wrong nonce for item 5
    bad = sealed.copy()
    bad[int(dst_off[3]) + 777] ^= 1
    bad[int(dst_off[4] + lens[4]) + 15] ^= 0x80
    n2 = nonces.copy()
    n2[5, 0] ^= 1
    _, ok = ctx.seal(PRK, bad, dst_off, slen, infos, n2, off, int(off[-1] + lens[-1]), open_=True)
    assert ok.tolist() == [1, 1, 1, 0, 0, 0]


@pytest.mark.gpu
def test_header_and_index_keys(ctx, oracle):
    # serialize_packfile (pack.rs:212-217): key from b"header", nonce = packfile id;
    # BlobIndex::flush (blob_index.rs:205-213): key from b"index", nonce = file number LE || 0^8
    for info, nonce in ((b"header", bytes(range(12))), (b"index", (7).to_bytes(4, "little") + bytes(8))):
        pt = splitmix_bytes(len(info), 5000)
        out = ctx.seal(PRK, pt, [0], [len(pt)], [np.frombuffer(info, np.uint8)], [np.frombuffer(nonce, np.uint8)],
                       [0], len(pt) + 16)
        assert out.tobytes() == oracle.seal_blob(PRK, info, nonce, pt)


@pytest.mark.gpu
def test_seal_device_resident(ctx, oracle):
    import torch
    lens = [1 << 20, 333, 2 * PIECE + 9]
    data, off, lens, infos, nonces = _items(lens, 14)
    dst_off, size = _sealed_layout(lens)
    d_src = torch.from_numpy(data).cuda()
    d_dst = torch.zeros(size, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    ctx.seal_device(PRK, d_src.data_ptr(), off, lens, infos, nonces, d_dst.data_ptr(), dst_off)
    torch.cuda.synchronize()
    out = d_dst.cpu().numpy()
    for i in range(len(lens)):
        pt = data[int(off[i]):int(off[i] + lens[i])]
        assert out[int(dst_off[i]):int(dst_off[i]) + int(lens[i]) + 16].tobytes() == \
            oracle.seal_blob(PRK, bytes(infos[i]), bytes(nonces[i]), pt)


@pytest.mark.gpu
def test_seal_argument_errors(ctx):
    from backuwup_amd._lib import BW_EINVAL, BwError
    with pytest.raises(BwError) as e:  # info longer than one HMAC block holds
        ctx.seal(PRK, b"x" * 10, [0], [10], [np.zeros(55, np.uint8)], [np.zeros(12, np.uint8)], [0], 26)
    assert e.value.rc == BW_EINVAL
    with pytest.raises(BwError) as e:  # shorter than a tag: decrypt_in_place would fail
        ctx.seal(PRK, b"x" * 10, [0], [10], [np.zeros(32, np.uint8)], [np.zeros(12, np.uint8)], [0], 10,
                 open_=True)
    assert e.value.rc == BW_EINVAL
