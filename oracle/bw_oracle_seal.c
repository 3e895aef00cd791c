/*
 * bw_oracle_seal.c -- CPU restatement of backuwup's blob sealing and packfile/index formats
 * (SURVEY.md §8f rows 3 and 4).  TEST INFRASTRUCTURE ONLY: loaded by tests/ and bench.py's
 * cpu_baseline leg through oracle/oracle.py; the product library never links it.
 *
 * What it restates (reference call sites; the arithmetic lives in RustCrypto crates that are not
 * in /root/reference):
 *   - Manager::compress_encrypt_blob, client/src/backup/filesystem/packfile/pack.rs:58-80:
 *       key   = KeyManager::derive_backup_key(&blob.hash)   (key_manager.rs:80-86:
 *               Hkdf::<Sha256>::from_prk(backup_secret_key).expand(info, 32 bytes))
 *       data  = Aes256Gcm::new(key).encrypt_in_place(nonce, b"", data)  = ciphertext || tag
 *   - the header / index keys: derive_backup_key(b"header") (pack.rs:212-213),
 *     derive_backup_key(b"index") (blob_index.rs:185,207)
 *   - unpack.rs:58-63 / blob_index.rs:187-191: decrypt_in_place (tag verified)
 * Crates (Cargo.lock): aes-gcm 0.10, hkdf 0.12, sha2 0.10 -- standard AES-256 (FIPS-197),
 * GCM (NIST SP 800-38D, 96-bit IV, 128-bit tag), HKDF-Expand (RFC 5869), HMAC-SHA-256
 * (RFC 2104, FIPS 180-4).
 *
 * PARITY: the algorithms are standards, so this restatement is pinned by published known
 * answers (FIPS-197 C.3, the GCM spec's AES-256 test cases, RFC 5869 test case 1, FIPS 180-2
 * SHA-256 "abc") and checked against an independent implementation available offline (OpenSSL
 * libcrypto via ctypes, Python's hashlib/hmac) in tests/test_seal.py.  The reference's own tests
 * hold no vectors for these paths.
 *
 * Written for clarity, not speed: byte-oriented AES with a computed S-box and the bitwise GF(2^128)
 * multiply of SP 800-38D Algorithm 1.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "bw_oracle.h"

/* ------------------------------------------------------------------ SHA-256 (FIPS 180-4) */

static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha256_block(uint32_t h[8], const uint8_t p[64]) {
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
        w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 64; i++) {
        const uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
        const uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
    for (int i = 0; i < 64; i++) {
        const uint32_t t1 = k + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
        const uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        k = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += k;
}

typedef struct {
    uint32_t h[8];
    uint8_t buf[64];
    size_t nbuf;
    uint64_t total;
} sha256_ctx;

static void sha256_init(sha256_ctx* s) {
    static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    memcpy(s->h, iv, sizeof iv);
    s->nbuf = 0;
    s->total = 0;
}

static void sha256_update(sha256_ctx* s, const uint8_t* p, size_t n) {
    s->total += n;
    while (n) {
        size_t k = 64 - s->nbuf < n ? 64 - s->nbuf : n;
        memcpy(s->buf + s->nbuf, p, k);
        s->nbuf += k;
        p += k;
        n -= k;
        if (s->nbuf == 64) {
            sha256_block(s->h, s->buf);
            s->nbuf = 0;
        }
    }
}

static void sha256_final(sha256_ctx* s, uint8_t out[32]) {
    const uint64_t bits = s->total * 8;
    uint8_t pad = 0x80, z = 0;
    sha256_update(s, &pad, 1);
    while (s->nbuf != 56) sha256_update(s, &z, 1);
    uint8_t len[8];
    for (int i = 0; i < 8; i++) len[i] = (uint8_t)(bits >> (56 - 8 * i));
    sha256_update(s, len, 8);
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)(s->h[i] >> 24);
        out[4 * i + 1] = (uint8_t)(s->h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(s->h[i] >> 8);
        out[4 * i + 3] = (uint8_t)s->h[i];
    }
}

void orc_sha256(const uint8_t* data, size_t len, uint8_t out[32]) {
    sha256_ctx s;
    sha256_init(&s);
    sha256_update(&s, data, len);
    sha256_final(&s, out);
}

/* HMAC-SHA-256 (RFC 2104); keys longer than the block are hashed first */
void orc_hmac_sha256(const uint8_t* key, size_t klen, const uint8_t* msg, size_t mlen, uint8_t out[32]) {
    uint8_t k[64] = {0}, ip[64], op[64], inner[32];
    if (klen > 64) orc_sha256(key, klen, k);
    else memcpy(k, key, klen);
    for (int i = 0; i < 64; i++) { ip[i] = k[i] ^ 0x36; op[i] = k[i] ^ 0x5c; }
    sha256_ctx s;
    sha256_init(&s);
    sha256_update(&s, ip, 64);
    sha256_update(&s, msg, mlen);
    sha256_final(&s, inner);
    sha256_init(&s);
    sha256_update(&s, op, 64);
    sha256_update(&s, inner, 32);
    sha256_final(&s, out);
}

/* Hkdf::<Sha256>::from_prk(prk).expand(info, okm) with okm = 32 bytes: T(1) = HMAC(prk, info||1) */
void orc_hkdf_expand32(const uint8_t prk[32], const uint8_t* info, size_t info_len, uint8_t out[32]) {
    uint8_t* m = (uint8_t*)malloc(info_len + 1);
    memcpy(m, info, info_len);
    m[info_len] = 1;
    orc_hmac_sha256(prk, 32, m, info_len + 1, out);
    free(m);
}

/* ------------------------------------------------------------------ AES-256 (FIPS-197) */

static uint8_t SBOX[256];

static uint8_t xtime(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0)); }

static uint8_t gmul8(uint8_t a, uint8_t b) {
    uint8_t r = 0;
    while (b) {
        if (b & 1) r ^= a;
        a = xtime(a);
        b >>= 1;
    }
    return r;
}

static void sbox_init(void) {
    if (SBOX[0] == 0x63) return;
    for (int x = 0; x < 256; x++) {
        uint8_t inv = 0;  /* multiplicative inverse in GF(2^8), 0 -> 0 */
        for (int y = 1; y < 256 && x; y++)
            if (gmul8((uint8_t)x, (uint8_t)y) == 1) { inv = (uint8_t)y; break; }
        uint8_t s = inv, r = inv;
        for (int i = 0; i < 4; i++) {  /* affine map: s ^= rotl(inv, 1..4); s ^= 0x63 */
            r = (uint8_t)((r << 1) | (r >> 7));
            s ^= r;
        }
        SBOX[x] = s ^ 0x63;
    }
}

/* 15 round keys x 16 bytes */
static void aes256_expand(const uint8_t key[32], uint8_t rk[240]) {
    sbox_init();
    memcpy(rk, key, 32);
    uint8_t rcon = 1;
    for (int i = 8; i < 60; i++) {
        uint8_t t[4];
        memcpy(t, rk + 4 * (i - 1), 4);
        if (i % 8 == 0) {
            const uint8_t u = t[0];
            t[0] = SBOX[t[1]] ^ rcon; t[1] = SBOX[t[2]]; t[2] = SBOX[t[3]]; t[3] = SBOX[u];
            rcon = xtime(rcon);
        } else if (i % 8 == 4) {
            for (int j = 0; j < 4; j++) t[j] = SBOX[t[j]];
        }
        for (int j = 0; j < 4; j++) rk[4 * i + j] = rk[4 * (i - 8) + j] ^ t[j];
    }
}

static void aes256_block(const uint8_t rk[240], const uint8_t in[16], uint8_t out[16]) {
    uint8_t s[16];
    for (int i = 0; i < 16; i++) s[i] = in[i] ^ rk[i];
    for (int r = 1; r <= 14; r++) {
        uint8_t t[16];
        for (int i = 0; i < 16; i++) t[i] = SBOX[s[i]];
        for (int c = 0; c < 4; c++)  /* ShiftRows: row i of column c <- column c+i */
            for (int i = 0; i < 4; i++) s[4 * c + i] = t[4 * ((c + i) % 4) + i];
        if (r != 14)
            for (int c = 0; c < 4; c++) {  /* MixColumns */
                const uint8_t a0 = s[4 * c], a1 = s[4 * c + 1], a2 = s[4 * c + 2], a3 = s[4 * c + 3];
                s[4 * c] = xtime(a0) ^ (xtime(a1) ^ a1) ^ a2 ^ a3;
                s[4 * c + 1] = a0 ^ xtime(a1) ^ (xtime(a2) ^ a2) ^ a3;
                s[4 * c + 2] = a0 ^ a1 ^ xtime(a2) ^ (xtime(a3) ^ a3);
                s[4 * c + 3] = (xtime(a0) ^ a0) ^ a1 ^ a2 ^ xtime(a3);
            }
        for (int i = 0; i < 16; i++) s[i] ^= rk[16 * r + i];
    }
    memcpy(out, s, 16);
}

void orc_aes256_encrypt_block(const uint8_t key[32], const uint8_t in[16], uint8_t out[16]) {
    uint8_t rk[240];
    aes256_expand(key, rk);
    aes256_block(rk, in, out);
}

/* ------------------------------------------------------------------ GCM (SP 800-38D) */

/* Z = X * Y in GF(2^128), GCM bit order (Algorithm 1) */
static void gf_mul(const uint8_t X[16], const uint8_t Y[16], uint8_t Z[16]) {
    uint8_t z[16] = {0}, v[16];
    memcpy(v, Y, 16);
    for (int i = 0; i < 128; i++) {
        if (X[i / 8] & (0x80 >> (i % 8)))
            for (int j = 0; j < 16; j++) z[j] ^= v[j];
        const int lsb = v[15] & 1;
        for (int j = 15; j > 0; j--) v[j] = (uint8_t)((v[j] >> 1) | (v[j - 1] << 7));
        v[0] >>= 1;
        if (lsb) v[0] ^= 0xe1;
    }
    memcpy(Z, z, 16);
}

static void ghash_blocks(const uint8_t H[16], uint8_t Y[16], const uint8_t* p, size_t n) {
    for (size_t off = 0; off < n; off += 16) {
        uint8_t b[16] = {0};
        memcpy(b, p + off, n - off < 16 ? n - off : 16);
        for (int j = 0; j < 16; j++) Y[j] ^= b[j];
        gf_mul(Y, H, Y);
    }
}

/* AES-256-GCM with a 96-bit nonce and empty AAD; tag over the ciphertext.  dec = 0: in is the
 * plaintext, out receives ciphertext || tag; dec = 1: in holds len bytes of ciphertext, tag_in
 * the received tag, out the plaintext; returns 0 or -1 (tag mismatch). */
static int gcm_crypt(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* in, size_t len, uint8_t* out,
                     int dec, const uint8_t* tag_in, uint8_t* tag_out) {
    uint8_t rk[240], H[16] = {0}, J[16], E0[16], Y[16] = {0};
    aes256_expand(key, rk);
    aes256_block(rk, H, H);
    memcpy(J, nonce, 12);
    J[12] = 0; J[13] = 0; J[14] = 0; J[15] = 1;
    aes256_block(rk, J, E0);
    if (dec) ghash_blocks(H, Y, in, len);
    for (size_t off = 0; off < len; off += 16) {
        uint32_t c = (uint32_t)J[12] << 24 | (uint32_t)J[13] << 16 | (uint32_t)J[14] << 8 | J[15];
        c++;  /* inc32 */
        J[12] = (uint8_t)(c >> 24); J[13] = (uint8_t)(c >> 16); J[14] = (uint8_t)(c >> 8); J[15] = (uint8_t)c;
        uint8_t ks[16];
        aes256_block(rk, J, ks);
        for (size_t j = 0; j < 16 && off + j < len; j++) out[off + j] = in[off + j] ^ ks[j];
    }
    if (!dec) ghash_blocks(H, Y, out, len);
    uint8_t L[16] = {0};
    const uint64_t bits = (uint64_t)len * 8;  /* len(A) = 0 || len(C) in bits, big-endian */
    for (int j = 0; j < 8; j++) L[8 + j] = (uint8_t)(bits >> (56 - 8 * j));
    ghash_blocks(H, Y, L, 16);
    uint8_t T[16];
    for (int j = 0; j < 16; j++) T[j] = Y[j] ^ E0[j];
    if (dec) {
        uint8_t d = 0;
        for (int j = 0; j < 16; j++) d |= T[j] ^ tag_in[j];
        return d ? -1 : 0;
    }
    memcpy(tag_out, T, 16);
    return 0;
}

void orc_aes256_gcm_seal(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* pt, size_t len,
                         uint8_t* out) {
    gcm_crypt(key, nonce, pt, len, out, 0, NULL, out + len);
}

int orc_aes256_gcm_open(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* ct, size_t len_with_tag,
                        uint8_t* out) {
    if (len_with_tag < 16) return -1;
    const size_t len = len_with_tag - 16;
    return gcm_crypt(key, nonce, ct, len, out, 1, ct + len, NULL);
}

/* compress_encrypt_blob's key derivation + encryption (pack.rs:70-80) for an already
 * compressed payload: out = AES-256-GCM(HKDF-Expand(prk, info, 32), nonce).seal(payload) */
void orc_seal_blob(const uint8_t prk[32], const uint8_t* info, size_t info_len, const uint8_t nonce[12],
                   const uint8_t* payload, size_t len, uint8_t* out) {
    uint8_t key[32];
    orc_hkdf_expand32(prk, info, info_len, key);
    orc_aes256_gcm_seal(key, nonce, payload, len, out);
}

int orc_open_blob(const uint8_t prk[32], const uint8_t* info, size_t info_len, const uint8_t nonce[12],
                  const uint8_t* sealed, size_t len_with_tag, uint8_t* out) {
    uint8_t key[32];
    orc_hkdf_expand32(prk, info, info_len, key);
    return orc_aes256_gcm_open(key, nonce, sealed, len_with_tag, out);
}
