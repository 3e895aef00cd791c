// bw_seal.hip -- per-blob sealing on gfx950: HKDF-SHA-256 key derivation + AES-256-GCM.
//
// Replaces the encryption half of Manager::compress_encrypt_blob (client/src/backup/filesystem/
// packfile/pack.rs:70-80):
//     key  = KEYS.derive_backup_key(&blob.hash)      key_manager.rs:80-86:
//            Hkdf::<Sha256>::from_prk(backup_secret_key).expand(info, [0u8; 32])
//     data = Aes256Gcm::new(key).encrypt_in_place(nonce, b"", data)   -> ciphertext || tag
// and its inverse (unpack.rs:58-63, blob_index.rs:185-191).  Crates aes-gcm 0.10 / hkdf 0.12 /
// sha2 0.10: standard AES-256, GCM with a 96-bit nonce and a 128-bit tag, RFC 5869 HKDF-Expand
// (L = 32 is one HMAC-SHA-256 block: T(1) = HMAC(prk, info || 0x01)).
//
//   k_seal_prep  one lane per item: HMAC-SHA-256 (the pads' states come from the host), AES-256
//                key schedule, H = E(0), E(J0), and the GHASH multipliers H^(2^k) (k <= 5),
//                H^64 and H^PIECE_BLOCKS.
//   k_seal_ctr   one wave per piece (up to PIECE_BLOCKS 16-byte blocks of one item): CTR
//                keystream + xor, and the piece's GHASH partial.  Lane l takes blocks
//                l, l+64, l+128, ... (every load and store is a coalesced 1 KiB per wave); each
//                lane runs Horner with the multiplier H^64 (Shoup 8-bit table in LDS, built per
//                piece), and a 6-level shuffle tree folds the 64 lane partials with H^(2^k)
//                (Shoup 4-bit tables).  AES is T-table: Te0 and Te1 as 32 lane replicas per
//                256-byte row at LDS address 0, so one v_perm_b32 forms a conflict-free lookup
//                address and Te1 is the same address + 128 (ds_read offset); Te2/Te3 are one
//                rotation of (Te0 ^ Te1) terms.
//   k_seal_tag   one lane per item: folds the piece partials with H^PIECE_BLOCKS (pieces are
//                cut from the item's end, so only the first is ragged), appends the length block and masks with E(J0); sealing
//                stores the tag after the ciphertext, opening compares it (ok flag).
//
// GF(2^128) elements are four big-endian words w0..w3 of the block (GCM bit order: the MSB of
// w0 is the coefficient of x^0); multiplication by x is a right shift by one with 0xE1 << 120
// folded in.
#include "bw_device.h"
#include "bw_internal.h"

#include <string.h>

namespace bw {

// ------------------------------------------------------------------ SHA-256 (FIPS 180-4)
__constant__ uint32_t c_k256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static const uint32_t h_k256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__host__ __device__ __forceinline__ uint32_t ror32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

template <typename KT>
__host__ __device__ __forceinline__ void sha256_compress(uint32_t h[8], const uint32_t in[16], const KT& K) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = in[i];
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            const uint32_t x = w[(i - 15) & 15], y = w[(i - 2) & 15];
            const uint32_t s0 = ror32(x, 7) ^ ror32(x, 18) ^ (x >> 3);
            const uint32_t s1 = ror32(y, 17) ^ ror32(y, 19) ^ (y >> 10);
            wi = w[i & 15] = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
        }
        const uint32_t t1 = k + (ror32(e, 6) ^ ror32(e, 11) ^ ror32(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + wi;
        const uint32_t t2 = (ror32(a, 2) ^ ror32(a, 13) ^ ror32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        k = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += k;
}

// ------------------------------------------------------------------ GF(2^128), GCM bit order
struct G4 {
    uint32_t w0, w1, w2, w3;
};

__device__ __forceinline__ G4 gxor(G4 a, G4 b) { return {a.w0 ^ b.w0, a.w1 ^ b.w1, a.w2 ^ b.w2, a.w3 ^ b.w3}; }

__device__ __forceinline__ G4 gmulx(G4 v) {
    const uint32_t lsb = v.w3 & 1;
    G4 r;
    r.w3 = __builtin_amdgcn_alignbit(v.w2, v.w3, 1);
    r.w2 = __builtin_amdgcn_alignbit(v.w1, v.w2, 1);
    r.w1 = __builtin_amdgcn_alignbit(v.w0, v.w1, 1);
    r.w0 = (v.w0 >> 1) ^ (lsb ? 0xe1000000u : 0u);
    return r;
}

// bitwise X * Y (SP 800-38D Algorithm 1): setup and the tag fold only, never per data block
__device__ G4 gmul_slow(G4 x, G4 y) {
    G4 z = {0, 0, 0, 0}, v = y;
    const uint32_t xw[4] = {x.w0, x.w1, x.w2, x.w3};
#pragma unroll
    for (int k = 0; k < 4; k++)
        for (int b = 31; b >= 0; b--) {
            const uint32_t m = 0u - ((xw[k] >> b) & 1u);
            z.w0 ^= v.w0 & m; z.w1 ^= v.w1 & m; z.w2 ^= v.w2 & m; z.w3 ^= v.w3 & m;
            v = gmulx(v);
        }
    return z;
}

// ------------------------------------------------------------------ AES-256 helpers
__device__ __forceinline__ uint32_t gf8_mul(uint32_t a, uint32_t b) {
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        r ^= (b & 1) ? a : 0;
        a = ((a << 1) ^ ((a & 0x80) ? 0x1b : 0)) & 0xff;
        b >>= 1;
    }
    return r;
}

// FIPS-197 S-box: affine map of the multiplicative inverse (x^254 in GF(2^8); 0 -> 0)
__device__ uint32_t aes_sbox(uint32_t x) {
    uint32_t x2 = gf8_mul(x, x), x3 = gf8_mul(x2, x), x6 = gf8_mul(x3, x3), x7 = gf8_mul(x6, x);
    uint32_t x14 = gf8_mul(x7, x7), x15 = gf8_mul(x14, x), x30 = gf8_mul(x15, x15), x31 = gf8_mul(x30, x);
    uint32_t x62 = gf8_mul(x31, x31), x63 = gf8_mul(x62, x), x126 = gf8_mul(x63, x63), x127 = gf8_mul(x126, x);
    const uint32_t inv = gf8_mul(x127, x127);  // x^254
    uint32_t s = inv, r = inv;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        r = ((r << 1) | (r >> 7)) & 0xff;
        s ^= r;
    }
    return s ^ 0x63;
}

// Te0[x] = (2s, s, s, 3s) big-endian, s = S[x]
__device__ __forceinline__ uint32_t aes_te0(uint32_t s) {
    const uint32_t s2 = ((s << 1) ^ ((s & 0x80) ? 0x1b : 0)) & 0xff;
    return (s2 << 24) | (s << 16) | (s << 8) | (s2 ^ s);
}

__device__ __forceinline__ void st4(uint32_t* d, G4 v) { d[0] = v.w0; d[1] = v.w1; d[2] = v.w2; d[3] = v.w3; }
__device__ __forceinline__ G4 ld4(const uint32_t* s) { return {s[0], s[1], s[2], s[3]}; }

// plain (unreplicated) T-table AES for the prep kernel
__device__ void aes_encrypt_plain(const uint32_t rk[60], const uint32_t* te, const uint32_t in[4], uint32_t out[4]) {
    uint32_t s0 = in[0] ^ rk[0], s1 = in[1] ^ rk[1], s2 = in[2] ^ rk[2], s3 = in[3] ^ rk[3];
#define TE(x, r) ror32(te[(x) & 0xff], (r))
    for (int r = 1; r < 14; r++) {
        const uint32_t t0 = TE(s0 >> 24, 0) ^ TE(s1 >> 16, 8) ^ TE(s2 >> 8, 16) ^ TE(s3, 24) ^ rk[4 * r];
        const uint32_t t1 = TE(s1 >> 24, 0) ^ TE(s2 >> 16, 8) ^ TE(s3 >> 8, 16) ^ TE(s0, 24) ^ rk[4 * r + 1];
        const uint32_t t2 = TE(s2 >> 24, 0) ^ TE(s3 >> 16, 8) ^ TE(s0 >> 8, 16) ^ TE(s1, 24) ^ rk[4 * r + 2];
        const uint32_t t3 = TE(s3 >> 24, 0) ^ TE(s0 >> 16, 8) ^ TE(s1 >> 8, 16) ^ TE(s2, 24) ^ rk[4 * r + 3];
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
#undef TE
#define SB(x) ((te[(x) & 0xff] >> 16) & 0xff)
    out[0] = ((SB(s0 >> 24) << 24) | (SB(s1 >> 16) << 16) | (SB(s2 >> 8) << 8) | SB(s3)) ^ rk[56];
    out[1] = ((SB(s1 >> 24) << 24) | (SB(s2 >> 16) << 16) | (SB(s3 >> 8) << 8) | SB(s0)) ^ rk[57];
    out[2] = ((SB(s2 >> 24) << 24) | (SB(s3 >> 16) << 16) | (SB(s0 >> 8) << 8) | SB(s1)) ^ rk[58];
    out[3] = ((SB(s3 >> 24) << 24) | (SB(s0 >> 16) << 16) | (SB(s1 >> 8) << 8) | SB(s2)) ^ rk[59];
#undef SB
}

// ------------------------------------------------------------------ k_seal_prep
__global__ __launch_bounds__(256) void k_seal_prep(const SealItem* __restrict__ items, uint64_t n, SealPads pads,
                                                   SealKey* __restrict__ keys) {
    __shared__ uint32_t s_te[256];
    s_te[threadIdx.x] = aes_te0(aes_sbox(threadIdx.x));
    __syncthreads();
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const SealItem& it = items[i];
    // HMAC inner: SHA-256(K ^ ipad || info || 0x01), the ipad block already compressed
    uint32_t m[16];
#pragma unroll
    for (int w = 0; w < 16; w++) m[w] = 0;
    const uint32_t il = it.info_len;
    for (uint32_t k = 0; k < il; k++) m[k >> 2] |= (uint32_t)it.info[k] << (24 - 8 * (k & 3));
    m[il >> 2] |= 0x01u << (24 - 8 * (il & 3));
    m[(il + 1) >> 2] |= 0x80u << (24 - 8 * ((il + 1) & 3));
    m[15] = (64 + il + 1) * 8;
    uint32_t h[8];
#pragma unroll
    for (int w = 0; w < 8; w++) h[w] = pads.istate[w];
    sha256_compress(h, m, c_k256);
    // HMAC outer: SHA-256(K ^ opad || inner)
#pragma unroll
    for (int w = 0; w < 8; w++) m[w] = h[w];
    m[8] = 0x80000000u;
#pragma unroll
    for (int w = 9; w < 15; w++) m[w] = 0;
    m[15] = (64 + 32) * 8;
#pragma unroll
    for (int w = 0; w < 8; w++) h[w] = pads.ostate[w];
    sha256_compress(h, m, c_k256);
    // AES-256 key schedule: the key bytes are the HMAC output, big-endian words
    uint32_t rk[60];
#pragma unroll
    for (int w = 0; w < 8; w++) rk[w] = h[w];
    uint32_t rcon = 1;
#pragma unroll
    for (int w = 8; w < 60; w++) {
        uint32_t t = rk[w - 1];
        if (w % 8 == 0 || w % 8 == 4) {
            if (w % 8 == 0) t = (t << 8) | (t >> 24);  // RotWord
            t = (((s_te[t >> 24] >> 16) & 0xff) << 24) | (((s_te[(t >> 16) & 0xff] >> 16) & 0xff) << 16) |
                (((s_te[(t >> 8) & 0xff] >> 16) & 0xff) << 8) | ((s_te[t & 0xff] >> 16) & 0xff);  // SubWord
            if (w % 8 == 0) {
                t ^= rcon << 24;
                rcon = ((rcon << 1) ^ ((rcon & 0x80) ? 0x1b : 0)) & 0xff;
            }
        }
        rk[w] = rk[w - 8] ^ t;
    }
    SealKey& K = keys[i];
#pragma unroll
    for (int w = 0; w < 60; w++) K.rk[w] = rk[w];
    const uint32_t zero[4] = {0, 0, 0, 0};
    const uint32_t j0[4] = {it.nonce[0], it.nonce[1], it.nonce[2], 1u};
    uint32_t hb[4], e0[4];
    {
        const uint32_t a0 = it.nonce[0] ^ rk[0], a1 = it.nonce[1] ^ rk[1], a2 = it.nonce[2] ^ rk[2];
#define TE(x, r) ror32(s_te[(x) & 0xff], (r))
        K.R1[0] = TE(a0 >> 24, 0) ^ TE(a1 >> 16, 8) ^ TE(a2 >> 8, 16) ^ rk[4];
        K.R1[1] = TE(a1 >> 24, 0) ^ TE(a2 >> 16, 8) ^ TE(a0, 24) ^ rk[5];
        K.R1[2] = TE(a2 >> 24, 0) ^ TE(a0 >> 8, 16) ^ TE(a1, 24) ^ rk[6];
        K.R1[3] = TE(a0 >> 16, 8) ^ TE(a1 >> 8, 16) ^ TE(a2, 24) ^ rk[7];
#undef TE
    }
    aes_encrypt_plain(rk, s_te, zero, hb);
    aes_encrypt_plain(rk, s_te, j0, e0);
    const G4 H = {hb[0], hb[1], hb[2], hb[3]};
    st4(K.H, H);
    st4(K.E0, {e0[0], e0[1], e0[2], e0[3]});
    G4 p = H;
    for (int k = 0; k < 6; k++) {
        st4(K.P[k], p);
        p = gmul_slow(p, p);
    }
    st4(K.H64, p);  // H^64
    for (uint32_t e = 64; e < PIECE_BLOCKS; e <<= 1) p = gmul_slow(p, p);
    st4(K.HP, p);
}

// ------------------------------------------------------------------ k_seal_ctr
struct SealLds {
    uint32_t te[256][64];       // [byte][Te0 x 32 replicas | Te1 x 32 replicas], at LDS address 0
    uint32_t gt[16][256][4];    // [wave][byte] Shoup 8-bit table of H^64 (contiguous: random bytes spread the banks)
    uint32_t g4[16][6][16][4];  // [wave][level][nibble] Shoup 4-bit tables of H^(2^k)
    uint32_t r8[256], r4[16];   // reduction of 8 / 4 shifted-out bits (xor into w0)
};

#define SEAL_SEL(k) (0x0c0c0000u | ((4u + (k)) << 8))          // (byte k of w) << 8 | lane_off

template <int OFF>
__device__ __forceinline__ uint32_t te_at(const SealLds& L, uint32_t addr) {
    return *(const uint32_t*)((const uint8_t*)&L.te[0][0] + addr + OFF);
}

// Two AES-256 encryptions of counter blocks (n0, n1, n2, ctr), words big-endian, interleaved so
// one block's LDS lookups overlap the other's xors.  Round 1 starts from r1 (its nonce-word
// terms, precomputed per item): only the counter word's four lookups remain.
__device__ __forceinline__ void aes_ctr2(const SealLds& L, const uint32_t* rk, const uint32_t* r1, uint32_t lane_off,
                                         uint32_t ca, uint32_t cb, uint32_t oa[4], uint32_t ob[4]) {
#define A0(w, k) te_at<0>(L, __builtin_amdgcn_perm((w), lane_off, SEAL_SEL(k)))
#define A1(w, k) te_at<128>(L, __builtin_amdgcn_perm((w), lane_off, SEAL_SEL(k)))
#define R16(x) __builtin_amdgcn_alignbit((x), (x), 16)
    uint32_t a0, a1, a2, a3, b0, b1, b2, b3;
    {
        const uint32_t xa = ca ^ rk[3], xb = cb ^ rk[3];
        a0 = r1[0] ^ R16(A1(xa, 0)); b0 = r1[0] ^ R16(A1(xb, 0));
        a1 = r1[1] ^ R16(A0(xa, 1)); b1 = r1[1] ^ R16(A0(xb, 1));
        a2 = r1[2] ^ A1(xa, 2);      b2 = r1[2] ^ A1(xb, 2);
        a3 = r1[3] ^ A0(xa, 3);      b3 = r1[3] ^ A0(xb, 3);
    }
#define COL(s0, s1, s2, s3, r) (A0(s0, 3) ^ A1(s1, 2) ^ R16(A0(s2, 1) ^ A1(s3, 0)) ^ (r))
#pragma unroll
    for (int r = 2; r < 14; r++) {
        const uint32_t ta0 = COL(a0, a1, a2, a3, rk[4 * r]), tb0 = COL(b0, b1, b2, b3, rk[4 * r]);
        const uint32_t ta1 = COL(a1, a2, a3, a0, rk[4 * r + 1]), tb1 = COL(b1, b2, b3, b0, rk[4 * r + 1]);
        const uint32_t ta2 = COL(a2, a3, a0, a1, rk[4 * r + 2]), tb2 = COL(b2, b3, b0, b1, rk[4 * r + 2]);
        const uint32_t ta3 = COL(a3, a0, a1, a2, rk[4 * r + 3]), tb3 = COL(b3, b0, b1, b2, rk[4 * r + 3]);
        a0 = ta0; a1 = ta1; a2 = ta2; a3 = ta3;
        b0 = tb0; b1 = tb1; b2 = tb2; b3 = tb3;
    }
    // last round: S-box bytes (byte 2 of Te0 and byte 0 of Te1 are S[x]), assembled by v_perm
#define LAST(s0, s1, s2, s3, r) \
    ((__builtin_amdgcn_perm(A0(s0, 3), A0(s1, 2), 0x06020c0cu) | __builtin_amdgcn_perm(A1(s2, 1), A1(s3, 0), 0x0c0c0400u)) ^ (r))
    oa[0] = LAST(a0, a1, a2, a3, rk[56]); ob[0] = LAST(b0, b1, b2, b3, rk[56]);
    oa[1] = LAST(a1, a2, a3, a0, rk[57]); ob[1] = LAST(b1, b2, b3, b0, rk[57]);
    oa[2] = LAST(a2, a3, a0, a1, rk[58]); ob[2] = LAST(b2, b3, b0, b1, rk[58]);
    oa[3] = LAST(a3, a0, a1, a2, rk[59]); ob[3] = LAST(b3, b0, b1, b2, rk[59]);
#undef LAST
#undef COL
#undef R16
#undef A1
#undef A0
}

// Byte f of the zstd store frame of the raw_len bytes at s (FHD 0x00, window descriptor, raw
// blocks of <= 128 KiB behind 3-byte headers with the last-block bit).
__device__ __forceinline__ uint32_t frame_byte(const uint8_t* s, uint32_t raw_len, uint32_t wd, uint32_t f) {
    if (f == 0) return 0;  // Frame_Header_Descriptor: no content size, no checksum, no dictionary
    if (f == 1) return wd;
    const uint32_t nb = raw_len ? (raw_len + ZSTD_BLOCK - 1) / ZSTD_BLOCK : 1;
    const uint32_t k = (f - 2) / ZSTD_STRIDE, r = (f - 2) - k * ZSTD_STRIDE;
    if (r < 3) {
        const uint32_t bl = k == nb - 1 ? raw_len - k * ZSTD_BLOCK : ZSTD_BLOCK;
        return (((bl << 3) | (k == nb - 1 ? 1u : 0u)) >> (8 * r)) & 0xff;  // Raw_Block
    }
    return s[(uint64_t)k * ZSTD_BLOCK + r - 3];
}

// CTR xor of block g of the item (keystream ks) from s to d; returns the GHASH input (the
// ciphertext, zero-padded past the end of the item).  FRAMED: the plaintext is the store frame
// of the raw bytes at s; a block inside one raw block's data is one (unaligned) 16-byte load.
template <bool DEC, bool FRAMED>
__device__ __forceinline__ G4 crypt_block(const uint8_t* s, uint8_t* d, uint64_t len, uint64_t g, const uint32_t ks[4],
                                          uint32_t raw_len, uint32_t wd) {
    const uint64_t at = 16 * g;
    uint32_t in[4];
    const bool full = at + 16 <= len;
    if (FRAMED) {
        const uint32_t f = (uint32_t)at;
        const uint32_t k0 = f >= 2 ? (f - 2) / ZSTD_STRIDE : 0, r0 = f >= 2 ? (f - 2) - k0 * ZSTD_STRIDE : 0;
        if (full && f >= 2 && r0 >= 3 && r0 + 16 <= ZSTD_STRIDE) {
            const uint4 v = *(const uint4*)(s + (uint64_t)k0 * ZSTD_BLOCK + r0 - 3);
            in[0] = __builtin_bswap32(v.x); in[1] = __builtin_bswap32(v.y);
            in[2] = __builtin_bswap32(v.z); in[3] = __builtin_bswap32(v.w);
        } else {
            const uint32_t nb = full ? 16 : (uint32_t)(len - at);
#pragma unroll
            for (int w = 0; w < 4; w++) {
                uint32_t x = 0;
#pragma unroll
                for (int b = 0; b < 4; b++)
                    if ((uint32_t)(4 * w + b) < nb) x |= frame_byte(s, raw_len, wd, f + 4 * w + b) << (24 - 8 * b);
                in[w] = x;
            }
        }
    } else if (full) {
        const uint4 v = *(const uint4*)(s + at);
        in[0] = __builtin_bswap32(v.x); in[1] = __builtin_bswap32(v.y);
        in[2] = __builtin_bswap32(v.z); in[3] = __builtin_bswap32(v.w);
    } else {
        const uint32_t nb = (uint32_t)(len - at);
#pragma unroll
        for (int w = 0; w < 4; w++) {
            uint32_t x = 0;
#pragma unroll
            for (int b = 0; b < 4; b++)
                if ((uint32_t)(4 * w + b) < nb) x |= (uint32_t)s[at + 4 * w + b] << (24 - 8 * b);
            in[w] = x;
        }
    }
    uint32_t out[4];
#pragma unroll
    for (int w = 0; w < 4; w++) out[w] = in[w] ^ ks[w];
    if (full) {
        *(uint4*)(d + at) = make_uint4(__builtin_bswap32(out[0]), __builtin_bswap32(out[1]), __builtin_bswap32(out[2]),
                                       __builtin_bswap32(out[3]));
    } else {
        const uint32_t nb = (uint32_t)(len - at);
        for (uint32_t b = 0; b < nb; b++) d[at + b] = (uint8_t)(out[b >> 2] >> (24 - 8 * (b & 3)));
#pragma unroll
        for (int w = 0; w < 4; w++) {
            const int v = (int)nb - 4 * w;  // valid bytes of word w (big-endian)
            out[w] &= v >= 4 ? ~0u : (v <= 0 ? 0u : ~0u << (32 - 8 * v));
        }
    }
    const uint32_t* c = DEC ? in : out;  // GHASH runs over the ciphertext
    return {c[0], c[1], c[2], c[3]};
}

// Z = X * H^64 with this wave's 8-bit table: Horner over the bytes of X from the last
__device__ __forceinline__ G4 gmul_h64(const SealLds& L, G4 x, uint32_t wid) {
    const uint8_t* gbase = (const uint8_t*)&L.gt[wid][0][0];
    const uint32_t xw[4] = {x.w0, x.w1, x.w2, x.w3};
    G4 z = {0, 0, 0, 0};
#pragma unroll
    for (int i = 15; i >= 0; i--) {
        if (i != 15) {
            const uint32_t rem = z.w3 & 0xff;
            z.w3 = __builtin_amdgcn_alignbyte(z.w2, z.w3, 1);
            z.w2 = __builtin_amdgcn_alignbyte(z.w1, z.w2, 1);
            z.w1 = __builtin_amdgcn_alignbyte(z.w0, z.w1, 1);
            z.w0 = (z.w0 >> 8) ^ L.r8[rem];
        }
        const uint32_t b = (xw[i >> 2] >> (8 * (3 - (i & 3)))) & 0xff;
        const uint4 m = *(const uint4*)(gbase + (b << 4));
        z.w0 ^= m.x; z.w1 ^= m.y; z.w2 ^= m.z; z.w3 ^= m.w;
    }
    return z;
}

// Z = X * T with a 4-bit table (16 entries)
__device__ __forceinline__ G4 gmul_t4(const SealLds& L, G4 x, const uint32_t (*t)[4]) {
    const uint32_t xw[4] = {x.w0, x.w1, x.w2, x.w3};
    G4 z = {0, 0, 0, 0};
#pragma unroll
    for (int i = 31; i >= 0; i--) {
        if (i != 31) {
            const uint32_t rem = z.w3 & 0xf;
            z.w3 = __builtin_amdgcn_alignbit(z.w2, z.w3, 4);
            z.w2 = __builtin_amdgcn_alignbit(z.w1, z.w2, 4);
            z.w1 = __builtin_amdgcn_alignbit(z.w0, z.w1, 4);
            z.w0 = (z.w0 >> 4) ^ L.r4[rem];
        }
        const uint32_t nib = (xw[i >> 3] >> (28 - 4 * (i & 7))) & 0xf;
        const uint4 m = *(const uint4*)t[nib];
        z.w0 ^= m.x; z.w1 ^= m.y; z.w2 ^= m.z; z.w3 ^= m.w;
    }
    return z;
}

__device__ __forceinline__ G4 shfl_down4(G4 v, int d) {
    return {(uint32_t)__shfl_down((int)v.w0, d, 64), (uint32_t)__shfl_down((int)v.w1, d, 64),
            (uint32_t)__shfl_down((int)v.w2, d, 64), (uint32_t)__shfl_down((int)v.w3, d, 64)};
}

template <bool DEC, bool FRAMED>
__global__ __launch_bounds__(SEAL_THREADS) void k_seal_ctr(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                           const SealItem* __restrict__ items, uint64_t n_items,
                                                           const SealKey* __restrict__ keys, uint64_t n_pieces,
                                                           uint32_t* __restrict__ parts) {
    __shared__ __attribute__((aligned(16))) SealLds L;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    // shared tables: S-box -> Te0/Te1 replicas, reductions
    if (tid < 256) {
        const uint32_t t0 = aes_te0(aes_sbox(tid));
        L.te[tid][0] = t0;
        L.te[tid][32] = ror32(t0, 8);
        G4 v = {0, 0, 0, tid};
        for (int k = 0; k < 8; k++) {
            v = gmulx(v);
            if (k == 3 && tid < 16) L.r4[tid] = v.w0;
        }
        L.r8[tid] = v.w0;
    }
    __syncthreads();
    for (uint32_t e = tid; e < 256 * 64; e += SEAL_THREADS) {
        const uint32_t row = e >> 6, col = e & 63;
        if (col != 0 && col != 32) L.te[row][col] = L.te[row][col < 32 ? 0 : 32];
    }
    __syncthreads();
    const uint32_t lane_off = (lane & 31) * 4;

    for (uint64_t p = (uint64_t)blockIdx.x * (SEAL_THREADS / 64) + wid; p < n_pieces;
         p += (uint64_t)gridDim.x * (SEAL_THREADS / 64)) {
        // item owning piece p (items[].piece0 ascending)
        uint64_t lo = 0, hi = n_items;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (items[mid].piece0 <= p) lo = mid + 1;
            else hi = mid;
        }
        const uint64_t ii = (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(lo - 1));
        const SealItem& it = items[ii];
        const SealKey& K = keys[ii];
        const uint64_t len = it.len, m = (len + 15) / 16;
        // pieces are cut from the end: the first takes the ragged remainder, so every later piece is
        // full and k_seal_tag folds them with the one multiplier H^PIECE_BLOCKS
        const uint64_t pi = p - it.piece0, np = (m + PIECE_BLOCKS - 1) / PIECE_BLOCKS;
        const uint64_t first = m - (np - 1) * PIECE_BLOCKS;
        const uint64_t b0 = pi == 0 ? 0 : first + (pi - 1) * PIECE_BLOCKS;
        const uint32_t q = (uint32_t)(pi == 0 ? first : PIECE_BLOCKS);
        // this wave's tables: 8-bit Shoup table of H^64 (4 entries per lane), 4-bit tables of H^(2^k)
        {
            G4 basis[8];
            basis[0] = ld4(K.H64);
#pragma unroll
            for (int j = 1; j < 8; j++) basis[j] = gmulx(basis[j - 1]);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const uint32_t b = lane + 64 * r;
                G4 e = {0, 0, 0, 0};
#pragma unroll
                for (int j = 0; j < 8; j++)
                    if (b & (0x80u >> j)) e = gxor(e, basis[j]);
                st4(L.gt[wid][b], e);
            }
            for (uint32_t pr = lane; pr < 96; pr += 64) {
                const uint32_t k = pr >> 4, nib = pr & 15;
                G4 v = ld4(K.P[k]), e = {0, 0, 0, 0};
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    if (nib & (0x8u >> j)) e = gxor(e, v);
                    v = gmulx(v);
                }
                st4(L.g4[wid][k][nib], e);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

        uint32_t rk[60];
#pragma unroll
        for (int w = 0; w < 60; w++) rk[w] = K.rk[w];
        const uint8_t* s = src + it.src_off;
        uint8_t* d = dst + it.dst_off;
        const uint32_t S = (q + 63) / 64, pad = 64 * S - q;
        G4 X = {0, 0, 0, 0};
        uint32_t r1[4];
#pragma unroll
        for (int w = 0; w < 4; w++) r1[w] = K.R1[w];
        // two blocks per lane per step (j, j + 1): their AES runs interleaved, GHASH stays in order
        for (uint32_t j = 0; j < S; j += 2) {
            const int32_t ra = (int32_t)(lane + 64 * j) - (int32_t)pad;  // >= -63; rb = ra + 64 >= 1
            const uint64_t ga = b0 + (uint32_t)(ra < 0 ? 0 : ra), gb = b0 + (uint32_t)(ra + 64);
            uint32_t ksa[4], ksb[4];
            aes_ctr2(L, rk, r1, lane_off, (uint32_t)(ga + 2), (uint32_t)(gb + 2), ksa, ksb);  // inc32 of J0 = nonce||1
            if (j) X = gmul_h64(L, X, wid);
            if (ra >= 0) X = gxor(X, crypt_block<DEC, FRAMED>(s, d, len, ga, ksa, it.raw_len, it.wd));
            if (j + 1 < S) {  // wave-uniform
                X = gmul_h64(L, X, wid);
                X = gxor(X, crypt_block<DEC, FRAMED>(s, d, len, gb, ksb, it.raw_len, it.wd));
            }
        }
        // fold the 64 lane partials: T = sum_l X_l * H^(63 - l)
#pragma unroll
        for (int k = 0; k < 6; k++) {
            const G4 y = shfl_down4(X, 1 << k);
            const G4 t = gmul_t4(L, X, L.g4[wid][k]);
            if ((lane & ((2u << k) - 1)) == 0) X = gxor(t, y);
        }
        if (lane == 0) st4(parts + 4 * p, X);
        __builtin_amdgcn_wave_barrier();  // the tables are rebuilt for the next piece
    }
}

// ------------------------------------------------------------------ k_seal_tag
template <bool DEC>
__global__ __launch_bounds__(256) void k_seal_tag(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                  const SealItem* __restrict__ items, uint64_t n,
                                                  const SealKey* __restrict__ keys, const uint32_t* __restrict__ parts,
                                                  uint8_t* __restrict__ ok) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const SealItem& it = items[i];
    const SealKey& K = keys[i];
    const uint64_t len = it.len, m = (len + 15) / 16;
    const uint64_t np = (m + PIECE_BLOCKS - 1) / PIECE_BLOCKS;
    const G4 H = ld4(K.H);
    G4 acc = {0, 0, 0, 0};
    const G4 HP = ld4(K.HP);
    for (uint64_t pi = 0; pi < np; pi++) {
        const G4 T = ld4(parts + 4 * (it.piece0 + pi));
        acc = pi == 0 ? T : gxor(gmul_slow(acc, HP), T);  // every piece after the first is full
    }
    const uint64_t bits = len * 8;
    const G4 Lb = {0, 0, (uint32_t)(bits >> 32), (uint32_t)bits};
    G4 y = gmul_slow(gxor(gmul_slow(acc, H), Lb), H);
    y = gxor(y, ld4(K.E0));
    const uint32_t tw[4] = {y.w0, y.w1, y.w2, y.w3};
    if (!DEC) {
        uint8_t* t = dst + it.dst_off + len;
        for (int b = 0; b < 16; b++) t[b] = (uint8_t)(tw[b >> 2] >> (24 - 8 * (b & 3)));
    } else {
        const uint8_t* t = src + it.src_off + len;
        uint32_t diff = 0;
        for (int b = 0; b < 16; b++) diff |= t[b] ^ (uint8_t)(tw[b >> 2] >> (24 - 8 * (b & 3)));
        ok[i] = diff == 0;
    }
}

// ------------------------------------------------------------------ host side
void seal_pads(const uint8_t prk[32], SealPads* pads) {
    uint32_t blk[16];
    for (int pass = 0; pass < 2; pass++) {
        const uint8_t x = pass ? 0x5c : 0x36;
        for (int w = 0; w < 16; w++) {
            uint32_t v = 0;
            for (int b = 0; b < 4; b++) {
                const int k = 4 * w + b;
                v |= (uint32_t)((k < 32 ? prk[k] : 0) ^ x) << (24 - 8 * b);
            }
            blk[w] = v;
        }
        uint32_t* st = pass ? pads->ostate : pads->istate;
        const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
        for (int w = 0; w < 8; w++) st[w] = iv[w];
        sha256_compress(st, blk, h_k256);
    }
}

uint64_t seal_pieces(uint64_t len) {
    const uint64_t m = (len + 15) / 16;
    return (m + PIECE_BLOCKS - 1) / PIECE_BLOCKS;
}

void seal_fill_item(SealItem* it, uint64_t src_off, uint64_t len, uint64_t dst_off, uint64_t piece0,
                    const uint8_t nonce[12], const uint8_t* info, uint32_t info_len) {
    memset(it, 0, sizeof(SealItem));
    it->src_off = src_off;
    it->len = len;
    it->dst_off = dst_off;
    it->piece0 = piece0;
    for (int w = 0; w < 3; w++)
        it->nonce[w] = (uint32_t)nonce[4 * w] << 24 | (uint32_t)nonce[4 * w + 1] << 16 |
                       (uint32_t)nonce[4 * w + 2] << 8 | nonce[4 * w + 3];
    it->info_len = info_len;
    memcpy(it->info, info, info_len);
}

uint32_t zstd_window_descriptor(uint64_t raw_len) {
    uint32_t wlog = raw_len > 1 ? 64 - __builtin_clzll(raw_len - 1) : 0;  // ceil(log2(raw_len))
    wlog = wlog < 10 ? 10 : (wlog > 21 ? 21 : wlog);  // level 3's windowLog, cut to the source size
    return (wlog - 10) << 3;
}

void launch_seal(hipStream_t st, bool dec, bool framed, const uint8_t* src, uint8_t* dst, const SealItem* it,
                 uint64_t n, const SealPads& pads, SealKey* k, uint64_t n_pieces, uint32_t* parts, uint8_t* ok) {
    if (!n) return;
    hipLaunchKernelGGL(k_seal_prep, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, it, n, pads, k);
    if (n_pieces) {
        uint64_t grid = (n_pieces + SEAL_THREADS / 64 - 1) / (SEAL_THREADS / 64);
        if (grid > 1024) grid = 1024;
        if (dec)
            hipLaunchKernelGGL((k_seal_ctr<true, false>), dim3((unsigned)grid), dim3(SEAL_THREADS), 0, st, src, dst, it,
                               n, k, n_pieces, parts);
        else if (framed)
            hipLaunchKernelGGL((k_seal_ctr<false, true>), dim3((unsigned)grid), dim3(SEAL_THREADS), 0, st, src, dst, it,
                               n, k, n_pieces, parts);
        else
            hipLaunchKernelGGL((k_seal_ctr<false, false>), dim3((unsigned)grid), dim3(SEAL_THREADS), 0, st, src, dst,
                               it, n, k, n_pieces, parts);
    }
    if (dec)
        hipLaunchKernelGGL(k_seal_tag<true>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, src, dst, it, n, k,
                           parts, ok);
    else
        hipLaunchKernelGGL(k_seal_tag<false>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, src, dst, it, n, k,
                           parts, ok);
}

}  // namespace bw
