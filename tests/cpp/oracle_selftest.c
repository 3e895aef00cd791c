/* oracle_selftest.c -- drives every entry point of the C restatement (oracle/) so that an
 * AddressSanitizer + UndefinedBehaviorSanitizer build of it (tests/test_sanitizers.py) walks the
 * same code the tests use: BLAKE3 (scalar and 16-way SIMD) at every tree shape, FastCDC at several
 * parameter sets on random data, zeros and odd tails, the batch driver on 4 threads with a seeded
 * index, and the sealing primitives (seal / open / tamper).  Exits non-zero on a failed check;
 * the sanitizers abort on any memory or UB error. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/bw_oracle.h"

static int fails = 0;
#define CHECK(c)                                                       \
    do {                                                               \
        if (!(c)) {                                                    \
            fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            fails++;                                                   \
        }                                                              \
    } while (0)

static void splitmix(uint64_t seed, uint8_t* out, size_t n) {
    uint64_t x = seed;
    for (size_t i = 0; i < n; i += 8) {
        x += 0x9E3779B97F4A7C15ull;
        uint64_t z = x;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        for (int k = 0; k < 8 && i + k < n; k++) out[i + k] = (uint8_t)(z >> (8 * k));
    }
}

static void blake3_shapes(const uint8_t* buf, size_t cap) {
    static const size_t lens[] = {0, 1, 63, 64, 65, 1023, 1024, 1025, 2048, 2049, 16 * 1024, 16 * 1024 + 1,
                                  33 * 1024 + 7, 64 * 1024, 1 << 20, (1 << 20) + 3, 3 << 20};
    const uint8_t empty_kat[32] = {0xaf, 0x13, 0x49, 0xb9, 0xf5, 0xf9, 0xa1, 0xa6, 0xa0, 0x40, 0x4d,
                                   0xea, 0x36, 0xdc, 0xc9, 0x49, 0x9b, 0xcb, 0x25, 0xc9, 0xad, 0xc1,
                                   0x12, 0xb7, 0xcc, 0x9a, 0x93, 0xca, 0xe4, 0x1f, 0x32, 0x62};
    uint8_t a[32], b[32];
    orc_blake3(buf, 0, a);
    CHECK(memcmp(a, empty_kat, 32) == 0);
    for (size_t i = 0; i < sizeof lens / sizeof lens[0]; i++) {
        if (lens[i] + 3 > cap) continue;
        for (size_t off = 0; off < 4; off += 3) {
            orc_blake3(buf + off, lens[i], a);
            orc_blake3_fast(buf + off, lens[i], b);
            CHECK(memcmp(a, b, 32) == 0);
        }
    }
}

static void fastcdc_cases(const uint8_t* buf, size_t n) {
    static const uint32_t P[][3] = {{64, 256, 1024}, {4096, 16384, 65536}, {262144, 1048576, 3145728}, {65, 300, 1024}};
    size_t cap = n / 32 + 4;
    uint64_t* h = malloc(cap * 8 * 3);
    for (size_t k = 0; k < sizeof P / sizeof P[0]; k++) {
        size_t cnt = 0;
        CHECK(orc_fastcdc_chunks(buf, n, P[k][0], P[k][1], P[k][2], h, h + cap, h + 2 * cap, cap, &cnt) == 0);
        uint64_t sum = 0;
        for (size_t i = 0; i < cnt; i++) {
            CHECK(h[cap + i] == sum);
            CHECK(h[2 * cap + i] <= P[k][2]);
            if (i + 1 < cnt) CHECK(h[2 * cap + i] >= (P[k][0] < P[k][2] ? P[k][0] / 2 * 2 : P[k][2]));
            sum += h[2 * cap + i];
        }
        CHECK(sum == n);
        /* odd tail and a short buffer */
        CHECK(orc_fastcdc_chunks(buf, n - 1, P[k][0], P[k][1], P[k][2], h, h + cap, h + 2 * cap, cap, &cnt) == 0);
        CHECK(orc_fastcdc_chunks(buf, 10, P[k][0], P[k][1], P[k][2], h, h + cap, h + 2 * cap, cap, &cnt) == 0);
        CHECK(cnt == 1 && h[2 * cap] == 10);
    }
    uint64_t ms, ml;
    CHECK(orc_fastcdc_masks(63, 256, 1024, &ms, &ml) != 0);  /* the crate's assert */
    uint8_t* zeros = calloc((8u << 20) + 5, 1);
    size_t cnt = 0;
    CHECK(orc_fastcdc_chunks(zeros, (8u << 20) + 5, 262144, 1048576, 3145728, h, h + cap, h + 2 * cap, cap, &cnt) == 0 &&
          cnt == 3);
    free(zeros);
    free(h);
}

static void batch_driver(const uint8_t* buf, size_t n) {
    enum { NF = 40 };
    uint64_t off[NF], len[NF];
    size_t pos = 0;
    for (int f = 0; f < NF; f++) {
        size_t l = (size_t)((f * 2654435761u) % (3u << 20));
        if (pos + l > n) l = 0;
        off[f] = pos;
        len[f] = l;
        pos += l / 2;  /* overlapping files: shared bytes = duplicate chunks */
    }
    uint8_t seed[64];
    orc_blake3(buf + off[3], len[3], seed);
    memset(seed + 32, 0xff, 32);
    orc_index* ix = orc_index_new(seed, 2);
    size_t cap = 4096, got = 0;
    orc_blob* out = calloc(cap, sizeof *out);
    CHECK(orc_process_files(buf, off, len, NF, 64, 256, 1024, 1024, ix, 4, out, cap, &got) == -2 || got <= cap);
    CHECK(orc_process_files(buf, off, len, NF, 262144, 1048576, 3145728, 1048576, ix, 4, out, cap, &got) == 0);
    CHECK(got >= NF);
    orc_index_free(ix);
    orc_set_blake3_simd(1);
    size_t got2 = 0;
    orc_blob* out2 = calloc(cap, sizeof *out2);
    CHECK(orc_process_files(buf, off, len, NF, 262144, 1048576, 3145728, 1048576, NULL, 3, out2, cap, &got2) == 0);
    orc_set_blake3_simd(0);
    CHECK(got2 == got);
    for (size_t i = 0; i < got && i < got2; i++) CHECK(memcmp(out[i].digest, out2[i].digest, 32) == 0);
    free(out);
    free(out2);
}

static void sealing(const uint8_t* buf) {
    uint8_t prk[32], nonce[12], key[32];
    memcpy(prk, buf, 32);
    memcpy(nonce, buf + 32, 12);
    orc_hkdf_expand32(prk, buf + 100, 32, key);
    static const size_t lens[] = {0, 1, 15, 16, 17, 4095, 70001};
    for (size_t i = 0; i < sizeof lens / sizeof lens[0]; i++) {
        size_t n = lens[i];
        uint8_t* ct = malloc(n + 16);
        uint8_t* pt = malloc(n + 1);
        orc_aes256_gcm_seal(key, nonce, buf + 200, n, ct);
        CHECK(orc_aes256_gcm_open(key, nonce, ct, n + 16, pt) == 0);
        CHECK(n == 0 || memcmp(pt, buf + 200, n) == 0);
        ct[n / 2] ^= 1;
        CHECK(orc_aes256_gcm_open(key, nonce, ct, n + 16, pt) != 0);
        free(ct);
        free(pt);
    }
    uint8_t d[32];
    orc_sha256(buf, 1000, d);
    orc_hmac_sha256(buf, 100, buf + 100, 1000, d);
}

int main(void) {
    const size_t n = (12u << 20) + 13;
    uint8_t* buf = malloc(n);
    splitmix(7, buf, n);
    blake3_shapes(buf, n);
    fastcdc_cases(buf, n);
    batch_driver(buf, n);
    sealing(buf);
    free(buf);
    if (fails) {
        fprintf(stderr, "%d check(s) failed\n", fails);
        return 1;
    }
    printf("oracle selftest ok\n");
    return 0;
}
