/*
 * bw_oracle.c -- CPU restatement (oracle) of backuwup's client-side dedup front end.
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg as the checker, never by the product path.  See bw_oracle.h for the
 * parity status ("unpinned by the reference"; pinned by spec KATs and derived constants).
 *
 * Sections:
 *   1. GEAR table from its derivation rule (own MD5), MASKS       -- fastcdc 3.0.3 v2020 consts
 *   2. fastcdc::v2020::cut + FastCDC iterator                     -- SURVEY.md A.1
 *   3. BLAKE3 (recursive subtree formulation of the spec)         -- SURVEY.md A.4
 *   4. BlobIndex: sorted `items` + binary search OR `blobs_queued` -- blob_index.rs:130-148
 *   5. process_file policy + add_blob dedup gate, batch driver     -- dir_packer.rs:231-311,
 *                                                                     pack.rs:31-39
 */
#include "bw_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- 1. constants */

static uint32_t md5_rotl(uint32_t x, int c) { return (x << c) | (x >> (32 - c)); }

/* Plain RFC 1321 MD5 of a message shorter than 56 bytes would not fit 64 B inputs; this is a
 * general single-call MD5 for short messages (<= 119 bytes), enough for the 64-byte GEAR rule. */
static void md5_short(const uint8_t* msg, size_t len, uint8_t out[16]) {
    static const uint32_t K[64] = {
        0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
        0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
        0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
        0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
        0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
        0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
        0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
        0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
    static const int R[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                              5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                              4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                              6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};
    uint8_t buf[128];
    size_t padded = ((len + 8) / 64 + 1) * 64;
    memset(buf, 0, sizeof buf);
    memcpy(buf, msg, len);
    buf[len] = 0x80;
    uint64_t bits = (uint64_t)len * 8;
    for (int i = 0; i < 8; i++) buf[padded - 8 + i] = (uint8_t)(bits >> (8 * i));
    uint32_t h0 = 0x67452301, h1 = 0xefcdab89, h2 = 0x98badcfe, h3 = 0x10325476;
    for (size_t off = 0; off < padded; off += 64) {
        uint32_t w[16];
        for (int i = 0; i < 16; i++)
            w[i] = (uint32_t)buf[off + 4 * i] | ((uint32_t)buf[off + 4 * i + 1] << 8) |
                   ((uint32_t)buf[off + 4 * i + 2] << 16) | ((uint32_t)buf[off + 4 * i + 3] << 24);
        uint32_t a = h0, b = h1, c = h2, d = h3;
        for (int i = 0; i < 64; i++) {
            uint32_t f;
            int g;
            if (i < 16) { f = (b & c) | (~b & d); g = i; }
            else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) % 16; }
            else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) % 16; }
            else { f = c ^ (b | ~d); g = (7 * i) % 16; }
            uint32_t tmp = d;
            d = c;
            c = b;
            b = b + md5_rotl(a + f + K[i] + w[g], R[i]);
            a = tmp;
        }
        h0 += a; h1 += b; h2 += c; h3 += d;
    }
    uint32_t hs[4] = {h0, h1, h2, h3};
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(hs[i] >> (8 * j));
}

static uint64_t GEAR[256], GEAR_LS[256];
static pthread_once_t gear_once = PTHREAD_ONCE_INIT;

/* fastcdc 3.0.3 src/v2020/mod.rs GEAR: be_u64(md5([i; 64])[0..8])  (SURVEY.md A.2). */
static void gear_init(void) {
    for (int i = 0; i < 256; i++) {
        uint8_t msg[64], d[16];
        memset(msg, i, sizeof msg);
        md5_short(msg, 64, d);
        uint64_t v = 0;
        for (int j = 0; j < 8; j++) v = (v << 8) | d[j];
        GEAR[i] = v;
        GEAR_LS[i] = v << 1;
    }
}

void orc_gear_table(uint64_t out[256]) {
    pthread_once(&gear_once, gear_init);
    memcpy(out, GEAR, sizeof GEAR);
}

/* fastcdc 3.0.3 src/v2020/mod.rs MASKS. */
static const uint64_t MASKS[26] = {
    0, 0, 0, 0, 0,
    0x0000000001804110ULL, 0x0000000001803110ULL, 0x0000000018035100ULL, 0x0000001800035300ULL,
    0x0000019000353000ULL, 0x0000590003530000ULL, 0x0000d90003530000ULL, 0x0000d90103530000ULL,
    0x0000d90303530000ULL, 0x0000d90313530000ULL, 0x0000d90f03530000ULL, 0x0000d90303537000ULL,
    0x0000d90703537000ULL, 0x0000d90707537000ULL, 0x0000d91707537000ULL, 0x0000d91747537000ULL,
    0x0000d91767537000ULL, 0x0000d93767537000ULL, 0x0000d93777537000ULL, 0x0000d93777577000ULL,
    0x0000db3777577000ULL,
};

/* FastCDC::with_level asserts (MINIMUM_MIN..MAXIMUM_MAX) and Level1 mask choice:
 * bits = round(log2(avg)); mask_s = MASKS[bits + 1]; mask_l = MASKS[bits - 1]. */
int orc_fastcdc_masks(uint32_t min, uint32_t avg, uint32_t max, uint64_t* mask_s, uint64_t* mask_l) {
    if (min < 64 || min > 1048576) return -1;
    if (avg < 256 || avg > 4194304) return -1;
    if (max < 1024 || max > 16777216) return -1;
    uint32_t bits = (uint32_t)lround(log2((double)avg));
    *mask_s = MASKS[bits + 1];
    *mask_l = MASKS[bits - 1];
    return 0;
}

/* ---------------------------------------------------------------- 2. FastCDC v2020 */

/* fastcdc::v2020::cut: two bytes per step, hash starts at 0 at min. */
size_t orc_fastcdc_cut(const uint8_t* src, size_t len, uint32_t min_size, uint32_t avg_size,
                       uint32_t max_size, uint64_t mask_s, uint64_t mask_l, uint64_t* out_hash) {
    pthread_once(&gear_once, gear_init);
    size_t remaining = len;
    if (remaining <= min_size) {
        *out_hash = 0;
        return remaining;
    }
    size_t center = avg_size;
    if (remaining > max_size) remaining = max_size;
    else if (remaining < center) center = remaining;
    const uint64_t mask_s_ls = mask_s << 1, mask_l_ls = mask_l << 1;
    size_t index = min_size / 2;
    uint64_t hash = 0;
    /* With avg > max and a source longer than max, `center` stays avg: the crate's first loop runs
     * past `remaining` (a cut there gives a chunk longer than max) and, when the source ends first,
     * indexes out of bounds -- a panic in Rust.  ORC_CUT_PANIC reports that. */
    while (index < center / 2) {
        size_t a = index * 2;
        if (a >= len) return ORC_CUT_PANIC;
        hash = (hash << 2) + GEAR_LS[src[a]];
        if ((hash & mask_s_ls) == 0) { *out_hash = hash; return a; }
        if (a + 1 >= len) return ORC_CUT_PANIC;
        hash = hash + GEAR[src[a + 1]];
        if ((hash & mask_s) == 0) { *out_hash = hash; return a + 1; }
        index++;
    }
    while (index < remaining / 2) {
        size_t a = index * 2;
        hash = (hash << 2) + GEAR_LS[src[a]];
        if ((hash & mask_l_ls) == 0) { *out_hash = hash; return a; }
        hash = hash + GEAR[src[a + 1]];
        if ((hash & mask_l) == 0) { *out_hash = hash; return a + 1; }
        index++;
    }
    *out_hash = hash;
    return remaining;
}

/* impl Iterator for FastCDC: repeated cut() from the running offset until the input is used. */
int orc_fastcdc_chunks(const uint8_t* src, size_t len, uint32_t min, uint32_t avg, uint32_t max,
                       uint64_t* out_hash, uint64_t* out_off, uint64_t* out_len, size_t cap,
                       size_t* n_out) {
    uint64_t ms, ml;
    if (orc_fastcdc_masks(min, avg, max, &ms, &ml) != 0) return -1;
    size_t n = 0, off = 0;
    while (off < len) {
        uint64_t h;
        size_t c = orc_fastcdc_cut(src + off, len - off, min, avg, max, ms, ml, &h);
        if (c == ORC_CUT_PANIC) return -3;  /* the crate panics (index out of bounds) */
        if (c == 0) break;
        if (n < cap) {
            out_hash[n] = h;
            out_off[n] = off;
            out_len[n] = c;
        }
        n++;
        off += c;
    }
    *n_out = n;
    return n > cap ? -2 : 0;
}

/* ---------------------------------------------------------------- 3. BLAKE3 */

enum { B3_CHUNK_START = 1, B3_CHUNK_END = 2, B3_PARENT = 4, B3_ROOT = 8 };
static const uint32_t B3_IV[8] = {0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A,
                                  0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19};
static const int B3_PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};

static uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

static void b3_g(uint32_t* v, int a, int b, int c, int d, uint32_t x, uint32_t y) {
    v[a] = v[a] + v[b] + x; v[d] = rotr32(v[d] ^ v[a], 16);
    v[c] = v[c] + v[d];     v[b] = rotr32(v[b] ^ v[c], 12);
    v[a] = v[a] + v[b] + y; v[d] = rotr32(v[d] ^ v[a], 8);
    v[c] = v[c] + v[d];     v[b] = rotr32(v[b] ^ v[c], 7);
}

/* compression function; writes the 8-word chaining value (first half of the output) */
static void b3_compress(const uint32_t cv[8], const uint8_t block[64], uint32_t block_len,
                        uint64_t counter, uint32_t flags, uint32_t out[8]) {
    uint32_t m[16], v[16];
    for (int i = 0; i < 16; i++)
        m[i] = (uint32_t)block[4 * i] | ((uint32_t)block[4 * i + 1] << 8) |
               ((uint32_t)block[4 * i + 2] << 16) | ((uint32_t)block[4 * i + 3] << 24);
    for (int i = 0; i < 8; i++) v[i] = cv[i];
    for (int i = 0; i < 4; i++) v[8 + i] = B3_IV[i];
    v[12] = (uint32_t)counter;
    v[13] = (uint32_t)(counter >> 32);
    v[14] = block_len;
    v[15] = flags;
    for (int r = 0; r < 7; r++) {
        b3_g(v, 0, 4, 8, 12, m[0], m[1]);
        b3_g(v, 1, 5, 9, 13, m[2], m[3]);
        b3_g(v, 2, 6, 10, 14, m[4], m[5]);
        b3_g(v, 3, 7, 11, 15, m[6], m[7]);
        b3_g(v, 0, 5, 10, 15, m[8], m[9]);
        b3_g(v, 1, 6, 11, 12, m[10], m[11]);
        b3_g(v, 2, 7, 8, 13, m[12], m[13]);
        b3_g(v, 3, 4, 9, 14, m[14], m[15]);
        uint32_t t[16];
        for (int i = 0; i < 16; i++) t[i] = m[B3_PERM[i]];
        memcpy(m, t, sizeof m);
    }
    for (int i = 0; i < 8; i++) out[i] = v[i] ^ v[i + 8];
}

/* one 1024-byte BLAKE3 chunk (<= 1024 bytes), chunk counter `t` */
static void b3_chunk_cv(const uint8_t* in, size_t len, uint64_t t, uint32_t extra_flags, uint32_t out[8]) {
    uint32_t cv[8];
    memcpy(cv, B3_IV, sizeof cv);
    size_t nblocks = len == 0 ? 1 : (len + 63) / 64;
    for (size_t b = 0; b < nblocks; b++) {
        uint8_t block[64];
        size_t bl = len - b * 64 < 64 ? len - b * 64 : 64;
        if (len == 0) bl = 0;
        memset(block, 0, sizeof block);
        memcpy(block, in + b * 64, bl);
        uint32_t flags = 0;
        if (b == 0) flags |= B3_CHUNK_START;
        if (b == nblocks - 1) flags |= B3_CHUNK_END | extra_flags;
        b3_compress(cv, block, (uint32_t)bl, t, flags, cv);
    }
    memcpy(out, cv, sizeof cv);
}

static void b3_parent_cv(const uint32_t l[8], const uint32_t r[8], uint32_t flags, uint32_t out[8]) {
    uint8_t block[64];
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 4; j++) {
            block[4 * i + j] = (uint8_t)(l[i] >> (8 * j));
            block[32 + 4 * i + j] = (uint8_t)(r[i] >> (8 * j));
        }
    b3_compress(B3_IV, block, 64, 0, B3_PARENT | flags, out);
}

/* subtree over `len` bytes starting at chunk counter `t`: the left subtree holds the largest
 * power of two number of chunks strictly less than the total (BLAKE3 spec §2.1). */
static void b3_subtree(const uint8_t* in, size_t len, uint64_t t, int root, uint32_t out[8]) {
    if (len <= 1024) {
        b3_chunk_cv(in, len, t, root ? B3_ROOT : 0, out);
        return;
    }
    uint64_t chunks = (len + 1023) / 1024, left = 1;
    while (left * 2 < chunks) left *= 2;
    uint32_t l[8], r[8];
    b3_subtree(in, left * 1024, t, 0, l);
    b3_subtree(in + left * 1024, len - left * 1024, t + left, 0, r);
    b3_parent_cv(l, r, root ? B3_ROOT : 0, out);
}

void orc_blake3_chunk_cv(const uint8_t* in, size_t len, uint64_t t, uint32_t out[8]) { b3_chunk_cv(in, len, t, 0, out); }

void orc_blake3_parent_cv(const uint32_t l[8], const uint32_t r[8], uint32_t flags, uint32_t out[8]) {
    uint32_t tmp[8];
    b3_parent_cv(l, r, flags, tmp);
    memcpy(out, tmp, sizeof tmp);
}

void orc_blake3(const uint8_t* data, size_t len, uint8_t out[32]) {
    uint32_t cv[8];
    b3_subtree(data, len, 0, 1, cv);
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(cv[i] >> (8 * j));
}

/* ---------------------------------------------------------------- 4. BlobIndex */

/* blob_index.rs:44-57: `items` (sorted prior (hash, packfile) pairs, binary-searched,
 * :143-148) and `blobs_queued` (HashSet of blobs queued this session, :52, :109). */
struct orc_index {
    uint8_t* items;  /* sorted digests, 32 B each */
    size_t n_items;
    uint8_t* set;    /* open addressing, 33 B per slot: used flag + digest */
    size_t cap, used;
};

static uint64_t digest_key(const uint8_t* d) {
    uint64_t k;
    memcpy(&k, d, 8);
    return k;
}

orc_index* orc_index_new(const uint8_t* sorted, size_t n) {
    orc_index* ix = (orc_index*)calloc(1, sizeof *ix);
    if (!ix) return NULL;
    ix->n_items = n;
    if (n) {
        ix->items = (uint8_t*)malloc(n * 32);
        memcpy(ix->items, sorted, n * 32);
    }
    ix->cap = 1024;
    ix->set = (uint8_t*)calloc(ix->cap, 33);
    return ix;
}

void orc_index_free(orc_index* ix) {
    if (!ix) return;
    free(ix->items);
    free(ix->set);
    free(ix);
}

static int set_contains(const orc_index* ix, const uint8_t* d) {
    size_t mask = ix->cap - 1, i = digest_key(d) & mask;
    for (;;) {
        const uint8_t* s = ix->set + i * 33;
        if (!s[0]) return 0;
        if (memcmp(s + 1, d, 32) == 0) return 1;
        i = (i + 1) & mask;
    }
}

static void set_put(orc_index* ix, const uint8_t* d) {
    size_t mask = ix->cap - 1, i = digest_key(d) & mask;
    for (;;) {
        uint8_t* s = ix->set + i * 33;
        if (!s[0]) {
            s[0] = 1;
            memcpy(s + 1, d, 32);
            ix->used++;
            return;
        }
        if (memcmp(s + 1, d, 32) == 0) return;
        i = (i + 1) & mask;
    }
}

/* BlobIndex::is_blob_duplicate (blob_index.rs:130-140) = blobs_queued.contains || find_packfile */
int orc_index_is_duplicate(orc_index* ix, const uint8_t d[32]) {
    if (set_contains(ix, d)) return 1;
    size_t lo = 0, hi = ix->n_items;
    while (lo < hi) {
        size_t mid = (lo + hi) / 2;
        int c = memcmp(ix->items + mid * 32, d, 32);
        if (c == 0) return 1;
        if (c < 0) lo = mid + 1;
        else hi = mid;
    }
    return 0;
}

/* BlobIndex::add_to_packfile -> blobs_queued.insert (blob_index.rs:109-111); returns -1 on the
 * reference's DuplicateBlob error. */
int orc_index_insert(orc_index* ix, const uint8_t d[32]) {
    if (set_contains(ix, d)) return -1;
    if ((ix->used + 1) * 2 > ix->cap) {
        uint8_t* old = ix->set;
        size_t oc = ix->cap;
        ix->cap *= 2;
        ix->set = (uint8_t*)calloc(ix->cap, 33);
        ix->used = 0;
        for (size_t i = 0; i < oc; i++)
            if (old[i * 33]) set_put(ix, old + i * 33 + 1);
        free(old);
    }
    set_put(ix, d);
    return 0;
}

/* ---------------------------------------------------------------- 5. batch driver */

typedef struct {
    const uint8_t* data;
    const uint64_t* foff;
    const uint64_t* flen;
    size_t n_files;
    uint32_t min, avg, max;
    uint64_t small;
    orc_blob** per_file;
    size_t* per_file_n;
    size_t next;
    pthread_mutex_t mu;
    int err;
} orc_job;

/* the baseline's BLAKE3: the scalar restatement, or the 16-way SIMD one (bw_oracle_simd.c) that
 * mirrors the crate's hash_many backends (orc_set_blake3_simd) */
static void (*b3_hash)(const uint8_t*, size_t, uint8_t*) = orc_blake3;

int orc_set_blake3_simd(int on) {
    b3_hash = on && orc_blake3_simd_available() ? orc_blake3_fast : orc_blake3;
    return b3_hash == orc_blake3_fast;
}

/* dir_packer.rs:231-282 process_file + :285-311 add_file_blob (hash part) for one file */
static int process_one_file(orc_job* j, size_t f) {
    const uint8_t* src = j->data + j->foff[f];
    size_t len = j->flen[f];
    if ((uint64_t)len > j->small) {  /* dir_packer.rs:246: len > BLOB_DESIRED_TARGET_SIZE */
        size_t mc = 2 * (j->min / 2) < j->max ? 2 * (j->min / 2) : j->max;
        size_t cap = len / mc + 2, n = 0;
        uint64_t* h = (uint64_t*)malloc(cap * 8 * 3);
        if (!h) return -4;
        if (orc_fastcdc_chunks(src, len, j->min, j->avg, j->max, h, h + cap, h + 2 * cap, cap, &n)) {
            free(h);
            return -1;
        }
        orc_blob* b = (orc_blob*)calloc(n ? n : 1, sizeof(orc_blob));
        for (size_t i = 0; i < n; i++) {
            b[i].file = f;
            b[i].gear_hash = h[i];
            b[i].offset = h[cap + i];
            b[i].length = h[2 * cap + i];
            b3_hash(src + b[i].offset, b[i].length, b[i].digest);
        }
        free(h);
        j->per_file[f] = b;
        j->per_file_n[f] = n;
    } else {  /* dir_packer.rs:267-271: whole (small or empty) file is one blob */
        orc_blob* b = (orc_blob*)calloc(1, sizeof(orc_blob));
        b->file = f;
        b->length = len;
        b3_hash(src, len, b->digest);
        j->per_file[f] = b;
        j->per_file_n[f] = 1;
    }
    return 0;
}

static void* worker(void* arg) {
    orc_job* j = (orc_job*)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        size_t f = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (f >= j->n_files) break;
        int e = process_one_file(j, f);
        if (e) j->err = e;
    }
    return NULL;
}

int orc_process_files(const uint8_t* data, const uint64_t* file_off, const uint64_t* file_len,
                      size_t n_files, uint32_t min, uint32_t avg, uint32_t max,
                      uint64_t small_file_threshold, orc_index* ix, int threads, orc_blob* out,
                      size_t cap, size_t* n_out) {
    uint64_t ms, ml;
    if (orc_fastcdc_masks(min, avg, max, &ms, &ml) != 0) return -1;
    orc_job j;
    memset(&j, 0, sizeof j);
    j.data = data; j.foff = file_off; j.flen = file_len; j.n_files = n_files;
    j.min = min; j.avg = avg; j.max = max; j.small = small_file_threshold;
    j.per_file = (orc_blob**)calloc(n_files ? n_files : 1, sizeof(orc_blob*));
    j.per_file_n = (size_t*)calloc(n_files ? n_files : 1, sizeof(size_t));
    pthread_mutex_init(&j.mu, NULL);
    if (threads < 1) threads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
    for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, worker, &j);
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    free(th);
    pthread_mutex_destroy(&j.mu);
    int rc = j.err;
    /* canonical-order dedup gate: pack.rs:37 is_blob_duplicate, then (for a new blob) the
     * eventual blobs_queued insert of write_packfiles (pack.rs:150, blob_index.rs:109). */
    orc_index* own = NULL;
    if (!ix) ix = own = orc_index_new(NULL, 0);
    size_t n = 0;
    for (size_t f = 0; f < n_files && rc == 0; f++) {
        for (size_t i = 0; i < j.per_file_n[f]; i++) {
            orc_blob* b = &j.per_file[f][i];
            b->is_dup = (uint8_t)orc_index_is_duplicate(ix, b->digest);
            if (!b->is_dup) orc_index_insert(ix, b->digest);
            if (n < cap) out[n] = *b;
            n++;
        }
    }
    for (size_t f = 0; f < n_files; f++) free(j.per_file[f]);
    free(j.per_file);
    free(j.per_file_n);
    orc_index_free(own);
    *n_out = n;
    if (rc) return rc;
    return n > cap ? -2 : 0;
}
