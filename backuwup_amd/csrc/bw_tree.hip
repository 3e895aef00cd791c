// bw_tree.hip -- tree blobs: the file and directory trees backuwup stores beside the chunks.
//
// Replaces split_serialize_tree + add_tree_to_blobs (client/src/backup/filesystem/
// dir_packer.rs:314-390) for many trees at once.  A tree (mod.rs:63-77) is serialized with
// bincode 1.3.3's legacy `bincode::serialize` (Cargo.lock:117-119): little endian, fixed-width
// integers, enum variants as u32, strings and sequences with a u64 length, Option as a one-byte
// tag, BlobHash = [u8; 32] as 32 raw bytes (shared/src/types.rs:31):
//
//   u32 kind | u64 name_len | name | (u8 tag [u64]) x 3 for size, mtime, ctime |
//   u64 n_children | 32 B x n_children | u8 tag [32 B next_sibling]
//
// A tree with more than TREE_BLOB_MAX_CHILDREN (10,000, dir_packer.rs:35) children is split into
// pieces of at most 10,000 children; every piece but the last carries the next piece's hash as
// next_sibling, so the pieces hash from the last one back (one batched GPU round per piece
// depth).  Every piece is a blob that goes through the dedup gate (add_blob, pack.rs:37) in
// canonical order: trees in the order given, pieces in order.  The tree's hash -- the value
// add_tree_to_blobs returns and the parent lists as a child -- is its first piece's hash.
//
// Serialization is host work (names and metadata come from the file system walk); the BLAKE3 of
// every piece and the index run on the GPU through the same kernels as the file blobs.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "../../include/backuwup_gpu.h"
#include "bw_internal.h"

namespace {

constexpr uint64_t TREE_BLOB_MAX_CHILDREN = 10000;

inline uint8_t* put_u32(uint8_t* p, uint32_t v) {
    for (int i = 0; i < 4; i++) p[i] = (uint8_t)(v >> (8 * i));
    return p + 4;
}
inline uint8_t* put_u64(uint8_t* p, uint64_t v) {
    for (int i = 0; i < 8; i++) p[i] = (uint8_t)(v >> (8 * i));
    return p + 8;
}
inline uint8_t* put_opt_u64(uint8_t* p, bool some, uint64_t v) {
    *p++ = some ? 1 : 0;
    return some ? put_u64(p, v) : p;
}

uint64_t piece_len(const bw_tree& t, uint64_t nch, bool sibling) {
    return 4 + 8 + t.name_len + (1 + ((t.flags & BW_TREE_HAS_SIZE) ? 8 : 0)) +
           (1 + ((t.flags & BW_TREE_HAS_MTIME) ? 8 : 0)) + (1 + ((t.flags & BW_TREE_HAS_CTIME) ? 8 : 0)) + 8 +
           32 * nch + 1 + (sibling ? 32 : 0);
}

// Tree{kind, name, metadata, children[first .. first + nch), next_sibling}
uint8_t* serialize_piece(uint8_t* p, const bw_tree& t, uint64_t first, uint64_t nch, const uint8_t* sibling) {
    p = put_u32(p, t.kind);
    p = put_u64(p, t.name_len);
    if (t.name_len) memcpy(p, t.name, t.name_len);
    p += t.name_len;
    p = put_opt_u64(p, (t.flags & BW_TREE_HAS_SIZE) != 0, t.size);
    p = put_opt_u64(p, (t.flags & BW_TREE_HAS_MTIME) != 0, t.mtime);
    p = put_opt_u64(p, (t.flags & BW_TREE_HAS_CTIME) != 0, t.ctime);
    p = put_u64(p, nch);
    if (nch) memcpy(p, t.children + 32 * first, 32 * nch);
    p += 32 * nch;
    *p++ = sibling ? 1 : 0;
    if (sibling) {
        memcpy(p, sibling, 32);
        p += 32;
    }
    return p;
}

bool valid(const bw_tree& t) {
    return t.kind <= 1 && (t.name_len == 0 || t.name) && (t.n_children == 0 || t.children);
}

}  // namespace

extern "C" int bw_tree_serialize(const bw_tree* t, const uint8_t* next_sibling, uint8_t* out, uint64_t cap,
                                 uint64_t* n_out) {
    if (!t || !n_out || !valid(*t)) return BW_EINVAL;
    const uint64_t need = piece_len(*t, t->n_children, next_sibling != nullptr);
    *n_out = need;
    if (need > cap || !out) return BW_ENOSPC;
    serialize_piece(out, *t, 0, t->n_children, next_sibling);
    return BW_OK;
}

extern "C" int bw_tree_blobs(bw_ctx* ctx, const bw_tree* trees, uint64_t n, uint32_t flags, uint8_t* tree_hashes,
                             bw_tree_blob* out, uint64_t cap, uint64_t* n_out) {
    if (!ctx || !n_out || (n && (!trees || !tree_hashes))) return BW_EINVAL;
    const bool timing = getenv("BW_TREE_TIMING") != nullptr;
    auto now = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    double t_ser = 0, t_hash = 0, t0 = now();
    for (uint64_t i = 0; i < n; i++)
        if (!valid(trees[i])) return BW_EINVAL;
    // canonical blob list: tree i's pieces 0 .. p_i - 1
    std::vector<uint64_t> first_blob(n + 1, 0);
    uint64_t max_pieces = 0;
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t nch = trees[i].n_children;
        const uint64_t p = nch <= TREE_BLOB_MAX_CHILDREN ? 1 : (nch + TREE_BLOB_MAX_CHILDREN - 1) / TREE_BLOB_MAX_CHILDREN;
        first_blob[i + 1] = first_blob[i] + p;
        max_pieces = std::max(max_pieces, p);
    }
    const uint64_t nblobs = first_blob[n];
    *n_out = nblobs;
    if (out && cap < nblobs) return BW_ENOSPC;
    const bool dedup = !(flags & BW_F_NO_DEDUP);
    if (max_pieces == 1) {
        std::vector<uint64_t> lens(n);
        // no tree is split: serialize every tree (in parallel) straight into pinned staging, then
        // one batch hashes them and gates them in order on the device
        std::vector<uint64_t> offs(n);
        uint64_t total = 0;
        for (uint64_t i = 0; i < n; i++) {
            offs[i] = total;
            lens[i] = piece_len(trees[i], trees[i].n_children, false);
            total += lens[i];
        }
        const double ts = now();
        uint8_t* buf = bw::message_stage(ctx, total + 16);
        if (!buf) return BW_ENOMEM;
        bw::parallel_ranges(n, [&](uint64_t lo, uint64_t hi) {
            for (uint64_t i = lo; i < hi; i++) serialize_piece(buf + offs[i], trees[i], 0, trees[i].n_children, nullptr);
        });
        const double th = now();
        std::vector<uint8_t> dup(n, 0);
        // one piece per tree: the piece hashes are the tree hashes
        if (int rc = bw::hash_messages(ctx, buf, total, offs.data(), lens.data(), n, dedup, tree_hashes, dup.data()))
            return rc;
        const double tw = now();
        if (out)
            bw::parallel_ranges(n, [&](uint64_t lo, uint64_t hi) {
                for (uint64_t i = lo; i < hi; i++) {
                    bw_tree_blob& o = out[i];
                    memset(&o, 0, sizeof o);
                    o.tree = i;
                    o.length = lens[i];
                    memcpy(o.hash, tree_hashes + i * 32, 32);
                    o.is_dup = dup[i];
                }
            });
        if (timing)
            fprintf(stderr, "bw_tree_blobs: %llu trees (one piece each), serialize %.2f ms, hash+gate %.2f ms, "
                    "total %.2f ms\n", (unsigned long long)n, th - ts, tw - th, now() - t0);
        return BW_OK;
    }
    std::vector<uint8_t> hashes(nblobs * 32);
    std::vector<uint64_t> lens(nblobs);
    // round r hashes piece p_i - 1 - r of every tree that has one: the last pieces first (no
    // next_sibling), then each earlier piece with its successor's hash
    std::vector<uint8_t> buf;
    std::vector<uint64_t> offs, ln, blob_of;
    for (uint64_t r = 0; r < max_pieces; r++) {
        offs.clear();
        ln.clear();
        blob_of.clear();
        uint64_t total = 0;
        for (uint64_t i = 0; i < n; i++) {
            const uint64_t p = first_blob[i + 1] - first_blob[i];
            if (p <= r) continue;
            const uint64_t k = p - 1 - r;
            const uint64_t nch = std::min<uint64_t>(TREE_BLOB_MAX_CHILDREN, trees[i].n_children - k * TREE_BLOB_MAX_CHILDREN);
            const uint64_t l = piece_len(trees[i], p == 1 ? trees[i].n_children : nch, r > 0);
            offs.push_back(total);
            ln.push_back(l);
            blob_of.push_back(first_blob[i] + k);
            total += l;
        }
        const double ts = now();
        buf.resize(total + 16);
        for (uint64_t j = 0, i = 0; i < n; i++) {
            const uint64_t p = first_blob[i + 1] - first_blob[i];
            if (p <= r) continue;
            const uint64_t k = p - 1 - r;
            const uint64_t nch = p == 1 ? trees[i].n_children
                                        : std::min<uint64_t>(TREE_BLOB_MAX_CHILDREN,
                                                             trees[i].n_children - k * TREE_BLOB_MAX_CHILDREN);
            const uint8_t* sib = r > 0 ? &hashes[(first_blob[i] + k + 1) * 32] : nullptr;
            serialize_piece(buf.data() + offs[j], trees[i], k * TREE_BLOB_MAX_CHILDREN, nch, sib);
            lens[blob_of[j]] = ln[j];
            j++;
        }
        std::vector<uint8_t> h(offs.size() * 32);
        const double th = now();
        t_ser += th - ts;
        if (int rc = bw_blake3_hash_many(ctx, buf.data(), total, offs.data(), ln.data(), offs.size(), h.data()))
            return rc;
        t_hash += now() - th;
        for (uint64_t j = 0; j < offs.size(); j++) memcpy(&hashes[blob_of[j] * 32], &h[j * 32], 32);
    }
    std::vector<uint8_t> dup(nblobs, 0);
    const double td = now();
    if (!(flags & BW_F_NO_DEDUP) && nblobs)
        if (int rc = bw_index_check_insert(ctx, hashes.data(), nblobs, dup.data())) return rc;
    if (timing)
        fprintf(stderr, "bw_tree_blobs: %llu trees, serialize %.2f ms, hash %.2f ms, gate %.2f ms, total %.2f ms\n",
                (unsigned long long)n, t_ser, t_hash, now() - td, now() - t0);
    for (uint64_t i = 0; i < n; i++) memcpy(tree_hashes + 32 * i, &hashes[first_blob[i] * 32], 32);
    if (out)
        for (uint64_t i = 0; i < n; i++)
            for (uint64_t b = first_blob[i]; b < first_blob[i + 1]; b++) {
                bw_tree_blob& o = out[b];
                memset(&o, 0, sizeof o);
                o.tree = i;
                o.piece = b - first_blob[i];
                o.length = lens[b];
                memcpy(o.hash, &hashes[b * 32], 32);
                o.is_dup = dup[b];
            }
    return BW_OK;
}
