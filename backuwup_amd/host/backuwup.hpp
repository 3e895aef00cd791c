// backuwup.hpp -- C++ host-side mirror of the reference's call sites, over the C ABI.
//
// The reference is Rust; there is no Rust toolchain in this image, so the host side of the
// boundary is written in C++ (the reference is compiled code) with the reference's names,
// argument meaning and error behaviour.  A Rust maintainer binds the same C ABI instead
// (INTEGRATION.md).  Header-only; link with -lbackuwup_amd.
//
//   fastcdc::v2020::FastCDC / Chunk    client/src/backup/filesystem/dir_packer.rs:254-266
//   blake3::hash                       dir_packer.rs:286
//   packfile::BlobIndex                packfile/blob_index.rs:44-148
//   packfile::Manager::add_blob gate   packfile/pack.rs:31-39
//   dir_packer::process_file           dir_packer.rs:231-282 (batched over many files)
//   Tree / split_serialize_tree / add_tree_to_blobs   filesystem/mod.rs:63-77, dir_packer.rs:314-390
//   Manager::write_packfiles / serialize_packfile      packfile/pack.rs:115-227
//   compress_encrypt_blob (zstd level 3) + write_packfiles   packfile/pack.rs:58-80
//   BlobIndex::flush / load (index files)              packfile/blob_index.rs:151-240
//   Pool (the drop-ins over every GPU of the node)     client/src/main.rs:43, dir_packer.rs:166
//   NodeSession (N ranks in one process)               client/src/backup/mod.rs:64, blob_index.rs:130-148
#pragma once

#include <algorithm>
#include <array>
#include <atomic>
#include <cstdint>
#include <exception>
#include <memory>
#include <mutex>
#include <optional>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/backuwup_gpu.h"

namespace backuwup {

using BlobHash = std::array<uint8_t, 32>;  // shared/src/types.rs:31

struct Error : std::runtime_error {
    int rc;
    Error(int r, const std::string& m) : std::runtime_error(m), rc(r) {}
};

inline void check(int rc, bw_ctx* ctx = nullptr) {
    if (rc != BW_OK) {
        std::string m = bw_strerror(rc);
        if (ctx) m += std::string(": ") + bw_last_error(ctx);
        throw Error(rc, m);
    }
}

// One GPU context: stream, workspaces, the in-HBM index.  Not thread-safe (the reference
// serialises index access under the packer mutex, packfile/mod.rs:77).
class Context {
public:
    explicit Context(int device = 0) { check(bw_create(device, &h_)); }
    ~Context() { bw_destroy(h_); }
    Context(const Context&) = delete;
    Context& operator=(const Context&) = delete;
    bw_ctx* get() const { return h_; }

private:
    bw_ctx* h_ = nullptr;
};

namespace fastcdc {
namespace v2020 {

constexpr uint32_t MINIMUM_MIN = BW_MINIMUM_MIN, MINIMUM_MAX = BW_MINIMUM_MAX;
constexpr uint32_t AVERAGE_MIN = BW_AVERAGE_MIN, AVERAGE_MAX = BW_AVERAGE_MAX;
constexpr uint32_t MAXIMUM_MIN = BW_MAXIMUM_MIN, MAXIMUM_MAX = BW_MAXIMUM_MAX;

struct Chunk {
    uint64_t hash;
    size_t offset;
    size_t length;
};

// FastCDC::new(source, min_size, avg_size, max_size): the crate panics on out-of-range sizes;
// here the constructor throws Error(BW_EINVAL).  Iterating yields the chunks in order.
class FastCDC {
public:
    FastCDC(Context& ctx, const uint8_t* source, size_t len, uint32_t min_size, uint32_t avg_size,
            uint32_t max_size) {
        const uint32_t s0 = 2 * (min_size / 2);
        const uint32_t mc = s0 < max_size ? s0 : max_size;
        std::vector<bw_chunk> out(len / (mc ? mc : 1) + 2);
        uint64_t n = 0;
        check(bw_fastcdc_chunks(ctx.get(), source, len, min_size, avg_size, max_size, out.data(), out.size(), &n),
              ctx.get());
        chunks_.reserve(n);
        for (uint64_t i = 0; i < n; i++) chunks_.push_back({out[i].hash, out[i].offset, out[i].length});
    }
    // The Rust drop-in's form (rust/backuwup-gpu FastCDC::new): chunks AND hashes the source in one
    // submit on a context of `pool` (any type with with_context, i.e. backuwup::Pool) and keeps the
    // digests until destruction, so Pool::hash of one of these chunk slices is answered without a
    // second trip (bw_fastcdc_chunks_hashed); the source must stay unchanged meanwhile.
    template <class P, class = decltype(std::declval<P&>().home_device())>
    FastCDC(P& pool, const uint8_t* source, size_t len, uint32_t min_size, uint32_t avg_size, uint32_t max_size) {
        const uint32_t s0 = 2 * (min_size / 2);
        const uint32_t mc = s0 < max_size ? s0 : max_size;
        std::vector<bw_chunk> out(len / (mc ? mc : 1) + 2);
        uint64_t n = 0;
        pool.with_context([&](Context& ctx) {
            check(bw_fastcdc_chunks_hashed(ctx.get(), source, len, min_size, avg_size, max_size, out.data(), out.size(),
                                           &n, &kept_),
                  ctx.get());
            return 0;
        });
        chunks_.reserve(n);
        for (uint64_t i = 0; i < n; i++) chunks_.push_back({out[i].hash, out[i].offset, out[i].length});
    }
    ~FastCDC() { bw_fastcdc_release(kept_); }
    FastCDC(const FastCDC&) = delete;
    FastCDC& operator=(const FastCDC&) = delete;
    std::vector<Chunk>::const_iterator begin() const { return chunks_.begin(); }
    std::vector<Chunk>::const_iterator end() const { return chunks_.end(); }
    size_t size() const { return chunks_.size(); }

private:
    std::vector<Chunk> chunks_;
    uint64_t kept_ = 0;  // bw_fastcdc_release(0) is a no-op
};

}  // namespace v2020
}  // namespace fastcdc

namespace blake3 {
inline BlobHash hash(Context& ctx, const uint8_t* data, size_t len) {
    BlobHash h{};
    check(bw_blake3_hash(ctx.get(), data, len, h.data()), ctx.get());
    return h;
}
}  // namespace blake3

// packfile::blob_index::BlobIndex -- lives in HBM; `load` seeds it with the prior backups'
// sorted items (blob_index.rs:167-200); `is_blob_duplicate` answers in canonical order and
// inserts a new blob (the blobs_queued insert of blob_index.rs:109).
class BlobIndex {
public:
    explicit BlobIndex(Context& ctx, uint64_t capacity_hint = 0) : ctx_(ctx) {
        check(bw_index_reset(ctx.get(), capacity_hint), ctx.get());
    }
    void load(const std::vector<BlobHash>& sorted_items) {
        check(bw_index_seed(ctx_.get(), sorted_items.empty() ? nullptr : sorted_items[0].data(), sorted_items.size()),
              ctx_.get());
    }
    bool is_blob_duplicate(const BlobHash& h) {
        uint8_t dup = 0;
        check(bw_index_check_insert(ctx_.get(), h.data(), 1, &dup), ctx_.get());
        return dup != 0;
    }
    std::vector<uint8_t> is_blob_duplicate_many(const std::vector<BlobHash>& hs) {
        std::vector<uint8_t> dup(hs.size());
        if (!hs.empty()) check(bw_index_check_insert(ctx_.get(), hs[0].data(), hs.size(), dup.data()), ctx_.get());
        return dup;
    }
    uint64_t size() {
        uint64_t n = 0;
        check(bw_index_size(ctx_.get(), &n), ctx_.get());
        return n;
    }

private:
    Context& ctx_;
};

struct BlobTooLarge : Error {
    BlobTooLarge() : Error(BW_EINVAL, "Blob too large") {}
};

// The dedup gate of packfile::Manager::add_blob (pack.rs:31-39): BlobTooLarge above 3 MiB,
// nullopt-like `false` for a duplicate (Ok(None)), `true` when the blob goes on to be packed.
inline bool add_blob_gate(BlobIndex& index, const BlobHash& h, size_t len) {
    if (len > BW_BLOB_MAX_UNCOMPRESSED_SIZE) throw BlobTooLarge();
    return !index.is_blob_duplicate(h);
}

// process_file for a batch of files laid out back to back: CDC for files > 1 MiB, one blob per
// smaller (or empty) file, blake3 per blob, dedup verdict per blob -- canonical order.
inline std::vector<bw_blob> process_files(Context& ctx, const uint8_t* data, size_t data_len,
                                          const std::vector<uint64_t>& file_off,
                                          const std::vector<uint64_t>& file_len, const bw_params* params = nullptr) {
    bw_params p;
    if (params) p = *params;
    else bw_params_default(&p);
    const uint32_t s0 = 2 * (p.min_size / 2);
    const uint64_t mc = s0 < p.max_size ? s0 : p.max_size;
    uint64_t cap = 1;
    for (uint64_t l : file_len) cap += l / (mc ? mc : 1) + 2;
    std::vector<bw_blob> out(cap);
    uint64_t n = 0;
    check(bw_process_files(ctx.get(), data, data_len, file_off.data(), file_len.data(), file_off.size(), &p,
                           out.data(), cap, &n),
          ctx.get());
    out.resize(n);
    return out;
}

enum class TreeKind : uint32_t { File = BW_TREE_FILE, Dir = BW_TREE_DIR };

struct TreeMetadata {  // filesystem/mod.rs:63-68
    std::optional<uint64_t> size, mtime, ctime;
};

struct Tree {  // filesystem/mod.rs:70-77 (next_sibling is set by the split, not by callers)
    TreeKind kind = TreeKind::File;
    std::string name;
    TreeMetadata metadata;
    std::vector<BlobHash> children;
};

inline bw_tree to_c(const Tree& t) {
    bw_tree c{};
    c.kind = (uint32_t)t.kind;
    c.flags = (t.metadata.size ? BW_TREE_HAS_SIZE : 0) | (t.metadata.mtime ? BW_TREE_HAS_MTIME : 0) |
              (t.metadata.ctime ? BW_TREE_HAS_CTIME : 0);
    c.size = t.metadata.size.value_or(0);
    c.mtime = t.metadata.mtime.value_or(0);
    c.ctime = t.metadata.ctime.value_or(0);
    c.name = (const uint8_t*)t.name.data();
    c.name_len = t.name.size();
    c.children = t.children.empty() ? nullptr : t.children[0].data();
    c.n_children = t.children.size();
    return c;
}

// bincode::serialize(&tree) of one piece (dir_packer.rs:318)
inline std::vector<uint8_t> serialize(const Tree& t, const BlobHash* next_sibling = nullptr) {
    const bw_tree c = to_c(t);
    uint64_t n = 0;
    const int rc = bw_tree_serialize(&c, next_sibling ? next_sibling->data() : nullptr, nullptr, 0, &n);
    if (rc != BW_ENOSPC) check(rc);
    std::vector<uint8_t> out(n);
    check(bw_tree_serialize(&c, next_sibling ? next_sibling->data() : nullptr, out.data(), n, &n));
    return out;
}

// add_tree_to_blobs for many trees: every piece through the dedup gate in canonical order;
// returns the hash each tree contributes to its parent (its first piece's hash).
inline std::vector<BlobHash> add_trees_to_blobs(Context& ctx, const std::vector<Tree>& trees,
                                                std::vector<bw_tree_blob>* pieces = nullptr) {
    std::vector<bw_tree> c;
    c.reserve(trees.size());
    uint64_t cap = 0;
    for (const Tree& t : trees) {
        c.push_back(to_c(t));
        cap += t.children.size() <= BW_TREE_BLOB_MAX_CHILDREN
                   ? 1
                   : (t.children.size() + BW_TREE_BLOB_MAX_CHILDREN - 1) / BW_TREE_BLOB_MAX_CHILDREN;
    }
    std::vector<BlobHash> hashes(trees.size());
    std::vector<bw_tree_blob> out(pieces ? cap : 0);
    uint64_t n = 0;
    check(bw_tree_blobs(ctx.get(), c.data(), c.size(), 0, hashes.empty() ? nullptr : hashes[0].data(),
                        pieces ? out.data() : nullptr, cap, &n),
          ctx.get());
    if (pieces) *pieces = std::move(out);
    return hashes;
}

// ------------------------------------------------------------------ packfiles (pack.rs:115-227)
using PackfileId = std::array<uint8_t, 12>;  // shared/src/types.rs
using BlobNonce = std::array<uint8_t, 12>;
enum class BlobKind : uint8_t { FileChunk = BW_BLOB_FILE_CHUNK, Tree = BW_BLOB_TREE };  // filesystem/mod.rs:13-17

struct Blob {  // filesystem/mod.rs:46-51 (data = the raw bytes; framed as zstd store on the GPU)
    BlobHash hash;
    BlobKind kind;
    std::vector<uint8_t> data;
};

// Manager::write_packfiles over a queue of unique blobs: nonces[i] and the packfile ids are the
// caller's random draws (the reference's getrandom, pack.rs:74-76, :207-208); ids must hold at
// least as many entries as packfiles result (packfile_count()).  Returns (id, bytes) per packfile.
inline size_t packfile_count(const std::vector<Blob>& blobs) {
    std::vector<uint64_t> lens;
    for (const Blob& b : blobs) lens.push_back(b.data.size());
    uint64_t n = 0, total = 0;
    const int rc = bw_pack_plan(lens.data(), lens.size(), BW_PACK_ZSTD_STORE, nullptr, 0, &n, &total);
    if (rc != BW_ENOSPC && rc != BW_OK) check(rc);
    return n;
}

inline std::vector<std::pair<PackfileId, std::vector<uint8_t>>> write_packfiles(
    Context& ctx, const std::array<uint8_t, 32>& prk, const std::vector<Blob>& blobs,
    const std::vector<BlobNonce>& nonces, const std::vector<PackfileId>& ids) {
    std::vector<uint64_t> lens, offs;
    std::vector<uint8_t> data, hashes, kinds, nb;
    for (size_t i = 0; i < blobs.size(); i++) {
        offs.push_back(data.size());
        lens.push_back(blobs[i].data.size());
        data.insert(data.end(), blobs[i].data.begin(), blobs[i].data.end());
        hashes.insert(hashes.end(), blobs[i].hash.begin(), blobs[i].hash.end());
        kinds.push_back((uint8_t)blobs[i].kind);
        nb.insert(nb.end(), nonces.at(i).begin(), nonces.at(i).end());
    }
    uint64_t np = 0, total = 0;
    std::vector<bw_packfile> plan(packfile_count(blobs));
    check(bw_pack_plan(lens.data(), lens.size(), BW_PACK_ZSTD_STORE, plan.data(), plan.size(), &np, &total));
    if (ids.size() < np) throw Error(BW_EINVAL, "not enough packfile ids");
    std::vector<uint8_t> idb, out(total);
    for (size_t k = 0; k < np; k++) idb.insert(idb.end(), ids[k].begin(), ids[k].end());
    check(bw_pack_build(ctx.get(), prk.data(), data.data(), offs.data(), lens.data(), lens.size(), hashes.data(),
                        kinds.data(), nb.data(), BW_PACK_ZSTD_STORE, plan.data(), np, idb.data(), out.data()),
          ctx.get());
    std::vector<std::pair<PackfileId, std::vector<uint8_t>>> res;
    for (size_t k = 0; k < np; k++)
        res.emplace_back(ids[k], std::vector<uint8_t>(out.begin() + plan[k].offset,
                                                      out.begin() + plan[k].offset + plan[k].size));
    return res;
}

// compress_encrypt_blob + write_packfiles with the reference's level-3 zstd (pack.rs:58-80,
// 115-227): the frames are made and staged on the GPU, the grouping runs over their sizes, and the
// packfiles are sealed from the staging.  ids must hold at least the resulting packfile count
// (8 per blob is always enough).  Returns (id, bytes) per packfile.
inline std::vector<std::pair<PackfileId, std::vector<uint8_t>>> write_packfiles_zstd(
    Context& ctx, const std::array<uint8_t, 32>& prk, const std::vector<Blob>& blobs,
    const std::vector<BlobNonce>& nonces, const std::vector<PackfileId>& ids) {
    std::vector<uint64_t> lens, offs, frame(blobs.size());
    std::vector<uint8_t> data, hashes, kinds, nb;
    for (size_t i = 0; i < blobs.size(); i++) {
        offs.push_back(data.size());
        lens.push_back(blobs[i].data.size());
        data.insert(data.end(), blobs[i].data.begin(), blobs[i].data.end());
        hashes.insert(hashes.end(), blobs[i].hash.begin(), blobs[i].hash.end());
        kinds.push_back((uint8_t)blobs[i].kind);
        nb.insert(nb.end(), nonces.at(i).begin(), nonces.at(i).end());
    }
    // all-empty queues (e.g. one empty file) leave `data` empty: hand the library a real pointer anyway
    static const uint8_t none[1] = {0};
    check(bw_pack_compress(ctx.get(), data.empty() ? none : data.data(), offs.data(), lens.data(), lens.size(),
                           frame.data()),
          ctx.get());
    uint64_t np = 0, total = 0;
    const int rc = bw_pack_plan(frame.data(), frame.size(), 0, nullptr, 0, &np, &total);
    if (rc != BW_ENOSPC && rc != BW_OK) check(rc);
    std::vector<bw_packfile> plan(np);
    check(bw_pack_plan(frame.data(), frame.size(), 0, plan.data(), plan.size(), &np, &total));
    if (ids.size() < np) throw Error(BW_EINVAL, "not enough packfile ids");
    std::vector<uint8_t> idb, out(total);
    for (size_t k = 0; k < np; k++) idb.insert(idb.end(), ids[k].begin(), ids[k].end());
    check(bw_pack_build_compressed_host(ctx.get(), prk.data(), hashes.data(), kinds.data(), nb.data(), plan.data(), np,
                                        idb.data(), out.data()),
          ctx.get());
    std::vector<std::pair<PackfileId, std::vector<uint8_t>>> res;
    for (size_t k = 0; k < np; k++)
        res.emplace_back(ids[k], std::vector<uint8_t>(out.begin() + plan[k].offset,
                                                      out.begin() + plan[k].offset + plan[k].size));
    return res;
}

// ------------------------------------------------------------------ index files (blob_index.rs)
using IndexEntry = std::pair<BlobHash, PackfileId>;

// BlobIndex::push for every entry, then the final unconditional flush: (file_num, bytes) per file
inline std::vector<std::pair<uint32_t, std::vector<uint8_t>>> index_flush(Context& ctx,
                                                                         const std::array<uint8_t, 32>& prk,
                                                                         const std::vector<IndexEntry>& entries,
                                                                         uint32_t last_file_num) {
    std::vector<uint8_t> e;
    for (const auto& x : entries) {
        e.insert(e.end(), x.first.begin(), x.first.end());
        e.insert(e.end(), x.second.begin(), x.second.end());
    }
    uint64_t nf = 0, total = 0;
    int rc = bw_index_files_build(ctx.get(), prk.data(), e.data(), entries.size(), last_file_num, nullptr, 0, nullptr,
                                  0, &nf, &total);
    if (rc != BW_ENOSPC) check(rc, ctx.get());
    std::vector<uint8_t> out(total);
    std::vector<bw_index_file> files(nf);
    check(bw_index_files_build(ctx.get(), prk.data(), e.data(), entries.size(), last_file_num, out.data(), total,
                               files.data(), nf, &nf, &total),
          ctx.get());
    std::vector<std::pair<uint32_t, std::vector<uint8_t>>> res;
    for (const auto& f : files)
        res.emplace_back(f.file_num, std::vector<uint8_t>(out.begin() + f.offset, out.begin() + f.offset + f.size));
    return res;
}

// BlobIndex::load: decrypt + parse the files on the GPU and seed the context's index; returns
// `items` sorted by hash as the reference keeps them (blob_index.rs:197).
inline std::vector<IndexEntry> index_load(Context& ctx, const std::array<uint8_t, 32>& prk,
                                          const std::vector<std::pair<uint32_t, std::vector<uint8_t>>>& files) {
    std::vector<uint8_t> data;
    std::vector<bw_index_file> tab;
    uint64_t cap = 0;
    for (const auto& f : files) {
        tab.push_back(bw_index_file{f.first, 0, data.size(), f.second.size(), 0});
        data.insert(data.end(), f.second.begin(), f.second.end());
        cap += f.second.size() / BW_INDEX_ENTRY_BYTES + 1;
    }
    std::vector<uint8_t> rec(cap * BW_INDEX_ENTRY_BYTES);
    uint64_t n = 0, bad = 0;
    check(bw_index_load_files(ctx.get(), prk.data(), data.data(), tab.data(), tab.size(), rec.data(), cap, &n, &bad),
          ctx.get());
    std::vector<IndexEntry> items(n);
    for (uint64_t i = 0; i < n; i++) {
        std::copy(rec.begin() + i * 44, rec.begin() + i * 44 + 32, items[i].first.begin());
        std::copy(rec.begin() + i * 44 + 32, rec.begin() + i * 44 + 44, items[i].second.begin());
    }
    std::sort(items.begin(), items.end(), [](const IndexEntry& a, const IndexEntry& b) { return a.first < b.first; });
    return items;
}

// ---------------------------------------------------------------- every GPU of the node
// The drop-ins' context pool (the Rust crate's Pool, INTEGRATION.md "Every GPU of the node"): the
// reference's tasks call FastCDC::new / blake3::hash with no context, one task per file on one
// worker thread per core (client/src/main.rs:43, dir_packer.rs:166).  `per_device` contexts per
// listed device (a device may repeat), context j on devices[j % n]; the k-th calling thread gets home
// slot k and home device devices[k % n]; with_context takes the first free context from the home
// slot on; hash() sends a small message to the home device's hash service with no context held
// (bw_blake3_hash_dropin_device), and BW_EAGAIN (a message over 64 KiB, a service that could not take
// it in time) through a pooled context's launch path.
class Pool {
public:
    explicit Pool(std::vector<int> devices = {}, int per_device = 16) : devices_(std::move(devices)) {
        if (devices_.empty()) {
            int n = 0;
            check(bw_device_count(&n));
            if (n <= 0) throw Error(BW_EINVAL, "no GPU for the drop-in pool");
            for (int d = 0; d < n; d++) devices_.push_back(d);
        }
        const size_t total = (size_t)std::max(per_device, 1) * devices_.size();
        for (size_t j = 0; j < total; j++) ctx_.emplace_back(new Context(devices_[j % devices_.size()]));
        mu_ = std::vector<std::mutex>(total);
    }
    const std::vector<int>& devices() const { return devices_; }
    size_t home_slot() const {
        thread_local size_t slot = next_slot().fetch_add(1);
        return slot;
    }
    int home_device() const { return devices_[home_slot() % devices_.size()]; }
    template <class F>
    auto with_context(F&& f) -> decltype(f(std::declval<Context&>())) {
        const size_t n = ctx_.size(), start = home_slot() % n;
        for (size_t k = 0; k < n; k++) {
            const size_t j = (start + k) % n;
            std::unique_lock<std::mutex> lk(mu_[j], std::try_to_lock);
            if (lk.owns_lock()) return f(*ctx_[j]);
        }
        std::lock_guard<std::mutex> lk(mu_[start]);
        return f(*ctx_[start]);
    }
    // blake3::hash(data) for read-only memory (kept chunk digests answer first)
    BlobHash hash(const uint8_t* data, size_t len) {
        BlobHash h{};
        const int rc = bw_blake3_hash_dropin_device(home_device(), data, len, h.data());
        if (rc == BW_OK) return h;
        if (rc != BW_EAGAIN) check(rc);
        return with_context([&](Context& c) {
            const uint64_t off = 0, n = len;
            static const uint8_t empty[16] = {0};
            check(bw_blake3_hash_many(c.get(), len ? data : empty, len, &off, &n, 1, h.data()), c.get());
            return h;
        });
    }

private:
    static std::atomic<size_t>& next_slot() {
        static std::atomic<size_t> n{0};
        return n;
    }
    std::vector<int> devices_;
    std::vector<std::unique_ptr<Context>> ctx_;
    std::vector<std::mutex> mu_;
};

// ---------------------------------------------------------------- N ranks in one process
// One backup session over N ranks of THIS process (the reference packs in one process,
// client/src/backup/mod.rs:64): rank r = a context on devices[r] whose index is rank r's shard of
// the session's BlobIndex (owner = digest[0] >> (8 - log2 N)) and a communicator from
// bw_comm_init_all (RCCL, one device per rank) or bw_comm_init_local (in-process transport).
// process_files shards the batch's files rank-major (contiguous, balanced by bytes), and each rank's
// thread submits its share with BW_F_NO_DEDUP, exchanges its digests and waits for its verdicts;
// the blobs come back in canonical order with `file` = the index in the batch.
class NodeSession {
public:
    NodeSession(const std::vector<int>& devices, bool rccl, uint64_t index_hint = 1u << 16,
                const bw_params* params = nullptr)
        : comms_(devices.size(), nullptr) {
        const size_t n = devices.size();
        if (n == 0 || (n & (n - 1))) throw Error(BW_EINVAL, "NodeSession: a power-of-two number of ranks");
        check(rccl ? bw_comm_init_all(devices.data(), (int)n, BW_COMM_DEFAULT_TIMEOUT_MS, comms_.data())
                   : bw_comm_init_local(devices.data(), (int)n, comms_.data()));
        for (int d : devices) {
            ctx_.emplace_back(new Context(d));
            check(bw_index_reset(ctx_.back()->get(), index_hint), ctx_.back()->get());
        }
        if (params) p_ = *params;
        else bw_params_default(&p_);
        p_.flags |= BW_F_NO_DEDUP;
    }
    ~NodeSession() {  // the communicators first: destroying one finishes its queued exchanges, which use the contexts
        for (bw_comm* c : comms_) bw_comm_destroy(c);
        ctx_.clear();
    }
    NodeSession(const NodeSession&) = delete;
    NodeSession& operator=(const NodeSession&) = delete;

    std::vector<bw_blob> process_files(const uint8_t* data, const std::vector<uint64_t>& file_off,
                                       const std::vector<uint64_t>& file_len) {
        const size_t n = ctx_.size(), nf = file_len.size();
        double total = 0;
        for (uint64_t l : file_len) total += (double)l + 1.0;  // (+1: empty files count too)
        std::vector<size_t> cut(n + 1, 0);
        double acc = 0;
        size_t f = 0;
        for (size_t r = 1; r < n; r++) {
            while (f < nf && acc + (double)file_len[f] + 1.0 <= total * (double)r / (double)n) acc += (double)file_len[f++] + 1.0;
            cut[r] = f;
        }
        cut[n] = nf;
        std::vector<std::vector<bw_blob>> out(n);
        std::vector<std::exception_ptr> err(n);
        std::vector<std::thread> th;
        for (size_t r = 0; r < n; r++)
            th.emplace_back([&, r] {
                try {
                    const size_t lo = cut[r], hi = cut[r + 1];
                    uint64_t a = 0, b = 0;
                    if (hi > lo) {
                        a = UINT64_MAX;
                        for (size_t i = lo; i < hi; i++) {
                            a = std::min(a, file_off[i]);
                            b = std::max(b, file_off[i] + file_len[i]);
                        }
                    }
                    std::vector<uint64_t> offs(hi - lo), lens(file_len.begin() + lo, file_len.begin() + hi);
                    uint64_t cap = 1;
                    for (size_t i = lo; i < hi; i++) {
                        offs[i - lo] = file_off[i] - a;
                        cap += file_len[i] / (p_.min_size ? p_.min_size : 1) + 2;
                    }
                    bw_ctx* c = ctx_[r]->get();
                    uint64_t t = 0, got = 0;
                    check(bw_submit_host(c, b > a ? data + a : nullptr, b - a, offs.data(), lens.data(), offs.size(), &p_, &t), c);
                    check(bw_exchange_dedup(c, comms_[r], t), c);
                    out[r].resize(cap);
                    check(bw_wait(c, t, out[r].data(), cap, &got), c);
                    out[r].resize(got);
                    for (auto& x : out[r]) x.file += lo;
                } catch (...) {
                    err[r] = std::current_exception();
                }
            });
        for (auto& t : th) t.join();
        for (auto& e : err)
            if (e) std::rethrow_exception(e);
        std::vector<bw_blob> all;
        for (auto& v : out) all.insert(all.end(), v.begin(), v.end());
        return all;
    }

private:
    std::vector<std::unique_ptr<Context>> ctx_;
    std::vector<bw_comm*> comms_;
    bw_params p_{};
};

}  // namespace backuwup
