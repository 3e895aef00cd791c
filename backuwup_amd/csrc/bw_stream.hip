// bw_stream.hip -- one long file split across the ranks of a communicator (SURVEY.md §8e "single long
// stream"; VERDICT r4 #2: behind the C ABI, so a Rust host can shard one VM image across GPUs).
//
// The reference chunks a file serially from its start (a new FastCDC per file, dir_packer.rs:
// 254-266).  Split over W ranks, rank r owns the file bytes [S_r, S_{r+1}), S_k = len * k / W, and
// holds the window [S_r - max, S_{r+1} + max) in HBM.  It chunks its window from a speculative start
// (the window's start; rank 0 from the file start); CDC resynchronises, so the chain soon equals the
// true one.  The ranks then settle where each true chain enters, in rounds of one 16-byte allgather:
//   every rank publishes P_r = its last cut <= S_{r+1} (the last rank: the file end) and whether it
//   rechunked; rank r takes entry = P_{r-1}; if entry is a cut of its chain (or its start), the
//   chain from entry on is the true one -- a cut depends only on its start and the bytes after it --
//   otherwise it rechunks its window from entry.  Rounds end when no rank rechunked.
// Random data settles in one round; data without content-defined cuts (zeros) carries the true
// phase one rank per round (at most W + 1 rounds).  The windows suffice: true chunks are <= max, so
// the true last cut <= S_{r+1} lies inside rank r+1's back halo, and a chunk starting before S_{r+1}
// is decided by bytes up to its start + max, inside rank r's forward halo.
// Rank r emits the chunks starting in [entry_r, P_r) (the last rank: to the file end), so the chunk
// straddling S_{r+1} is hashed once, by rank r+1, which holds it whole.  In rank order the emitted
// chunks are the file's chunks in offset order -- canonical order for bw_exchange_dedup, which sends
// only them.  The Python form of the same settlement (backuwup_amd/stream_split.py) drives the gloo
// tests with the oracle's chunker.
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "bw_internal.h"

using namespace bw;

extern "C" int bw_stream_window(uint64_t file_len, int rank, int world, uint32_t max_size, uint64_t* lo,
                                uint64_t* hi) {
    if (!lo || !hi || world < 1 || rank < 0 || rank >= world) return BW_EINVAL;
    const unsigned __int128 L = file_len;
    const uint64_t s0 = (uint64_t)(L * (unsigned)rank / (unsigned)world);
    const uint64_t s1 = (uint64_t)(L * (unsigned)(rank + 1) / (unsigned)world);
    *lo = s0 > max_size ? s0 - max_size : 0;
    *hi = std::min<uint64_t>(file_len, s1 + max_size);
    return BW_OK;
}

namespace {

struct Chain {
    uint64_t start = 0, ticket = 0;
    std::vector<uint64_t> cuts;  // absolute chunk ends, ascending
};

// Chunk file[start, hi) of the window (file byte x at d_window + x - lo) as a file of its own: one
// batch, CDC forced (a file split across ranks is far above the small-file rule), hashed, no index.
int chunk_from(bw_ctx* c, const uint8_t* d_window, uint64_t lo, uint64_t hi, uint64_t start, const bw_params* prm,
               Chain& ch, std::vector<bw_blob>& tmp) {
    bw_params p = *prm;
    p.small_file_threshold = 0;
    p.flags |= BW_F_NO_DEDUP;
    p.flags &= ~BW_F_NO_HASH;
    const uintptr_t at = (uintptr_t)(d_window + (start - lo));
    const uint64_t mis = at & 15;  // the library reads from 16-byte aligned batch pointers
    const uint8_t* base = (const uint8_t*)(at - mis);
    const uint64_t flen = hi - start, foff = mis;
    if (int rc = bw_submit_device(c, base, mis + flen, &foff, &flen, 1, &p, &ch.ticket)) return rc;
    const uint64_t cap = flen / std::min<uint64_t>(2 * (p.min_size / 2), p.max_size) + 2;
    if (tmp.size() < cap) tmp.resize(cap);
    uint64_t n = 0;
    if (int rc = bw_wait(c, ch.ticket, tmp.data(), tmp.size(), &n)) return rc;
    ch.start = start;
    ch.cuts.resize(n);
    for (uint64_t i = 0; i < n; i++) ch.cuts[i] = start + tmp[i].offset + tmp[i].length;
    return BW_OK;
}

}  // namespace

extern "C" int bw_chunk_stream_shard(bw_ctx* c, bw_comm* comm, const uint8_t* d_window, uint64_t file_len,
                                     const bw_params* params, bw_stream_shard* out) {
    if (!c || !comm || !out) return BW_EINVAL;
    memset(out, 0, sizeof *out);
    bw_params def;
    if (!params) {
        bw_params_default(&def);
        params = &def;
    }
    if (params->min_size < BW_MINIMUM_MIN || params->min_size > BW_MINIMUM_MAX || params->avg_size < BW_AVERAGE_MIN ||
        params->avg_size > BW_AVERAGE_MAX || params->max_size < BW_MAXIMUM_MIN || params->max_size > BW_MAXIMUM_MAX)
        return BW_EINVAL;
    // the halos are max wide: with min > max a truncated window's last chunk (<= min, returned whole
    // by cut()) is not the file's, and its true chain can enter before lo (the header's note)
    if (params->min_size > params->max_size || params->avg_size > params->max_size) return BW_EINVAL;
    if (comm_failed(comm)) return BW_ECOMM;
    const int r = comm_rank(comm), W = comm_world(comm);
    if (comm_device(comm) != ctx_device(c)) return BW_EINVAL;
    std::string err;
    uint64_t lo = 0, hi = 0;
    bw_stream_window(file_len, r, W, params->max_size, &lo, &hi);
    const unsigned __int128 L = file_len;
    const uint64_t S_r = (uint64_t)(L * (unsigned)r / (unsigned)W);
    const uint64_t S_next = (uint64_t)(L * (unsigned)(r + 1) / (unsigned)W);
    if (file_len && !d_window) return BW_EINVAL;
    Chain ch;
    std::vector<bw_blob> tmp;
    std::vector<uint64_t> all(2 * W);
    if (file_len && hi > lo)  // every rank chunks from its window's start (rank 0 from the file's)
        if (int rc = chunk_from(c, d_window, lo, hi, r == 0 ? 0 : lo, params, ch, tmp)) return rc;
    uint64_t entry = 0, last = 0;
    for (uint32_t round = 1;; round++) {
        // P_r: the last cut <= S_{r+1} on the current chain (its start if none); the last rank: the end
        uint64_t P = file_len;
        if (r != W - 1) {
            auto it = std::upper_bound(ch.cuts.begin(), ch.cuts.end(), S_next);
            P = it == ch.cuts.begin() ? ch.start : *(it - 1);
        }
        uint64_t mine[2] = {P, 0};
        if (int rc = comm_allgather2(comm, mine, all.data(), err)) return rc;
        entry = r == 0 ? 0 : all[2 * (r - 1)];
        last = all[2 * r];
        if (entry < lo || entry > S_r) return BW_EHIP;  // cannot happen (see the window argument)
        bool changed = false;
        if (file_len && entry != ch.start && !std::binary_search(ch.cuts.begin(), ch.cuts.end(), entry)) {
            if (int rc = chunk_from(c, d_window, lo, hi, entry, params, ch, tmp)) return rc;
            changed = true;
        }
        mine[0] = P;
        mine[1] = changed;
        if (int rc = comm_allgather2(comm, mine, all.data(), err)) return rc;
        bool any = false;
        for (int k = 0; k < W; k++) any |= all[2 * k + 1] != 0;
        out->rounds = round;
        if (!any) break;
        if (round > (uint32_t)W + 2) return BW_EHIP;  // the phase travels one rank per round at most
    }
    if (!file_len) return BW_OK;
    // the chunks starting in [entry, stop): chunk i spans [cut_{i-1}, cut_i), cut_{-1} = start
    const uint64_t stop = r == W - 1 ? file_len : last;
    uint64_t first = ~0ull, n = 0;
    for (uint64_t i = 0; i < ch.cuts.size(); i++) {
        const uint64_t s = i ? ch.cuts[i - 1] : ch.start;
        if (s >= entry && s < stop) {
            if (first == ~0ull) first = i;
            n++;
        }
    }
    if (first == ~0ull) first = 0;
    out->ticket = ch.ticket;
    out->first_blob = first;
    out->n_blobs = n;
    out->chain_start = ch.start;
    return batch_set_exchange_range(c, ch.ticket, first, n);
}
