// Host-side C++ mirror exercised the way the reference calls it (dir_packer.rs:254-286,
// pack.rs:31-39).  Prints one line per result; tests/test_cpp_host.py compares with the oracle.
#include <algorithm>
#include <cstdio>
#include <string>
#include <thread>
#include <vector>

#include "../../backuwup_amd/host/backuwup.hpp"

static std::vector<uint8_t> splitmix(uint64_t seed, size_t n) {
    std::vector<uint8_t> out(n);
    uint64_t x = seed;
    for (size_t i = 0; i < n; i += 8) {
        x += 0x9E3779B97F4A7C15ull;
        uint64_t z = x;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        for (int k = 0; k < 8 && i + k < n; k++) out[i + k] = (uint8_t)(z >> (8 * k));
    }
    return out;
}

int main() {
    using namespace backuwup;
    Context ctx(0);
    auto data = splitmix(0, 8400953);
    fastcdc::v2020::FastCDC chunker(ctx, data.data(), data.size(), 262144, 1048576, 3145728);
    for (const auto& c : chunker) {
        BlobHash h = blake3::hash(ctx, data.data() + c.offset, c.length);
        printf("chunk %llu %zu %zu ", (unsigned long long)c.hash, c.offset, c.length);
        for (auto b : h) printf("%02x", b);
        printf("\n");
    }
    try {
        fastcdc::v2020::FastCDC bad(ctx, data.data(), 1000, 63, 256, 1024);
        printf("invalid-params not rejected\n");
    } catch (const Error& e) {
        printf("invalid-params rc=%d\n", e.rc);
    }
    BlobIndex index(ctx);
    BlobHash a = blake3::hash(ctx, data.data(), 100), b = blake3::hash(ctx, data.data(), 101);
    index.load({a});
    const int g1 = add_blob_gate(index, a, 100);  // seeded -> duplicate (Ok(None))
    const int g2 = add_blob_gate(index, b, 101);  // new
    const int g3 = add_blob_gate(index, b, 101);  // now a duplicate
    printf("gate %d %d %d %d\n", g1, g2, g3, (int)index.size());
    try {
        add_blob_gate(index, a, BW_BLOB_MAX_UNCOMPRESSED_SIZE + 1);
    } catch (const BlobTooLarge&) {
        printf("too-large ok\n");
    }
    // the file tree of the A.5 file (dir_packer.rs:237-274): chunk hashes as children
    Tree ft;
    ft.kind = TreeKind::File;
    ft.name = "a5.bin";
    ft.metadata.size = data.size();
    ft.metadata.mtime = 1700000000;
    for (const auto& c : chunker) ft.children.push_back(blake3::hash(ctx, data.data() + c.offset, c.length));
    auto bytes = serialize(ft);
    printf("tree-bytes ");
    for (auto x : bytes) printf("%02x", x);
    printf("\n");
    auto th = add_trees_to_blobs(ctx, {ft, ft});
    printf("tree-hash ");
    for (auto x : th[0]) printf("%02x", x);
    printf("\n");
    // two packfiles' worth of blobs (pack.rs:115-227), then their index entries as files
    std::array<uint8_t, 32> prk;
    for (int k = 0; k < 32; k++) prk[k] = (uint8_t)(0x40 + k);
    std::vector<Blob> blobs;
    std::vector<BlobNonce> nonces;
    const size_t sizes[4] = {0, 1000, 3 << 20, 70000};
    for (size_t i = 0; i < 4; i++) {
        Blob bl;
        bl.data.assign(data.begin() + 5 * i, data.begin() + 5 * i + sizes[i]);
        bl.hash = blake3::hash(ctx, bl.data.data(), bl.data.size());
        bl.kind = i == 3 ? BlobKind::Tree : BlobKind::FileChunk;
        blobs.push_back(bl);
        BlobNonce nn;
        for (int k = 0; k < 12; k++) nn[k] = (uint8_t)(7 * i + k);
        nonces.push_back(nn);
    }
    std::vector<PackfileId> ids(packfile_count(blobs));
    for (size_t p = 0; p < ids.size(); p++)
        for (int k = 0; k < 12; k++) ids[p][k] = (uint8_t)(0xa0 + 16 * p + k);
    auto packs = write_packfiles(ctx, prk, blobs, nonces, ids);
    std::vector<IndexEntry> entries;
    for (const auto& pk : packs) {
        printf("packfile %zu ", pk.second.size());
        for (auto x : pk.second) printf("%02x", x);
        printf("\n");
    }
    for (size_t i = 0; i < blobs.size(); i++) entries.push_back({blobs[i].hash, ids[i < 3 ? 0 : 1]});
    auto files = index_flush(ctx, prk, entries, 9);
    for (const auto& f : files) {
        printf("index %u ", f.first);
        for (auto x : f.second) printf("%02x", x);
        printf("\n");
    }
    auto items = index_load(ctx, prk, files);
    printf("index-load %zu %d\n", items.size(), (int)std::is_sorted(items.begin(), items.end()));
    // the level-3 chain over compressible blobs (tests/test_cpp_host.py rebuilds the same bytes)
    std::vector<Blob> zb;
    std::vector<BlobNonce> zn;
    const size_t zsizes[4] = {0, 5000, 200000, (1u << 20) + 17};
    for (size_t j = 0; j < 4; j++) {
        Blob bl;
        bl.data.resize(zsizes[j]);
        for (size_t i = 0; i < zsizes[j]; i++) bl.data[i] = (uint8_t)('a' + ((i * (j + 3)) / 7) % 26);
        bl.hash = blake3::hash(ctx, bl.data.data(), bl.data.size());
        bl.kind = BlobKind::FileChunk;
        zb.push_back(bl);
        BlobNonce nn;
        for (int k = 0; k < 12; k++) nn[k] = (uint8_t)(3 * j + k + 1);
        zn.push_back(nn);
    }
    std::vector<PackfileId> zids(8);
    for (size_t p = 0; p < zids.size(); p++)
        for (int k = 0; k < 12; k++) zids[p][k] = (uint8_t)(0x30 + 16 * p + k);
    for (const auto& pk : write_packfiles_zstd(ctx, prk, zb, zn, zids)) {
        printf("packfile-zstd %zu ", pk.second.size());
        for (auto x : pk.second) printf("%02x", x);
        printf("\n");
    }
    // a queue of nothing but one empty file: the mirror's staging vector stays empty
    Blob empty;
    empty.hash = blake3::hash(ctx, data.data(), 0);
    empty.kind = BlobKind::FileChunk;
    for (const auto& pk : write_packfiles_zstd(ctx, prk, {empty}, {zn[0]}, zids)) {
        printf("packfile-zstd-empty %zu ", pk.second.size());
        for (auto x : pk.second) printf("%02x", x);
        printf("\n");
    }
    // ---- N ranks in one process (NodeSession over bw_comm_init_local: four ranks on device 0), a
    // corpus of small files with CDC files between them and 30 % copies; three batches, the third
    // repeating the first, one with fewer files than ranks (tests/test_cpp_host.py: one oracle index)
    {
        const size_t nfiles = 603;
        std::vector<uint64_t> off(nfiles), len(nfiles);
        std::vector<uint8_t> corpus;
        for (size_t i = 0; i < nfiles; i++) {
            const size_t src = (i < 600 && i % 10 == 3) ? i - 3 : i;  // a copy of the file three before
            const size_t n = src < 600 ? 4096 + (src * 7919) % 61440 : (1u << 20) + 1 + src * 12345;
            auto bytes = splitmix(1000 + src, n);
            off[i] = corpus.size();
            len[i] = n;
            corpus.insert(corpus.end(), bytes.begin(), bytes.end());
        }
        NodeSession ns({0, 0, 0, 0}, false, 1u << 14);
        const size_t batches[3][2] = {{0, 301}, {600, 603}, {0, 301}};
        for (int bi = 0; bi < 3; bi++) {
            const size_t lo = batches[bi][0], hi = batches[bi][1];
            std::vector<uint64_t> bo(off.begin() + lo, off.begin() + hi), bl(len.begin() + lo, len.begin() + hi);
            // the big files first in the second batch: ranks get 0 or 1 files each
            auto blobs = ns.process_files(corpus.data(), bo, bl);
            for (const auto& b : blobs) {
                printf("ns %d %llu %llu %llu %llu ", bi, (unsigned long long)(b.file + lo), (unsigned long long)b.offset,
                       (unsigned long long)b.length, (unsigned long long)b.gear_hash);
                for (auto x : b.digest) printf("%02x", x);
                printf(" %d\n", (int)b.is_dup);
            }
        }
        // ---- the drop-in pool over the device list [0, 0]: 8 threads, small messages (home device's
        // service) and a few over 64 KiB (a pooled context), every digest printed
        Pool pool({0, 0}, 2);
        const size_t nm = 400;
        std::vector<BlobHash> got(nm);
        std::vector<std::thread> th;
        for (int t = 0; t < 8; t++)
            th.emplace_back([&, t] {
                for (size_t i = t; i < nm; i += 8) {
                    const size_t n = (i % 50 == 7) ? 70000 + i : (i * 331) % 65537;
                    got[i] = pool.hash(corpus.data() + i * 1000, n);
                }
            });
        for (auto& x : th) x.join();
        for (size_t i = 0; i < nm; i++) {
            const size_t n = (i % 50 == 7) ? 70000 + i : (i * 331) % 65537;
            printf("ph %zu %zu ", i * 1000, n);
            for (auto x : got[i]) printf("%02x", x);
            printf("\n");
        }
        // the reference's loop exactly as the Rust drop-ins run it (dir_packer.rs:254-266 -> :286):
        // FastCDC::new on a pooled context (chunks and digests in one submit), then blake3::hash of
        // every chunk slice answered from the kept digests; the three big files, one thread each
        const uint64_t hits0 = bw_blake3_kept_hits();
        std::vector<std::vector<std::string>> lines(3);
        std::vector<std::thread> tf;
        for (int t = 0; t < 3; t++)
            tf.emplace_back([&, t] {
                const size_t f = 600 + t;
                fastcdc::v2020::FastCDC chunker(pool, corpus.data() + off[f], len[f], 262144, 1048576, 3145728);
                for (const auto& c : chunker) {
                    BlobHash h = pool.hash(corpus.data() + off[f] + c.offset, c.length);
                    char buf[160];
                    int k = snprintf(buf, sizeof buf, "pf %zu %llu %zu %zu ", f, (unsigned long long)c.hash, c.offset, c.length);
                    for (auto x : h) k += snprintf(buf + k, sizeof buf - k, "%02x", x);
                    lines[t].push_back(buf);
                }
            });
        for (auto& x : tf) x.join();
        for (auto& v : lines)
            for (auto& l : v) printf("%s\n", l.c_str());
        printf("pf-kept %llu\n", (unsigned long long)(bw_blake3_kept_hits() - hits0));
    }
    return 0;
}
