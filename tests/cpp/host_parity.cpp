// Host-side C++ mirror exercised the way the reference calls it (dir_packer.rs:254-286,
// pack.rs:31-39).  Prints one line per result; tests/test_cpp_host.py compares with the oracle.
#include <cstdio>
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
    return 0;
}
