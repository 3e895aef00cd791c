/* Experiment (CPU, not product code): how many rounds does a block-parallel speculative dfast
 * parse need before every block of a blob matches the serial parse?
 *
 * Round r parses every block k of a blob from (a) the hash tables block k-1 ended with in round
 * r-1 and (b) block k-1's repeat offsets of round r-1 (block 0 starts from empty tables and the
 * initial offsets, so it is exact in round 1).  Table writes of the dfast parse are monotonic in
 * position, so "the tables after block k-1" is exactly block k's input in the serial parse once
 * every earlier block has converged: block k is exact by round k+1 at the latest.  The question is
 * how much earlier the chain settles on real data.
 *
 *   gcc -O2 -o /tmp/zspec tools/zstd_spec_rounds.c && /tmp/zspec <file> [blob_bytes]
 */
#include "../oracle/bw_oracle_zstd.c"

#include <stdio.h>

typedef struct {
    uint32_t* hl;  /* tables at the block's end */
    uint32_t* hs;
    uint32_t rep[3];
    uint64_t sig;  /* digest of the block's sequences */
    size_t nseq;
} blockstate;

static uint64_t seq_sig(const zseqstore* ss, size_t lastLL) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < ss->nseq; i++) {
        h = (h ^ ss->seq[i].litLength) * 1099511628211ull;
        h = (h ^ ss->seq[i].offset) * 1099511628211ull;
        h = (h ^ ss->seq[i].mlBase) * 1099511628211ull;
    }
    return (h ^ lastLL) * 1099511628211ull;
}

static int rounds_for_blob(const uint8_t* src, size_t n, int* nblocks_out, int verbose) {
    zparams const p = zstd_params(n);
    const size_t BS = ZB_BLOCK_MAX, nb = (n + BS - 1) / BS;
    const size_t nl = (size_t)1 << p.hlog, ns = (size_t)1 << p.clog;
    zseqstore ss;
    ss.seq = malloc(sizeof(zseq) * (BS / 3 + 2));
    ss.lit = malloc(BS + 8);
    blockstate* truth = calloc(nb, sizeof(blockstate));
    blockstate* prev = calloc(nb, sizeof(blockstate));
    blockstate* cur = calloc(nb, sizeof(blockstate));
    for (size_t k = 0; k < nb; k++) {
        truth[k].hl = calloc(nl, 4); truth[k].hs = calloc(ns, 4);
        prev[k].hl = calloc(nl, 4); prev[k].hs = calloc(ns, 4);
        cur[k].hl = calloc(nl, 4); cur[k].hs = calloc(ns, 4);
    }
    zms ms;
    ms.p = p;
    ms.base = src - 1;
    ms.dictLimit = 1;
    /* serial truth (every block treated as compressed: the reps always carry) */
    {
        uint32_t* hl = calloc(nl, 4); uint32_t* hs = calloc(ns, 4);
        uint32_t rep[3] = {1, 4, 8};
        for (size_t k = 0; k < nb; k++) {
            const size_t bs = k + 1 < nb ? BS : n - k * BS;
            ss.nseq = 0; ss.nlit = 0;
            ms.hashLong = hl; ms.hashSmall = hs;
            size_t lastLL = bs >= 7 ? dfast_block(&ms, &ss, rep, src + k * BS, bs) : bs;
            truth[k].sig = seq_sig(&ss, lastLL);
            truth[k].nseq = ss.nseq;
            memcpy(truth[k].rep, rep, sizeof rep);
        }
        free(hl); free(hs);
    }
    int round = 0;
    for (;;) {
        round++;
        int ok = 0, first_bad = -1;
        for (size_t k = 0; k < nb; k++) {
            const size_t bs = k + 1 < nb ? BS : n - k * BS;
            uint32_t rep[3] = {1, 4, 8};
            if (k == 0 || round == 1) {
                memset(cur[k].hl, 0, nl * 4); memset(cur[k].hs, 0, ns * 4);
            } else {
                memcpy(cur[k].hl, prev[k - 1].hl, nl * 4); memcpy(cur[k].hs, prev[k - 1].hs, ns * 4);
            }
            if (k && round > 1) memcpy(rep, prev[k - 1].rep, sizeof rep);
            ss.nseq = 0; ss.nlit = 0;
            ms.hashLong = cur[k].hl; ms.hashSmall = cur[k].hs;
            size_t lastLL = bs >= 7 ? dfast_block(&ms, &ss, rep, src + k * BS, bs) : bs;
            cur[k].sig = seq_sig(&ss, lastLL);
            memcpy(cur[k].rep, rep, sizeof rep);
            const int good = cur[k].sig == truth[k].sig && !memcmp(cur[k].rep, truth[k].rep, sizeof rep);
            ok += good;
            if (!good && first_bad < 0) first_bad = (int)k;
        }
        if (verbose) printf("  round %d: %d/%zu blocks equal to serial, first wrong %d\n", round, ok, nb, first_bad);
        blockstate* t = prev; prev = cur; cur = t;
        if (ok == (int)nb) break;
    }
    for (size_t k = 0; k < nb; k++) {
        free(truth[k].hl); free(truth[k].hs); free(prev[k].hl); free(prev[k].hs); free(cur[k].hl); free(cur[k].hs);
    }
    free(truth); free(prev); free(cur); free(ss.seq); free(ss.lit);
    *nblocks_out = (int)nb;
    return round;
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    fseek(f, 0, SEEK_END);
    size_t n = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t* buf = malloc(n);
    if (fread(buf, 1, n, f) != n) return 2;
    fclose(f);
    size_t blob = argc > 2 ? (size_t)atoll(argv[2]) : n;
    int verbose = argc > 3;
    for (size_t o = 0; o < n; o += blob) {
        size_t len = n - o < blob ? n - o : blob;
        int nbk = 0;
        int r = rounds_for_blob(buf + o, len, &nbk, verbose);
        printf("blob @%zu len %zu blocks %d rounds %d\n", o, len, nbk, r);
    }
    return 0;
}
