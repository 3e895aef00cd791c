#!/bin/bash
# Round-3 session s: the §8(f) rows on the final tree -- sealing, packing (store frames and the level-3
# zstd chain) of C2's unique blobs, file trees of the C4 batch -- and C1 with two batches in flight.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a "$OUT/summary.txt"; return $rc; }
run c2_seal 400 python bench.py --no-cpu-baseline --no-calibrate --steps 40 --seal || exit 1
run c2_pack 400 python bench.py --no-cpu-baseline --no-calibrate --steps 40 --pack || exit 1
run c2_pack_l3 500 python bench.py --no-cpu-baseline --no-calibrate --steps 20 --pack-l3 || exit 1
run c4_trees 500 python bench.py --workload c4 --no-cpu-baseline --no-calibrate --steps 20 --trees || exit 1
run c1_s2 200 python bench.py --workload c1 --streams 2 --steps 1500 --no-cpu-baseline || exit 1
