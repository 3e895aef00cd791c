#!/bin/bash
# Round-3 session l: bench lines after the bench loop's prebuilt ctypes calls (no library change):
# C1 one batch in flight x3, C1 three in flight, C2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a "$OUT/summary.txt"; return $rc; }
for r in 1 2 3; do run c1s1_r$r 200 python bench.py --workload c1 --streams 1 --steps 1500 --no-cpu-baseline || exit 1; done
run c1s3 200 python bench.py --workload c1 --steps 1500 --no-cpu-baseline || exit 1
run c2 300 python bench.py || exit 1
