#!/bin/bash
# Round-3 session o: C4 (1 M small files) with 1, 2 and 4 BLAKE3 leaves per lane (BW_OPT_B3_GROUP).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a "$OUT/summary.txt"; return $rc; }
for g in 1 2 4 1 2; do run c4_g${g}_$RANDOM 400 python bench.py --workload c4 --no-cpu-baseline --no-calibrate --b3-group $g || exit 1; done
