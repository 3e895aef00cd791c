#!/bin/bash
# Round-3 session k: same-box A/B of the s09 library (build_ab/libbw_s09.so, before the 2 x max
# segments, the group -> blob map and the table-upload kernel) against the current one, C1 with one
# batch in flight and C2, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a "$OUT/summary.txt"; return $rc; }
for r in 1 2; do
  BW_LIB=$GRAFT_REPO_ROOT/build_ab/libbw_s09.so run c1s1_old_r$r 200 python bench.py --workload c1 --streams 1 --steps 1500 --no-cpu-baseline --no-calibrate || exit 1
  run c1s1_new_r$r 200 python bench.py --workload c1 --streams 1 --steps 1500 --no-cpu-baseline --no-calibrate || exit 1
done
for r in 1 2; do
  BW_LIB=$GRAFT_REPO_ROOT/build_ab/libbw_s09.so run c2_old_r$r 300 python bench.py --no-cpu-baseline --no-calibrate || exit 1
  run c2_new_r$r 300 python bench.py --no-cpu-baseline --no-calibrate || exit 1
done
