#!/bin/bash
# Round-3 session m: same-box A/B of the library before the last stream-operation cuts
# (build_ab/libbw_prev.so: upload event, hipMemsetAsync) against the final one; C1 one in flight, C2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a "$OUT/summary.txt"; return $rc; }
for r in 1 2 3; do
  BW_LIB=$GRAFT_REPO_ROOT/build_ab/libbw_prev.so run c1s1_old_r$r 200 python bench.py --workload c1 --streams 1 --steps 1500 --no-cpu-baseline --no-calibrate || exit 1
  run c1s1_new_r$r 200 python bench.py --workload c1 --streams 1 --steps 1500 --no-cpu-baseline --no-calibrate || exit 1
done
BW_LIB=$GRAFT_REPO_ROOT/build_ab/libbw_prev.so run c2_old 300 python bench.py --no-cpu-baseline --no-calibrate || exit 1
run c2_new 300 python bench.py --no-cpu-baseline --no-calibrate || exit 1
