#!/bin/bash
# Round-3 session n: every GPU test, then a same-box A/B of event scopes (build_ab/libbw_prev.so:
# default-flag events; the tree: device-scope ordering events, fence-free timing marks) on C1 one and
# three in flight and C2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a "$OUT/summary.txt"; return $rc; }
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread || exit 1
for r in 1 2 3; do
  BW_LIB=$GRAFT_REPO_ROOT/build_ab/libbw_prev.so run c1s1_old_r$r 200 python bench.py --workload c1 --streams 1 --steps 1500 --no-cpu-baseline --no-calibrate || exit 1
  run c1s1_new_r$r 200 python bench.py --workload c1 --streams 1 --steps 1500 --no-cpu-baseline --no-calibrate || exit 1
done
BW_LIB=$GRAFT_REPO_ROOT/build_ab/libbw_prev.so run c1s3_old 200 python bench.py --workload c1 --steps 1500 --no-cpu-baseline --no-calibrate || exit 1
run c1s3_new 200 python bench.py --workload c1 --steps 1500 --no-cpu-baseline --no-calibrate || exit 1
BW_LIB=$GRAFT_REPO_ROOT/build_ab/libbw_prev.so run c2_old 300 python bench.py --no-cpu-baseline --no-calibrate || exit 1
run c2_new 300 python bench.py --no-cpu-baseline --no-calibrate || exit 1
