#!/bin/bash
# A/B of the scan strip (bytes per lane) on small (C1) and large (C2) batches: parity tests and
# benches for each variant library under build_ab/ (BW_LIB) and the default build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" >> "$OUT/summary.txt"; return $rc; }
for v in S1024 S512 base; do
  if [ $v = base ]; then unset BW_LIB; else export BW_LIB="$GRAFT_REPO_ROOT/build_ab/lib$v.so"; fi
  run tests_$v 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_configs.py -k "not c2_full" || exit 1
  run c1_$v 300 python bench.py --workload c1 --no-cpu-baseline || exit 1
  run c2_$v 300 python bench.py --no-cpu-baseline || exit 1
done
