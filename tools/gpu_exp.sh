#!/bin/bash
# Experiment session: parity tests first, then each "name|bench args" variant; each GPU step
# has its own time limit and the chain stops at the first failure.  Variant args may set
# BW_LIB=<path> as a leading token to pick an alternate library build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest_gpu rc=$rc" >> "$OUT/summary.txt"; [ $rc = 0 ] || exit 1
fi
for spec in "$@"; do
  name="${spec%%|*}"; args="${spec#*|}"
  envs=""
  if [[ "$args" == BW_LIB=* ]]; then envs="${args%% *}"; args="${args#* }"; fi
  env $envs timeout -k 10 500 python bench.py $args > "$OUT/bench_$name.log" 2>&1
  rc=$?; echo "bench_$name rc=$rc" >> "$OUT/summary.txt"; [ $rc = 0 ] || exit 1
done
