#!/bin/bash
# A/B session: GPU tests on the current library (B), then benches of build_ab/libA.so and B,
# B also with two batches in flight.  Each GPU step has its own time limit; stop at a failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" >> "$OUT/summary.txt"; return $rc; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread || exit 1
fi
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then export BW_LIB="$GRAFT_REPO_ROOT/build_ab/libA.so"; else unset BW_LIB; fi
    run bench_${v}_$r 300 python bench.py --no-cpu-baseline --no-check --steps 8 ${BENCH_ARGS} || exit 1
  done
done
unset BW_LIB
run bench_B_s2 300 python bench.py --no-cpu-baseline --no-check --steps 8 --streams 2 ${BENCH_ARGS} || exit 1
exit 0
