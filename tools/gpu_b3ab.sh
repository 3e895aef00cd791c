#!/bin/bash
# A/B of the BLAKE3 leaf loaders on C2: parity tests of all three loaders, the bench line with
# block pairs (1) and aligned lines (2) alternating, then FETCH_SIZE of each leaf kernel.  Every
# GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a "$OUT/summary.txt"; return $rc; }
if [[ "${SKIP_TESTS:-0}" != 1 ]]; then
  run pytest_b3 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "blake3 or variants or c2 or fastcdc_backuwup" || exit 1
fi
for r in 1 2; do
  for l in 1 2; do
    run bench_l${l}_r${r} 300 python bench.py --b3-loads $l --steps ${STEPS:-160} --no-cpu-baseline ${BENCH_ARGS:-} || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
for l in 1 2; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc_fetch_l$l" -o run --pmc FETCH_SIZE -- python3 "$GRAFT_REPO_ROOT/bench.py" --b3-loads $l --steps 4 --warmup 1 --no-cpu-baseline --no-check --no-power > "$OUT/pmc_fetch_l$l.log" 2>&1 || exit 1
  echo "pmc_l$l rc=0" >> "$OUT/summary.txt"
done
# C1 with one batch in flight: the per-batch timeline (kernel trace) and the bench line
if [[ "${C1:-1}" == 1 ]]; then
  cd "$GRAFT_REPO_ROOT"
  run bench_c1_s1 300 python bench.py --workload c1 --streams 1 --steps 1500 --no-cpu-baseline || exit 1
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_c1s1" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload c1 --streams 1 --steps 300 --no-cpu-baseline --no-check --no-power > "$OUT/prof_c1s1.log" 2>&1 || exit 1
  cd "$GRAFT_REPO_ROOT" && python3 tools/trace_batches.py "$(ls $OUT/prof_c1s1/*/run_kernel_trace.csv $OUT/prof_c1s1/run_kernel_trace.csv 2>/dev/null | head -1)" 20 "$OUT/c1s1_batches.json" > "$OUT/c1s1_batches.log" 2>&1
  echo "c1 trace rc=$?" >> "$OUT/summary.txt"
fi
