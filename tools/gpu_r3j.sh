#!/bin/bash
# Round-3 session j: GPU tests, BW_OPT_B3_MAP A/B on C1 (one in flight) and C2, C4, and the C1
# one-in-flight batch timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a "$OUT/summary.txt"; return $rc; }
if [[ "${SKIP_TESTS:-0}" != 1 ]]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} || exit 1
fi
for r in 1 2; do
  for m in 1 0; do run c1s1_m${m}_r$r 200 python bench.py --workload c1 --streams 1 --steps 1500 --no-cpu-baseline --b3-map $m || exit 1; done
done
for m in 1 0; do run c2_m$m 300 python bench.py --no-cpu-baseline --b3-map $m || exit 1; done
run c4 400 python bench.py --workload c4 --no-cpu-baseline || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_c1s1" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload c1 --streams 1 --steps 300 --no-cpu-baseline --no-check --no-power --no-calibrate > "$OUT/prof_c1s1.log" 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT" && python3 tools/trace_batches.py "$(ls $OUT/prof_c1s1/*/run_kernel_trace.csv $OUT/prof_c1s1/run_kernel_trace.csv 2>/dev/null | head -1)" 20 "$OUT/c1s1_batches.json" 1 > "$OUT/c1s1_batches.log" 2>&1
echo "c1 trace rc=$?" >> "$OUT/summary.txt"
