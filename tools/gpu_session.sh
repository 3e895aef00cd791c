#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel trace.  Each GPU step runs under
# its own time limit and the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
MODE="${1:-all}"
run() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a "$OUT/summary.txt"; return $rc; }
: > "$OUT/summary.txt"
if [[ "$MODE" == *tests* || "$MODE" == all ]]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread || exit 1
fi
if [[ "$MODE" == *smoke* || "$MODE" == all ]]; then
  run smoke 300 python __graft_entry__.py || exit 1
fi
if [[ "$MODE" == *bench* || "$MODE" == all ]]; then
  run bench 600 python bench.py ${BENCH_ARGS:-} || exit 1
fi
if [[ "$MODE" == *prof* || "$MODE" == all ]]; then
  cd /tmp && export TMPDIR=/tmp
  # the bench command itself (default steps / batches in flight), so the per-launch durations of
  # the timed region can be compared with the bench line (tools/trace_split.py)
  run rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline || exit 1
  # the leaf pass's timed launches from the trace: mean, union per step, achieved on the union
  T=$(find "$OUT/prof" -name "*kernel_trace.csv" | head -1)
  [ -n "$T" ] && python3 "$GRAFT_REPO_ROOT/tools/trace_split.py" "$T" k_b3_lines 2 320 17179869184 > "$OUT/trace_split.json" 2>&1
fi
