#!/bin/bash
# Round-2 GPU session: each step under its own time limit, the chain stops at the first failure.
# Usage: gpu_r2.sh STEP... where STEP is tests | smoke | c2 | c1 | c3 | c4 | c5 | exchange | prof
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
run() { local name=$1 t=$2; shift 2; echo "== $name $(date +%T)" >&2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a "$OUT/summary.txt"; return $rc; }
: > "$OUT/summary.txt"
for step in "$@"; do
  case "$step" in
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread || exit 1 ;;
    smoke) run smoke 300 python __graft_entry__.py || exit 1 ;;
    c2) run bench_c2 600 python bench.py || exit 1 ;;
    c1) run bench_c1 600 python bench.py --workload c1 || exit 1 ;;
    c3) run bench_c3 900 python bench.py --workload c3 || exit 1 ;;
    c4) run bench_c4 900 python bench.py --workload c4 || exit 1 ;;
    c5) run bench_c5 900 python bench.py --workload c5 || exit 1 ;;
    pmc) run pmc 900 bash tools/gpu_pmc.sh || exit 1 ;;
    debug) run debug_check 600 python tools/debug_check.py || exit 1 ;;
    exchange) BW_HOST_TIMING=1 run bench_exchange 600 python bench.py --exchange --no-cpu-baseline || exit 1 ;;
    prof) cd /tmp && export TMPDIR=/tmp
          run rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline || exit 1
          cd "$GRAFT_REPO_ROOT" ;;
    *) echo "unknown step $step" >&2; exit 2 ;;
  esac
done
