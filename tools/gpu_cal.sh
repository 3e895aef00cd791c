#!/bin/bash
# Session: FETCH_SIZE calibration of the hot path's read patterns (tools/fetch_cal.hip), then a
# rocprofv3 kernel trace of the bench.  Each step has its own limit; the chain stops on failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" >> "$OUT/summary.txt"; return $rc; }
run cal_time 120 ./build_ab/fetch_cal || exit 1
cd /tmp && export TMPDIR=/tmp
run cal_fetch 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/cal_fetch" -o run --pmc FETCH_SIZE -- "$GRAFT_REPO_ROOT/build_ab/fetch_cal" || exit 1
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-check || exit 1
exit 0
