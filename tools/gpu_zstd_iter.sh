#!/bin/bash
# zstd iteration on the GPU: parity tests, then the bench on the text corpus at 1 and 8 GiB, the
# random corpus, and (ZSTD_PROF=1) a rocprofv3 kernel trace.  Each step has its own time limit;
# the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; echo "== $name $(date +%T)" >&2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a "$OUT/summary.txt"; return $rc; }
run zstd_tests 300 python -u -m pytest tests/test_zstd.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread || exit 1
run zstd_text1 300 python tools/zstd_bench.py --kind text --gib 1 --reps 3 || exit 1
run zstd_text8 400 python tools/zstd_bench.py --kind text --gib 8 --reps 2 --cpu-sample-mib 8 --check 4 || exit 1
run zstd_random 300 python tools/zstd_bench.py --kind random --gib 1 --reps 3 --cpu-sample-mib 8 || exit 1
if [ -n "$ZSTD_PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  run zstd_prof 400 rocprofv3 --kernel-trace --stats -d "$OUT/zprof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/zstd_bench.py" --kind text --gib 8 --reps 1 --cpu-sample-mib 1 --check 1 || exit 1
fi
