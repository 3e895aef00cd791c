#!/bin/bash
# zstd level-3 measurements: tools/zstd_bench.py per corpus kind, then a rocprofv3 kernel trace of
# the text corpus.  Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; echo "== $name $(date +%T)" >&2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a "$OUT/summary.txt"; return $rc; }
for k in ${ZSTD_KINDS:-text mixed random}; do
  run zstd_$k 400 python tools/zstd_bench.py --kind $k --gib ${ZSTD_GIB:-1} ${ZSTD_ARGS:-} || exit 1
done
if [ -n "$ZSTD_PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  run zstd_prof 400 rocprofv3 --kernel-trace --stats -d "$OUT/zprof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/zstd_bench.py" --kind text --gib ${ZSTD_GIB:-1} --reps 2 --cpu-sample-mib 8 --check 1 || exit 1
fi
