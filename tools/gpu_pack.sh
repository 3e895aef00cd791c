#!/bin/bash
# Pack session: pack tests, bench --pack, rocprofv3 kernel trace of the same command.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" >> "$OUT/summary.txt"; return $rc; }
run test_pack 300 python -u -m pytest tests/test_pack.py tests/test_seal.py tests/test_cpp_host.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread || exit 1
run bench_pack 400 python bench.py --pack --seal --steps 4 --no-cpu-baseline ${BENCH_ARGS} || exit 1
cd /tmp && export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --pack --gib 4 --steps 2 --warmup 1 --no-cpu-baseline --no-check"
run prof_pack 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_pack" -o run -- $B || exit 1
exit 0
