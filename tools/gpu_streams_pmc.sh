#!/bin/bash
# Session: bench at 1/2/3 batches in flight, then rocprofv3 kernel-trace stats and the
# FETCH_SIZE / WRITE_SIZE passes (separate runs) at the bench's default size, summarised into
# gpurun_out/pmc_traffic.json.  Each GPU step has its own limit; the chain stops on failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" >> "$OUT/summary.txt"; return $rc; }
GIB=${GIB:-16}
for s in ${STREAMS:-1 2 3}; do
  run bench_s$s 400 python bench.py --no-cpu-baseline --no-check --steps 8 --streams $s || exit 1
done
[ "${PMC:-1}" = 1 ] || exit 0
cd /tmp && export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --gib $GIB --steps 3 --warmup 1 --no-cpu-baseline --no-check"
run trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $B || exit 1
run pmc_fetch 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run --pmc FETCH_SIZE -- $B || exit 1
run pmc_write 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run --pmc WRITE_SIZE -- $B || exit 1
python3 "$GRAFT_REPO_ROOT/tools/pmc_traffic.py" "$OUT/pmc_fetch" "$OUT/pmc_write" $GIB "$OUT/pmc_traffic.json" > "$OUT/pmc_traffic.log" 2>&1
exit 0
