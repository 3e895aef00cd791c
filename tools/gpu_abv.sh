#!/bin/bash
# A/B of diagnostic library variants against the release library on one workload: alternating
# benches (ROUNDS rounds), then one FETCH_SIZE pass per library when PMC=1.  Each GPU step has its
# own time limit and the chain stops at the first failure.
#   VARIANTS="scannt other" ROUNDS=2 BENCH_ARGS="--workload c1" PMC=1 bash tools/gpu_abv.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
[ -n "${TAG:-}" ] || [ "${KEEP_SUMMARY:-0}" = 1 ] || : > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" >> "$OUT/summary.txt"; return $rc; }
libof() { if [ "$1" = base ]; then echo "$GRAFT_REPO_ROOT/backuwup_amd/libbackuwup_amd.so"; else echo "$GRAFT_REPO_ROOT/backuwup_amd/libbackuwup_amd_$1.so"; fi; }
for r in $(seq 1 "${ROUNDS:-2}"); do
  for v in base $VARIANTS; do
    BW_LIB=$(libof $v) run "${TAG:-}bench_${v}_$r" 300 python bench.py --no-cpu-baseline --no-check ${BENCH_ARGS} || exit 1
  done
done
if [ "${PMC:-0}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  for v in base $VARIANTS; do
    BW_LIB=$(libof $v) timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/${TAG:-}pmc_$v" -o run --pmc FETCH_SIZE -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 4 --warmup 1 --no-cpu-baseline --no-check ${BENCH_ARGS} > "$OUT/${TAG:-}pmc_$v.log" 2>&1 || exit 1
  done
fi
exit 0
