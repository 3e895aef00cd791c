#!/bin/bash
# Seal session: seal tests, bench --seal, rocprofv3 kernel trace + one SQ counter pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" >> "$OUT/summary.txt"; return $rc; }
run test_seal 300 python -u -m pytest tests/test_seal.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread || exit 1
run bench_seal 400 python bench.py --seal --steps 4 --no-cpu-baseline ${BENCH_ARGS} || exit 1
cd /tmp && export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --seal --gib 4 --steps 2 --warmup 1 --no-cpu-baseline --no-check"
run prof_seal 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_seal" -o run -- $B || exit 1
run pmc_seal 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc_seal" -o run --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- $B || exit 1
exit 0
