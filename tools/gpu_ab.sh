#!/bin/bash
# A/B + counters session: tests on the current library, bench of library A (build_ab/libA.so)
# and B (current), then rocprofv3 PMC passes on B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" >> "$OUT/summary.txt"; return $rc; }
fatal() { case $1 in 124|137|134|139) exit 1;; esac; }
run pytest_gpu 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider || exit 1
for v in A B; do
  if [ $v = A ]; then export BW_LIB="$GRAFT_REPO_ROOT/build_ab/libA.so"; else unset BW_LIB; fi
  run bench_$v 400 python bench.py --no-cpu-baseline --no-check --steps 8 || exit 1
done
unset BW_LIB
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > "$OUT/counters.txt" 2>&1
B="python3 $GRAFT_REPO_ROOT/bench.py --gib 4 --steps 2 --warmup 1 --no-cpu-baseline --no-check"
run pmc1 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc1" -o run --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- $B; fatal $?
run pmc2 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc2" -o run --pmc FETCH_SIZE -- $B; fatal $?
run pmc3 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc3" -o run --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY TA_BUSY_avr -- $B; fatal $?
exit 0
