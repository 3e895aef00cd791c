#!/bin/bash
# Profiling session: ablation microbenchmarks, then rocprofv3 kernel trace + PMC passes on a
# 4 GiB bench run.  A step that times out/faults ends the session.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" >> "$OUT/summary.txt"; return $rc; }
fatal() { case $1 in 0) ;; 124|137|134|139) exit 1;; esac; }
if [ -x build_ab/ablate ]; then run ablate 300 ./build_ab/ablate; fatal $?; fi
cd /tmp && export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --gib ${PROF_GIB:-4} --steps 2 --warmup 1 --no-cpu-baseline --no-check"
run trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $B; fatal $?
run pmc1 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc1" -o run --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- $B; fatal $?
run pmc2 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc2" -o run --pmc FETCH_SIZE -- $B; fatal $?
run pmc3 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc3" -o run --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY TA_BUSY_avr SQ_INSTS_SALU -- $B; fatal $?
exit 0
