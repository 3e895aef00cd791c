#!/bin/bash
# SQ counters of the zstd kernels (tools/zstd_bench.py, text corpus, 1 warm-up + 1 timed call), two
# passes of at most 8 SQ counters each, every pass killed if it hangs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
B="python3 $GRAFT_REPO_ROOT/tools/zstd_bench.py --kind ${ZSTD_KIND:-text} --gib ${ZSTD_GIB:-1} --reps 1 --cpu-sample-mib 1 --check 0"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/zpmc1" -o run --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- $B > "$OUT/zpmc1.log" 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/zpmc2" -o run --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES -- $B > "$OUT/zpmc2.log" 2>&1 || exit 1
