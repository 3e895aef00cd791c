#!/bin/bash
# Round-3 session t: counters of C1 with one batch in flight (for the next round's plan): HBM fetch per
# kernel, and SQ wave occupancy / busy cycles / VALU instructions, in separate passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
B="python3 $GRAFT_REPO_ROOT/bench.py --workload c1 --streams 1 --steps 40 --warmup 2 --no-cpu-baseline --no-check --no-calibrate --no-power"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc_c1_fetch" -o run --pmc FETCH_SIZE -- $B > "$OUT/pmc_c1_fetch.log" 2>&1 || exit 1
echo "fetch rc=0" >> "$OUT/summary.txt"
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc_c1_sq" -o run --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE -- $B > "$OUT/pmc_c1_sq.log" 2>&1 || exit 1
echo "sq rc=0" >> "$OUT/summary.txt"
