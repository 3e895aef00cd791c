#!/bin/bash
# Samples the GPU's power and clocks (amd-smi, read-only) while the C2 bench runs, to tell a
# power/clock-bound pipeline from a unit-bound one.  Output: gpurun_out/clock_probe.log
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
timeout -k 5 30 amd-smi metric --help > "$OUT/amdsmi_help.log" 2>&1
timeout -k 5 30 amd-smi metric -p -c > "$OUT/amdsmi_idle.log" 2>&1
( for i in $(seq 1 400); do echo "T $(date +%s.%N)"; timeout -k 2 5 amd-smi metric -p -c 2>&1; sleep 0.05; done ) > "$OUT/clock_probe.log" 2>&1 &
P=$!
timeout -k 10 300 python bench.py --no-cpu-baseline --no-check --steps 2000 > "$OUT/bench_probe.log" 2>&1
RC=$?
kill $P 2>/dev/null
wait $P 2>/dev/null
exit $RC
