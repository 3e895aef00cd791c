#!/bin/bash
# HBM traffic per launch (FETCH_SIZE and WRITE_SIZE in separate passes: 3 + 2 TCC counters do not
# fit one pass) on the default C2 bench command, summarised into gpurun_out/pmc_traffic.json with
# the source digest of the measured kernels.  Each pass is killed if it hangs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
B="python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-check --no-holds"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run --pmc FETCH_SIZE -- $B > "$OUT/pmc_fetch.log" 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run --pmc WRITE_SIZE -- $B > "$OUT/pmc_write.log" 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT" && python3 tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" 16 "$OUT/pmc_traffic.json" > "$OUT/pmc_traffic.log" 2>&1
