#!/bin/bash
# Energy per byte of each pass: build_ab/ablate holds the scan alone, BLAKE3 alone, then both on
# two streams, each for HOLD seconds, while amd-smi samples socket power and clocks.
# Build first: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I backuwup_amd/csrc tools/ablate.hip -o build_ab/ablate
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
HOLD=${HOLD:-8}
for w in ${WHAT:-scan b3 both}; do
  ( for i in $(seq 1 200); do echo "T $(date +%s.%N)"; timeout -k 2 5 amd-smi metric -p -c 2>&1; sleep 0.1; done ) > "$OUT/power_$w.log" 2>&1 &
  P=$!
  sleep 1
  timeout -k 10 120 ./build_ab/ablate $w $HOLD > "$OUT/ablate_$w.log" 2>&1
  RC=$?
  sleep 1
  kill $P 2>/dev/null
  wait $P 2>/dev/null
  [ $RC -eq 0 ] || exit $RC
done
[ -n "${WHAT:-}" ] || timeout -k 10 300 ./build_ab/ablate > "$OUT/ablate_times.log" 2>&1
