#!/bin/bash
# VERDICT r3 #3 measurement: the BLAKE3 leaf pass over bytes the scan just brought into the Infinity
# Cache (slab pipeline) against the product's order (whole scan, then whole hash), on an 8 GiB
# C2-shaped stream.  Per arrangement: rate, socket power while it is held (amdsmi, beside it) ->
# pJ/B; then rocprofv3 FETCH_SIZE per kernel.  Every GPU step has its own time limit; the script
# stops at the first failure.  Build first (CPU): hipcc --offload-arch=gfx950 -O3 -std=c++17
# -I backuwup_amd/csrc tools/slab.hip -o build_ab/slab
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/slab_summary.txt"
HOLD=${HOLD:-10}
CONFIGS=${CONFIGS:-"cold:0:4 cold:0:1 slab:64:1 slab:128:1 slab:96:2 slab:192:1 slab:64:4 scan:0:4 hash:0:4"}
for cfg in $CONFIGS; do
  IFS=: read -r mode s g <<< "$cfg"
  name="${mode}_${s}_${g}"
  ( sleep 3; timeout -k 5 $((HOLD)) python3 tools/power_sample.py $((HOLD - 5)) "$OUT/power_$name.json" ) &
  P=$!
  timeout -k 10 120 ./build_ab/slab "$mode" "$s" "$g" "$HOLD" > "$OUT/slab_$name.log" 2>&1
  RC=$?
  wait $P
  echo "$name rc=$RC $(head -1 "$OUT/slab_$name.log")" >> "$OUT/slab_summary.txt"
  [ $RC -eq 0 ] || exit 1
done
cd /tmp && export TMPDIR=/tmp
PMC_CONFIGS=${PMC_CONFIGS:-"cold:0:1 slab:128:1 slab:192:1 cold:0:4"}
for cfg in $PMC_CONFIGS; do
  IFS=: read -r mode s g <<< "$cfg"
  name="${mode}_${s}_${g}"
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc_$name" -o run --pmc FETCH_SIZE -- \
    "$GRAFT_REPO_ROOT/build_ab/slab" "$mode" "$s" "$g" > "$OUT/pmc_$name.log" 2>&1 || exit 1
  echo "pmc $name rc=0" >> "$OUT/slab_summary.txt"
done
exit 0
