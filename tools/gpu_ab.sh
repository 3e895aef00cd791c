#!/bin/bash
# A/B of bench variants: for each "name|bench args" pair, the bench line (C2 default) and a
# FETCH_SIZE pass (rocprofv3, 4 steps).  Every GPU step has its own time limit; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
for v in "$@"; do
  name="${v%%|*}"; args="${v#*|}"
  echo "== $name: $args $(date +%T)" >&2
  timeout -k 10 600 python bench.py --no-cpu-baseline $args > "$OUT/ab_$name.log" 2>&1 || { echo "$name bench rc=$?"; exit 1; }
  if [ -n "$AB_PMC" ]; then
    (cd /tmp && TMPDIR=/tmp timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/ab_pmc_$name" -o run --pmc FETCH_SIZE -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-check --steps 4 --warmup 1 $args > "$OUT/ab_pmc_$name.log" 2>&1) || { echo "$name pmc rc=$?"; exit 1; }
  fi
done
