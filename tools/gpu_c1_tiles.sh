#!/bin/bash
# C1 with the per-batch tile choice (half-size tiles below 4 GiB) vs forced full-size tiles,
# alternating, 4 runs each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py --workload c1 --no-cpu-baseline --no-check > gpurun_out/c1_full_$i.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --workload c1 --no-cpu-baseline --no-check > gpurun_out/c1_half_$i.log 2>&1 || exit 1
done
