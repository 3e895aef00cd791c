#!/bin/bash
# Round-3 session q: the bench's exchange path (RCCL at world size 1) and --gpus 1, on the final tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a "$OUT/summary.txt"; return $rc; }
run c2_exchange 300 python bench.py --no-cpu-baseline --exchange || exit 1
run c2_gpus1 300 python bench.py --gpus 1 --no-cpu-baseline --steps 100 || exit 1
run c1_exchange 200 python bench.py --workload c1 --no-cpu-baseline --exchange --steps 500 || exit 1
