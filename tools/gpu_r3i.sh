#!/bin/bash
# Round-3 session i: BW_OPT_ORDER_HASH (scans and leaf passes of the session's contexts serialized)
# A/B on C2 and C1 (2 and 3 in flight), and C2 with the RCCL exchange at world size 1.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a "$OUT/summary.txt"; return $rc; }
for r in 1 2; do
  for o in 0 1; do run c2_o${o}_r$r 300 python bench.py --no-cpu-baseline --order-hash $o || exit 1; done
done
for o in 0 1; do run c1s2_o$o 200 python bench.py --workload c1 --streams 2 --steps 1500 --no-cpu-baseline --order-hash $o || exit 1; done
for o in 0 1; do run c1s3_o$o 200 python bench.py --workload c1 --streams 3 --steps 1500 --no-cpu-baseline --order-hash $o || exit 1; done
run c2_exchange 300 python bench.py --no-cpu-baseline --exchange || exit 1
