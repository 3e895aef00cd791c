#!/bin/bash
# Round-3 session o: BLAKE3 leaves per lane on small batches, same box: one leaf per lane (G=1)
# against the automatic two (G=2) on C1 with one and three batches in flight, and on C4.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a "$OUT/summary.txt"; return $rc; }
for r in 1 2 3; do
  run c1s1_g2_r$r 200 python bench.py --workload c1 --streams 1 --steps 1500 --no-cpu-baseline --no-calibrate || exit 1
  run c1s1_g1_r$r 200 python bench.py --workload c1 --streams 1 --steps 1500 --no-cpu-baseline --no-calibrate --b3-group 1 || exit 1
done
run c1s3_g2 200 python bench.py --workload c1 --steps 1500 --no-cpu-baseline --no-calibrate || exit 1
run c1s3_g1 200 python bench.py --workload c1 --steps 1500 --no-cpu-baseline --no-calibrate --b3-group 1 || exit 1
run c4_g2 300 python bench.py --workload c4 --no-cpu-baseline --no-calibrate || exit 1
run c4_g1 300 python bench.py --workload c4 --no-cpu-baseline --no-calibrate --b3-group 1 || exit 1
