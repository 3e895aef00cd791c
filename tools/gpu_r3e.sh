#!/bin/bash
# Round-3 session e: GPU tests (BLAKE3 + pipeline), then BW_OPT_B3_GROUP (4/2/1 leaves per lane)
# on C1 with one batch in flight, C1 three in flight, C2 and C4.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a "$OUT/summary.txt"; return $rc; }
if [[ "${SKIP_TESTS:-0}" != 1 ]]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} || exit 1
fi
for r in 1 2; do
  for g in 4 2 1; do run c1s1_g${g}_r$r 200 python bench.py --workload c1 --streams 1 --steps 1500 --no-cpu-baseline --b3-group $g || exit 1; done
done
for g in 4 2 1; do run c1s3_g$g 200 python bench.py --workload c1 --steps 1500 --no-cpu-baseline --b3-group $g || exit 1; done
for g in 4 2; do run c2_g$g 300 python bench.py --no-cpu-baseline --b3-group $g || exit 1; done
for g in 4 2; do run c4_g$g 400 python bench.py --workload c4 --no-cpu-baseline --b3-group $g || exit 1; done
