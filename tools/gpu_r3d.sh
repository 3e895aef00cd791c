#!/bin/bash
# Round-3 session d: GPU tests, then the fused-upper A/B (BW_OPT_B3_UPPER) on C1 (one in flight), C2, C4.
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
  for u in 0 1; do run c1s1_u${u}_r$r 200 python bench.py --workload c1 --streams 1 --steps 1500 --no-cpu-baseline --b3-upper $u || exit 1; done
done
for u in 0 1; do run c2_u$u 300 python bench.py --no-cpu-baseline --b3-upper $u || exit 1; done
for u in 0 1; do run c4_u$u 400 python bench.py --workload c4 --no-cpu-baseline --b3-upper $u || exit 1; done
