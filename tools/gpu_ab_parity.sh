#!/bin/bash
# GPU tests on the release library, the BLAKE3 parity tests on each variant in VARIANTS, then the
# variant benches (tools/gpu_abv.sh with the same environment).  Each GPU step has its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" >> "$OUT/summary.txt"; return $rc; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  run pytest_gpu 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread || exit 1
fi
for v in $VARIANTS; do
  BW_LIB="$GRAFT_REPO_ROOT/backuwup_amd/libbackuwup_amd_$v.so" run "pytest_$v" 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "${PARITY_K:-blake3 or process_files or c1 or c2}" || exit 1
done
KEEP_SUMMARY=1 bash tools/gpu_abv.sh
