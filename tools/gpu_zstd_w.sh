#!/bin/bash
# zstd parse experiment: parity tests, then section timers for WMIN = 2 / 8 at 1 and 8 GiB of text
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_zstd.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/zstd_tests.log 2>&1 || exit 1
for v in ${ZVARIANTS:-ztime_w2 ztime}; do
  for g in 1 8; do
    BW_LIB=$PWD/backuwup_amd/libbackuwup_amd_$v.so timeout -k 10 300 python tools/zstd_bench.py --kind text --gib $g --reps 1 --check 1 --cpu-sample-mib 1 > gpurun_out/${v}_$g.log 2>&1 || exit 1
  done
done
