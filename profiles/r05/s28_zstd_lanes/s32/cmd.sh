set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s32; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
ZL="python -u tools/zstd_bench.py --gib 1 --kind text --reps 3 --check 2 --cpu-sample-mib 64"
timeout -k 10 300 $ZL --lanes 6 > $O/l6.log 2>&1 && timeout -k 10 300 $ZL --lanes 4 > $O/l4.log 2>&1 && echo lanes ok
