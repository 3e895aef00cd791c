set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s27
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s27/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/s27/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/s27/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/s27/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/s27/smoke.log; exit 1; }
tail -1 gpurun_out/s27/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/s27/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/s27/bench.log; exit 1; }
tail -1 gpurun_out/s27/bench.log
