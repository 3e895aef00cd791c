set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s39; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
