set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s25
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "service or small_hash or coalesced" > gpurun_out/s25/pytest_service.log 2>&1 || { echo pytest rc=$?; tail -30 gpurun_out/s25/pytest_service.log; exit 1; }
tail -3 gpurun_out/s25/pytest_service.log
SVC_KINDS=low bash tools/gpu_svc_stream.sh || exit 1
for v in "low 500000" "low 50000" "cumask 500000"; do
  set -- $v
  BW_SVC_STREAM=$1 BW_SVC_LIFE_US=$2 DROPIN_PARTS=c4 bash tools/gpu_dropin.sh || { echo "c4 $v failed"; cat gpurun_out/dropin_summary.txt; exit 1; }
  cp gpurun_out/dropin_c4.log gpurun_out/s25/c4_$1_$2.log
  echo "== c4 $v"; grep -iE "GB/s" gpurun_out/s25/c4_$1_$2.log
done
