set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s26
n=0
for v in sleep yield sleep yield; do
  n=$((n+1))
  BW_SVC_WAIT=$v DROPIN_PARTS=c4 bash tools/gpu_dropin.sh || { echo "c4 $v failed"; cat gpurun_out/dropin_summary.txt; exit 1; }
  cp gpurun_out/dropin_c4.log gpurun_out/s26/c4_${n}_$v.log
  echo "== c4 $n $v"; grep -E "GB/s" gpurun_out/s26/c4_${n}_$v.log
done
