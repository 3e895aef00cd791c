set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s31; mkdir -p $O
ZL="python -u tools/zstd_bench.py --gib 1 --kind text --reps 3 --check 1 --cpu-sample-mib 1"
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; return $rc; }
step l8a 300 $ZL --lanes 8 && step l6a 300 $ZL --lanes 6 && step l8b 300 $ZL --lanes 8 && step l6b 300 $ZL --lanes 6 &&
step l8_q8 300 env GPU_MAX_HW_QUEUES=8 $ZL --lanes 8
