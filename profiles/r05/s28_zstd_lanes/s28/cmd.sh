set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s28; mkdir -p $O
ZL="python -u tools/zstd_bench.py --gib 1 --kind text --reps 3 --check 1 --cpu-sample-mib 1 --lanes 3"
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; grep -iE "GB/s" $O/$n.log | tail -4; return $rc; }
step high1 300 $ZL && step normal1 300 env BW_ZSTD_LANE_PRIO=normal $ZL && step high2 300 $ZL && step normal2 300 env BW_ZSTD_LANE_PRIO=normal $ZL && step normal_q8 300 env BW_ZSTD_LANE_PRIO=normal GPU_MAX_HW_QUEUES=8 $ZL &&
step zstd_tests 600 python -u -m pytest tests/test_zstd.py tests/test_pack.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
