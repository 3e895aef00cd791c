set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s29; mkdir -p $O
ZL="python -u tools/zstd_bench.py --gib 1 --kind text --reps 3 --check 1 --cpu-sample-mib 1"
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; return $rc; }
step l4a 300 $ZL --lanes 4 && step l3a 300 $ZL --lanes 3 && step l4b 300 $ZL --lanes 4 && step l3b 300 $ZL --lanes 3 &&
step zstd_tests 600 python -u -m pytest tests/test_zstd.py tests/test_pack.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
