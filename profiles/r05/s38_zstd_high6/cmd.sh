set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s38; mkdir -p $O
ZL="python -u tools/zstd_bench.py --gib 1 --kind text --reps 3 --check 1 --cpu-sample-mib 1 --lanes 6"
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; return $rc; }
step h4a 300 $ZL && step h6a 300 env BW_ZSTD_HIGH_LANES=6 $ZL && step h4b 300 $ZL && step h6b 300 env BW_ZSTD_HIGH_LANES=6 $ZL
