set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p $OUT; : > $OUT/summary.txt
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" >> "$OUT/summary.txt"; return $rc; }
for r in 1 2; do
run c1_split1_r$r 200 python bench.py --workload c1 --streams 1 --steps 1500 --no-cpu-baseline --split 1 || exit 1
run c1_split2w8_r$r 200 python bench.py --workload c1 --streams 1 --steps 1500 --no-cpu-baseline --split 2 --scan-waves 8 || exit 1
run c1_split1_s3_r$r 200 python bench.py --workload c1 --streams 3 --steps 1500 --no-cpu-baseline --split 1 || exit 1
run c1_split1_s2_r$r 200 python bench.py --workload c1 --streams 2 --steps 1500 --no-cpu-baseline --split 1 || exit 1
done
