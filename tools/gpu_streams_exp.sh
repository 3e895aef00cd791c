set -o pipefail
mkdir -p gpurun_out
for w in c1 c2; do for s in 2 3 4; do
  timeout -k 10 300 python bench.py --workload $w --streams $s --no-cpu-baseline > gpurun_out/${w}_s$s.log 2>&1 || exit 1
done; done
