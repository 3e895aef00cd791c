#!/bin/bash
# Round-3 evidence session: every GPU test, smoke, the default bench line (C2 + CPU baseline), the
# other configurations, the rocprofv3 kernel-trace stats of the default bench command, and the
# FETCH_SIZE / WRITE_SIZE passes behind roofline.traffic.  Every GPU step has its own time limit;
# the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a "$OUT/summary.txt"; return $rc; }
if [[ "${SKIP_TESTS:-0}" != 1 ]]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} || exit 1
  run smoke 300 python __graft_entry__.py || exit 1
fi
run bench_c2 400 python bench.py || exit 1
if [[ "${CONFIGS:-1}" == 1 ]]; then
  run bench_c1_s1 200 python bench.py --workload c1 --streams 1 --steps 1500 --no-cpu-baseline || exit 1
  run bench_c1_s1_b 200 python bench.py --workload c1 --streams 1 --steps 1500 --no-cpu-baseline || exit 1
  run bench_c1 200 python bench.py --workload c1 --steps 1500 --no-cpu-baseline || exit 1
  run bench_c3 400 python bench.py --workload c3 --no-cpu-baseline || exit 1
  run bench_c4 400 python bench.py --workload c4 --no-cpu-baseline || exit 1
  run bench_c5 400 python bench.py --workload c5 --no-cpu-baseline || exit 1
fi
cd /tmp && export TMPDIR=/tmp
run rocprof 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline || exit 1
B="python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-check --no-calibrate --no-power"
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run --pmc FETCH_SIZE -- $B > "$OUT/pmc_fetch.log" 2>&1 || exit 1
echo "pmc_fetch rc=0" >> "$OUT/summary.txt"
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run --pmc WRITE_SIZE -- $B > "$OUT/pmc_write.log" 2>&1 || exit 1
echo "pmc_write rc=0" >> "$OUT/summary.txt"
cd "$GRAFT_REPO_ROOT" && python3 tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" 16 "$OUT/pmc_traffic.json" > "$OUT/pmc_traffic.log" 2>&1
echo "pmc_traffic rc=$?" >> "$OUT/summary.txt"
