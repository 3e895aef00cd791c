#!/bin/bash
# Round-3 session p: C1-shaped batches with one batch in flight driven from C++ (tools/c1_inflight.cpp),
# next to bench.py's Python-driven line on the same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a "$OUT/summary.txt"; return $rc; }
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -std=c++17 -I include tools/c1_inflight.cpp -L backuwup_amd -lbackuwup_amd \
  -Wl,-rpath,$GRAFT_REPO_ROOT/backuwup_amd -o "$OUT/c1_inflight" > "$OUT/build_c1_inflight.log" 2>&1 || exit 1
python3 -c "
import sys, numpy as np; sys.path.insert(0, '.')
from backuwup_amd import synth
d, o, l = synth.tree_corpus(1 << 30, seed=0x6261636B)
o = np.asarray(o, np.uint64); l = np.asarray(l, np.uint64)
open('$OUT/c1_table.bin', 'wb').write(np.array([len(o)], np.uint64).tobytes() + o.tobytes() + l.tobytes())
" > "$OUT/c1_table.log" 2>&1 || exit 1
for r in 1 2; do run cpp_c1s1_bench_table_r$r 200 "$OUT/c1_inflight" 1500 20 "$OUT/c1_table.bin" || exit 1; done
run cpp_c1s1_own_table 200 "$OUT/c1_inflight" 1500 20 || exit 1
for r in 1 2; do run py_c1s1_r$r 200 python bench.py --workload c1 --streams 1 --steps 1500 --no-cpu-baseline --no-calibrate || exit 1; done
rm -f "$OUT/c1_inflight" "$OUT/c1_table.bin"
