#!/bin/bash
# the reference's unchanged call sites on C1 (tools/dropin_c1.cpp, 16 threads, one
# context each, pageable memory), then bench.py's C1 line for the 16-core CPU baseline on the same
# files.  Build first (CPU): see tools/dropin_c1.cpp.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/dropin_summary.txt"
python3 - <<'EOF' > "$OUT/corpus.log" 2>&1 || exit 1
import numpy as np, sys
sys.path.insert(0, ".")
from backuwup_amd.synth import tree_corpus
d, o, l = tree_corpus(1 << 30, seed=0x6261636B)  # bench.py --workload c1, rank 0
with open("/tmp/c1.bin", "wb") as f:
    np.array([len(o)], np.uint64).tofile(f)
    np.asarray(o, np.uint64).tofile(f)
    np.asarray(l, np.uint64).tofile(f)
    d.tofile(f)
print("files", len(o), "bytes", int(np.sum(l)))
EOF
for cfg in ${DROPIN_CFGS:-16:0 8:0 16:8 16:4 32:8}; do
  IFS=: read -r t mib <<< "$cfg"
  timeout -k 10 300 ./build_ab/dropin_c1 /tmp/c1.bin $t 3 $mib > "$OUT/dropin_t${t}_s${mib}.log" 2>&1
  rc=$?; echo "dropin t=$t stage=$mib rc=$rc" >> "$OUT/dropin_summary.txt"; [ $rc -eq 0 ] || exit 1
done
[ -n "${DROPIN_ONLY:-}" ] && exit 0
timeout -k 10 600 python3 bench.py --workload c1 --steps 300 > "$OUT/bench_c1.log" 2>&1
rc=$?; echo "bench c1 rc=$rc" >> "$OUT/dropin_summary.txt"; [ $rc -eq 0 ] || exit 1
exit 0
