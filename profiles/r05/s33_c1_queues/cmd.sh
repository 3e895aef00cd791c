set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s33; mkdir -p $O
python3 - <<'PY' > $O/corpus.log 2>&1 || exit 1
import numpy as np, sys
sys.path.insert(0, ".")
from backuwup_amd.synth import tree_corpus
d, o, l = tree_corpus(1 << 30, seed=0x6261636B)
with open("/tmp/c1.bin", "wb") as f:
    np.array([len(o)], np.uint64).tofile(f)
    np.asarray(o, np.uint64).tofile(f)
    np.asarray(l, np.uint64).tofile(f)
    d.tofile(f)
print("files", len(o))
PY
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; grep -E "GB/s" $O/$n.log | tail -2; return $rc; }
step q4a 300 ./build_ab/dropin_c1 /tmp/c1.bin 16 3 0 0 && step q16a 300 env GPU_MAX_HW_QUEUES=16 ./build_ab/dropin_c1 /tmp/c1.bin 16 3 0 0 &&
step q4b 300 ./build_ab/dropin_c1 /tmp/c1.bin 16 3 0 0 && step q16b 300 env GPU_MAX_HW_QUEUES=16 ./build_ab/dropin_c1 /tmp/c1.bin 16 3 0 0
