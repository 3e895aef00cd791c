#!/bin/bash
# The reference's unchanged call sites through the drop-ins.
#   C1 (tools/dropin_c1.cpp): per file FastCDC::new + blake3::hash per chunk, at 16 threads with one
#      context each, and at 64 / 256 threads (tokio's default is one worker per core) with one
#      context each and with the Rust shim's pool of 16 contexts; HBM per context.
#   C4 (tools/dropin_c4.cpp): 1 M small files, blake3::hash of each file and of its Tree blob, at
#      16 / 64 / 256 threads over a pool of 16 contexts (small calls served by the library's hash
#      service; BW_DROPIN_SERVICE=0 selects the round-5 coalescer).
#   CPU on the same files: bench.py's cpu_baseline (C1; C4 with --cpu-trees).
# Build first (CPU): see the two tools' headers.  DROPIN_PARTS picks parts (default "c1 c4 cpu"; "c1reg"
# after "c1": the BW_DROPIN_REGISTER_MIB A/B and the [0,0] device pool; DROPIN_C4_DEVICES=0,0 runs C4
# through the device pool's policy; "c4ab" after "c4": the hash service's completers yielding vs
# spinning; "c4cpu": the CPU on C4 alone).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/dropin_summary.txt"
PARTS=${DROPIN_PARTS:-"c1 c4 cpu"}
run() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc" >> "$OUT/dropin_summary.txt"; return $rc
}
if [[ " $PARTS " == *" c1 "* ]]; then
  python3 - <<'PY' > "$OUT/corpus_c1.log" 2>&1 || exit 1
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
PY
  for cfg in ${DROPIN_CFGS:-16:0 64:0 256:0 64:16 256:16}; do
    IFS=: read -r t p <<< "$cfg"
    run dropin_c1_t${t}_p${p} 600 ./build_ab/dropin_c1 /tmp/c1.bin $t 3 0 $p || exit 1
  done
fi
if [[ " $PARTS " == *" c1reg "* ]]; then  # round 6: page-locking in place, alternating A/B
  [ -f /tmp/c1.bin ] || { echo "c1reg needs the c1 part first" >> "$OUT/dropin_summary.txt"; exit 1; }
  for rep in 1 2; do
    for t in 16 64 256; do
      run c1_t${t}_pool16_plain_$rep 300 ./build_ab/dropin_c1 /tmp/c1.bin $t 3 0 16 || exit 1
      run c1_t${t}_pool16_reg64_$rep 300 env BW_DROPIN_REGISTER_MIB=64 ./build_ab/dropin_c1 /tmp/c1.bin $t 3 0 16 || exit 1
      run c1_t${t}_pool16_reg4_$rep 300 env BW_DROPIN_REGISTER_MIB=4 ./build_ab/dropin_c1 /tmp/c1.bin $t 3 0 16 || exit 1
    done
  done
  run c1_t16_devices00 300 ./build_ab/dropin_c1 /tmp/c1.bin 16 3 0 8 --devices=0,0 || exit 1
fi
if [[ " $PARTS " == *" c4 "* ]]; then
  python3 - <<'PY' > "$OUT/corpus_c4.log" 2>&1 || exit 1
import numpy as np, sys
sys.path.insert(0, ".")
from backuwup_amd.synth import small_files_table
u, o, l = small_files_table(1000000, seed=3)  # bench.py --workload c4, rank 0 (bytes: splitmix seed 3)
with open("/tmp/c4_table.bin", "wb") as f:
    np.array([len(o), u, 3], np.uint64).tofile(f)
    np.asarray(o, np.uint64).tofile(f)
    np.asarray(l, np.uint64).tofile(f)
print("files", len(o), "unique bytes", u, "file bytes", int(np.sum(l)))
PY
  run dropin_c4 900 stdbuf -oL ./build_ab/dropin_c4 /tmp/c4_table.bin ${DROPIN_C4_THREADS:-16,64,256} 16 ${DROPIN_C4_REPS:-1} \
    ${DROPIN_C4_DEVICES:+--devices=$DROPIN_C4_DEVICES} || exit 1
fi
if [[ " $PARTS " == *" c4ab "* ]]; then  # round 6: the service's completers yielding (default) vs spinning, alternating
  [ -f /tmp/c4_table.bin ] || { echo "c4ab needs the c4 part first" >> "$OUT/dropin_summary.txt"; exit 1; }
  for rep in 1 2; do
    run c4_yield_$rep 600 stdbuf -oL ./build_ab/dropin_c4 /tmp/c4_table.bin 16,64,256 16 1 --devices=0,0 || exit 1
    run c4_spin_$rep 600 env BW_SVC_COMPLETER=spin stdbuf -oL ./build_ab/dropin_c4 /tmp/c4_table.bin 16,64,256 16 1 \
      --devices=0,0 || exit 1
  done
fi
if [[ " $PARTS " == *" c4cpu "* ]]; then
  run bench_c4_cpu 900 python3 bench.py --workload c4 --steps 20 --cpu-trees || exit 1
fi
if [[ " $PARTS " == *" cpu "* ]]; then
  run bench_c1_cpu 600 python3 bench.py --workload c1 --steps 300 || exit 1
  run bench_c4_cpu 900 python3 bench.py --workload c4 --steps 20 --cpu-trees || exit 1
fi
exit 0
