#!/bin/bash
# One GPU session of several steps (rounds 4-5), chosen by STEPS (default: all).  Every step runs under
# its own time limit; a step that times out, aborts or faults (rc 124/134/137/139 or a signal) ends
# the session there, any other failure is recorded and the next step runs.  Results go to
# gpurun_out/ (summary.txt lists each step's rc).
#   tests    pytest -m gpu                       smoke   __graft_entry__.smoke()
#   collide  tools/collide.hip (BLAKE3 8-byte prefix collision -> gpurun_out/*.json)
#   slab     tools/gpu_slab.sh (Infinity-Cache reuse of the leaf pass)
#   dropin   tools/gpu_dropin.sh (the reference's call sites on C1)
#   bench    python bench.py $BENCH_ARGS         prof    rocprofv3 --kernel-trace --stats of the bench
#   pmc      tools/gpu_pmc.sh (FETCH_SIZE / WRITE_SIZE passes -> pmc_traffic.json)
#   debug    tools/debug_check.py (BW_DEBUG + BW_DIAG library)
#   rehearse bench.py --gpus 2 / 4 --transport host on one GPU (the N > 1 path end to end)
#   zstd     tools/zstd_bench.py on 1 GiB and 8 GiB of text (level-3 frames, oracle-checked sample)
#   zstream  the same 1 GiB batch with 2, 3 and 4 calls in flight
#   zspmc    SQ counter passes of the zstd kernels (1 GiB of text)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
STEPS=${STEPS:-"tests smoke slab dropin bench"}
step() {
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)" >&2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a "$OUT/summary.txt" >&2
  case $rc in
    0|1|2|3|4|5) return 0 ;;
    *) echo "stopping after $name (rc=$rc)" >> "$OUT/summary.txt"; exit 1 ;;
  esac
}
for s in $STEPS; do
  case $s in
    tests) step pytest_gpu 900 python -u -m pytest tests -m gpu --maxfail 20 -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    smoke) step smoke 300 python __graft_entry__.py ;;
    sel) step pytest_sel 600 python -u -m pytest ${PYTEST_SEL:-tests/test_gpu_dropin_pool.py} -m gpu -v -p no:cacheprovider \
           --timeout 240 --timeout-method thread ;;
    full) step pytest_full 600 python -u -m pytest tests/test_gpu_full_configs.py -m gpu -v -p no:cacheprovider \
           --timeout 300 --timeout-method thread ;;
    bench20) step bench20 300 python bench.py --steps 20 --no-cpu-baseline ;;
    collide) step collide 120 ./build_ab/collide "$OUT/blake3_prefix_collision.json" 14 32768 1 ;;
    slab) step slab 900 bash tools/gpu_slab.sh ;;
    dropin) step dropin 1100 bash tools/gpu_dropin.sh ;;
    bench) step bench 600 python bench.py ${BENCH_ARGS:-} ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run \
        --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-holds) || exit 1
      T=$(find "$OUT/prof" -name "*kernel_trace.csv" | head -1)
      [ -n "$T" ] && python3 tools/trace_split.py "$T" k_b3_lines 2 320 17179869184 > "$OUT/trace_split.json" 2>&1 ;;
    pmc) step pmc 900 bash tools/gpu_pmc.sh ;;
    slabpmc) step slabpmc 600 env CONFIGS=" " bash tools/gpu_slab.sh ;;
    dropsweep) step dropsweep 600 env DROPIN_ONLY=1 bash tools/gpu_dropin.sh ;;
    configs)
      step bench_c1_1 600 python bench.py --workload c1 --streams 1 --steps 1500 --no-cpu-baseline &&
      step bench_c3 600 python bench.py --workload c3 --steps 40 --no-cpu-baseline &&
      step bench_c4 600 python bench.py --workload c4 --steps 60 --no-cpu-baseline &&
      step bench_c5 600 python bench.py --workload c5 --steps 3 --no-cpu-baseline ;;
    debug) step debug_check 600 python tools/debug_check.py ;;
    rehearse)  # round 6: the driver's N > 1 bench path on one GPU (host transport, ranks share the GPU)
      step bench_n2_host 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29533 bench.py --gpus 2 --transport host --steps 20 --warmup 2 --no-holds &&
      step bench_n4_host 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
        --master-port 29534 bench.py --gpus 4 --transport host --steps 10 --warmup 2 --no-holds ;;
    attrib)  # round 5, VERDICT r4 #4: what limits the overlap of the scan and the leaf pass (build first:
             # python backuwup_amd/build.py --clock); then the bench at the driver's 20 steps, the
             # default 320 and 2,000 (18 s), each with its power and clock samples
      step clock_windows 300 python tools/clock_windows.py --steps 400 --window 24 &&
      step bench_s20 300 python bench.py --steps 20 --no-cpu-baseline --no-calibrate &&
      step bench_s320 300 python bench.py --steps 320 --no-cpu-baseline --no-calibrate &&
      step bench_s2000 600 python bench.py --steps 2000 --no-cpu-baseline --no-calibrate ;;
    exch)  # round 5: the exactly sized, deferred exchange (host transport + RCCL world 1) and the bench's
           # exchange path at world size 1
      step exch_tests 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_stream_split.py tests/test_gpu_parity.py \
        -m gpu -k "exchange or shard or split or dropin or coalesced" -v -p no:cacheprovider --timeout 300 \
        --timeout-method thread &&
      step bench_exch 600 python bench.py --exchange --steps 60 --no-cpu-baseline &&
      step bench_split 600 python bench.py --workload c3 --gib 1 --split-files --steps 5 ;;
    zsdiag)  # diagnostic zstd variants: section timers (BW_ZSTD_TIMING) and the step fences dropped
             # (build first: python backuwup_amd/build.py --ztime; build(variant="zsnofence", defines=("-DBW_ZS_NOFENCE",)))
      step zstd_ztime 600 env BW_LIB="$GRAFT_REPO_ROOT/backuwup_amd/libbackuwup_amd_ztime.so" python tools/zstd_bench.py \
        --gib 1 --kind text --reps 1 --check 4 &&
      step zstd_nofence 600 env BW_LIB="$GRAFT_REPO_ROOT/backuwup_amd/libbackuwup_amd_zsnofence.so" python tools/zstd_bench.py \
        --gib 1 --kind text --reps 2 --check 16 ;;
    zstream)  # 1 GiB text batches with 2 / 3 / 4 calls in flight (one context and host thread each)
      step zstd_if2 600 python tools/zstd_bench.py --gib 1 --kind text --reps 2 --check 2 --cpu-sample-mib 16 --inflight 2 &&
      step zstd_if3 600 python tools/zstd_bench.py --gib 1 --kind text --reps 2 --check 2 --cpu-sample-mib 16 --inflight 3 &&
      step zstd_if4 600 python tools/zstd_bench.py --gib 1 --kind text --reps 2 --check 2 --cpu-sample-mib 16 --inflight 4 ;;
    zspmc)  # SQ counters of the zstd kernels (1 GiB of text, one timed call), two passes of 8
      Z="$GRAFT_REPO_ROOT/tools/zstd_bench.py --kind text --gib 1 --reps 1 --cpu-sample-mib 1 --check 0"
      (cd /tmp && export TMPDIR=/tmp &&
        step zspmc1 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/zpmc1" -o run --pmc SQ_WAVES SQ_INSTS_VALU \
          SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- python3 $Z &&
        step zspmc2 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/zpmc2" -o run --pmc SQ_INSTS_SALU \
          SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES -- python3 $Z) || exit 1 ;;
    zsab)  # A/B of the zstd parse: the product library against libbackuwup_amd_zsold.so (built by hand
           # from the previous bw_zstd.hip), alternating
      ZB="python tools/zstd_bench.py --gib 1 --kind text --reps 2 --cpu-sample-mib 1"
      ZOLD="$GRAFT_REPO_ROOT/backuwup_amd/libbackuwup_amd_zsold.so"
      step zstd_tests 600 python -u -m pytest tests/test_zstd.py tests/test_pack.py -m gpu -x -q -p no:cacheprovider \
        --timeout 300 --timeout-method thread &&
      step zsab_new1 300 $ZB --check 16 && step zsab_old1 300 env BW_LIB="$ZOLD" $ZB --check 2 &&
      step zsab_new2 300 $ZB --check 2 && step zsab_old2 300 env BW_LIB="$ZOLD" $ZB --check 2 &&
      step zsab_new_if3 600 $ZB --check 2 --inflight 3 ;;
    zstests)  # the zstd and pack GPU tests alone
      step zstd_tests 600 python -u -m pytest tests/test_zstd.py tests/test_pack.py -m gpu -x -q -p no:cacheprovider \
        --timeout 300 --timeout-method thread ;;
    zsab8)  # the same A/B on 8 GiB of text (the throughput case: ~6.8 k blobs, several waves per SIMD)
      ZB8="python tools/zstd_bench.py --gib 8 --kind text --reps 1 --cpu-sample-mib 1 --check 2"
      ZOLD="$GRAFT_REPO_ROOT/backuwup_amd/libbackuwup_amd_zsold.so"
      step zsab8_new1 300 $ZB8 && step zsab8_old1 300 env BW_LIB="$ZOLD" $ZB8 &&
      step zsab8_new2 300 $ZB8 && step zsab8_old2 300 env BW_LIB="$ZOLD" $ZB8 ;;
    zlanes)  # 1 GiB text batches through one context's asynchronous lanes, one host thread
      step zstd_lanes3 600 python tools/zstd_bench.py --gib 1 --kind text --reps 3 --check 2 --cpu-sample-mib 1 --lanes 3 ;;
    lanesq)  # the zstd lanes from one host thread with HIP's default 4 hardware queues and with 8
      ZL="python tools/zstd_bench.py --gib 1 --kind text --reps 3 --check 1 --cpu-sample-mib 1 --lanes 3"
      step lanes_q4 300 $ZL && step lanes_q8 300 env GPU_MAX_HW_QUEUES=8 $ZL ;;
    zprof)  # rocprofv3 kernel trace + stats of one 1 GiB text zstd call (and its warm-up)
      (cd /tmp && export TMPDIR=/tmp && step zprof 300 rocprofv3 --kernel-trace --stats -d "$OUT/zprof" -o run \
        --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/zstd_bench.py" --gib 1 --kind text --reps 1 --check 1 \
        --cpu-sample-mib 1) || exit 1 ;;
    zstd) step zstd_text1 600 python tools/zstd_bench.py --gib 1 --kind text --reps 2 --check 16 &&
          step zstd_text8 600 python tools/zstd_bench.py --gib 8 --kind text --reps 1 --check 4 ;;
  esac
done
exit 0
