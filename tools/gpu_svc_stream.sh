#!/bin/bash
# A/B of the hash service's stream (BW_SVC_STREAM): the CU-masked stream (its own hardware queue, but
# a blocking stream), a plain non-blocking stream, a least-priority non-blocking stream.  For each:
# the drop-in's latency, a neighbour on 8 non-blocking streams, the legacy null stream.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
for kind in ${SVC_KINDS:-cumask plain low}; do
  for t in ${SVC_THREADS:-1 16}; do
    BW_SVC_STREAM=$kind BW_SVC_TRACE=1 timeout -k 10 180 ./build_ab/dropin_lat 96,4096,65536 4000 $t \
      > "$OUT/svc_${kind}_t$t.log" 2>&1 || { echo "$kind t$t rc=$?"; exit 1; }
    echo "== $kind t$t"; grep -E "dropin|neighbour|null|max|stream" "$OUT/svc_${kind}_t$t.log"
  done
done
