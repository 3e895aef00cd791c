#!/bin/bash
# Host-side helper: run one gpurun call; retry ONLY when the infrastructure reports a transient
# failure before anything ran (status=transient / no box free, exit 3), honouring the
# back-off it announces.  Never retries a command that actually ran on the GPU.
cmd="$1"; tmo="${2:-1200}"
for i in 1 2 3 4 5 6 7 8; do
  # keep the previous call's results out of the way (not deleted: copy what matters to profiles/)
  if [ -n "$(ls -A gpurun_out 2>/dev/null)" ]; then d=/tmp/gpurun_prev_$(date +%s); mkdir -p $d; mv gpurun_out/* $d/; fi
  out=$(/usr/local/graft/bin/gpurun --timeout "$tmo" -- "$cmd" 2>&1); rc=$?
  echo "[$(date +%T) attempt $i rc=$rc]"; echo "$out" | tail -4
  if [ $rc = 3 ] || echo "$out" | grep -q "status=transient"; then
    w=$(echo "$out" | grep -o "retry in [0-9]*s" | grep -o "[0-9]*" | tail -1)
    sleep $(( ${w:-40} + 10 )); continue
  fi
  exit $rc
done
exit 99
