#!/bin/bash
# Host-side helper: run one gpurun call; retry ONLY when the infrastructure reports a transient
# failure before anything ran (status=transient / no box free, exit 3), honouring the
# back-off it announces.  Never retries a command that actually ran on the GPU.
cmd="$1"; tmo="${2:-1200}"
for i in $(seq 1 ${GPU_TRIES:-40}); do
  # archive the previous call's scratch where the judge can read it: every file (the verdict
  # .last_call.json and any .graft_* marker included) goes to profiles/<round>/calls/<time>/; files
  # over 8 MiB (raw traces) are listed there by size instead of copied
  if [ -n "$(ls -A gpurun_out 2>/dev/null)" ]; then
    d=profiles/${GPU_ROUND:-r06}/calls/$(date +%Y%m%d_%H%M%S); mkdir -p "$d"
    (cd gpurun_out && find . -type f -size -8M -exec cp --parents {} "../$d" \;)
    (cd gpurun_out && find . -type f -size +8M -printf '%s %p\n') > "$d/_large_files.txt"
    rm -rf gpurun_out/* gpurun_out/.[!.]*
  fi
  out=$(/usr/local/graft/bin/gpurun --timeout "$tmo" -- "$cmd" 2>&1); rc=$?
  echo "[$(date +%T) attempt $i rc=$rc]"; echo "$out" | tail -4
  if [ $rc = 3 ] || echo "$out" | grep -q "status=transient"; then
    w=$(echo "$out" | grep -o "retry in [0-9]*s" | grep -o "[0-9]*" | tail -1)
    sleep $(( ${w:-40} + 10 )); continue
  fi
  exit $rc
done
exit 99
