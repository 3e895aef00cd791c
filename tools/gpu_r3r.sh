#!/bin/bash
# Round-3 session r: the BW_DEBUG build (device bounds asserts) over the parity inputs, final tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/summary.txt"
run() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a "$OUT/summary.txt"; return $rc; }
run debug_check 600 python -u tools/debug_check.py || exit 1
