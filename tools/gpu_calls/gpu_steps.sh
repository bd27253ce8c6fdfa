#!/bin/bash
# Runs GPU steps with per-step time limits; stops the whole call at the first fatal exit
# (fault / abort / segfault / timeout), continues past ordinary failures (rc 1/2).
# usage: source tools/gpu_calls/gpu_steps.sh; step NAME SECONDS cmd args...
set -u
REPO="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$REPO/gpurun_out"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {
  local name=$1 t=$2; shift 2
  local t0=$(date +%s)
  mkdir -p "$(dirname "$OUT/$name.log")"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[step] $name rc=$rc $(( $(date +%s) - t0 ))s"
  tail -n 4 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "[step] fatal exit in $name; no further GPU steps"
    exit $rc
  fi
  return 0
}
