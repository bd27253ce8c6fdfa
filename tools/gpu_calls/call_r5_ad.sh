#!/bin/bash
# round 5 AD: kernel stats of the final Inception-v3 fp8 plan (3 lanes) under rocprofv3.
REPO="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$REPO/gpurun_out/r05_ad"
mkdir -p "$OUT"
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "[step] $name" >&2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> "$OUT/rc.txt"
  if [ $rc -gt 1 ]; then echo "[step] $name ended with $rc: stopping" >&2; exit $rc; fi
  return 0
}
cd /tmp && export TMPDIR=/tmp
step prof_inc 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_inc" -o run -- python3 "$REPO/bench.py" --model inception_v3 --steps 30 --warmup 5
echo done >&2
