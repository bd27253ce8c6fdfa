#!/bin/bash
# round 5 R: Inception-v3 fp8 on 3 lanes, cache-resident slice sizes 24 / 28 / 30 / 32 / 40
# (per-slice tile counts against the chip's resident-workgroup slots); interleaved.
OUT=gpurun_out/r05_r
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
INC="python bench.py --model inception_v3 --steps 30 --warmup 5"
for r in 1 2; do
  for c in 32 24 28 30 40; do
    step c${c}_$r 200 env FT_CHAIN_BATCH=$c $INC
  done
done
echo done >&2
