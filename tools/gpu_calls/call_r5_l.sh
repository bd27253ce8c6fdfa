#!/bin/bash
# round 5 L: Inception-v3 fp8 operating points: the cache-resident slice size of the
# 149x149..71x71 chain (32 default / 64 / off) and three compute lanes; interleaved.
OUT=gpurun_out/r05_l
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
  step inc_c32_$r 200 $INC
  step inc_c64_$r 200 env FT_CHAIN_BATCH=64 $INC
  step inc_c0_$r 200 env FT_CHAIN_BATCH=0 $INC
  step inc_l3_$r 200 $INC --lanes 3
done
echo done >&2
