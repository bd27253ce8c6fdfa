#!/bin/bash
# round 5 Q: Inception-v3 fp8 on 3 lanes: slicing off, depth 4, staggered lane start.
OUT=gpurun_out/r05_q
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
  step l3_$r 200 $INC
  step l3c0_$r 200 env FT_CHAIN_BATCH=0 $INC
  step l3d4_$r 200 $INC --depth 4
  step l3st_$r 200 $INC --stagger-lanes
done
echo done >&2
