#!/bin/bash
# round 5 M: lanes x slice size.  Inception-v3 fp8: 3 lanes with 32 / 64-image slices, 4
# lanes; ResNet-50: 2 vs 3 lanes (driver window); interleaved.
OUT=gpurun_out/r05_m
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
  step inc_l3c32_$r 200 $INC --lanes 3
  step inc_l3c64_$r 200 env FT_CHAIN_BATCH=64 $INC --lanes 3
  step inc_l4c32_$r 200 $INC --lanes 4 --depth 4
  step inc_l2c64_$r 200 env FT_CHAIN_BATCH=64 $INC
  step rn_l2_$r 150 python bench.py
  step rn_l3_$r 150 python bench.py --lanes 3
  step rn_l3d4_$r 150 python bench.py --lanes 3 --depth 4
done
step inc_l3_dyn 200 $INC --lanes 3 --dynamic
step inc_l2_dyn 200 $INC --dynamic
echo done >&2
