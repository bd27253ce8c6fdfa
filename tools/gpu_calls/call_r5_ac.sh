#!/bin/bash
# round 5 AC: Inception-v3 fp8 (3 lanes): fp8 conv_lite layers that would launch fewer than two
# workgroups per CU (the 8x8 modules) on narrower channel tiles (temporary switch); A/B.
OUT=gpurun_out/r05_ac
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
for r in 1 2 3; do
  step def_$r 200 $INC
  step fill_$r 200 env FTM_AB_LITE_FILL=1 $INC
done
step layers_fill 300 env FTM_AB_LITE_FILL=1 python -u tools/layer_table.py --model inception_v3 --reps 3 --out "$OUT/layers_fill.md"
echo done >&2
