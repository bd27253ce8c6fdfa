#!/bin/bash
# round 5 N: host staging for the headline's window: native gather threads 8 (default) / 12 /
# 16 and pipeline depth 4, ResNet-50 driver window; Inception-v3 (3 lanes) with 16 threads.
OUT=gpurun_out/r05_n
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
for r in 1 2; do
  step rn_g8_$r 150 python bench.py
  step rn_g12_$r 150 python bench.py --gather-threads 12
  step rn_g16_$r 150 python bench.py --gather-threads 16
  step rn_d4_$r 150 python bench.py --depth 4
  step inc_g8_$r 200 python bench.py --model inception_v3 --steps 30 --warmup 5
  step inc_g16_$r 200 python bench.py --model inception_v3 --steps 30 --warmup 5 --gather-threads 16
done
echo done >&2
