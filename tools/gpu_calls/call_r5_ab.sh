#!/bin/bash
# round 5 AB (information only): ResNet-50 micro-batch 512 vs the headline's 256, 2 lanes.
OUT=gpurun_out/r05_ab
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
  step b256_$r 150 python bench.py
  step b512_$r 200 python bench.py --batch 512
done
echo done >&2
