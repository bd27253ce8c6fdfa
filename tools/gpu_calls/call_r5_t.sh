#!/bin/bash
# round 5 T: does the window's start-up ramp vanish with more warm-up?  20-step windows with
# 5 / 30 / 100 warm-up steps, batch timelines; two rounds.
OUT=gpurun_out/r05_t
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
  step w5_$r 150 python bench.py --timeline --steps 20 --warmup 5
  step w30_$r 150 python bench.py --timeline --steps 20 --warmup 30
  step w100_$r 150 python bench.py --timeline --steps 20 --warmup 100
done
echo done >&2
