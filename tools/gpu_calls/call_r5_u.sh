#!/bin/bash
# round 5 U: lane phase at the window start: the second lane's first batch delayed by
# 0 / 1000 / 1800 / 2600 µs (stream-ordered delay kernel), ResNet-50 driver window with batch
# timelines; two rounds; then Inception-v3 (3 lanes) with 0 / 800 / 1400 µs.
OUT=gpurun_out/r05_u
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
  for o in 0 1000 1800 2600; do
    step rn_o${o}_$r 150 python bench.py --timeline --steps 20 --warmup 5 --lane-offset-us $o
  done
done
for r in 1 2; do
  for o in 0 800 1400; do
    step inc_o${o}_$r 200 python bench.py --model inception_v3 --steps 30 --warmup 5 --lane-offset-us $o
  done
done
echo done >&2
