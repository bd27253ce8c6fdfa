#!/bin/bash
# round 5 W: bottleneck3 v4 (the 3x3 bank as register A fragments, W3 in LDS): numerics,
# per-boundary A/B, ResNet-50 on / off interleaved (three rounds).
OUT=gpurun_out/r05_w
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
PYT="python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider"
step new_tests 300 $PYT -m gpu tests/test_bottleneck.py
step micro 200 python -u bench/bottleneck3_ab.py
for r in 1 2 3; do
  step rn_f_$r 150 python bench.py
  step rn_u_$r 150 env FT_FUSE_CONV3_TAILS=0 python bench.py
done
echo done >&2
