#!/bin/bash
# round 5 K: bottleneck3 v3 (next tile's residual double-buffered, in flight for the whole
# tile): numerics, per-boundary A/B, ResNet-50 on / off; Inception fp8 with the direct
# convs at 4 vs 8 waves (the one-tile-per-workgroup kernel restored).
OUT=gpurun_out/r05_k
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
step new_tests 300 $PYT -m gpu tests/test_bottleneck.py tests/test_dconv.py
step micro 200 python -u bench/bottleneck3_ab.py
step rn_f 150 python bench.py
step rn_u 150 env FT_FUSE_CONV3_TAILS=0 python bench.py
step rn_f2 150 python bench.py
step rn_u2 150 env FT_FUSE_CONV3_TAILS=0 python bench.py
step inc_w4 200 env FT_DCONV_WAVES=4 python bench.py --model inception_v3 --steps 30 --warmup 5
step inc_w8 200 env FT_DCONV_WAVES=8 python bench.py --model inception_v3 --steps 30 --warmup 5
step inc_w4b 200 env FT_DCONV_WAVES=4 python bench.py --model inception_v3 --steps 30 --warmup 5
step inc_w8b 200 env FT_DCONV_WAVES=8 python bench.py --model inception_v3 --steps 30 --warmup 5
echo done >&2
