#!/bin/bash
# round 5 J: bottleneck3 v2 (K-split 3x3, next patch prefetched a whole tile ahead): numerics,
# the per-boundary A/B, ResNet-50 on / off interleaved; Inception (fp8 direct convs now on
# 4-wave tiles) with the persistent direct conv on / off.
OUT=gpurun_out/r05_j
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
step inc_p 200 env FT_DCONV_PERSIST=1 python bench.py --model inception_v3 --steps 30 --warmup 5
step inc_t 200 python bench.py --model inception_v3 --steps 30 --warmup 5
step inc_p2 200 env FT_DCONV_PERSIST=1 python bench.py --model inception_v3 --steps 30 --warmup 5
step inc_t2 200 python bench.py --model inception_v3 --steps 30 --warmup 5
echo done >&2
