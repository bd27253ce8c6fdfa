#!/bin/bash
# round 5 H: persistent direct conv (filter bank resident, grid-stride tile loop): numerics
# (bit-identical to one tile per workgroup), the per-layer A/B, then Inception-v3 fp8 and
# ResNet-50 end to end with it on / off, interleaved.
OUT=gpurun_out/r05_h
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
step new_tests 300 $PYT -m gpu tests/test_dconv.py
step micro 300 python -u bench/dconv_persist_ab.py
step inc_p 200 env FT_DCONV_PERSIST=1 python bench.py --model inception_v3 --steps 30 --warmup 5
step inc_t 200 python bench.py --model inception_v3 --steps 30 --warmup 5
step inc_p2 200 env FT_DCONV_PERSIST=1 python bench.py --model inception_v3 --steps 30 --warmup 5
step inc_t2 200 python bench.py --model inception_v3 --steps 30 --warmup 5
step rn_p 150 env FT_DCONV_PERSIST=1 python bench.py
step rn_t 150 python bench.py
step rn_p2 150 env FT_DCONV_PERSIST=1 python bench.py
step rn_t2 150 python bench.py
echo done >&2
