#!/bin/bash
# round 5 Y: Inception-v3 fp8 (3 lanes) — extent of the cache-resident slice chain: without the
# resolution-leaving edge layers, from 73x73 up, from 147x147 up; two interleaved rounds.
OUT=gpurun_out/r05_y
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
  step def_$r 200 $INC
  step noedge_$r 200 env FT_CHAIN_EDGE=0 $INC
  step min73_$r 200 env FT_CHAIN_MIN_HW=5329 $INC
  step min147_$r 200 env FT_CHAIN_MIN_HW=21609 $INC
done
echo done >&2
