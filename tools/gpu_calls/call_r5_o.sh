#!/bin/bash
# round 5 O: ResNet-50, the LDS-exclusive persistent kernels (gemm_pp 132 KB, block tails
# 144 KB, conv3x3c64 117 KB, pw_res) vs their overlappable fallbacks, on 2 and 3 lanes.
OUT=gpurun_out/r05_o
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
for L in 2 3; do
  step l${L}_base 150 python bench.py --lanes $L
  step l${L}_nopp 150 env FTM_AB_NO_GEMM_PP=1 python bench.py --lanes $L
  step l${L}_nopw 150 env FT_PW_RES_KERNEL=0 python bench.py --lanes $L
  step l${L}_noc64 150 env FT_CONV3X3C64_KERNEL=0 python bench.py --lanes $L
  step l${L}_notail 150 env FT_FUSE_BLOCK_TAILS=0 python bench.py --lanes $L
  step l${L}_none 150 env FTM_AB_NO_GEMM_PP=1 FT_PW_RES_KERNEL=0 FT_CONV3X3C64_KERNEL=0 FT_FUSE_BLOCK_TAILS=0 python bench.py --lanes $L
done
step l2_base2 150 python bench.py --lanes 2
echo done >&2
