#!/bin/bash
# round 5 F: the whole GPU suite on the current tree, then Inception-v3 fp8 A/B of the two
# new stem fusions (pool+1x1 kernel, preprocess folded into the s2d stem), interleaved,
# and the Inception layer table.
OUT=gpurun_out/r05_f
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
step new_tests 300 $PYT -m gpu tests/test_fp8.py::test_stem_from_raw_uint8_equals_preprocess_then_conv_gpu tests/test_fp8.py::test_inception_v3_fp8_plan_gpu tests/test_fp8.py::test_pool_conv1x1_fp8_gpu
step gpu_suite 780 $PYT -m gpu tests --maxfail 10
INC="python bench.py --model inception_v3 --steps 30 --warmup 5"
step inc_all 200 $INC
step inc_nopc 200 env FT_POOL_CONV_FUSION=0 $INC
step inc_nopre 200 env FT_FUSE_PREPROCESS_STEM=0 $INC
step inc_none 200 env FT_POOL_CONV_FUSION=0 FT_FUSE_PREPROCESS_STEM=0 $INC
step inc_all2 200 $INC
step inc_nopc2 200 env FT_POOL_CONV_FUSION=0 $INC
step inc_nopre2 200 env FT_FUSE_PREPROCESS_STEM=0 $INC
step inc_none2 200 env FT_POOL_CONV_FUSION=0 FT_FUSE_PREPROCESS_STEM=0 $INC
step layers_inc 300 python -u tools/layer_table.py --model inception_v3 --reps 3 --out "$OUT/layers_inc.md"
echo done >&2
