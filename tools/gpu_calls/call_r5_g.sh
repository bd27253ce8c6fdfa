#!/bin/bash
# round 5 G: the preprocess folded into ResNet-50's pool-fused s2d stem (bilinear resize in
# the patch builder): numerics, then the headline A/B interleaved, the ResNet layer table,
# Inception once more.
OUT=gpurun_out/r05_g
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
step new_tests 300 $PYT -m gpu tests/test_fp8.py::test_stem_from_raw_uint8_equals_preprocess_then_conv_gpu tests/test_arena.py tests/test_fp8.py::test_inception_v3_fp8_plan_gpu
step rn_fused 150 python bench.py
step rn_sep 150 env FT_FUSE_PREPROCESS_STEM=0 python bench.py
step rn_fused2 150 python bench.py
step rn_sep2 150 env FT_FUSE_PREPROCESS_STEM=0 python bench.py
step rn_fused_300 200 python bench.py --steps 300
step layers_rn 300 python -u tools/layer_table.py --model resnet50 --reps 3 --out "$OUT/layers_rn.md"
step inc 200 python bench.py --model inception_v3 --steps 30 --warmup 5
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
echo done >&2
