# round 4 J: the unrolled 3x3 / stride-1 average-pool epilogue kernel (Inception's commuted
# AvgPool branches) and the unrolled global average pools (ResNet-50 bf16, Inception fp8):
# correctness, per-layer tables, benches
source tools/gpu_calls/gpu_steps.sh
step test_pool 300 python -u -m pytest tests/test_fp8.py tests/test_kernels_gpu.py tests/test_compiler.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
if ! grep -q " passed" "$OUT/test_pool.log" || grep -q "failed" "$OUT/test_pool.log"; then
  echo "[call] tests did not pass; no benches"; exit 1
fi
step layers_inc 300 python -u tools/layer_table.py --model inception_v3 --reps 5 --out "$OUT/layers_inc.md"
step layers_rn 300 python -u tools/layer_table.py --reps 5 --out "$OUT/layers_rn.md"
step bench_inc_a 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step bench_inc_b 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step bench_inc_dyn 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --dynamic
step bench_rn_a 300 python -u bench.py --steps 20 --warmup 5
step bench_rn_b 300 python -u bench.py --steps 20 --warmup 5
