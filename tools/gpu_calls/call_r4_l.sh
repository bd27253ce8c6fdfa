# round 4 L: conv3x3c64 (ResNet-50 stage-1 3x3) patch loads through a buffer descriptor
# (no branch around each load); the igemm GEMM-mode version of the same change measured
# slower in call K and is reverted here
source tools/gpu_calls/gpu_steps.sh
step test_l 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_compiler.py -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread
if ! grep -q " passed" "$OUT/test_l.log" || grep -q "failed" "$OUT/test_l.log"; then
  echo "[call] tests did not pass; no benches"; exit 1
fi
step layers_rn 300 python -u tools/layer_table.py --reps 5 --out "$OUT/layers_rn.md"
step bench_rn_a 300 python -u bench.py --steps 20 --warmup 5
step bench_rn_b 300 python -u bench.py --steps 20 --warmup 5
