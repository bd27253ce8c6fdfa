# round 4 K: the register-staged igemm's GEMM mode (ResNet-50's 1x1 convs outside the fused
# kernels: stage-1 entry reduce, stage-2 reduces, stage-4 expands) reads X and W through
# buffer descriptors instead of per-element guarded loads (a branch around every load)
source tools/gpu_calls/gpu_steps.sh
step test_k 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_compiler.py tests/test_fullsize_numerics.py tests/test_pw_res.py tests/test_bottleneck.py -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread
if ! grep -q " passed" "$OUT/test_k.log" || grep -q "failed" "$OUT/test_k.log"; then
  echo "[call] tests did not pass; no benches"; exit 1
fi
step layers_rn 300 python -u tools/layer_table.py --reps 5 --out "$OUT/layers_rn.md"
step probe_1x1 300 python -u bench/conv_layer_probe.py --layers s2_reduce,s4_expand,s1_reduce --impls igemm --reps 20
step bench_rn_a 300 python -u bench.py --steps 20 --warmup 5
step bench_rn_b 300 python -u bench.py --steps 20 --warmup 5
step bench_rn_300 300 python -u bench.py --steps 300 --warmup 10
