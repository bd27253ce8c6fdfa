# round 4 S: halo-staged 3x3 conv (kernels/conv3x3h.hip) — numerics, per-layer time against
# conv_lite, then the ResNet-50 bench (it routes the 10 stride-1 stage 2-4 3x3 convs there)
source tools/gpu_calls/gpu_steps.sh
step test_c3h 300 python -u -m pytest tests/test_conv3x3h.py -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
step probe 120 python -u bench/conv_layer_probe.py --layers s2_3x3,s3_3x3,s4_3x3 --impls lite,halo,lite,halo --reps 20
step bench_rn1 300 python -u bench.py --steps 20 --warmup 5
step bench_rn2 300 python -u bench.py --steps 20 --warmup 5
step bench_inc 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
