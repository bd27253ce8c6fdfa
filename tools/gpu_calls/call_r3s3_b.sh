# round 3 (session 3) B: LDS fragment reads hoisted ahead of the MFMAs (sched_group_barrier
# pipelining) in conv_lite, the stage-1 bottleneck tails, pw_res and conv3x3c64: numerics,
# then ResNet-50 / Inception-v3 A/B against the previous kernel library (ab/_hip_base.so)
source tools/gpu_calls/gpu_steps.sh
SO=$(ls flink_tensorflow_amd/_hip.cpython-*.so)
cp "$SO" /tmp/_hip_new.so
step pytest_b 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_conv_pp.py tests/test_bottleneck.py tests/test_pw_res.py tests/test_kernels_gpu.py tests/test_fp8.py tests/test_compiler.py tests/test_fullsize_numerics.py
for i in a b; do
  cp /tmp/_hip_new.so "$SO"; step rn_new_$i 300 python -u bench.py --steps 20 --warmup 5
  cp ab/_hip_base.so "$SO"; step rn_base_$i 300 python -u bench.py --steps 20 --warmup 5
done
cp /tmp/_hip_new.so "$SO"; step rn_new_300 300 python -u bench.py --steps 300 --warmup 10
cp ab/_hip_base.so "$SO"; step rn_base_300 300 python -u bench.py --steps 300 --warmup 10
cp /tmp/_hip_new.so "$SO"; step inc_new 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
cp ab/_hip_base.so "$SO"; step inc_base 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
cp /tmp/_hip_new.so "$SO"
step layers_new 300 python -u bench/layer_table.py --model resnet50
