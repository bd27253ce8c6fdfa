# round 3 (session 3) K: gemm_train with both K-steps' fragments read before the MFMAs
# (one wave per SIMD in the W&D grids) — numerics, W&D A/B against ab/_hip_base.so
source tools/gpu_calls/gpu_steps.sh
SO=$(ls flink_tensorflow_amd/_hip.cpython-*.so)
cp "$SO" /tmp/_hip_new.so
step pytest_k 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gemm_train.py tests/test_widedeep.py
step gtb_new 300 python -u bench/gemm_train_bench.py
cp ab/_hip_base.so "$SO"; step gtb_base 300 python -u bench/gemm_train_bench.py
for i in a b c; do
  cp /tmp/_hip_new.so "$SO"; step wd_new_$i 300 python -u bench.py --model widedeep --steps 200 --warmup 20
  cp ab/_hip_base.so "$SO"; step wd_base_$i 300 python -u bench.py --model widedeep --steps 200 --warmup 20
done
cp /tmp/_hip_new.so "$SO"
