# round 3 (session 3) J: conv_lite's 8-wave 256x128 tile (96 KiB; a quarter fewer LDS image
# bytes per MFMA) — numerics, per-layer probe, end-to-end A/B (EngineConfig.conv_lite_wide)
source tools/gpu_calls/gpu_steps.sh
step pytest_j 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_conv_pp.py
step probe_j 300 python -u bench/conv_layer_probe.py --layers s2_3x3,s3_3x3,s4_3x3,s3_3x3s2 --impls lite,lite256 --reps 20
for i in a b; do
  step w0_$i 300 python -u bench.py --steps 20 --warmup 5
  step w1_$i 300 env FT_CONV_LITE_WIDE=1 python -u bench.py --steps 20 --warmup 5
done
step w0_300 300 python -u bench.py --steps 300 --warmup 10
step w1_300 300 env FT_CONV_LITE_WIDE=1 python -u bench.py --steps 300 --warmup 10
step w1_l1 300 env FT_CONV_LITE_WIDE=1 python -u bench.py --steps 100 --warmup 10 --lanes 1
step w0_l1 300 python -u bench.py --steps 100 --warmup 10 --lanes 1
