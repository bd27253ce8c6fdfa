# round 3 (session 3) F: conv_lite 32-deep K-tile on FOUR LDS stages (3 K-tiles of DMA in
# flight, still 64 KiB / two workgroups per CU) vs the 64-deep two-stage default
source tools/gpu_calls/gpu_steps.sh
step pytest_f 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_conv_pp.py
step probe_f 300 python -u bench/conv_layer_probe.py --layers s2_3x3,s3_3x3,s4_3x3,s3_3x3s2 --impls lite,lite32 --reps 20
for i in a b; do
  step bk64_$i 300 python -u bench.py --steps 20 --warmup 5
  step bk32_$i 300 env FT_CONV_LITE_BK=32 python -u bench.py --steps 20 --warmup 5
done
step bk64_300 300 python -u bench.py --steps 300 --warmup 10
step bk32_300 300 env FT_CONV_LITE_BK=32 python -u bench.py --steps 300 --warmup 10
step bk32_l1 300 env FT_CONV_LITE_BK=32 python -u bench.py --steps 100 --warmup 10 --lanes 1
step bk64_l1 300 python -u bench.py --steps 100 --warmup 10 --lanes 1
