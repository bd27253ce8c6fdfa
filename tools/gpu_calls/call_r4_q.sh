# round 4 Q: where a conv_lite_fp8 K-tile's time goes (in-kernel s_memtime stamps per phase)
# on Inception-v3 layer shapes; fp8 tests (the STAMP build shares the kernel source)
source tools/gpu_calls/gpu_steps.sh
step test_fp8 300 python -u -m pytest tests/test_fp8.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
step stamp_fp8 120 python -u bench/conv_stamp_probe.py --fp8
