# round 4 U+V in one call: the halo conv with the row-aware swizzle key, and conv_lite on
# eight waves with the DMA / MFMA roles split (tile 4): numerics, per-layer times, counters,
# ResNet-50 bench A/B (FT_* environment overrides of the engine config)
source tools/gpu_calls/gpu_steps.sh
step test_c3h 300 python -u -m pytest tests/test_conv3x3h.py tests/test_conv_pp.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
step probe 180 python -u bench/conv_layer_probe.py --layers s2_3x3,s3_3x3,s4_3x3,s3_3x3s2 --impls lite,halo,ws,lite,halo,ws --reps 20
step pmc_b 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAVE_CYCLES --kernel-trace --output-format csv -d "$OUT/pmc_b" -o run -- python3 bench/conv_layer_probe.py --layers s3_3x3,s2_3x3 --impls lite,halo,ws --reps 3
step bench_base 300 python -u bench.py --steps 20 --warmup 5
step bench_ws 300 env FT_CONV_LITE_WS=1 python -u bench.py --steps 20 --warmup 5
step bench_halo 300 env FT_CONV3X3_HALO=1 python -u bench.py --steps 20 --warmup 5
