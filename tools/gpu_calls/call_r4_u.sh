# round 4 U: halo conv with the row-aware swizzle key (bank conflicts at row ends removed):
# numerics, per-layer time against conv_lite, LDS counters, ResNet-50 bench
source tools/gpu_calls/gpu_steps.sh
step test_c3h 300 python -u -m pytest tests/test_conv3x3h.py -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
step probe 120 python -u bench/conv_layer_probe.py --layers s2_3x3,s3_3x3,s4_3x3 --impls lite,halo,lite,halo --reps 20
step pmc_b 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAVE_CYCLES --kernel-trace --output-format csv -d "$OUT/pmc_b" -o run -- python3 bench/conv_layer_probe.py --layers s3_3x3,s2_3x3 --impls lite,halo --reps 3
step bench_rn1 300 python -u bench.py --steps 20 --warmup 5
