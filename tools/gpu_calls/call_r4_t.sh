# round 4 T: conv_lite vs the halo-staged 3x3 conv under SQ counters (stage 2 / 3 3x3, B=256);
# halo kernel numerics (tail shapes fixed)
source tools/gpu_calls/gpu_steps.sh
step test_c3h 300 python -u -m pytest tests/test_conv3x3h.py -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
step pmc_a 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAVES --kernel-trace --output-format csv -d "$OUT/pmc_a" -o run -- python3 bench/conv_layer_probe.py --layers s3_3x3,s2_3x3 --impls lite,halo --reps 3
step pmc_b 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAVE_CYCLES --kernel-trace --output-format csv -d "$OUT/pmc_b" -o run -- python3 bench/conv_layer_probe.py --layers s3_3x3,s2_3x3 --impls lite,halo --reps 3
step pmc_c 120 timeout -s KILL 100 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc_c" -o run -- python3 bench/conv_layer_probe.py --layers s3_3x3,s2_3x3 --impls lite,halo --reps 3
