# round 3 (session 2) E: conv_lite numerics + per-layer probe vs igemm / conv_pp; SQ counters of conv_lite
source tools/gpu_calls/gpu_steps.sh
step pytest_convpp 300 python -u -m pytest tests/test_conv_pp.py -q -m gpu --timeout 120 --timeout-method thread
step probe 200 python -u bench/conv_layer_probe.py --layers s2_3x3,s3_3x3,s4_3x3,s3_3x3s2,s3_reduce,s2_reduce --impls igemm,lite,pp --reps 20
cd /tmp && export TMPDIR=/tmp && cd "$REPO"
step pmc_lite 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAVES --kernel-trace --output-format csv -d "$OUT/pmc_lite" -o run -- python3 bench/conv_layer_probe.py --layers s3_3x3 --impls lite --reps 3
step pmc_lite2 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAVE_CYCLES --kernel-trace --output-format csv -d "$OUT/pmc_lite2" -o run -- python3 bench/conv_layer_probe.py --layers s3_3x3 --impls lite --reps 3
