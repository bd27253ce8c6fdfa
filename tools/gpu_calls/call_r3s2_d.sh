# round 3 (session 2) D: NUMA-bound staging + gather threads A/B (20-step window), 3x3 conv
# layer probe (igemm vs conv_pp) and SQ counters of both on the stage-3 3x3 layer
source tools/gpu_calls/gpu_steps.sh
step rn_numa_a 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_nonuma 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-numa
step rn_numa_b 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_g16 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --gather-threads 16
step rn_g4 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --gather-threads 4
step probe 200 python -u bench/conv_layer_probe.py --layers s2_3x3,s3_3x3,s4_3x3,s3_reduce,s2_reduce --impls igemm,pp --reps 20
cd /tmp && export TMPDIR=/tmp && cd "$REPO"
step pmc_ig 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAVES --kernel-trace --output-format csv -d "$OUT/pmc_ig" -o run -- python3 bench/conv_layer_probe.py --layers s3_3x3,s2_3x3 --impls igemm --reps 3
step pmc_pp 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAVES --kernel-trace --output-format csv -d "$OUT/pmc_pp" -o run -- python3 bench/conv_layer_probe.py --layers s3_3x3,s2_3x3 --impls pp --reps 3
step pmc_ig2 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAVE_CYCLES --kernel-trace --output-format csv -d "$OUT/pmc_ig2" -o run -- python3 bench/conv_layer_probe.py --layers s3_3x3,s2_3x3 --impls igemm --reps 3
