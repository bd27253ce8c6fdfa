# round 5 E: Winograd PMC counters (one pass per run, kernel-trace only)
source tools/gpu_calls/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$REPO"
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
step pmc1 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS -d "$OUT/pmc1" -o p -- python3 -u bench/wino_bench.py --reps 5 --layers 56,7 --wino-only
step pmc2 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_WAVES TCC_HIT_sum TCC_MISS_sum -d "$OUT/pmc2" -o p -- python3 -u bench/wino_bench.py --reps 5 --layers 56,7 --wino-only
