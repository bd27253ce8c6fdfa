# gemm_pp per-shape counters (one shape per run; counters in their own passes)
source tools/gpu_calls/gpu_steps.sh
step plain 300 python -u bench/gemm_pp_bench.py --shapes bert_qkv,bert_ffn1,bert_ffn1_plain,k768_n2304_m49152,bert_ffn2 --ours-only
cd /tmp && export TMPDIR=/tmp
for sh in bert_qkv bert_ffn1_plain; do
  step sq_$sh 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAVES --kernel-trace --output-format csv -d "$OUT/pmc_sq_$sh" -o run -- python "$REPO/bench/gemm_pp_bench.py" --shapes $sh --ours-only --rounds 2 --reps 5
  step tcc_$sh 120 timeout -s KILL 100 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc_tcc_$sh" -o run -- python "$REPO/bench/gemm_pp_bench.py" --shapes $sh --ours-only --rounds 2 --reps 5
done
