# gemm_pp epilogue A/B: LDS-staged (0) vs direct from registers (1)
source tools/gpu_calls/gpu_steps.sh
FTM_GEMM_EPI=1 step epi_tests 300 python -u -m pytest tests/test_gemm_pp.py -x -q -m gpu --timeout 120 --timeout-method thread
step epi0 300 python -u bench/gemm_pp_bench.py --shapes bert_qkv,bert_o,bert_ffn1,bert_ffn2,bert_packed_o,sq4096,rn_s3_c1
FTM_GEMM_EPI=1 step epi1 300 python -u bench/gemm_pp_bench.py --shapes bert_qkv,bert_o,bert_ffn1,bert_ffn2,bert_packed_o,sq4096,rn_s3_c1
step bert_epi0 300 python -u bench.py --model bert --steps 30 --warmup 5
FTM_GEMM_EPI=1 step bert_epi1 300 python -u bench.py --model bert --steps 30 --warmup 5
step bert_epi0b 300 python -u bench.py --model bert --steps 30 --warmup 5
FTM_GEMM_EPI=1 step bert_epi1b 300 python -u bench.py --model bert --steps 30 --warmup 5
