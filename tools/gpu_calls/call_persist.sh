# gemm_pp persistent tile walk A/B
source tools/gpu_calls/gpu_steps.sh
FTM_GEMM_PERSIST=1 step pst_tests 300 python -u -m pytest tests/test_gemm_pp.py -x -q -m gpu --timeout 120 --timeout-method thread
step pst0 300 python -u bench/gemm_pp_bench.py --shapes bert_qkv,bert_o,bert_ffn1,bert_ffn2,bert_packed_o,sq4096,rn_s3_c1
FTM_GEMM_PERSIST=1 step pst1 300 python -u bench/gemm_pp_bench.py --shapes bert_qkv,bert_o,bert_ffn1,bert_ffn2,bert_packed_o,sq4096,rn_s3_c1
step bert_p0 300 python -u bench.py --model bert --steps 30 --warmup 5
FTM_GEMM_PERSIST=1 step bert_p1 300 python -u bench.py --model bert --steps 30 --warmup 5
step rn_p0 300 python -u bench.py --steps 30 --warmup 5
FTM_GEMM_PERSIST=1 step rn_p1 300 python -u bench.py --steps 30 --warmup 5
