# native exp2 / rcp activations: full GPU suite, FFN1 GEMM, BERT
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
step gemm 300 python -u bench/gemm_pp_bench.py --shapes bert_ffn1,bert_ffn1_plain,bert_qkv
step bert 300 python -u bench.py --model bert --steps 30 --warmup 5
step bert_b 300 python -u bench.py --model bert --steps 30 --warmup 5
step bert_graph 300 python -u bench.py --model bert_graph --steps 30 --warmup 5
