source tools/gpu_calls/gpu_steps.sh
step bench_pp 400 python -u bench/gemm_pp_bench.py
