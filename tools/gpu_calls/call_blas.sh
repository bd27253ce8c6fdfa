source tools/gpu_calls/gpu_steps.sh
step blas 300 python bench/probe_hipblaslt.py
