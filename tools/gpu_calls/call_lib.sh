source tools/gpu_calls/gpu_steps.sh
step probe_lib 400 python -u bench/probe_lib_convs.py
