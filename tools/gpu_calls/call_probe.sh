source tools/gpu_calls/gpu_steps.sh
step probe 120 python tools/probe_tr.py
