# round 3 (session 2) W: debug the multi-output fp8 conv against its host reference
source tools/gpu_calls/gpu_steps.sh
step multi_probe 120 python -u tools/probes/multi_probe.py
