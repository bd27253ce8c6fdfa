source tools/gpu_calls/gpu_steps.sh
step df_stage1 300 python -u bench/depth_first_probe.py
FETCH=block2/unit4/conv3/Relu:0 step df_stage2 300 python -u bench/depth_first_probe.py
FETCH=top_k:1 step df_all 300 python -u bench/depth_first_probe.py
