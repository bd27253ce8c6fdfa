#!/bin/bash
# Round 6 call AJ: soak runs — 3,000-step ResNet-50 and Inception-v3 windows, and 100,000
# JPEG files through the ResNet-50 job.
source tools/gpu_calls/gpu_steps.sh
step r06_aj/rn_3000 300 python bench.py --steps 3000 --warmup 10
step r06_aj/inc_3000 300 python bench.py --model inception_v3 --steps 3000 --warmup 10
step r06_aj/jpeg_100k 600 python bench/jpeg_e2e.py --files 100000
