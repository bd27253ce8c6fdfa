#!/bin/bash
# Round 6 call AB: JPEG end to end with 32 file-read threads (Inception-v3 and ResNet-50).
source tools/gpu_calls/gpu_steps.sh
step r06_ab/jpeg_inc 500 python bench/jpeg_e2e.py --files 20000 --model inception_v3
step r06_ab/jpeg_rn 400 python bench/jpeg_e2e.py --files 20000
