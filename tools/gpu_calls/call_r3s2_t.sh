# round 3 (session 2) T: fp8 conv implementations per Inception layer (which kernel for the
# 147x147 / 73x73 layers now that conv_lite_fp8 has 64/96-wide tiles)
source tools/gpu_calls/gpu_steps.sh
step fp8_probe 300 python -u bench/fp8_conv_probe.py --impls dconv4,dconv8,lite,cfg0,cfg1,cfg2
