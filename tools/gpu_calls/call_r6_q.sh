#!/bin/bash
# Round 6 call Q: Inception-v3 fp8 on 4 compute lanes (3 is the default), and ResNet-50 on 3.
source tools/gpu_calls/gpu_steps.sh
step r06_q/inc_l3 300 python bench.py --model inception_v3 --steps 30 --warmup 5
step r06_q/inc_l4 300 python bench.py --model inception_v3 --steps 30 --warmup 5 --lanes 4 --depth 4
step r06_q/inc_l4d5 300 python bench.py --model inception_v3 --steps 30 --warmup 5 --lanes 4 --depth 5
step r06_q/inc_l3b 300 python bench.py --model inception_v3 --steps 30 --warmup 5
step r06_q/inc_l4b 300 python bench.py --model inception_v3 --steps 30 --warmup 5 --lanes 4 --depth 4
step r06_q/rn_l2 200 python bench.py --steps 20 --warmup 5
step r06_q/rn_l3 200 python bench.py --steps 20 --warmup 5 --lanes 3 --depth 4
