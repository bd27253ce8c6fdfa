# round 4 O: compute lane 0 on a high-priority HIP stream (EngineConfig.lane_priority),
# interleaved A/B against the default on ResNet-50 and Inception-v3
source tools/gpu_calls/gpu_steps.sh
step rn_base_a 300 python -u bench.py --steps 20 --warmup 5
FT_LANE_PRIORITY=1 step rn_prio_a 300 python -u bench.py --steps 20 --warmup 5
step rn_base_b 300 python -u bench.py --steps 20 --warmup 5
FT_LANE_PRIORITY=1 step rn_prio_b 300 python -u bench.py --steps 20 --warmup 5
FT_LANE_PRIORITY=1 step rn_prio_300 300 python -u bench.py --steps 300 --warmup 10
step rn_base_300 300 python -u bench.py --steps 300 --warmup 10
step inc_base 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
FT_LANE_PRIORITY=1 step inc_prio 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
