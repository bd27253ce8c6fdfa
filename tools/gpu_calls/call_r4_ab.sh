# round 4 AB: persistent kernels (conv3x3c64, bottleneck_tail, pw_res) on fewer CUs, leaving
# room for the other compute lane's kernels (EngineConfig.persistent_cus); ResNet-50 A/B,
# alternating settings on one box
source tools/gpu_calls/gpu_steps.sh
step p256a 300 python -u bench.py --steps 20 --warmup 5
step p192a 300 env FT_PERSISTENT_CUS=192 python -u bench.py --steps 20 --warmup 5
step p224a 300 env FT_PERSISTENT_CUS=224 python -u bench.py --steps 20 --warmup 5
step p160a 300 env FT_PERSISTENT_CUS=160 python -u bench.py --steps 20 --warmup 5
step p256b 300 python -u bench.py --steps 20 --warmup 5
step p192b 300 env FT_PERSISTENT_CUS=192 python -u bench.py --steps 20 --warmup 5
step p224b 300 env FT_PERSISTENT_CUS=224 python -u bench.py --steps 20 --warmup 5
step p160b 300 env FT_PERSISTENT_CUS=160 python -u bench.py --steps 20 --warmup 5
