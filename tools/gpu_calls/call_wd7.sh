# gather_into on raw buffer views: W&D + ResNet benches
source tools/gpu_calls/gpu_steps.sh
step bench_wd 300 python -u bench.py --model widedeep --steps 50 --warmup 10
step bench_wd_b 300 python -u bench.py --model widedeep --steps 50 --warmup 10
step bench_rn 300 python -u bench.py --steps 30 --warmup 5
step rn_stream 300 python -u examples/resnet50_stream.py --records 100000
