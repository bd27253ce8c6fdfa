# A/B of the staging-slot preprocess head through the DataStream runtime and bench.py (interleaved)
source tools/gpu_calls/gpu_steps.sh
step stream_on1 300 python examples/resnet50_stream.py --records 80000
FTM_HEAD_BYPASS=0 step stream_off1 300 python examples/resnet50_stream.py --records 80000
step stream_on2 300 python examples/resnet50_stream.py --records 80000
FTM_HEAD_BYPASS=0 step stream_off2 300 python examples/resnet50_stream.py --records 80000
step bench_on 300 python bench.py --steps 40 --warmup 8
FTM_HEAD_BYPASS=0 step bench_off 300 python bench.py --steps 40 --warmup 8
