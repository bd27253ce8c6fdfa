source tools/gpu_calls/gpu_steps.sh
step pytest_lib 300 python -u -m pytest tests/test_bottleneck.py tests/test_compiler.py -x -v -m gpu --timeout 200 --timeout-method thread
step bench_resnet 300 python bench.py --steps 30 --warmup 5
step bench_resnet_nolib 300 env FTM_CONV_LIB=0 python bench.py --steps 30 --warmup 5
step bench_resnet2 300 python bench.py --steps 30 --warmup 5
