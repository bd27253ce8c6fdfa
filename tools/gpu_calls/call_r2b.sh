# W&D packed collation + captured DP step; dynamic buckets; open-loop latency
source tools/gpu_calls/gpu_steps.sh
step pytest_wd 300 python -u -m pytest tests/test_rccl.py tests/test_widedeep.py -x -v -m gpu --timeout 120 --timeout-method thread
step bench_wd 300 python -u bench.py --model widedeep --steps 30 --warmup 5
step bench_inc_dyn32 600 python -u bench.py --model inception_v3 --dynamic --buckets 64,96,128,160,192,224 --steps 30 --warmup 5
step bench_inc_dyn_old 600 python -u bench.py --model inception_v3 --dynamic --buckets 64,128 --steps 30 --warmup 5
step bench_rn_open 300 python -u bench.py --offered-rate 40000 --buckets 32,64,96,128,160,192,224 --max-delay-ms 2 --steps 40 --warmup 10
step bench_rn_open60 300 python -u bench.py --offered-rate 60000 --buckets 32,64,96,128,160,192,224 --max-delay-ms 2 --steps 40 --warmup 10
step transport_slab 300 python -u bench/transport_bench.py --workers 8 --records 80000
FTM_SLAB_BYTES=0 step transport_pickle 300 python -u bench/transport_bench.py --workers 8 --records 80000
step stream_inproc 300 python -u examples/resnet50_stream.py --records 80000
step stream_proc 300 python -u examples/resnet50_stream.py --records 80000 --processes
