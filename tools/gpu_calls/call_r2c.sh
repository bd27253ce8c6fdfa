# full GPU suite, transport + stream in worker process, headline benches
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
step transport_slab 300 python -u bench/transport_bench.py --workers 8 --records 120000
FTM_SLAB_BYTES=0 step transport_pickle 300 python -u bench/transport_bench.py --workers 8 --records 120000
step stream_inproc 300 python -u examples/resnet50_stream.py --records 100000
step stream_proc 300 python -u examples/resnet50_stream.py --records 100000 --processes
step bench_rn 300 python -u bench.py --steps 30 --warmup 5
step bench_bert 300 python -u bench.py --model bert --steps 30 --warmup 5
step bench_inc 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
