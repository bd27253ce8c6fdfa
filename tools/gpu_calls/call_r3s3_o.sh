# round 3 (session 3) O: record transport with the streaming-store slab scatter (8 workers;
# coordinator source and in-worker parallel source), ResNet stream through worker processes
source tools/gpu_calls/gpu_steps.sh
step transport8 300 python -u bench/transport_bench.py --workers 8 --records 80000
step transport8_wsrc 300 python -u bench/transport_bench.py --workers 8 --records 400000 --remote-source
step transport16_wsrc 300 python -u bench/transport_bench.py --workers 16 --records 800000 --remote-source
step stream_proc 400 python -u examples/resnet50_stream.py --records 200000 --processes
step stream_wsrc 400 python -u examples/resnet50_stream.py --records 200000 --worker-source
