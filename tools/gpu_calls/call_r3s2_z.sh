# round 3 (session 2) Z: worker maps a message's slab records as slices of one base array
# (one frombuffer + finalizer per batch instead of per record): stream --processes and
# transport; Inception lanes 2 vs 3 at 300 steps
source tools/gpu_calls/gpu_steps.sh
step stream_proc 300 python -u examples/resnet50_stream.py --records 200000 --processes
step stream_proc_b 300 python -u examples/resnet50_stream.py --records 200000 --processes
step stream_chain 300 python -u examples/resnet50_stream.py --records 200000
step transport8 300 python -u bench/transport_bench.py --workers 8 --records 80000
step transport1 300 python -u bench/transport_bench.py --workers 1 --records 40000
step inc_l2_300 300 python -u bench.py --model inception_v3 --steps 300 --warmup 10
step inc_l3_300 300 python -u bench.py --model inception_v3 --steps 300 --warmup 10 --lanes 3
step inc_l3_30 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --lanes 3
step inc_l2_30 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
