# round 3 (session 2) K: operating-point sweep with conv_lite (lanes x depth), and the
# ResNet-50 stream modes at 200k records (a steady window long enough to compare with bench.py)
source tools/gpu_calls/gpu_steps.sh
step l2d3 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --lanes 2 --depth 3
step l3d4 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --lanes 3 --depth 4
step l2d4 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --lanes 2 --depth 4
step l3d5 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --lanes 3 --depth 5
step l2d3b 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --lanes 2 --depth 3
step l3d4_inc 200 env FT_CONV_IMPL=incumbent python -u bench.py --gpus 1 --steps 20 --warmup 5 --lanes 3 --depth 4
step stream_inproc 300 python -u examples/resnet50_stream.py --records 200000
step stream_wsrc 300 python -u examples/resnet50_stream.py --records 200000 --worker-source
step stream_proc 300 python -u examples/resnet50_stream.py --records 200000 --processes
