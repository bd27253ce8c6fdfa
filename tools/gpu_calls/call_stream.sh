source tools/gpu_calls/gpu_steps.sh
step stream_rn 600 python examples/resnet50_stream.py --records 80000 --batch 256
