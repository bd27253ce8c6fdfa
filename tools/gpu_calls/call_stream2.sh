# ResNet-50 through the full DataStream runtime (source -> batched model operator -> sink)
source tools/gpu_calls/gpu_steps.sh
step stream_rn 400 python examples/resnet50_stream.py --records 80000
