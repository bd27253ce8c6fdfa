# round 3 (session 2) M: framework-owned HIP streams for runner lanes and hipGraph captures
# (fixes pooled-stream collisions between sibling GPU subtasks); GPU suite + default benches
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench_rn 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_bert 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --model bert_graph
step stream_chain 300 python -u examples/resnet50_stream.py --records 200000
