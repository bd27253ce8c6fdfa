source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_resnet 300 python bench.py --steps 30 --warmup 5
step bench_bert 300 python bench.py --model bert --steps 30 --warmup 5
step bench_inc 300 python bench.py --model inception_v3 --steps 20 --warmup 5
step stream_rn 600 python examples/resnet50_stream.py --records 80000 --batch 256
