# Validation after the block-boundary / library-GEMM / odd-s2d changes
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_resnet 500 python bench.py --steps 30 --warmup 5
step bench_resnet_b128 500 python bench.py --steps 30 --warmup 5 --batch 128
step bench_resnet_l1 500 python bench.py --steps 30 --warmup 5 --lanes 1
step bench_bert 500 python bench.py --model bert --steps 30 --warmup 5
step bench_bert_l1 500 python bench.py --model bert --steps 30 --warmup 5 --lanes 1
step bench_wd 500 python bench.py --model widedeep --steps 50 --warmup 10
step bench_inc_fp8 500 python bench.py --model inception_v3 --steps 20 --warmup 5
step bench_inc_l1 500 python bench.py --model inception_v3 --steps 20 --warmup 5 --lanes 1
step stream_rn 500 python examples/resnet50_stream.py --records 80000
