# end of round 2 (late): GPU suite, smoke, every bench config, kernel stats for W&D (fused)
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_resnet 300 python -u bench.py --steps 30 --warmup 5
step bench_bert 300 python -u bench.py --model bert --steps 30 --warmup 5
step bench_bert_graph 300 python -u bench.py --model bert_graph --steps 30 --warmup 5
step bench_wd 300 python -u bench.py --model widedeep --steps 50 --warmup 10
step bench_inc 300 python -u bench.py --model inception_v3 --steps 20 --warmup 5
step bench_inc_dyn 300 python -u bench.py --model inception_v3 --steps 20 --warmup 5 --dynamic
step bench_rn_open 300 python -u bench.py --steps 200 --warmup 20 --offered-rate 40000 --buckets 32,64,96,128,160,192,224,256
step bert_stream 300 python -u examples/bert_stream.py --records 196608 --batch 256 --steady
step rn_stream_sm 300 python -u examples/resnet50_stream.py --records 100000 --savedmodel
