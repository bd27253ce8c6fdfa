# BERT stream steady state vs the GPU-only number of the same compiled graph
source tools/gpu_calls/gpu_steps.sh
step bert_stream_steady 300 python -u examples/bert_stream.py --records 196608 --batch 256 --steady
step bert_graph_bench 300 python -u bench.py --model bert_graph --steps 30 --warmup 5
