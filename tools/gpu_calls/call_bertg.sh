# BERT GraphDef/SavedModel through the compiler: GPU tests, bench vs the hand-built padded encoder
source tools/gpu_calls/gpu_steps.sh
step pytest_bg 600 python -u -m pytest tests/test_bert_graph.py tests/test_compiler.py tests/test_fp8.py tests/test_model_function_compiled.py -x -v -s -m gpu --timeout 300 --timeout-method thread
step bench_bg 600 python -u bench.py --model bert_graph --steps 30 --warmup 5
step bench_bert_pad 300 python -u bench.py --model bert --no-pack --steps 30 --warmup 5
