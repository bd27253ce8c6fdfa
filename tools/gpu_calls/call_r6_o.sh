#!/bin/bash
# Round 6 call O: JPEG end to end with the 2x decoder + background decode; job vs SPMD with
# plan summaries (BERT SavedModel vs GraphDef) and the cheaper result conversion.
source tools/gpu_calls/gpu_steps.sh
step r06_o/jpeg_async32 400 python bench/jpeg_e2e.py --files 20000 --decode-threads 32
step r06_o/jpeg_async64 400 python bench/jpeg_e2e.py --files 20000 --decode-threads 64
step r06_o/jpeg_reader12 400 python bench/jpeg_e2e.py --files 20000 --decode reader --readers 12
step r06_o/bench_bert_job 300 python bench.py --model bert_graph --job --steps 30 --warmup 5
step r06_o/bench_bert 300 python bench.py --model bert_graph --steps 30 --warmup 5
step r06_o/bench_rn_job 300 python bench.py --job --steps 20 --warmup 5
step r06_o/bench_rn 200 python bench.py --gpus 1 --steps 20 --warmup 5
