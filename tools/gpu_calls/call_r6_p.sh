#!/bin/bash
# Round 6 call P: BERT job on the 2048-token granule, Inception job vs SPMD (plans), the
# JPEG workload on the reference example's model (Inception-v3) and with Flink's
# coordinator monitor.
source tools/gpu_calls/gpu_steps.sh
step r06_p/bench_bert_job 300 python bench.py --model bert_graph --job --steps 30 --warmup 5
step r06_p/bench_inc_job 300 python bench.py --model inception_v3 --job --steps 30 --warmup 5
step r06_p/bench_inc 300 python bench.py --model inception_v3 --steps 30 --warmup 5
step r06_p/jpeg_inc 500 python bench/jpeg_e2e.py --files 20000 --model inception_v3
step r06_p/jpeg_coord 400 python bench/jpeg_e2e.py --files 20000 --monitor coordinator
