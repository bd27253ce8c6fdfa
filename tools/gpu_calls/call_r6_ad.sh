#!/bin/bash
# Round 6 call AD: BERT-base 2 vs 3 compute lanes, interleaved twice more.
source tools/gpu_calls/gpu_steps.sh
for i in 1 2; do
step r06_ad/bert_l2_$i 300 python bench.py --model bert_graph --steps 30 --warmup 5 --lanes 2
step r06_ad/bert_l3_$i 300 python bench.py --model bert_graph --steps 30 --warmup 5 --lanes 3
done
