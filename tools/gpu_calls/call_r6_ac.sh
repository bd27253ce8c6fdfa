#!/bin/bash
# Round 6 call AC: BERT-base (TF GraphDef, token-packed) on 2 / 3 / 4 compute lanes.
source tools/gpu_calls/gpu_steps.sh
step r06_ac/bert_l3 300 python bench.py --model bert_graph --steps 30 --warmup 5
step r06_ac/bert_l2 300 python bench.py --model bert_graph --steps 30 --warmup 5 --lanes 2
step r06_ac/bert_l4 300 python bench.py --model bert_graph --steps 30 --warmup 5 --lanes 4 --depth 4
step r06_ac/bert_l3b 300 python bench.py --model bert_graph --steps 30 --warmup 5
