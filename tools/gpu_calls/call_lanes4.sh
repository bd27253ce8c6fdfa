# operating points: BERT lanes 3/4, ResNet lanes 2/3 with the current kernels
source tools/gpu_calls/gpu_steps.sh
step bert_l3 300 python -u bench.py --model bert --steps 30 --warmup 5
step bert_l4 300 python -u bench.py --model bert --steps 30 --warmup 5 --lanes 4
step bert_l2 300 python -u bench.py --model bert --steps 30 --warmup 5 --lanes 2
step rn_l2 300 python -u bench.py --steps 30 --warmup 5
step rn_l3 300 python -u bench.py --steps 30 --warmup 5 --lanes 3
step rn_l2b 300 python -u bench.py --steps 30 --warmup 5
