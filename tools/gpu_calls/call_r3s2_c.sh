# round 3 (session 2) C: copy-pool gather (host ms per batch), ResNet-50 default window x3,
# 300-step steady state, packed BERT graph with 3 lanes / 2048-token capacities
source tools/gpu_calls/gpu_steps.sh
step rn_a 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_b 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_c 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_300 200 python -u bench.py --gpus 1 --steps 300 --warmup 10
step bertg 400 python -u bench.py --model bert_graph --steps 50 --warmup 5
step bertg_l2 400 python -u bench.py --model bert_graph --steps 50 --warmup 5 --lanes 2
step bert_zoo 300 python -u bench.py --model bert --steps 50 --warmup 5
