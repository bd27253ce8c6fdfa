# Multi-rank rehearsal of bench.py after the node-level histogram merge (2 ranks on one GPU over
# gloo: RCCL needs one GPU per rank), then two more 1-GPU ResNet-50 runs for the range.
source tools/gpu_steps.sh
export FTM_DIST_BACKEND=gloo
step dp2_resnet50 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3
step dp2_bert 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --model bert --steps 5 --warmup 2
unset FTM_DIST_BACKEND
step bench_resnet_a 300 python bench.py --steps 40 --warmup 8
step bench_resnet_b 300 python bench.py --steps 40 --warmup 8
