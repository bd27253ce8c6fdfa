# Multi-rank rehearsal on one GPU: 2 ranks over gloo (RCCL needs one GPU per rank)
source tools/gpu_steps.sh
export FTM_DIST_BACKEND=gloo
for m in resnet50 bert widedeep inception_v3; do
  step dp2_$m 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --model $m
done
