source tools/gpu_steps.sh
export FTM_DIST_BACKEND=gloo
step build 400 python -c "import __graft_entry__ as g; g.build()"
step dp2_resnet 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3
step dp2_bert 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --model bert --steps 5 --warmup 2
step dp2_wd 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --model widedeep --steps 10 --warmup 3
step dp2_inc 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29536 bench.py --gpus 2 --model inception_v3 --steps 5 --warmup 2
