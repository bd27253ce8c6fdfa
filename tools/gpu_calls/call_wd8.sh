# fused W&D under data parallelism: replica check (2 ranks, loopback comm, one GPU) + bench rehearsal
source tools/gpu_calls/gpu_steps.sh
step wd_dp 400 python -u -m pytest tests/test_widedeep.py -x -q -m gpu -k "dp_replicas" --timeout 350 --timeout-method thread
TR="python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
step rehearse_wd 400 $TR --master-port 29542 bench.py --gpus 2 --model widedeep --steps 10 --warmup 3 --no-graph --rehearse-fake-comm
