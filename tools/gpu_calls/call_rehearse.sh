# 2-rank rehearsal of bench.py's multi-rank control flow on one GPU (loopback comm, not RCCL)
source tools/gpu_calls/gpu_steps.sh
TR="python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
step rehearse_rn 400 $TR --master-port 29541 bench.py --gpus 2 --steps 10 --warmup 3 --rehearse-fake-comm
step rehearse_wd 400 $TR --master-port 29542 bench.py --gpus 2 --model widedeep --steps 10 --warmup 3 --no-graph --rehearse-fake-comm
step rehearse_bert 400 $TR --master-port 29543 bench.py --gpus 2 --model bert --steps 10 --warmup 3 --rehearse-fake-comm
