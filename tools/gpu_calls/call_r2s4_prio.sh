# igemm: s_setprio(1) around each K-tile's MFMA cluster (FTM_IGEMM_PRIO) — per-layer and end to end
source tools/gpu_calls/gpu_steps.sh
step layers_p0 300 python -u bench/layer_table.py --model resnet50
step layers_p1 300 env FTM_IGEMM_PRIO=1 python -u bench/layer_table.py --model resnet50
for i in 1 2 3; do
step abp0_$i 300 python -u bench.py --steps 300 --warmup 10
step abp1_$i 300 env FTM_IGEMM_PRIO=1 python -u bench.py --steps 300 --warmup 10
done
