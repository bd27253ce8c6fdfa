# ResNet-50 operating-point sweep: compute lanes x pipeline depth x micro-batch
source tools/gpu_calls/gpu_steps.sh
for cfg in "2 3 256" "3 3 256" "4 4 256" "2 4 256" "3 4 256" "2 3 384" "3 4 384" "2 3 512"; do
  set -- $cfg
  step "sw_l$1_d$2_b$3" 200 python bench.py --steps 40 --warmup 8 --lanes $1 --depth $2 --batch $3
done
step sw_wide 200 env FTM_TAIL_WIDE=1 python bench.py --steps 40 --warmup 8
