# end-to-end A/B of the pooled stem tile height, longer timed windows, interleaved
source tools/gpu_calls/gpu_steps.sh
for i in 1 2 3; do
step ab7_$i 300 env FTM_STEM_POOL_ROWS=7 python -u bench.py --steps 300 --warmup 10
step ab14_$i 300 env FTM_STEM_POOL_ROWS=14 python -u bench.py --steps 300 --warmup 10
done
