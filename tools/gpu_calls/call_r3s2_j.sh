# round 3 (session 2) J: stage-2 fused tail (expand + next reduce, weights streamed; moves
# ~200 MB less per boundary) in the 2-lane plan — does fewer bytes beat a slower kernel?
source tools/gpu_calls/gpu_steps.sh
step rn_def_a 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_wide_a 200 env FT_FUSE_WIDE_TAILS=1 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_def_b 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_wide_b 200 env FT_FUSE_WIDE_TAILS=1 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_wide_300 200 env FT_FUSE_WIDE_TAILS=1 python -u bench.py --gpus 1 --steps 300 --warmup 10
step rn_def_300 200 python -u bench.py --gpus 1 --steps 300 --warmup 10
