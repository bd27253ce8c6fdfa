# round 3 (session 2) J: stage-2 fused tail (expand + next reduce, weights streamed; moves
# ~200 MB less per boundary) in the 2-lane plan — does fewer bytes beat a slower kernel?
source tools/gpu_calls/gpu_steps.sh
step rn_def_a 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_wide_a 200 env FT_FUSE_WIDE_TAILS=1 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_def_b 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_wide_b 200 env FT_FUSE_WIDE_TAILS=1 python -u bench.py --gpus 1 --steps 20 --warmup 5
step rn_wide_300 200 env FT_FUSE_WIDE_TAILS=1 python -u bench.py --gpus 1 --steps 300 --warmup 10
step rn_def_300 200 python -u bench.py --gpus 1 --steps 300 --warmup 10
step stream_inproc 300 python -u examples/resnet50_stream.py --records 40000
step stream_proc 300 python -u examples/resnet50_stream.py --records 40000 --processes
step stream_wsrc 300 python -u examples/resnet50_stream.py --records 40000 --worker-source
step transport8 300 python -u bench/transport_bench.py --workers 8 --records 80000
step transport8_wsrc 300 python -u bench/transport_bench.py --workers 8 --records 400000 --remote-source
source tools/gpu_calls/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$REPO"
step pmc_fetch 150 timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py --gpus 1 --steps 3 --warmup 1 --lanes 1
step pmc_write 150 timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py --gpus 1 --steps 3 --warmup 1 --lanes 1
step pmc_ea 150 timeout -s KILL 140 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc_ea" -o run -- python3 bench.py --gpus 1 --steps 3 --warmup 1 --lanes 1
