# round 3 (session 2) I: HBM / fabric bytes per kernel of one ResNet-50 lane (TCC counters),
# to see whether the 2-lane plan is bound by memory traffic rather than MFMA time
source tools/gpu_calls/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$REPO"
step pmc_fetch 150 timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py --gpus 1 --steps 3 --warmup 1 --lanes 1
step pmc_write 150 timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py --gpus 1 --steps 3 --warmup 1 --lanes 1
step pmc_ea 150 timeout -s KILL 140 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc_ea" -o run -- python3 bench.py --gpus 1 --steps 3 --warmup 1 --lanes 1
