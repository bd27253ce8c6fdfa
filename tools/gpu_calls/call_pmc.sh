source tools/gpu_calls/gpu_steps.sh
step build 400 python -c "import __graft_entry__ as g; g.build()"
step pytest_fp8 300 python -m pytest tests/test_fp8.py -q -m gpu -x
cd /tmp && export TMPDIR=/tmp
step pmc_l2 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d "$OUT/pmc_l2" -o run -- python "$REPO/bench/ablate_v2.py"
step pmc_ta 300 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum --output-format csv -d "$OUT/pmc_ta" -o run -- python "$REPO/bench/ablate_v2.py"
cd "$REPO"
step bench_inc_fp8 500 python bench.py --model inception_v3 --steps 20 --warmup 5
