# round 4 AF: validation of the final tree on a fresh box (the fp8 192-wide tile is now the
# default) — the whole GPU suite, smoke, the BASELINE benches — plus the fewest-staged-rows
# fp8 tile chooser (FT_FP8_LITE_WIDE=2) A/B on Inception-v3
source tools/gpu_calls/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests/ -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_rn_a 300 python -u bench.py --steps 20 --warmup 5
step inc_w1_a 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_w2_a 300 env FT_FP8_LITE_WIDE=2 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_w1_b 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_w2_b 300 env FT_FP8_LITE_WIDE=2 python -u bench.py --model inception_v3 --steps 30 --warmup 5
step inc_w1_dyn 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --dynamic
step inc_w2_dyn 300 env FT_FP8_LITE_WIDE=2 python -u bench.py --model inception_v3 --steps 30 --warmup 5 --dynamic
step bench_rn_b 300 python -u bench.py --steps 20 --warmup 5
step bench_bert_graph 300 python -u bench.py --model bert_graph --steps 30 --warmup 5
step bench_wd 300 python -u bench.py --model widedeep --steps 50 --warmup 10
