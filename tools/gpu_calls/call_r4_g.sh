# round 4 G: where conv_lite's K-tile time goes (in-kernel s_memtime stamps of wave 0 per
# phase), and a BERT GraphDef kernel trace per replay (the CLS gather is now a HIP kernel:
# no at::native kernel expected per replay)
source tools/gpu_calls/gpu_steps.sh
step test_conv 300 python -u -m pytest tests/test_conv_pp.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
step stamp 120 python -u bench/conv_stamp_probe.py --layers s2_3x3,s3_3x3,s4_3x3
cd /tmp && export TMPDIR=/tmp
step rocprof_bert 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bert" -o run -- python "$REPO/bench.py" --model bert_graph --steps 20 --warmup 3
