# round 4 AG: the GPU tests that build Inception-v3 fp8 plans, on the new default tile chooser
source tools/gpu_calls/gpu_steps.sh
step test_inc 400 python -u -m pytest tests/test_fp8.py tests/test_fullsize_numerics.py tests/test_chain.py tests/test_examples.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread
step inc_default 300 python -u bench.py --model inception_v3 --steps 30 --warmup 5
