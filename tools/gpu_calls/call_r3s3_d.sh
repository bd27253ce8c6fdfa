# round 3 (session 3) D: persistent kernels (stage-1 tails, pw_res, conv3x3c64) on a subset
# of the CUs (EngineConfig.persistent_cus) so the sibling lane's kernels can co-run
source tools/gpu_calls/gpu_steps.sh
step pt_test 300 env FT_PERSISTENT_CUS=128 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_bottleneck.py tests/test_pw_res.py tests/test_compiler.py
for i in a b; do
  for c in 0 128 192 160 96; do
    step pc${c}_$i 300 env FT_PERSISTENT_CUS=$c python -u bench.py --steps 20 --warmup 5
  done
done
for c in 0 128 192; do
  step pc${c}_300 300 env FT_PERSISTENT_CUS=$c python -u bench.py --steps 300 --warmup 10
done
step pc128_1lane 300 env FT_PERSISTENT_CUS=128 python -u bench.py --steps 100 --warmup 10 --lanes 1
step pc0_1lane 300 env FT_PERSISTENT_CUS=0 python -u bench.py --steps 100 --warmup 10 --lanes 1
