# round 3 (session 3) H: non-temporal (streaming) stores in the host staging gather, A/B
# against the previous native library (ab/_native_base.so) in the driver's window
source tools/gpu_calls/gpu_steps.sh
export FTM_NO_AUTOBUILD=1
NSO=$(ls flink_tensorflow_amd/_native.cpython-*.so)
cp "$NSO" /tmp/_native_new.so
for i in a b c; do
  cp /tmp/_native_new.so "$NSO"; step nt_$i 300 python -u bench.py --steps 20 --warmup 5
  cp ab/_native_base.so "$NSO"; step base_$i 300 python -u bench.py --steps 20 --warmup 5
done
cp /tmp/_native_new.so "$NSO"; step nt_300 300 python -u bench.py --steps 300 --warmup 10
cp ab/_native_base.so "$NSO"; step base_300 300 python -u bench.py --steps 300 --warmup 10
cp /tmp/_native_new.so "$NSO"; step nt_l1 300 python -u bench.py --steps 100 --warmup 10 --lanes 1
cp ab/_native_base.so "$NSO"; step base_l1 300 python -u bench.py --steps 100 --warmup 10 --lanes 1
cp /tmp/_native_new.so "$NSO"
step pytest_h 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_remote.py tests/test_runtime.py
