# round 3 (session 3) P: streaming-store native library vs the previous one on the record
# transport and the worker-process ResNet stream (same box, alternating)
source tools/gpu_calls/gpu_steps.sh
export FTM_NO_AUTOBUILD=1
NSO=$(ls flink_tensorflow_amd/_native.cpython-*.so)
cp "$NSO" /tmp/_native_new.so
for i in a b; do
  cp /tmp/_native_new.so "$NSO"; step t8_new_$i 300 python -u bench/transport_bench.py --workers 8 --records 80000
  cp ab/_native_base.so "$NSO"; step t8_base_$i 300 python -u bench/transport_bench.py --workers 8 --records 80000
  cp /tmp/_native_new.so "$NSO"; step ws_new_$i 400 python -u examples/resnet50_stream.py --records 200000 --worker-source
  cp ab/_native_base.so "$NSO"; step ws_base_$i 400 python -u examples/resnet50_stream.py --records 200000 --worker-source
done
cp /tmp/_native_new.so "$NSO"
