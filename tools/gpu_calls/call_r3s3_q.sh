# round 3 (session 3) Q: conv_lite without s_setprio around its MFMAs (wave priority may
# widen the skew the per-K-tile barrier waits on) vs the default, same box, alternating
source tools/gpu_calls/gpu_steps.sh
SO=$(ls flink_tensorflow_amd/_hip.cpython-*.so)
cp "$SO" /tmp/_hip_new.so
step probe_noprio 300 python -u bench/conv_layer_probe.py --layers s2_3x3,s3_3x3,s4_3x3 --impls lite --reps 20
cp ab/_hip_base.so "$SO"; step probe_prio 300 python -u bench/conv_layer_probe.py --layers s2_3x3,s3_3x3,s4_3x3 --impls lite --reps 20
for i in a b; do
  cp /tmp/_hip_new.so "$SO"; step np_$i 300 python -u bench.py --steps 20 --warmup 5
  cp ab/_hip_base.so "$SO"; step p_$i 300 python -u bench.py --steps 20 --warmup 5
done
cp /tmp/_hip_new.so "$SO"; step np_300 300 python -u bench.py --steps 300 --warmup 10
cp ab/_hip_base.so "$SO"; step p_300 300 python -u bench.py --steps 300 --warmup 10
cp /tmp/_hip_new.so "$SO"
