# round 3 (session 3) M: gc.freeze() of the setup objects after the plans compile (the
# runner default now) vs the GC left alone, in the driver's 20-step window; window timelines
source tools/gpu_calls/gpu_steps.sh
for i in a b c d; do
  step fz_$i 300 python -u bench.py --steps 20 --warmup 5
  step nofz_$i 300 python -u bench.py --steps 20 --warmup 5 --no-gc-freeze
done
step fz_300 300 python -u bench.py --steps 300 --warmup 10
step nofz_300 300 python -u bench.py --steps 300 --warmup 10 --no-gc-freeze
step win_fz_40 300 python -u bench/window_probe.py --steps 40 --warmup 5
step wd_fz 300 python -u bench.py --model widedeep --steps 200 --warmup 20
step wd_nofz 300 python -u bench.py --model widedeep --steps 200 --warmup 20 --no-gc-freeze
