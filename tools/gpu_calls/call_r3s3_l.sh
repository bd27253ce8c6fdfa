# round 3 (session 3) L: per-batch timeline of the driver's 20-step window (submit, H2D done,
# compute done) — where the ~2.4 ms of fill / drain go
source tools/gpu_calls/gpu_steps.sh
step window_a 300 python -u bench/window_probe.py --steps 20 --warmup 5
step window_b 300 python -u bench/window_probe.py --steps 20 --warmup 5
step window_40 300 python -u bench/window_probe.py --steps 40 --warmup 5
