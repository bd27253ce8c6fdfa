#!/bin/bash
# Round 6 call K: where the stage 2-4 3x3 conv_lite spends its time — the kernel without
# MFMAs, without DMA, with MFMAs only, and the two-wave tile, per layer.
source tools/gpu_calls/gpu_steps.sh
step r06_k/probe 200 python -u bench/conv_layer_probe.py --layers s2_3x3,s3_3x3,s4_3x3 --impls lite:2,lite:3,lite:4,lite:5,lite:6 --reps 20
step r06_k/jpeg_part32 400 python bench/jpeg_e2e.py --files 20000 --decode-threads 32
step r06_k/jpeg_part48 400 python bench/jpeg_e2e.py --files 20000 --decode-threads 48
step r06_k/jpeg_coord32 400 python bench/jpeg_e2e.py --files 20000 --decode-threads 32 --monitor coordinator
