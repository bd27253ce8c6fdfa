#!/usr/bin/env python3
"""Per-layer A/B: Winograd F(2x2,3x3) (kernels/wino3x3.hip) against the incumbent kernels
on ResNet-50's stride-1 3x3 layers at micro-batch B: conv3x3c64 (stage 1) and conv_lite
(stages 2-4).  Reports µs per launch, the direct-conv-equivalent TFLOP/s (9 * Cin MACs per
output, as the model counts them) and the max error of each against an fp32 conv."""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flink_tensorflow_amd.ops import kernels as K  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--layers", default="56,28,14,7", help="spatial sizes to run (56: 64 ch, 28: 128, 14: 256, 7: 512)")
    ap.add_argument("--wino-only", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda")
    B = a.batch
    chans = {56: 64, 28: 128, 14: 256, 7: 512}
    for H in [int(v) for v in a.layers.split(",")]:
        C = chans[H]
        g = torch.Generator().manual_seed(H)
        x = torch.randn(B, H, H, C, generator=g).to(dev, torch.bfloat16)
        w = torch.randn(3, 3, C, C, generator=g) * (2.0 / (9 * C)) ** 0.5
        b = (torch.randn(C, generator=g) * 0.1).to(dev)
        w_ohwi = w.permute(3, 0, 1, 2).contiguous().to(dev, torch.bfloat16)
        u = K.wino_f23_weights(w).to(dev)
        y_w = torch.empty(B, H, H, C, dtype=torch.bfloat16, device=dev)
        y_i = torch.empty_like(y_w)
        if C == 64:
            inc_name = "conv3x3c64"

            def inc():
                K.conv3x3_c64(x, w_ohwi, b, K.ACT_RELU, out=y_i)
        else:
            inc_name = "conv_lite"
            cl = K.ConvPP([(tuple(x.shape), (3, 3), (1, 1), (1, 1), (1, 1))], C, (H, H), dev, tile=2)
            w2 = w_ohwi.reshape(C, -1)

            def inc():
                cl([x], w2, b, None, K.ACT_RELU, out=y_i)

        def win():
            K.wino_f23(x, u, C, b, K.ACT_RELU, out=y_w)

        t_w = timeit(win, a.reps)
        if a.wino_only:
            print(json.dumps({"layer": f"{H}x{H}x{C}", "wino_us": round(t_w, 1)}), flush=True)
            continue
        t_i = timeit(inc, a.reps)
        flops = 2.0 * B * H * H * C * C * 9
        nref = min(B, 16)
        ref = torch.relu(F.conv2d(x[:nref].float().permute(0, 3, 1, 2), w.permute(3, 2, 0, 1).to(dev), b,
                                  padding=1)).permute(0, 2, 3, 1)
        sc = ref.abs().max().item()
        print(json.dumps({"layer": f"{H}x{H}x{C}", "batch": B, "wino_us": round(t_w, 1), inc_name + "_us": round(t_i, 1),
                          "speedup": round(t_i / t_w, 3), "wino_tflops_equiv": round(flops / t_w / 1e6, 1),
                          "incumbent_tflops": round(flops / t_i / 1e6, 1),
                          "wino_err": round((y_w[:nref].float() - ref).abs().max().item() / sc, 5),
                          "incumbent_err": round((y_i[:nref].float() - ref).abs().max().item() / sc, 5)}), flush=True)


if __name__ == "__main__":
    main()
