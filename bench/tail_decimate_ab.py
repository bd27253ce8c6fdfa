#!/usr/bin/env python3
"""A/B of the stage-1 -> stage-2 block tail (kernels/bottleneck.hip, TP 64 / CN 128) with the
256-channel output stored whole vs decimated (only the even-(h, w) pixels the stride-2
projection reads), ResNet-50 shapes at micro-batch 256.  HIP-event timing, interleaved."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from flink_tensorflow_amd.ops import kernels as K  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    N, H, W = 256, 56, 56
    g = torch.Generator(device=dev).manual_seed(0)
    x2 = torch.randn(N, H, W, 64, device=dev, generator=g).bfloat16()
    res = torch.randn(N, H, W, 256, device=dev, generator=g).bfloat16()
    w3 = (torch.randn(256, 64, device=dev, generator=g) / 8).bfloat16()
    w1 = (torch.randn(128, 256, device=dev, generator=g) / 16).bfloat16()
    b3 = torch.randn(256, device=dev, generator=g)
    b1 = torch.randn(128, device=dev, generator=g)
    y3 = torch.empty(N, H, W, 256, device=dev, dtype=torch.bfloat16)
    y3d = torch.empty(N, H // 2, W // 2, 256, device=dev, dtype=torch.bfloat16)
    y1 = torch.empty(N, H, W, 128, device=dev, dtype=torch.bfloat16)
    runs = {"full": lambda: K.bottleneck_tail(x2, res, w3, b3, w1, b1, y3=y3, y1=y1),
            "decimated": lambda: K.bottleneck_tail(x2, res, w3, b3, w1, b1, y3=y3d, y1=y1, y3_decimated=True)}
    for f in runs.values():
        f()
    torch.cuda.synchronize()
    times = {k: [] for k in runs}
    for _ in range(10):
        for k, f in runs.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(5):
                f()
            b.record()
            b.synchronize()
            times[k].append(a.elapsed_time(b) * 1000 / 5)
    out = {k: round(sorted(v)[len(v) // 2], 1) for k, v in times.items()}
    print(json.dumps({"tail_us_median": out}))


if __name__ == "__main__":
    main()
