#!/usr/bin/env python3
"""Inception-v3's MaxPool_3a -> Conv2d_3b_1x1 (147x147x64 -> 73x73x64 -> 73x73x80, e4m3)
at micro-batch B: the fused kernel (``kernels/poolconv.hip``) against the two kernels it
replaces (``pool2d_nhwc_fp8`` + the fp8 1x1 ``conv_lite_fp8``).  Prints µs per launch,
the fused kernel's effective bandwidth (pre-pool read + output write) and the max byte
difference of the two outputs."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flink_tensorflow_amd.ops import fp8 as Q  # noqa: E402


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
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--cout", type=int, default=80)
    a = ap.parse_args()
    dev = torch.device("cuda")
    B, H, W, C, Co = a.batch, 147, 147, 64, a.cout
    g = torch.Generator().manual_seed(0)
    x = Q.to_fp8_bytes(torch.randn(B, H, W, C, generator=g).relu() * 3).to(dev)
    wq, ws = Q.quantize_weight(torch.randn(Co, C, generator=g) / 8)
    wq, ws = wq.to(dev), ws.to(dev)
    xs, os_ = 0.02, 0.05
    cs = (ws * xs).float().contiguous()
    b = (torch.randn(Co, generator=g) * 0.1).to(dev)
    Hp, Wp = (H - 3) // 2 + 1, (W - 3) // 2 + 1
    y_f = torch.empty(B, Hp, Wp, Co, dtype=torch.uint8, device=dev)
    y_u = torch.empty_like(y_f)
    pooled = torch.empty(B, Hp, Wp, C, dtype=torch.uint8, device=dev)

    def fused():
        Q.pool_conv1x1_fp8(x, wq, cs, b, "relu", out_scale=os_, out=y_f)

    def unfused():
        Q.pool2d_nhwc_fp8(x, (3, 3), (2, 2), (0, 0, 0, 0), "max", out=pooled)
        Q.conv2d_nhwc_fp8(pooled, xs, wq.reshape(Co, C), (1, 1), ws, b, act="relu", out=y_u, out_scale=os_,
                          chan_scale=cs, cfg=11)

    tf, tu = timeit(fused, a.reps), timeit(unfused, a.reps)
    nbytes = x.numel() + y_f.numel()
    diff = (Q.from_fp8_bytes(y_f.cpu()) - Q.from_fp8_bytes(y_u.cpu())).abs()
    ref = Q.from_fp8_bytes(y_u.cpu()).abs()
    print(json.dumps({"batch": B, "cout": Co, "fused_us": round(tf, 1), "unfused_us": round(tu, 1),
                      "speedup": round(tu / tf, 3), "fused_TBps": round(nbytes / tf / 1e6, 2),
                      "max_rel_diff": round(float((diff / (ref + 1e-2)).max()), 4)}), flush=True)


if __name__ == "__main__":
    main()
