#!/usr/bin/env python3
"""Persistent identity-residual expand conv (kernels/pw_res.hip) vs the tiled implicit-GEMM
kernel (igemm_bf16.hip) on ResNet-50's stage-2/3 expand shapes at micro-batch 256.
HIP-event timing, interleaved; prints achieved TB/s of the minimum traffic."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from flink_tensorflow_amd.ops import kernels as K  # noqa: E402


def time_us(f, reps=5, rounds=9):
    ts = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            f()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1000 / reps)
    return sorted(ts)[len(ts) // 2]


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    for name, (N, H, W, Cin, Cout, tp) in {"s2_expand": (256, 28, 28, 128, 512, 0),
                                           "s3_expand_tp128": (256, 14, 14, 256, 1024, 128),
                                           "s3_expand": (256, 14, 14, 256, 1024, 0)}.items():
        x = torch.randn(N, H, W, Cin, device=dev, generator=g).bfloat16()
        w = (torch.randn(Cout, Cin, device=dev, generator=g) / Cin ** 0.5).bfloat16()
        b = torch.randn(Cout, device=dev, generator=g)
        r = torch.randn(N, H, W, Cout, device=dev, generator=g).bfloat16()
        o1, o2 = torch.empty_like(r), torch.empty_like(r)
        f_ig = lambda: K.conv2d_nhwc(x, w.reshape(Cout, 1, 1, Cin), b, r, act="relu", out=o1)  # noqa: E731
        f_pw = lambda: K.pw_res(x, w, b, r, out=o2, tp=tp)  # noqa: E731
        f_ig(), f_pw()
        torch.cuda.synchronize()
        err = ((o1.float() - o2.float()).abs().max() / o1.float().abs().max()).item()
        t_ig, t_pw = time_us(f_ig), time_us(f_pw)
        t_ig2, t_pw2 = time_us(f_ig), time_us(f_pw)
        nbytes = (x.numel() + 2 * r.numel()) * 2 + w.numel() * 2
        print(json.dumps({"layer": name, "igemm_us": [round(t_ig, 1), round(t_ig2, 1)],
                          "pw_res_us": [round(t_pw, 1), round(t_pw2, 1)],
                          "pw_res_TBps": round(nbytes / min(t_pw, t_pw2) / 1e6, 2), "max_rel_diff": round(err, 4)}))



if __name__ == "__main__":
    main()
