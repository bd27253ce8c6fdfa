"""Where a conv_lite K-tile's time goes: per-phase clocks of wave 0 of the first 64
workgroups (kernels/conv_pp.hip ``STAMP``: s_memtime before / after the vmcnt wait, after
the barrier, after the next tile's DMA issue, after the MFMA issue), on ResNet-50 3x3
layer shapes at B=256.  Prints, per layer, the median cycles of each phase over K-tiles
2..nk-2 of all sampled workgroups, and the spread across workgroups.

    python bench/conv_stamp_probe.py --layers s2_3x3,s3_3x3
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from flink_tensorflow_amd.ops import kernels as K  # noqa: E402

LAYERS = {  # name: (H, W, Cin, Cout, k, stride)
    "s2_3x3": (28, 28, 128, 128, 3, 1),
    "s3_3x3": (14, 14, 256, 256, 3, 1),
    "s4_3x3": (7, 7, 512, 512, 3, 1),
}
# fp8 (conv_lite_fp8, fp8 out, ReLU): Inception-v3 shapes — (H, W, Cin, Cout, (kh, kw), pads t/b/l/r)
FP8_LAYERS = {
    "i35_3x3_96": (35, 35, 96, 96, (3, 3), (1, 1, 1, 1)),
    "i17_7x1_192": (17, 17, 192, 192, (7, 1), (3, 3, 0, 0)),
    "i17_1x7_160": (17, 17, 160, 160, (1, 7), (0, 0, 3, 3)),
    "i8_3x3_384": (8, 8, 448, 384, (3, 3), (1, 1, 1, 1)),
}


def _summary(name, t, nk):
    body = t[:, 2:-1] if t.shape[1] > 4 else t
    ph = {
        "vmcnt_wait": np.median(body[..., 1] - body[..., 0]),
        "barrier": np.median(body[..., 2] - body[..., 1]),
        "dma_issue": np.median(body[..., 3] - body[..., 2]),
        "mfma_issue": np.median(body[..., 4] - body[..., 3]),
        "loop_tail": np.median(np.diff(body[..., 0], axis=1)) if body.shape[1] > 1 else 0,
    }
    per_wg = (t[:, -1, 4] - t[:, 0, 0]).astype(np.float64)
    return {"layer": name, "nk": nk, **{k2: float(v) for k2, v in ph.items()},
            "wg_cycles_median": float(np.median(per_wg)), "wg_cycles_p10": float(np.percentile(per_wg, 10)),
            "wg_cycles_p90": float(np.percentile(per_wg, 90))}


def fp8_main(layers, B):
    from flink_tensorflow_amd.ops import fp8 as Q

    dev = torch.device("cuda")
    stamp = torch.zeros(64 * 64 * 5, dtype=torch.int64, device=dev)
    for name in layers:
        H, W, Cin, Cout, (kh, kw), pads = FP8_LAYERS[name]
        x = torch.randint(0, 120, (B, H, W, Cin), dtype=torch.uint8, device=dev)
        wq = torch.randint(0, 120, (Cout, kh * kw * Cin), dtype=torch.uint8, device=dev)
        ws = torch.full((Cout,), 1e-3, device=dev)
        b = torch.zeros(Cout, device=dev)

        def run():
            Q.conv2d_nhwc_fp8(x, 0.01, wq, (kh, kw), ws, b, (1, 1), pads, act="relu", out_scale=0.05, cfg=8)

        for _ in range(3):
            run()
        torch.cuda.synchronize()
        K._hip().conv_lite_fp8_stamp(stamp.data_ptr())
        try:
            run()
            torch.cuda.synchronize()
        finally:
            K._hip().conv_lite_fp8_stamp(0)
        nk = -(-kh * kw * Cin // 128)
        t = stamp.view(64, 64, 5).cpu().numpy()[:, : min(nk, 64)].astype(np.int64)
        print(json.dumps(_summary(name, t, nk)), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", default="s2_3x3,s3_3x3,s4_3x3")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--fp8", action="store_true", help="conv_lite_fp8 on Inception-v3 layer shapes")
    a = ap.parse_args()
    if a.fp8:
        fp8_main(a.layers.split(",") if a.layers != ap.get_default("layers") else list(FP8_LAYERS), a.batch)
        return
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    stamp = torch.zeros(64 * 64 * 5, dtype=torch.int64, device=dev)
    for name in a.layers.split(","):
        H, W, Cin, Cout, k, s = LAYERS[name]
        pad = k // 2
        B = a.batch
        x = torch.randn((B, H, W, Cin), device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn((Cout, k, k, Cin), device=dev, generator=g) * 0.05).to(torch.bfloat16).reshape(Cout, -1)
        b = torch.zeros(Cout, device=dev)
        y = torch.empty((B, H, W, Cout), dtype=torch.bfloat16, device=dev)
        cp = K.ConvPP([((B, H, W, Cin), (k, k), (s, s), (pad, pad), (1, 1))], Cout, (H, W), dev, tile=2)
        for _ in range(3):
            cp([x], w, b, None, K.ACT_RELU, out=y)  # warm
        torch.cuda.synchronize()
        K._hip().conv_lite_stamp(stamp.data_ptr())
        try:
            cp([x], w, b, None, K.ACT_RELU, out=y)
            torch.cuda.synchronize()
        finally:
            K._hip().conv_lite_stamp(0)
        nk = Cin * k * k // 64
        t = stamp.view(64, 64, 5).cpu().numpy()[:, : min(nk, 64)].astype(np.int64)
        body = t[:, 2:-1] if t.shape[1] > 4 else t
        ph = {
            "vmcnt_wait": np.median(body[..., 1] - body[..., 0]),
            "barrier": np.median(body[..., 2] - body[..., 1]),
            "dma_issue": np.median(body[..., 3] - body[..., 2]),
            "mfma_issue": np.median(body[..., 4] - body[..., 3]),
            "loop_tail": np.median(np.diff(body[..., 0], axis=1)) if body.shape[1] > 1 else 0,
        }
        per_wg = (t[:, -1, 4] - t[:, 0, 0]).astype(np.float64)
        out = {"layer": name, "nk": nk, **{k2: float(v) for k2, v in ph.items()},
               "wg_cycles_median": float(np.median(per_wg)), "wg_cycles_p10": float(np.percentile(per_wg, 10)),
               "wg_cycles_p90": float(np.percentile(per_wg, 90))}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
