"""One ResNet-50 layer shape per process for counter runs (``rocprofv3 --pmc``): the
incumbent implicit-GEMM conv (``igemm``) and the ping-pong conv (``pp``) on the stage 2/3/4
3x3 layers at B=256, --reps launches each, plus a µs line per kernel on stdout.

    python bench/conv_layer_probe.py --layers s3_3x3 --impls igemm,lite:2,lite:4,lite:5,lite:6 --reps 10

(``lite:4`` / ``5`` / ``6``: tile 2 without MFMAs / without DMA after the first K-tile /
MFMAs only — a decomposition of where its time goes; outputs meaningless.)
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from flink_tensorflow_amd.ops import kernels as K  # noqa: E402

LAYERS = {  # name: (H, W, Cin, Cout, k, stride)
    "s2_3x3": (28, 28, 128, 128, 3, 1),
    "s3_3x3": (14, 14, 256, 256, 3, 1),
    "s4_3x3": (7, 7, 512, 512, 3, 1),
    "s3_3x3s2": (28, 28, 256, 256, 3, 2),
    "s3_reduce": (14, 14, 1024, 256, 1, 1),
    "s2_reduce": (28, 28, 512, 128, 1, 1),
    "s4_expand": (7, 7, 512, 2048, 1, 1, True),  # + identity residual (units 2 / 3)
    "s1_reduce": (56, 56, 64, 64, 1, 1),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", default="s2_3x3,s3_3x3,s4_3x3")
    ap.add_argument("--impls", default="igemm,lite")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    B = a.batch
    for name in a.layers.split(","):
        H, W, Cin, Cout, k, s, *opt = LAYERS[name]
        pad = k // 2 if s == 1 else (0 if k == 1 else 1)
        OH, OW = (H + 2 * pad - k) // s + 1, (W + 2 * pad - k) // s + 1
        x = torch.randn((B, H, W, Cin), device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn((Cout, k, k, Cin), device=dev, generator=g) * 0.05).to(torch.bfloat16)
        b = torch.zeros(Cout, device=dev)
        y = torch.empty((B, OH, OW, Cout), dtype=torch.bfloat16, device=dev)
        res = torch.randn((B, OH, OW, Cout), device=dev, generator=g).to(torch.bfloat16) if opt and opt[0] else None
        flops = 2.0 * B * OH * OW * Cout * k * k * Cin
        for impl in a.impls.split(","):
            if impl == "igemm":
                def fn():
                    K.conv2d_nhwc(x, w, b, res, (s, s), (pad, pad, pad, pad), (1, 1), K.ACT_RELU, out=y)
            else:  # lite[:tile]: the 128x128 LDS-DMA tile (2; 4..6 diagnostics)
                tile = int(impl.split(":")[1]) if ":" in impl else None
                cp = K.ConvPP([((B, H, W, Cin), (k, k), (s, s), (pad, pad), (1, 1))], Cout, (OH, OW), dev, tile=tile)
                w2 = w.reshape(Cout, -1)

                def fn(cp=cp, w2=w2):
                    cp([x], w2, b, res, K.ACT_RELU, out=y)
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.reps
            print(json.dumps({"layer": name, "impl": impl, "us": round(us, 1), "tflops": round(flops / us / 1e6, 1)}),
                  flush=True)


if __name__ == "__main__":
    main()
