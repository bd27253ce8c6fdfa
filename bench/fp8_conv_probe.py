"""fp8 conv implementations on single Inception-v3 layer shapes (B=256): the direct LDS conv
(``dconv``, 4 / 8 waves), the 4-wave LDS-DMA implicit GEMM (``lite`` = cfg 8, channel tile
chosen by the kernel) and the register-staged igemm configs 0/1/2.
Prints one JSON line per (layer, impl) with µs per launch.

    python bench/fp8_conv_probe.py --layers 2a,2b,3b --impls dconv4,dconv8,lite,cfg0
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from flink_tensorflow_amd.ops import fp8 as Q  # noqa: E402
from flink_tensorflow_amd.ops import kernels as K  # noqa: E402

LAYERS = {  # name: (H, W, Cin, Cout, (kh, kw), stride, pads t/b/l/r)
    "2a": (149, 149, 32, 32, (3, 3), 1, (0, 0, 0, 0)),
    "2b": (147, 147, 32, 64, (3, 3), 1, (1, 1, 1, 1)),
    "3b": (73, 73, 64, 80, (1, 1), 1, (0, 0, 0, 0)),
    "4a": (73, 73, 80, 192, (3, 3), 1, (0, 0, 0, 0)),
    "5b_b2": (35, 35, 64, 96, (3, 3), 1, (1, 1, 1, 1)),
    "5b_b1": (35, 35, 48, 64, (5, 5), 1, (2, 2, 2, 2)),
    "6b_17": (17, 17, 128, 192, (1, 7), 1, (0, 0, 3, 3)),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", default=",".join(LAYERS))
    ap.add_argument("--impls", default="dconv4,dconv8,lite,cfg0,cfg2")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    dev = torch.device("cuda")
    B = a.batch
    for name in a.layers.split(","):
        H, W, Cin, Cout, (kh, kw), s, pads = LAYERS[name]
        torch.manual_seed(0)
        x = torch.randn(B, H, W, Cin, device=dev).relu()
        sx = Q.scale_for(float(x.max()))
        xq = Q.quantize(x.to(torch.bfloat16), sx)
        del x
        wq, ws = Q.quantize_weight(torch.randn(Cout, kh, kw, Cin) / (kh * kw * Cin) ** 0.5)
        wq, ws = wq.to(dev), ws.to(dev)
        b = torch.zeros(Cout, device=dev)
        cs = (ws * sx).contiguous()
        Ho, Wo = K.conv_out_hw(H, W, kh, kw, s, s, pads[0], pads[2], 1, 1, pads[1], pads[3])
        y = torch.empty((B, Ho, Wo, Cout), dtype=torch.uint8, device=dev)
        flops = 2.0 * B * Ho * Wo * Cout * kh * kw * Cin
        for impl in a.impls.split(","):
            if impl.startswith("dconv"):
                if not K.dconv_eligible(Cin, kh, kw, (s, s), (1, 1), 1):
                    continue
                bn = 64 if Cout >= 64 else 32
                arr = K.dconv_weights(wq, Cout, 1, bn)
                waves = int(impl[5:])

                def fn(arr=arr, bn=bn, waves=waves):
                    K.conv2d_direct(xq, arr, (kh, kw), Cout, b, (s, s), pads, "relu", out=y, bn=bn, chan_scale=cs,
                                    out_scale=0.05, waves=waves)
            else:
                cfg = 8 if impl == "lite" else int(impl[3:])

                def fn(cfg=cfg):
                    Q.conv2d_nhwc_fp8(xq, sx, wq, (kh, kw), ws, b, (s, s), pads, (1, 1), "relu", out_scale=0.05,
                                      out=y, cfg=cfg, chan_scale=cs)
            try:
                fn()
                torch.cuda.synchronize()
            except (ValueError, RuntimeError) as e:
                print(json.dumps({"layer": name, "impl": impl, "error": str(e)[:120]}), flush=True)
                continue
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
