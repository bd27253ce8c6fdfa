"""Direct conv (kernels/dconv.hip, BN 32/64, 4- or 8-wave tiles) vs the implicit-GEMM auto path on the narrow
layers of ResNet-50 and Inception-v3 at B=256 (random data, interleaved rounds)."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/bench/", 1)[0])
from flink_tensorflow_amd.ops import fp8 as Q  # noqa: E402
from flink_tensorflow_amd.ops import kernels as K  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
# name, es, H, W, Cin, Cout, (kh, kw), stride, pad
LAYERS = [
    ("rn_stem_s2d", 2, 112, 112, 16, 64, (4, 4), 1, (1, 2, 1, 2)),
    ("rn_s1_c2", 2, 56, 56, 64, 64, (3, 3), 1, (1, 1, 1, 1)),
    ("inc_stem", 2, 299, 299, 8, 32, (3, 3), 2, (0, 0, 0, 0)),
    ("inc_2a", 1, 149, 149, 32, 32, (3, 3), 1, (0, 0, 0, 0)),
    ("inc_2b", 1, 147, 147, 32, 64, (3, 3), 1, (1, 1, 1, 1)),
    ("inc_5b_3x3a", 1, 35, 35, 64, 96, (3, 3), 1, (1, 1, 1, 1)),
    ("inc_5b_3x3b", 1, 35, 35, 96, 96, (3, 3), 1, (1, 1, 1, 1)),
    ("inc_6b_1x7", 1, 17, 17, 128, 128, (1, 7), 1, (0, 0, 3, 3)),
]


def timeit(fn, reps=10):
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / reps * 1e3)
    return sorted(ts)[2]


def main():
    dev = torch.device("cuda", 0)
    for name, es, H, W, Cin, Cout, (kh, kw), s, pad in LAYERS:
        Ho, Wo = K.conv_out_hw(H, W, kh, kw, s, s, pad[0], pad[2], 1, 1, pad[1], pad[3])
        b = torch.zeros(Cout, device=dev)
        res = {}
        if es == 2:
            x = torch.randn(B, H, W, Cin, device=dev).to(torch.bfloat16)
            w = (torch.randn(Cout, kh, kw, Cin, device=dev) / 10).to(torch.bfloat16)
            y = torch.empty(B, Ho, Wo, Cout, device=dev, dtype=torch.bfloat16)
            fns = {"auto": lambda: K.conv2d_nhwc(x, w, b, None, (s, s), pad, (1, 1), "relu", out=y)}
            for bn in (32, 64):
                arr = K.dconv_bf16_weight_bytes(w.float(), bn)
                for wv in (4, 8):
                    fns[f"d{bn}w{wv}"] = (lambda arr=arr, bn=bn, wv=wv: K.conv2d_direct(
                        x, arr, (kh, kw), Cout, b, (s, s), pad, "relu", out=y, bn=bn, waves=wv))
        else:
            x = torch.randint(0, 120, (B, H, W, Cin), dtype=torch.uint8, device=dev)
            wq = torch.randint(0, 120, (Cout, kh * kw * Cin), dtype=torch.uint8, device=dev)
            ws = torch.full((Cout,), 1e-3, device=dev)
            cs = ws * 0.01
            y = torch.empty(B, Ho, Wo, Cout, device=dev, dtype=torch.uint8)
            fns = {"auto": lambda: Q.conv2d_nhwc_fp8(x, 0.01, wq, (kh, kw), ws, b, (s, s), pad, act="relu",
                                                     out_scale=0.05, out=y, chan_scale=cs)}
            for bn in (32, 64):
                arr = K.dconv_weights(wq, Cout, 1, bn)
                for wv in (4, 8):
                    fns[f"d{bn}w{wv}"] = (lambda arr=arr, bn=bn, wv=wv: K.conv2d_direct(
                        x, arr, (kh, kw), Cout, b, (s, s), pad, "relu", out=y, bn=bn, chan_scale=cs, out_scale=0.05,
                        waves=wv))
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        for k, f in fns.items():
            res[k] = round(timeit(f), 1)
        flops = 2.0 * B * Ho * Wo * Cout * kh * kw * Cin
        best = min(res, key=res.get)
        print(json.dumps({"layer": name, "us": res, "best": best, "best_tflops": round(flops / res[best] / 1e6, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
