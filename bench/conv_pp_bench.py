"""conv_pp vs the round-1 implicit-GEMM conv (igemm_bf16 via conv2d_nhwc) on the ResNet-50
v1.5 layer shapes at B=256 / 224: per-layer µs and TFLOP/s, both tile shapes and the
split-K choice of the cost model.  One JSON line per layer."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from flink_tensorflow_amd.ops import kernels as K  # noqa: E402

B = int(os.environ.get("B", 256))
# (name, H, W, Cin, Cout, k, stride, residual)
LAYERS = [
    ("s2_3x3s2", 56, 56, 128, 128, 3, 2, False),
    ("s2_3x3", 28, 28, 128, 128, 3, 1, False),
    ("s2_reduce", 28, 28, 512, 128, 1, 1, False),
    ("s2_expand_res", 28, 28, 128, 512, 1, 1, True),
    ("s1to2_reduce", 56, 56, 256, 128, 1, 1, False),
    ("s3_3x3s2", 28, 28, 256, 256, 3, 2, False),
    ("s3_3x3", 14, 14, 256, 256, 3, 1, False),
    ("s3_expand_res", 14, 14, 256, 1024, 1, 1, True),
    ("s3_reduce", 14, 14, 1024, 256, 1, 1, False),
    ("s4_3x3s2", 14, 14, 512, 512, 3, 2, False),
    ("s4_3x3", 7, 7, 512, 512, 3, 1, False),
    ("s4_expand_res", 7, 7, 512, 2048, 1, 1, True),
    ("s4_reduce", 7, 7, 2048, 512, 1, 1, False),
    ("s2_proj_s2", 56, 56, 256, 512, 1, 2, False),
]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    dev = torch.device("cuda")
    for name, H, W, Cin, Cout, k, s, res in LAYERS:
        pad = (k // 2) if s == 1 else (0 if k == 1 else 1)
        OH, OW = (H + 2 * pad - k) // s + 1, (W + 2 * pad - k) // s + 1
        if k == 3 and s == 2:  # TF SAME for even sizes: pad bottom/right only
            pt = 0
            OH, OW = H // 2, W // 2
        else:
            pt = pad
        x = torch.randn(B, H, W, Cin, device=dev).to(torch.bfloat16)
        w = (torch.randn(Cout, k, k, Cin, device=dev) / (k * k * Cin) ** 0.5).to(torch.bfloat16)
        b = torch.randn(Cout, device=dev)
        r = torch.randn(B, OH, OW, Cout, device=dev).to(torch.bfloat16) if res else None
        out = torch.empty(B, OH, OW, Cout, dtype=torch.bfloat16, device=dev)
        flops = 2.0 * B * OH * OW * Cout * k * k * Cin
        ph_b = max(0, (OH - 1) * s + k - H - pt)
        t_old = timeit(lambda: K.conv2d_nhwc(x, w, b, r, (s, s), (pt, ph_b, pt, ph_b), (1, 1), "relu", out=out))
        ref = out.float().clone()
        row = {"layer": name, "M": B * OH * OW, "N": Cout, "K": k * k * Cin, "igemm_us": round(t_old, 1),
               "igemm_tflops": round(flops / t_old / 1e6, 1)}
        w2 = w.reshape(Cout, -1)
        for tile in (0, 1):
            cp = K.ConvPP([((B, H, W, Cin), (k, k), (s, s), (pt, pt), (1, 1))], Cout, (OH, OW), dev, tile=tile)
            t = timeit(lambda: cp([x], w2, b, r, "relu", out=out))
            err = (out.float() - ref).abs().max().item() / max(1e-6, ref.abs().max().item())
            row[f"pp_t{tile}_us"] = round(t, 1)
            row[f"pp_t{tile}_tflops"] = round(flops / t / 1e6, 1)
            row[f"pp_t{tile}_splits"] = cp.splits
            row[f"pp_t{tile}_relerr"] = round(err, 4)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
