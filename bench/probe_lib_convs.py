"""Same-GPU yardstick for the ResNet-50 conv layers (B=256): the hand-written implicit
GEMM (ops.kernels.conv2d_nhwc, auto tile) vs hipBLASLt (1x1 stride-1 layers as a plain
GEMM with fused bias+ReLU, torch._addmm_activation) and MIOpen (torch conv2d,
channels_last bf16, conv only).  Decides where a library call beats the HIP kernel."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/bench/", 1)[0])
from flink_tensorflow_amd.ops import kernels as K  # noqa: E402

B = 256
LAYERS = [  # name, H, W, Cin, Cout, k, stride, pad
    ("s1_c1", 56, 56, 256, 64, 1, 1, 0), ("s2_c1", 56, 56, 256, 128, 1, 1, 0),
    ("s2_c1b", 28, 28, 512, 128, 1, 1, 0), ("s3_c1", 28, 28, 512, 256, 1, 1, 0),
    ("s3_c1b", 14, 14, 1024, 256, 1, 1, 0), ("s4_c1", 14, 14, 1024, 512, 1, 1, 0),
    ("s4_c1b", 7, 7, 2048, 512, 1, 1, 0),
    ("s2_c2", 28, 28, 128, 128, 3, 1, 1), ("s3_c2", 14, 14, 256, 256, 3, 1, 1), ("s4_c2", 7, 7, 512, 512, 3, 1, 1),
]


def timeit(f, n=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            f()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / n * 1e3)
    return round(best, 1)


def main():
    dev = torch.device("cuda", 0)
    for name, H, W, Cin, Cout, k, s, p in LAYERS:
        x = torch.randn(B, H, W, Cin, device=dev).to(torch.bfloat16)
        w = (torch.randn(Cout, k, k, Cin, device=dev) / (k * k * Cin) ** 0.5).to(torch.bfloat16)
        b = torch.randn(Cout, device=dev)
        y = torch.empty(B, H, W, Cout, device=dev, dtype=torch.bfloat16)
        flops = 2.0 * B * H * W * Cout * k * k * Cin
        r = {"layer": name, "ours": timeit(lambda: K.conv2d_nhwc(x, w, b, None, (s, s), (p, p, p, p), (1, 1), "relu",
                                                                 out=y))}
        if k == 1:
            x2, w2, bb = x.reshape(-1, Cin), w.reshape(Cout, Cin), b.to(torch.bfloat16)
            r["hipblaslt"] = timeit(lambda: torch._addmm_activation(bb, x2, w2.t()))
        xc = x.permute(0, 3, 1, 2)  # NCHW view of NHWC memory = channels_last
        wc = w.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        r["miopen"] = timeit(lambda: torch.nn.functional.conv2d(xc, wc, None, s, p))
        r["ours_tflops"] = round(flops / r["ours"] / 1e6, 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
