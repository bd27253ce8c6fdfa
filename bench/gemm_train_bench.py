"""Times the Wide&Deep training GEMMs (batch 4096, MLP 1024-512-256 over an 896-wide input)
on ``gemm_train`` (per layout, cost-model split-K) against torch.mm (hipBLASLt), HIP
events around 20 back-to-back launches.  One JSON line per shape."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from flink_tensorflow_amd.ops import kernels as K  # noqa: E402

CASES = [  # name, M, N, K, x_t, w_t, fp32 out
    ("fwd0", 4096, 1024, 896, False, False, False), ("fwd1", 4096, 512, 1024, False, False, False),
    ("fwd2", 4096, 256, 512, False, False, False),
    ("dX2", 4096, 512, 256, False, True, False), ("dX1", 4096, 1024, 512, False, True, False),
    ("dX0", 4096, 832, 1024, False, True, False),
    ("dW2", 256, 512, 4096, True, True, True), ("dW1", 512, 1024, 4096, True, True, True),
    ("dW0", 1024, 896, 4096, True, True, True),
]


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


def main():
    dev = torch.device("cuda", 0)
    forced = os.environ.get("SPLITS")
    for name, M, N, Kd, xt, wt, f32 in CASES:
        x = torch.randn((Kd, M) if xt else (M, Kd), device=dev).to(torch.bfloat16)
        w = torch.randn((Kd, N) if wt else (N, Kd), device=dev).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
        s = int(forced) if forced else K.gemm_train_splits(M, N, Kd)
        ws = torch.empty(max(1, s) * M * N, device=dev)
        us = timeit(lambda: K.gemm_train(x, w, x_t=xt, w_t=wt, out=out, splits=s, ws=ws))
        X = x.t() if xt else x
        W = w if wt else w.t()
        if f32:
            lib = timeit(lambda: torch.mm(X, W, out_dtype=torch.float32, out=out))
        else:
            lib = timeit(lambda: torch.mm(X, W, out=out))
        tf = 2.0 * M * N * Kd / us / 1e6
        print(json.dumps({"case": name, "M": M, "N": N, "K": Kd, "splits": s, "gemm_train_us": round(us, 2),
                          "tflops": round(tf, 1), "torch_mm_us": round(lib, 2)}), flush=True)


if __name__ == "__main__":
    main()
