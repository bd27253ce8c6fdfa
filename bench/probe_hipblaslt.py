"""Same-GPU yardstick: torch (hipBLASLt) bf16 GEMM rates on the BERT-base projection
shapes, to decide where a library GEMM beats the hand-written MFMA kernels."""
import json

import torch

dev = torch.device("cuda", 0)
for name, M, N, K, gelu in [("qkv", 32768, 2304, 768, False), ("out", 32768, 768, 768, False),
                            ("ffn1", 32768, 3072, 768, True), ("ffn2", 32768, 768, 3072, False)]:
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = torch.randn(N, K, device=dev).to(torch.bfloat16)
    b = torch.randn(N, device=dev).to(torch.bfloat16)
    fns = {"linear": lambda: torch.nn.functional.linear(x, w, b),
           "mm": lambda: x @ w.t()}
    if gelu:
        fns["addmm_gelu"] = lambda: torch._addmm_activation(b, x, w.t(), use_gelu=True)
    res = {}
    for k, f in fns.items():
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                f()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / 10 * 1e3)
        us = sorted(ts)[2]
        res[k] = {"us": round(us, 1), "tflops": round(2.0 * M * N * K / us / 1e6, 1)}
    print(json.dumps({"gemm": name, **res}), flush=True)
