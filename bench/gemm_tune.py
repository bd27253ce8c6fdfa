"""bf16 GEMM tile configurations on the BERT-base / Wide&Deep shapes (random data,
interleaved rounds): register-staged igemm tiles 0..4 vs the pipelined LDS-DMA kernel 16/17."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/bench/", 1)[0])
from flink_tensorflow_amd import _ext  # noqa: E402
from flink_tensorflow_amd.ops import kernels as K  # noqa: E402

SHAPES = [  # name, M, N, K, act, residual
    ("bert_qkv", 32768, 2304, 768, "none", False),
    ("bert_out", 32768, 768, 768, "none", True),
    ("bert_ffn1", 32768, 3072, 768, "gelu", False),
    ("bert_ffn2", 32768, 768, 3072, "none", True),
    ("wd_l1", 4096, 1024, 848, "relu", False),
    ("wd_l2", 4096, 512, 1024, "relu", False),
]


def main():
    dev = torch.device("cuda", 0)
    ncfg = _ext.hip().igemm_num_configs
    tot = {}
    for name, M, N, Kd, act, res in SHAPES:
        x = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, Kd, device=dev) / Kd ** 0.5).to(torch.bfloat16)
        b = torch.randn(N, device=dev)
        r = torch.randn(M, N, device=dev).to(torch.bfloat16) if res else None
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        cfgs = list(range(ncfg)) + list(K.V2_CONFIGS) + [-1]
        med = {}
        for c in cfgs:
            K.gemm(x, w, b, r, act, out=y, cfg=c)
        torch.cuda.synchronize()
        times = {c: [] for c in cfgs}
        for _ in range(5):
            for c in cfgs:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    K.gemm(x, w, b, r, act, out=y, cfg=c)
                e1.record()
                e1.synchronize()
                times[c].append(e0.elapsed_time(e1) / 10 * 1e3)
        med = {c: sorted(v)[2] for c, v in times.items()}
        best = min([c for c in cfgs if c >= 0], key=med.get)
        fl = 2.0 * M * N * Kd
        print(json.dumps({"gemm": name, "us": {str(c): round(v, 1) for c, v in med.items()}, "best": best,
                          "best_tflops": round(fl / med[best] / 1e6, 1), "auto_tflops": round(fl / med[-1] / 1e6, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
