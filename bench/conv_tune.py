"""Times every implicit-GEMM tile configuration on the ResNet-50 layer shapes (B=256).

Interleaved rounds in one process (guide §5.4 rule 24); random bf16 data (rule 25).
Prints per-layer the best config vs the auto heuristic.
"""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/bench/", 1)[0])
from flink_tensorflow_amd import _ext  # noqa: E402
from flink_tensorflow_amd.ops import kernels as K  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
# (name, H, W, Cin, Cout, k, stride, pad(t,b,l,r), residual)
LAYERS = [
    ("stem_s2d", 112, 112, 16, 64, 4, 1, (1, 2, 1, 2), False),
    ("s1_c1_first", 56, 56, 64, 64, 1, 1, (0, 0, 0, 0), False),
    ("s1_c1", 56, 56, 256, 64, 1, 1, (0, 0, 0, 0), False),
    ("s1_c2", 56, 56, 64, 64, 3, 1, (1, 1, 1, 1), False),
    ("s1_c3_res", 56, 56, 64, 256, 1, 1, (0, 0, 0, 0), True),
    ("s1_sc", 56, 56, 64, 256, 1, 1, (0, 0, 0, 0), False),
    ("s2_c1", 56, 56, 256, 128, 1, 1, (0, 0, 0, 0), False),
    ("s2_c2_s2", 56, 56, 128, 128, 3, 2, (0, 1, 0, 1), False),
    ("s2_sc_s2", 56, 56, 256, 512, 1, 2, (0, 0, 0, 0), False),
    ("s2_c1b", 28, 28, 512, 128, 1, 1, (0, 0, 0, 0), False),
    ("s2_c2", 28, 28, 128, 128, 3, 1, (1, 1, 1, 1), False),
    ("s2_c3_res", 28, 28, 128, 512, 1, 1, (0, 0, 0, 0), True),
    ("s3_c2", 14, 14, 256, 256, 3, 1, (1, 1, 1, 1), False),
    ("s3_c3_res", 14, 14, 256, 1024, 1, 1, (0, 0, 0, 0), True),
    ("s3_c1b", 14, 14, 1024, 256, 1, 1, (0, 0, 0, 0), False),
    ("s4_c2", 7, 7, 512, 512, 3, 1, (1, 1, 1, 1), False),
    ("s4_c3_res", 7, 7, 512, 2048, 1, 1, (0, 0, 0, 0), True),
    ("s4_c1b", 7, 7, 2048, 512, 1, 1, (0, 0, 0, 0), False),
]


def main():
    dev = torch.device("cuda", 0)
    ncfg = _ext.hip().igemm_num_configs
    out = []
    for name, H, W, Cin, Cout, k, s, pad, res in LAYERS:
        x = torch.randn(B, H, W, Cin, device=dev).to(torch.bfloat16)
        w = (torch.randn(Cout, k, k, Cin, device=dev) / (k * k * Cin) ** 0.5).to(torch.bfloat16)
        b = torch.randn(Cout, device=dev)
        Ho, Wo = K.conv_out_hw(H, W, k, k, s, s, pad[0], pad[2], 1, 1, pad[1], pad[3])
        r = torch.randn(B, Ho, Wo, Cout, device=dev).to(torch.bfloat16) if res else None
        y = torch.empty(B, Ho, Wo, Cout, device=dev, dtype=torch.bfloat16)
        flops = 2.0 * B * Ho * Wo * Cout * k * k * Cin
        nbytes = x.numel() * 2 + y.numel() * 2 * (2 if res else 1) + w.numel() * 2
        cfgs = list(range(ncfg)) + [-1]
        times = {c: [] for c in cfgs}
        for c in cfgs:  # warmup
            K.conv2d_nhwc(x, w, b, r, (s, s), pad, (1, 1), "relu", out=y, cfg=c)
        torch.cuda.synchronize()
        for _ in range(5):
            for c in cfgs:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    K.conv2d_nhwc(x, w, b, r, (s, s), pad, (1, 1), "relu", out=y, cfg=c)
                e1.record()
                e1.synchronize()
                times[c].append(e0.elapsed_time(e1) / 10 * 1e3)
        med = {c: sorted(v)[len(v) // 2] for c, v in times.items()}
        best = min([c for c in cfgs if c >= 0], key=lambda c: med[c])
        row = {"layer": name, "us": {str(c): round(med[c], 1) for c in cfgs}, "best": best,
               "auto_us": round(med[-1], 1), "best_us": round(med[best], 1),
               "best_tflops": round(flops / med[best] / 1e6, 1), "best_gbps": round(nbytes / med[best] / 1e3, 1)}
        out.append(row)
        print(json.dumps(row), flush=True)
    tot_auto = sum(r["auto_us"] for r in out)
    tot_best = sum(r["best_us"] for r in out)
    print(json.dumps({"sum_auto_us": round(tot_auto, 1), "sum_best_us": round(tot_best, 1)}))


if __name__ == "__main__":
    main()
