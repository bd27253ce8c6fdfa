"""Ablation timing of the pipelined conv kernel (igemm_v2): full / no-MFMA / no-DMA /
no-ds_read variants on one bf16 and one fp8 3x3 conv (random data, interleaved rounds)."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/bench/", 1)[0])
from flink_tensorflow_amd import _ext  # noqa: E402

CASES = [  # es, B, H, W, Cin, Cout
    (2, 256, 56, 56, 64, 64),
    (2, 256, 28, 28, 128, 128),
    (1, 256, 35, 35, 96, 96),
    (1, 256, 17, 17, 160, 192),
]


def main():
    hip = _ext.hip(required=True)
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream().cuda_stream
    for es, B, H, W, Cin, Cout in CASES:
        dt = torch.bfloat16 if es == 2 else torch.uint8
        if es == 2:
            x = torch.randn(B, H, W, Cin, device=dev).to(dt)
            w = torch.randn(Cout, 3, 3, Cin, device=dev).to(dt)
        else:
            x = torch.randint(0, 120, (B, H, W, Cin), device=dev, dtype=dt)
            w = torch.randint(0, 120, (Cout, 9 * Cin), device=dev, dtype=dt)
        sc = torch.ones(Cout, device=dev)
        b = torch.zeros(Cout, device=dev)
        y = torch.empty(B * H * W * Cout * (2 if es == 2 else 1), dtype=torch.uint8, device=dev)
        res = {}
        for abl in (0, 1, 2, 4, 6):
            def run():
                hip.igemm_v2_ablate(x.data_ptr(), w.data_ptr(), sc.data_ptr(), b.data_ptr(), y.data_ptr(), es, B, H, W,
                                    Cin, Cout, 3, 3, 1, 1, H, W, abl, st)
            run()
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    run()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) / 10 * 1e3)
            res[abl] = round(sorted(ts)[2], 1)
        flops = 2.0 * B * H * W * Cout * 9 * Cin
        print(json.dumps({"es": es, "shape": [B, H, W, Cin, Cout], "us": res,
                          "full_tflops": round(flops / res[0] / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
