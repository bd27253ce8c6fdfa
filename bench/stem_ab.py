"""Times the pooled ResNet-50 stem (space-to-depth 4x4 conv 16->64 + ReLU + fused 3x3/s2 max
pool; B=256 at 224x224 = 112x112x16 input) on the direct LDS conv kernel (dconv.hip).

Measured history (1x MI355X, profiles/r01_s3/stem.md): 237 us with a float compare per
element in the pooled epilogue and two runtime integer divides per K-step; 213 us with the
packed u16 max; 181 us with the host-built K-offset table.  A persistent variant (filter
bank resident, two 4-wave tile pipelines per CU, double-buffered patches) measured 194 us
(only 2 waves per SIMD) and was dropped.  Round 2: 8-wave workgroups with 14 x 8 pooled
pixels (pool_rows=14) fetch the filter bank half as often: 181.2 -> 160.9 us, bit-identical
output (profiles/r02_stem_rows)."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/bench/", 1)[0])
from flink_tensorflow_amd.ops import kernels as K  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    x = torch.randn(B, 112, 112, 16, device=dev).to(torch.bfloat16)
    w = torch.randn(64, 4, 4, 16) / 16.0
    arr = K.dconv_bf16_weight_bytes(w, 64).to(dev)
    b = torch.randn(64, device=dev) * 0.1
    times = {7: [], 14: []}
    outs = {}
    for rnd in range(8):  # interleaved rounds: 7-row (4-wave) vs 14-row (8-wave) pooled tiles
        for rows in (7, 14):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                outs[rows] = K.conv2d_direct(x, arr, (4, 4), 64, b, (1, 1), (2, 1, 2, 1), "relu", bn=64,
                                             maxpool_pad=(0, 1, 0, 1), pool_rows=rows)
            e1.record()
            e1.synchronize()
            if rnd:
                times[rows].append(e0.elapsed_time(e1) / 10 * 1e3)
    flops = 2.0 * B * 112 * 112 * 64 * 4 * 4 * 16
    for rows in (7, 14):
        us = sorted(times[rows])[len(times[rows]) // 2]
        print(json.dumps({"batch": B, "pool_rows": rows, "stem_us": round(us, 1),
                          "tflops_s2d_conv": round(flops / us / 1e6, 1), "out_shape": list(outs[rows].shape),
                          "equal_to_7": bool(torch.equal(outs[rows], outs[7]))}))


if __name__ == "__main__":
    main()
