"""ResNet-50 stage 1 at B=256 (56x56): the block's 3x3 (conv3x3c64) + its fused tail as two
launches vs the one bottleneck3 kernel, for the three stage-1 boundaries.  Interleaved."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/bench/", 1)[0])
from flink_tensorflow_amd.ops import kernels as K  # noqa: E402


def timeit(fn, reps=10):
    ts = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / reps * 1e3)
    return sorted(ts)[3]


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    dev = torch.device("cuda", 0)
    bf = lambda *s: (torch.randn(*s, device=dev) / 8).to(torch.bfloat16)  # noqa: E731
    y1, x2 = bf(B, 56, 56, 64).relu(), torch.empty(B, 56, 56, 64, device=dev, dtype=torch.bfloat16)
    w2, b2 = bf(64, 3, 3, 64), torch.zeros(64, device=dev)
    for name, dual, cn, dec in (("unit1_dual", True, 64, False), ("unit2", False, 64, False),
                                ("unit3_to_stage2", False, 128, True)):
        second = bf(B, 56, 56, 64 if dual else 256)
        w3, b3 = bf(256, 128 if dual else 64), torch.zeros(256, device=dev)
        w1, b1 = bf(cn, 256), torch.zeros(cn, device=dev)
        y3 = torch.empty(B, 28 if dec else 56, 28 if dec else 56, 256, device=dev, dtype=torch.bfloat16)
        yo = torch.empty(B, 56, 56, cn, device=dev, dtype=torch.bfloat16)
        kw = dict(xs=second if dual else None, y3_decimated=dec)
        res = None if dual else second

        def pair():
            K.conv3x3_c64(y1, w2, b2, "relu", out=x2)
            K.bottleneck_tail(x2, res, w3, b3, w1, b1, y3=y3, y1=yo, **kw)

        def c3():
            K.conv3x3_c64(y1, w2, b2, "relu", out=x2)

        def tail():
            K.bottleneck_tail(x2, res, w3, b3, w1, b1, y3=y3, y1=yo, **kw)

        def fused():
            K.bottleneck3(y1, w2, b2, res, w3, b3, w1, b1, y3=y3, y1_out=yo, **kw)

        fns = {"pair": pair, "fused": fused, "c3": c3, "tail": tail}
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        res_us = {k: [] for k in fns}
        for _ in range(3):
            for k, f in fns.items():
                res_us[k].append(timeit(f))
        us = {k: round(sorted(v)[1], 1) for k, v in res_us.items()}
        print(json.dumps({"boundary": name, "batch": B, "us": us, "speedup": round(us["pair"] / us["fused"], 3)}),
              flush=True)


if __name__ == "__main__":
    main()
