"""gemm_pp (hand-written ping-pong MFMA GEMM) vs hipBLASLt (torch.addmm) on the hot-path
shapes.  Interleaved rounds in one process (guide §5.4 rule 24), random operands (rule
25).  Prints one JSON line per shape: median / min µs and TFLOP/s for both."""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flink_tensorflow_amd.ops import kernels as K

SHAPES = {
    "bert_qkv": (32768, 2304, 768, None, False),
    "bert_o": (32768, 768, 768, None, True),
    "bert_ffn1": (32768, 3072, 768, "gelu", False),
    "bert_ffn1_plain": (32768, 3072, 768, None, False),
    "k768_n2304_m49152": (49152, 2304, 768, None, False),
    "bert_ffn2": (32768, 768, 3072, None, True),
    "bert_packed_o": (24576, 768, 768, None, True),
    "sq4096": (4096, 4096, 4096, None, False),
    "sq8192": (8192, 8192, 8192, None, False),
    "rn_s3_c1": (12544, 256, 1024, "relu", False),
    "rn_s4_c1": (3136, 512, 2048, "relu", False),
    "rn_fc": (256, 1000, 2048, None, False),
}


def timeit(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--ours-only", action="store_true", help="skip the library arm (profiling)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for name in a.shapes.split(","):
        M, N, Kd, act, res = SHAPES[name]
        x = (torch.rand(M, Kd, device=dev) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, Kd, device=dev) * 2 - 1) / Kd ** 0.5).to(torch.bfloat16)
        b = torch.randn(N, device=dev)
        b16 = b.to(torch.bfloat16)
        r = torch.randn(M, N, device=dev).to(torch.bfloat16) if res else None
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        out2 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)

        def ours():
            K.gemm_pp(x, w, b, r, act, out=out)

        def lib():
            if act == "gelu":
                y = torch._addmm_activation(b16, x, w.t(), use_gelu=True)
            elif act == "relu":
                y = torch._addmm_activation(b16, x, w.t())
            else:
                y = torch.addmm(b16, x, w.t(), out=out2)
            if r is not None:
                y.add_(r)

        if a.ours_only:
            lib = ours  # noqa: F811
        ours(); lib(); torch.cuda.synchronize()
        t_o, t_l = [], []
        for _ in range(a.rounds):
            t_o.append(timeit(ours, a.reps))
            t_l.append(timeit(lib, a.reps))
        fl = 2.0 * M * N * Kd
        err = (out.float() - K._apply_act_ref(x.float() @ w.float().t() + b + (r.float() if r is not None else 0),
                                              K.act_code(act))).abs().max().item()
        print(json.dumps({"shape": name, "M": M, "N": N, "K": Kd, "act": act, "res": res,
                          "ours_us_med": round(statistics.median(t_o), 2), "ours_us_min": round(min(t_o), 2),
                          "lib_us_med": round(statistics.median(t_l), 2), "lib_us_min": round(min(t_l), 2),
                          "ours_tflops": round(fl / statistics.median(t_o) / 1e6, 1),
                          "lib_tflops": round(fl / statistics.median(t_l) / 1e6, 1),
                          "speedup_vs_lib": round(statistics.median(t_l) / statistics.median(t_o), 3),
                          "max_abs_err": round(err, 4)}), flush=True)


if __name__ == "__main__":
    main()
