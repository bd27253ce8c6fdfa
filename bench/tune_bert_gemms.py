"""Pre-tunes the BERT-base projection GEMMs (hipBLASLt / rocBLAS solutions via PyTorch
TunableOp) for every token capacity of the padding-free encoder, and reports the default
vs tuned times.  The resulting solution table is loaded by the encoder at plan build
(``flink_tensorflow_amd/data/tunableop_gfx950.csv``) so no tuning runs in a stream job.

    python bench/tune_bert_gemms.py [--granule 2048] [--out path] [--shapes-only]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def shapes(granule: int, full: int = 256 * 128, h: int = 768, inter: int = 3072):
    for m in range(granule, full + granule, granule):
        m = min(m, full)
        yield m, h, 3 * h, "bias"       # QKV
        yield m, h, h, "bias"           # attention output
        yield m, h, inter, "gelu"       # FFN up (+GELU epilogue)
        yield m, inter, h, "bias"       # FFN down


def run(m, k, n, kind, dev, iters=20):
    import torch

    x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
    w = torch.randn(n, k, device=dev, dtype=torch.bfloat16) * 0.02
    b = torch.randn(n, device=dev, dtype=torch.bfloat16)
    out = torch.empty(m, n, device=dev, dtype=torch.bfloat16)

    def f():
        if kind == "gelu":
            return torch._addmm_activation(b, x, w.t(), use_gelu=True)
        return torch.addmm(b, x, w.t(), out=out)

    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--granule", type=int, default=2048)
    ap.add_argument("--out", default=os.path.join(ROOT, "flink_tensorflow_amd", "data", "tunableop_gfx950.csv"))
    ap.add_argument("--compare", action="store_true", help="time default vs the solutions in --out (no tuning)")
    a = ap.parse_args()
    import torch

    dev = torch.device("cuda", 0)
    todo = list(shapes(a.granule))
    tun = torch.cuda.tunable
    t0 = time.time()
    if not a.compare:  # tuning pass: results are flushed to the file at interpreter exit
        tun.enable(True)
        tun.tuning_enable(True)
        tun.set_max_tuning_duration(60)
        tun.set_max_tuning_iterations(50)
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        tun.set_filename(a.out)
        for s in todo:
            run(*s, dev, iters=1)
            print(f"[tune] {s} {time.time() - t0:.0f}s", flush=True)
        return
    base = {s: run(*s, dev) for s in todo}
    tun.enable(True)
    tun.tuning_enable(False)
    tun.read_file(a.out)
    tuned = {s: run(*s, dev) for s in todo}
    tot_b = sum(base.values())
    tot_t = sum(tuned.values())
    for s in todo:
        print(json.dumps({"m": s[0], "k": s[1], "n": s[2], "epi": s[3], "default_us": round(base[s], 1),
                          "tuned_us": round(tuned[s], 1)}), flush=True)
    print(json.dumps({"sum_default_us": round(tot_b, 1), "sum_tuned_us": round(tot_t, 1),
                      "tuning_s": round(time.time() - t0, 1), "file": a.out}), flush=True)


if __name__ == "__main__":
    main()
