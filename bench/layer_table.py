"""Per-layer table of a compiled CNN plan: device time of every step (HIP event pair around
each launch, median of --reps eager runs via ``CompiledFunction.profile``), the MACs it
performs (fused shortcut projections and fused next-block reduce convs included), the
bytes it must move at least once (activations in + out, weights) and the resulting
TFLOP/s and TB/s.  Prints a markdown table and writes one JSON line per step to --jsonl.

    python bench/layer_table.py [--model resnet50|inception_v3] [--batch 256] [--reps 5]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flink_tensorflow_amd.graph.compiler import CompiledFunction  # noqa: E402
from flink_tensorflow_amd.graph.graph import Graph  # noqa: E402


def _elems(shape):
    n = 1
    for s in shape:
        n *= int(s)
    return n


def _bytes(v):
    es = 1 if v.qscale is not None or v.dtype in (torch.uint8, torch.int8) else (v.dtype.itemsize if v.dtype else 2)
    return _elems(v.shape) * es


def _filter_shape(plan, node):
    if node is None or node.op != "Conv2D" or len(node.inputs) < 2:
        return None
    src = node.inputs[1]
    v = plan.vals.get((src[0], src[1]) if isinstance(src, tuple) else (src, 0))
    return tuple(v.shape) if v is not None else None


def step_work(plan, step):
    """(MACs, weight elements) of a step, or (None, 0) when it is not a conv / GEMM."""
    node = plan.graph.nodes.get(step.name)
    f = _filter_shape(plan, node)
    if f is None:
        if step.kind == "gemm" and step.inputs and step.outputs:  # 1x1 conv / FC as a GEMM
            k = step.inputs[0].shape[-1]
            n = step.outputs[0].shape[-1]
            m = _elems(step.outputs[0].shape) // n
            return m * n * k, n * k
        return None, 0
    kh, kw, cin, cout = f
    out = step.meta.get("conv_out") or step.outputs[0].shape  # fused-pool stem: pre-pool grid
    m = _elems(out) // out[-1]
    macs, wel = m * cout * kh * kw * cin, kh * kw * cin * cout
    if len(step.inputs) > 1 and step.inputs[1].shape[-1] != out[-1]:  # fused projection shortcut
        c_sc = step.inputs[1].shape[-1]
        macs += m * c_sc * cout
        wel += c_sc * cout
    if step.meta.get("impl") == "bottleneck_tail" and len(step.outputs) > 1:  # + next block's reduce
        c2 = step.outputs[1].shape[-1]
        macs += m * cout * c2
        wel += cout * c2
    return macs, wel


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "inception_v3"])
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--jsonl", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    if a.model == "resnet50":
        from flink_tensorflow_amd.models.zoo.resnet import resnet50_graph_def

        hw, precision = 256, "bf16"
        g = Graph.from_graph_def(resnet50_graph_def(image_hw=(hw, hw), top_k=5, seed=0))
        calib = None
    else:
        from flink_tensorflow_amd.models.zoo.inception_v3 import inception_v3_graph_def

        hw, precision = 299, "fp8"
        g = Graph.from_graph_def(inception_v3_graph_def(image_hw=(hw, hw), top_k=5, seed=0))
        calib = {"images:0": torch.randint(0, 256, (64, hw, hw, 3), dtype=torch.uint8).repeat(-(-a.batch // 64), 1, 1, 1)[: a.batch]}
    feed = {"images:0": ((a.batch, hw, hw, 3), "UINT8")}
    plan = CompiledFunction(g, feed, ["top_k:0", "top_k:1"], dev, strict=True, precision=precision, calibration=calib)
    imgs = torch.randint(0, 256, (a.batch, hw, hw, 3), dtype=torch.uint8, device=dev)
    plan.profile({"images:0": imgs})
    runs = []
    for _ in range(a.reps):
        md = plan.profile({"images:0": imgs})
        runs.append([ns.op_end_rel_micros for ns in md.step_stats.dev_stats[0].node_stats])
    us = [statistics.median(col) for col in zip(*runs)]
    rows, tot_us, tot_macs = [], 0.0, 0
    for st, t in zip(plan.steps, us):
        macs, wel = step_work(plan, st)
        act = sum(_bytes(v) for v in st.inputs + st.outputs if not v.is_const)
        wbytes = wel * (1 if precision == "fp8" else 2)
        nbytes = act + wbytes
        r = {"step": st.name, "kind": st.kind, "impl": st.meta.get("impl", ""), "us": round(t, 1),
             "out": list(st.outputs[0].shape) if st.outputs else None, "gmacs": round(macs / 1e9, 3) if macs else None,
             "tflops": round(2 * macs / t / 1e6, 1) if macs and t else None, "mbytes": round(nbytes / 1e6, 1),
             "tbps": round(nbytes / t / 1e6, 2) if t else None}
        rows.append(r)
        tot_us += t
        tot_macs += macs or 0
    print(f"| # | step | kind | out | µs | GMAC | TFLOP/s | MB | TB/s |")
    print("|---|---|---|---|---|---|---|---|---|")
    for i, r in enumerate(rows):
        print(f"| {i} | {r['step']} | {r['kind']}{('/' + r['impl']) if r['impl'] else ''} | {r['out']} | {r['us']} | "
              f"{r['gmacs'] if r['gmacs'] is not None else ''} | {r['tflops'] if r['tflops'] is not None else ''} | "
              f"{r['mbytes']} | {r['tbps']} |")
    print(f"\n{a.model} {precision} B={a.batch}: {len(rows)} steps, {tot_us:.0f} µs of step time (one lane, eager "
          f"launches), {2 * tot_macs / 1e12:.2f} TFLOP -> {2 * tot_macs / tot_us / 1e6:.0f} TFLOP/s", flush=True)
    if a.jsonl:
        with open(a.jsonl, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
