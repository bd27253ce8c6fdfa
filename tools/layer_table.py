"""Per-layer device times of a compiled CNN plan (ResNet-50 v1.5 at micro-batch 256 by
default, as bench.py builds it): one eager pass with a HIP event pair around every launch
(``CompiledFunction.profile``), repeated ``--reps`` times, median per step.  Prints one JSON
line per step (name, kind, kernel, output shape, µs, TF/s) and a markdown table; a step
named after a Conv2D gets its FLOPs from the graph (2 * B*Ho*Wo*Cout * KH*KW*Cin) on the
grid the kernel computes: a stem conv with a fused max pool is counted on its full-resolution
(pre-pool) output (the step's ``conv_out``), not on the pooled tensor it stores; steps that
fuse several convs into one launch (stage-1 tails) report time only.

    python tools/layer_table.py [--model resnet50|inception_v3] [--batch 256] [--reps 5]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "inception_v3"])
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=None, help="also write the markdown table here")
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--hw", type=int, default=None)
    a = ap.parse_args()
    import numpy as np
    import torch

    from flink_tensorflow_amd.graph.compiler import CompiledFunction
    from flink_tensorflow_amd.graph.graph import Graph

    dev = torch.device(a.device)
    B = a.batch
    if a.model == "resnet50":
        from flink_tensorflow_amd.models.zoo.resnet import resnet50_graph_def

        HW, prec = a.hw or 256, "bf16"
        graph = Graph.from_graph_def(resnet50_graph_def(image_hw=(HW, HW), top_k=5, seed=0))
        calib = None
    else:
        from flink_tensorflow_amd.models.zoo.inception_v3 import inception_v3_graph_def

        HW, prec = a.hw or 299, "fp8"
        graph = Graph.from_graph_def(inception_v3_graph_def(image_hw=(HW, HW), top_k=5, seed=0))
        rng = np.random.default_rng(5)
        calib = {"images:0": torch.from_numpy(rng.integers(0, 256, (64, HW, HW, 3), dtype=np.uint8)).repeat(
            -(-B // 64), 1, 1, 1)[:B]}
    plan = CompiledFunction(graph, {"images:0": ((B, HW, HW, 3), "UINT8")}, ["top_k:0", "top_k:1"], dev,
                            use_graph=False, strict=True, precision=prec, calibration=calib)
    imgs = torch.from_numpy(np.random.default_rng(0).integers(0, 256, (B, HW, HW, 3), dtype=np.uint8)).to(dev)
    plan.profile({"images:0": imgs})  # warm-up
    runs = []
    for _ in range(a.reps):
        md = plan.profile({"images:0": imgs})
        runs.append([(s.node_name, s.timeline_label, s.op_end_rel_micros) for s in md.step_stats.dev_stats[0].node_stats])
    total = 0.0
    rows = []
    for i, st in enumerate(plan.steps):
        us = float(np.median([r[i][2] for r in runs]))
        total += us
        # a stage-1 tail launch also runs the next block's reduce: time only
        out = st.outputs[0].shape if st.outputs and hasattr(st.outputs[0], "shape") else None
        grid = st.meta.get("conv_out") or out  # the computed grid (pre-pool for a pool-fused stem)
        flops = 0.0
        node = graph.nodes.get(st.name)
        if node is not None and node.op == "Conv2D" and out is not None and st.meta.get("impl") != "bottleneck_tail":
            from flink_tensorflow_amd.graph.tensor_proto import tensor_from_proto

            wn = graph.nodes.get(node.inputs[1][0])
            if wn is not None and wn.op == "Const":
                KH, KW, Cin, Cout = tensor_from_proto(wn.tensor_attr("value")).shape
                flops = 2.0 * grid[0] * grid[1] * grid[2] * Cout * KH * KW * Cin
        rows.append({"i": i, "name": st.name, "kind": st.kind, "impl": st.meta.get("impl", ""),
                     "out": list(out) if out is not None else None,
                     "grid": list(grid) if grid is not None and grid is not out else None, "us": round(us, 1),
                     "tflops": round(flops / us / 1e6, 1) if flops and us else None})
    for r in rows:
        print(json.dumps(r))
    print(json.dumps({"total_us": round(total, 1), "steps": len(rows), "batch": B, "model": a.model}))
    lines = ["| # | step | kind / kernel | output (computed grid) | µs | TF/s |", "|---|---|---|---|---|---|"]
    for r in rows:
        shown = f"{r['out']} (grid {r['grid']})" if r["grid"] else f"{r['out']}"
        lines.append(f"| {r['i']} | {r['name']} | {r['kind']} {r['impl']} | {shown} | {r['us']} | "
                     f"{r['tflops'] if r['tflops'] is not None else ''} |")
    lines.append(f"| | **total** | | | **{round(total, 1)}** | |")
    md = "\n".join(lines)
    print(md)
    if a.out:
        with open(a.out, "w") as f:
            f.write(md + "\n")


if __name__ == "__main__":
    main()
