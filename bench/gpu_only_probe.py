"""Diagnostic (not the benchmark): the GPU-only rate of the compiled ResNet-50 plans with
the input already in HBM — no host gather, no H2D, no D2H — replayed on 1..3 lanes (one
HIP stream each).  Compared with ``bench.py`` it separates the GPU bound from the input
pipeline's cost.  Prints one JSON line per lane count."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from flink_tensorflow_amd.batching.arena import DeviceArena  # noqa: E402
from flink_tensorflow_amd.config import EngineConfig  # noqa: E402
from flink_tensorflow_amd.graph.compiler import CompiledFunction  # noqa: E402
from flink_tensorflow_amd.graph.graph import Graph  # noqa: E402
from flink_tensorflow_amd.models.zoo.resnet import resnet50_graph_def  # noqa: E402
from flink_tensorflow_amd.utils.streams import dedicated_stream  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--lanes", default="1,2,3")
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = Graph.from_graph_def(resnet50_graph_def(image_hw=(256, 256), top_k=5, seed=0))
    nmax = max(int(x) for x in a.lanes.split(","))
    budget = EngineConfig().arena_bytes(dev) // nmax
    plans = [CompiledFunction(g, {"images:0": ((a.batch, 256, 256, 3), "UINT8")}, ["top_k:0", "top_k:1"], dev,
                              strict=True, arena=DeviceArena(dev, budget, name=f"probe{i}")) for i in range(nmax)]
    src = torch.randint(0, 255, (a.batch, 256, 256, 3), dtype=torch.uint8, device=dev)
    streams = [dedicated_stream(dev, owner=p) for p in plans]
    for n in [int(x) for x in a.lanes.split(",")]:
        for warm in (True, False):
            iters = 20 if warm else a.iters
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for i in range(iters):
                k = i % n
                with torch.cuda.stream(streams[k]):
                    plans[k].replay_from("images:0", src)
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t0
        print(json.dumps({"lanes": n, "batches": a.iters, "ms_per_batch": round(dt / a.iters * 1e3, 3),
                          "records_per_s": round(a.iters * a.batch / dt, 1)}), flush=True)


if __name__ == "__main__":
    main()
