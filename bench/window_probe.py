"""Diagnostic: where the driver's 20-step window loses time against the steady rate.
Runs bench.py's ResNet-50 configuration (2 lanes, B = 256, warmup, drain), then K timed
steps, and prints per batch: host submit time, the H2D completion and the compute
completion on the GPU (timing events recorded right after each submit on the copy stream
and on the batch's lane stream), all in ms from the start of the window."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from flink_tensorflow_amd.batching.arena import DeviceArena  # noqa: E402
from flink_tensorflow_amd.batching.engine import PipelinedGpuRunner  # noqa: E402
from flink_tensorflow_amd.config import EngineConfig  # noqa: E402
from flink_tensorflow_amd.graph.compiler import CompiledFunction  # noqa: E402
from flink_tensorflow_amd.graph.graph import Graph  # noqa: E402
from flink_tensorflow_amd.models.zoo.resnet import resnet50_graph_def  # noqa: E402
from flink_tensorflow_amd.parallel import comm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--lanes", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm.bind_to_gpu_numa(dev)
    B, HW = 256, 256
    g = Graph.from_graph_def(resnet50_graph_def(image_hw=(HW, HW), top_k=5, seed=0))
    budget = EngineConfig().arena_bytes(dev) // a.lanes
    lanes = [{B: CompiledFunction(g, {"images:0": ((B, HW, HW, 3), "UINT8")}, ["top_k:0", "top_k:1"], dev,
                                  strict=True, arena=DeviceArena(dev, budget, name=f"lane{i}"))}
             for i in range(a.lanes)]
    pool = np.random.default_rng(1234).integers(0, 256, size=(512, HW, HW, 3), dtype=np.uint8)
    records = [pool[i] for i in range(512)]
    runner = PipelinedGpuRunner(lanes, "images:0", lambda p: p.output_tensors(), (HW, HW, 3), torch.uint8,
                                depth=3, device=dev)
    cursor = 0

    def step(log=None):
        nonlocal cursor
        batch = [records[(cursor + i) % 512] for i in range(B)]
        cursor += B
        ts = np.full(B, time.perf_counter())
        lane = runner._lane
        res = runner.poll() + runner.submit(batch, ts)
        if log is not None:
            ec, eh = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            eh.record(runner.copy_stream)
            ec.record(runner.compute_streams[lane])
            log.append((lane, time.perf_counter(), eh, ec))
        return res

    for _ in range(a.warmup):
        step()
    for _ in runner.drain():
        pass
    torch.cuda.synchronize(dev)
    e0 = torch.cuda.Event(enable_timing=True)
    e0.record(torch.cuda.current_stream(dev))
    t0 = time.perf_counter()
    log = []
    for _ in range(a.steps):
        step(log)
    for _ in runner.drain():
        pass
    torch.cuda.synchronize(dev)
    el = (time.perf_counter() - t0) * 1e3
    rows = [{"i": i, "lane": ln, "submitted_ms": round((t - t0) * 1e3, 3), "h2d_done_ms": round(e0.elapsed_time(eh), 3),
             "done_ms": round(e0.elapsed_time(ec), 3)} for i, (ln, t, eh, ec) in enumerate(log)]
    for r in rows:
        print(json.dumps(r))
    print(json.dumps({"window_ms": round(el, 3), "records_per_s": round(a.steps * B / el * 1e3, 1),
                      "host_ms_per_batch": {k: round(v * 1e3 / max(1, runner.batches), 3)
                                            for k, v in runner.host_s.items()}}), flush=True)


if __name__ == "__main__":
    main()
