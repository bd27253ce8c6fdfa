"""tests/test_arena.py::test_two_compute_lanes_keep_order_gpu step by step (prints after
every step, faulthandler on) to name the step of a segfault."""
import faulthandler
import gc
import sys

faulthandler.enable()
sys.path.insert(0, ".")
import numpy as np  # noqa: E402
import torch  # noqa: E402

from flink_tensorflow_amd.batching.arena import DeviceArena  # noqa: E402
from flink_tensorflow_amd.batching.engine import PipelinedGpuRunner  # noqa: E402
from flink_tensorflow_amd.graph.compiler import CompiledFunction  # noqa: E402
from flink_tensorflow_amd.graph.graph import Graph  # noqa: E402
from flink_tensorflow_amd.models.zoo.resnet import resnet50_graph_def  # noqa: E402


def say(*a):
    print(*a, flush=True)


g = Graph.from_graph_def(resnet50_graph_def(depth=26, image_hw=(48, 48), num_classes=32))
dev = torch.device("cuda", 0)
feeds = {"images:0": ((4, 48, 48, 3), "UINT8")}


def lane():
    return {4: CompiledFunction(g, feeds, ["top_k:0", "top_k:1"], dev, strict=True, arena=DeviceArena(dev, 4 << 30))}


rng = np.random.default_rng(0)
batches = [[rng.integers(0, 256, (48, 48, 3), dtype=np.uint8) for _ in range(4)] for _ in range(7)]
say("graph built")
lanes = lane()
say("plan compiled")
r = PipelinedGpuRunner(lanes, "images:0", lambda p: p.output_tensors(), (48, 48, 3), depth=3, device=dev)
say("runner", r.copy_stream, r.compute_streams)
out = []
for i, b in enumerate(batches):
    out += r.submit(b, np.full(4, float(i)), [i] * 4)
    say("submitted", i)
out += r.drain()
say("drained", len(out))
del r
gc.collect()
say("runner collected")
torch.cuda.synchronize()
say("synced")
two = [lane(), lane()]
say("two lanes compiled")
r = PipelinedGpuRunner(two, "images:0", lambda p: p.output_tensors(), (48, 48, 3), depth=3, device=dev)
out2 = []
for i, b in enumerate(batches):
    out2 += r.submit(b, np.full(4, float(i)), [i] * 4)
    say("submitted2", i)
out2 += r.drain()
say("done", [x.tags[0] for x in out2])
