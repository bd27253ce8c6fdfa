"""Step-by-step check of framework-owned HIP streams (utils/streams.py) on one GPU: prints
a line after each step so a fault names the step that caused it."""
import faulthandler
import gc
import sys

faulthandler.enable()
sys.path.insert(0, ".")
import torch  # noqa: E402

from flink_tensorflow_amd import _ext  # noqa: E402
from flink_tensorflow_amd.utils.streams import capture_stream, dedicated_stream  # noqa: E402


def say(*a):
    print(*a, flush=True)


dev = torch.device("cuda", 0)
x = torch.ones(1024, device=dev)
torch.cuda.synchronize()
lib = _ext.hip()
say("lib", lib.__file__)
ptr = lib.stream_create(0)
say("raw stream", hex(ptr))
s = torch.cuda.ExternalStream(ptr, device=dev)
say("external stream", s, s.cuda_stream)
with torch.cuda.stream(s):
    y = x * 2
s.synchronize()
say("kernel on raw stream ok", float(y.sum()))
lib.stream_destroy(ptr)
say("destroyed raw stream")


class Owner:
    pass


o = Owner()
s2 = dedicated_stream(dev, owner=o)
with torch.cuda.stream(s2):
    z = x + 1
ev = torch.cuda.Event()
ev.record(s2)
ev.synchronize()
say("dedicated stream ok", float(z.sum()))
cs = capture_stream(dev)
say("capture stream", cs.cuda_stream)
g = torch.cuda.CUDAGraph()
static = torch.zeros(1024, device=dev)
from flink_tensorflow_amd.utils.tracing import graph_capture  # noqa: E402

with graph_capture(g):
    static.add_(x)
say("captured")
with torch.cuda.stream(s2):
    g.replay()
s2.synchronize()
say("replayed on dedicated stream", float(static.sum()))
del o
gc.collect()
say("owner collected (stream released)")
torch.cuda.synchronize()
say("done")
