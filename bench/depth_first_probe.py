"""Does running ResNet-50's stem + stage 1 in sub-batches (activations resident in the
256 MB Infinity Cache between layers) beat the full micro-batch?  Times the compiled
plan truncated at the stage-1 output for 256 images as 1 x 256, 2 x 128, 4 x 64 and
8 x 32 back-to-back hipGraph replays.  One JSON line per split."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from flink_tensorflow_amd.graph.compiler import CompiledFunction  # noqa: E402
from flink_tensorflow_amd.graph.graph import Graph  # noqa: E402
from flink_tensorflow_amd.models.zoo.resnet import resnet50_graph_def  # noqa: E402

FETCH = os.environ.get("FETCH", "block1/unit3/conv3/Relu:0")


def main():
    dev = torch.device("cuda", 0)
    g = Graph.from_graph_def(resnet50_graph_def(image_hw=(256, 256), top_k=5, seed=0))
    imgs = torch.randint(0, 256, (256, 256, 256, 3), dtype=torch.uint8, device=dev)
    for b in (256, 128, 64, 32):
        p = CompiledFunction(g, {"images:0": ((b, 256, 256, 3), "UINT8")}, [FETCH], dev, strict=True)
        n = 256 // b
        inb = p.input_buffer("images:0")
        inb.copy_(imgs[:b])

        def run():
            for _ in range(n):
                p.replay()

        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 10
        print(json.dumps({"fetch": FETCH, "sub_batch": b, "chunks": n, "us_per_256_images": round(us, 1),
                          "steps": p.summary()["kinds"]}), flush=True)
        del p


if __name__ == "__main__":
    main()
