"""BASELINE config 1: MNIST-MLP SavedModel inference in the local mini-cluster on CPU.

Compares the reference's execution model (one ``Session.run`` per record at batch 1 inside
``mapWithModel``) with the micro-batching operator, at parallelism 1..P.
Prints one JSON line per configuration (records/s, p50 latency).
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flink_tensorflow_amd.models.zoo.mnist import MnistModel, export_mnist_mlp  # noqa: E402
from flink_tensorflow_amd.runtime import StreamExecutionEnvironment  # noqa: E402


def run(path, n, parallelism, batched, imgs):
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(parallelism)
    src = env.from_collection(list(range(n))).rebalance()
    model = MnistModel(path)
    if batched:
        s = src.map_with_model_batched(model, lambda m, ids: m.classify(torch.from_numpy(imgs[ids]))[0].tolist(),
                                       max_batch=256, max_delay_ms=2, name="mnist")
    else:
        s = src.map_with_model(model, lambda i, m: int(m.classify(torch.from_numpy(imgs[i:i + 1]))[0]), name="mnist")
    sink = s.collect_into()
    t0 = time.perf_counter()
    res = env.execute("mnist")
    el = time.perf_counter() - t0
    assert len(sink.results()) == n
    lat = [v["histograms"].get("latency_s", {}).get("p50") for k, v in res.metrics.items() if k.startswith("mnist")]
    return {"config": "mnist-mlp-cpu", "mode": "micro-batched" if batched else "per-record (reference model)",
            "parallelism": parallelism, "records": n, "records_per_s": round(n / el, 1),
            "p50_latency_ms": round(1e3 * float(np.nanmedian([x for x in lat if x is not None])), 3) if batched
            and any(x is not None for x in lat) else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=20000)
    ap.add_argument("--max-parallelism", type=int, default=4)
    a = ap.parse_args()
    torch.set_num_threads(1)
    d = export_mnist_mlp(os.path.join(tempfile.mkdtemp(), "mnist"))
    imgs = np.random.default_rng(0).random((a.records, 784), dtype=np.float32)
    for p in sorted({1, a.max_parallelism}):
        print(json.dumps(run(d, min(a.records, 5000), p, False, imgs)), flush=True)
        print(json.dumps(run(d, a.records, p, True, imgs)), flush=True)


if __name__ == "__main__":
    main()
