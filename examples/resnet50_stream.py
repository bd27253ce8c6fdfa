#!/usr/bin/env python3
"""ResNet-50 bf16 image-classification stream on the full DataStream runtime.

    python examples/resnet50_stream.py [--records N] [--batch 256] [--delay-ms 5] [--parallelism P]

synthetic decoded-image source → map_with_model_batched(ResNet50Model) → sink.  On a GPU
the model is compiled per batch bucket and run by the pipelined pinned-H2D / hipGraph
runner; prints throughput and the per-record latency histogram of the model operator.
(``bench.py`` times the same engine step-by-step for the headline number.)

``--parallelism P``: the reference's data parallelism (``env.setParallelism``,
``inception.scala:22-23``) the MI355X way — P worker-process subtasks, one GPU each, every
subtask's source chained into its worker, the model operator with ``distributed_weights``
(subtask 0 compiles, its weights are broadcast over the operator's RCCL group).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flink_tensorflow_amd.models.zoo.image_classifier import ResNet50Model  # noqa: E402
from flink_tensorflow_amd.runtime import StreamExecutionEnvironment  # noqa: E402
from flink_tensorflow_amd.runtime.sources import ThroughputSink  # noqa: E402




def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=20000)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--delay-ms", type=float, default=5.0)
    ap.add_argument("--hw", type=int, default=256)
    ap.add_argument("--depth-layers", type=int, default=50)
    ap.add_argument("--savedmodel", action="store_true",
                    help="export ResNet-50 as a TF SavedModel and serve its serving_default signature "
                         "through SignatureBatchedModel (the path a user's own SavedModel takes)")
    ap.add_argument("--processes", action="store_true",
                    help="run the model operator in a worker process (records cross through the tensor slab)")
    ap.add_argument("--worker-source", action="store_true",
                    help="run the source inside the model's worker process too (a chained source: records are "
                         "produced where the GPU operator consumes them; implies --processes)")
    ap.add_argument("--parallelism", type=int, default=1,
                    help="P GPU subtasks in worker processes (implies --worker-source), one RCCL group, "
                         "rank 0's weights broadcast")
    ap.add_argument("--no-chain", action="store_true",
                    help="disable operator chaining: the in-process source runs in its own thread and hands "
                         "records to the model thread through a queue")
    a = ap.parse_args()
    hw, n_rec = a.hw, a.records

    def images(idx, par, start):
        # built where the source runs (the coordinator, or the worker with --worker-source)
        pool = np.random.default_rng(idx).integers(0, 256, (256, hw, hw, 3), dtype=np.uint8)
        for k, i in enumerate(range(idx, n_rec, par)):
            if k >= start:
                yield pool[i % len(pool)]

    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(a.parallelism)
    dist = a.parallelism > 1
    if dist:
        a.worker_source = True
        env.enable_job_communicator(True)
    if a.no_chain:
        env.disable_operator_chaining()
    if a.savedmodel:
        import tempfile

        from flink_tensorflow_amd.models import SignatureBatchedModel
        from flink_tensorflow_amd.models.zoo.resnet import export_resnet50_saved_model

        d = export_resnet50_saved_model(os.path.join(tempfile.mkdtemp(), "rn50"), image_hw=(a.hw, a.hw),
                                        depth=a.depth_layers)
        model = SignatureBatchedModel(d, buckets=(a.batch,), output_keys=["classes", "scores"],
                                      distributed_weights=dist)
    else:
        model = ResNet50Model(image_hw=(a.hw, a.hw), buckets=(a.batch,), depth_layers=a.depth_layers,
                              distributed_weights=dist)
    src = env.generate(images)
    if a.worker_source:
        src = src.run_in_processes()
    op = src.map_with_model_batched(model, None, max_batch=a.batch, max_delay_ms=a.delay_ms, name="resnet50")
    if a.processes or a.worker_source:
        op = op.run_in_processes()
    op.add_sink(sink := ThroughputSink())
    t0 = time.time()
    res = env.execute("resnet50-stream")
    el = time.time() - t0
    m = [v for k, v in res.metrics.items() if k.startswith("resnet50")][0]
    steady = sink.rate(0.2)  # steady state: skip the first fifth (compile, capture, pipeline fill)
    print(json.dumps({"records": a.records, "parallelism": a.parallelism, "savedmodel": a.savedmodel, "worker_process": a.processes or a.worker_source,
                      "worker_source": a.worker_source, "chained": not a.no_chain, "seconds": round(el, 3), "records_per_s": round(a.records / el, 1),
                      "steady_records_per_s": round(steady, 1) if steady else None,
                      "latency_s": m["histograms"].get("latency_s"), "batch": m["histograms"].get("batch_size")}))


if __name__ == "__main__":
    main()
