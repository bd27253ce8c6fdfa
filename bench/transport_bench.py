"""Coordinator -> worker-process record transport: decoded-image records (256x256x3 uint8,
196 KB) streamed through ``run_in_processes()`` subtasks (tensor slab: payload written once
into shared memory, descriptors through the ring) vs the pickle path (FTM_SLAB_BYTES=0).
The generator source is splittable, so by default the executor relocates it into the
worker processes (``LocalExecutor._relocate_sources``: records are produced where they are
consumed); ``--no-relocate`` measures the coordinator -> slab -> worker copy path.
Prints one JSON line: aggregate GB/s and records/s of the whole job."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _touch(v):
    return int(v[0, 0, 0]) + int(v[-1, -1, -1])  # reads both ends of the payload


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--records", type=int, default=40000)
    ap.add_argument("--hw", type=int, default=256)
    ap.add_argument("--remote-source", action="store_true",
                    help="the parallel source runs inside the worker processes, chained with the map "
                         "(records are produced where they are consumed; nothing crosses the coordinator)")
    ap.add_argument("--no-chain", action="store_true", help="disable operator chaining (source and proxy threads)")
    ap.add_argument("--no-relocate", action="store_true",
                    help="keep the generator source in the coordinator (env.relocate_sources = False): every "
                         "record is produced there and copied into the workers' slabs")
    a = ap.parse_args()
    from flink_tensorflow_amd.runtime import StreamExecutionEnvironment
    from flink_tensorflow_amd.runtime.sources import ThroughputSink

    pool = [np.random.default_rng(i).integers(0, 256, (a.hw, a.hw, 3), dtype=np.uint8) for i in range(64)]
    n = a.records

    hw = a.hw

    def images(idx, par, start):
        # this subtask's share of the n records; ``start`` = how many of them it already emitted
        import numpy as _np

        local = [_np.random.default_rng(i).integers(0, 256, (hw, hw, 3), dtype=_np.uint8) for i in range(16)]
        for k, i in enumerate(range(idx, n, par)):
            if k >= start:
                yield local[i % len(local)].copy()  # a freshly produced record (decode / read), not a shared buffer

    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(a.workers)
    if a.no_chain:
        env.disable_operator_chaining()
    env.relocate_sources = not a.no_relocate
    sink = ThroughputSink(every=512)
    src = env.generate(images)
    if a.remote_source:
        src = src.run_in_processes()
    src.map(_touch).run_in_processes().add_sink(sink, parallelism=1)
    from flink_tensorflow_amd.runtime.executor import LocalExecutor

    t0 = time.perf_counter()
    ex = LocalExecutor(env, "transport")
    ex.execute()
    el = time.perf_counter() - t0
    got = sink.count() if hasattr(sink, "count") else n
    steady = sink.rate(0.3)  # after worker spawn / import and pipeline fill
    print(json.dumps({"workers": a.workers, "records": got, "record_bytes": pool[0].nbytes, "seconds": round(el, 3),
                      "steady_records_per_s": round(steady, 1),
                      "steady_GB_per_s": round(steady * pool[0].nbytes / 1e9, 2),
                      "slab": os.environ.get("FTM_SLAB_BYTES", "default") != "0", "cpus": os.cpu_count(),
                      "mode": "in-worker parallel source" if a.remote_source else "coordinator source -> workers",
                      "relocated_sources": ex.relocated, "chained": not a.no_chain}),
          flush=True)
    assert got == n


if __name__ == "__main__":
    main()
