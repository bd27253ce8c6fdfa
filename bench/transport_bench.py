"""Coordinator -> worker-process record transport: decoded-image records (256x256x3 uint8,
196 KB) streamed through ``run_in_processes()`` subtasks (tensor slab: payload written once
into shared memory, descriptors through the ring) vs the pickle path (FTM_SLAB_BYTES=0).
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
    a = ap.parse_args()
    from flink_tensorflow_amd.runtime import StreamExecutionEnvironment
    from flink_tensorflow_amd.runtime.sources import ThroughputSink

    pool = [np.random.default_rng(i).integers(0, 256, (a.hw, a.hw, 3), dtype=np.uint8) for i in range(64)]
    n = a.records

    def images(idx, par, start):
        for i in range(start, n):
            if i % par == idx:
                yield pool[i % len(pool)]

    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(a.workers)
    sink = ThroughputSink(every=512)
    env.generate(images).map(_touch).run_in_processes().add_sink(sink, parallelism=1)
    t0 = time.perf_counter()
    env.execute("transport")
    el = time.perf_counter() - t0
    got = sink.count() if hasattr(sink, "count") else n
    steady = sink.rate(0.3)  # after worker spawn / import and pipeline fill
    print(json.dumps({"workers": a.workers, "records": got, "record_bytes": pool[0].nbytes, "seconds": round(el, 3),
                      "steady_records_per_s": round(steady, 1),
                      "steady_GB_per_s": round(steady * pool[0].nbytes / 1e9, 2),
                      "slab": os.environ.get("FTM_SLAB_BYTES", "default") != "0", "cpus": os.cpu_count()}),
          flush=True)
    assert got == n


if __name__ == "__main__":
    main()
