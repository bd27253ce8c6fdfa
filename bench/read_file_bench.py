#!/usr/bin/env python3
"""``env.read_file`` -> ``map_with_model`` at parallelism P in worker processes, with the
readers chained into the workers (default) or left in the coordinator (``--unchained``:
operator chaining disabled, so every decoded image crosses the coordinator -> worker
transport).  Reports records/s and the coordinator -> worker bytes per record (ring
messages + tensor slab; ``runtime/remote.py`` TRANSPORT_STATS).

    python bench/read_file_bench.py [--files 2000] [--hw 256] [--parallelism 4] [--unchained]
"""
import argparse
import io
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _Shape:
    """A stand-in model: the decoded image's shape and a checksum (no GPU needed)."""

    def run(self, img):
        a = np.asarray(img)
        return a.shape, int(a[::17, ::13].sum())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=2000)
    ap.add_argument("--hw", type=int, default=256)
    ap.add_argument("--parallelism", type=int, default=4)
    ap.add_argument("--unchained", action="store_true")
    a = ap.parse_args()
    from PIL import Image

    from flink_tensorflow_amd.models.zoo.inception import ImageInputFormat
    from flink_tensorflow_amd.runtime import PROCESS_ONCE, StreamExecutionEnvironment
    from flink_tensorflow_amd.runtime.remote import TRANSPORT_STATS

    d = tempfile.mkdtemp(prefix="ftm-rf-")
    try:
        rng = np.random.default_rng(0)
        pool = [rng.integers(0, 256, (a.hw, a.hw, 3), dtype=np.uint8) for _ in range(16)]
        for i in range(a.files):
            buf = io.BytesIO()
            Image.fromarray(pool[i % 16]).save(buf, format="JPEG", quality=90)
            with open(os.path.join(d, f"img{i:06d}.jpg"), "wb") as f:
                f.write(buf.getvalue())
        env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(a.parallelism)
        if a.unchained:
            env.disable_operator_chaining()
        sink = (env.read_file(ImageInputFormat(), d, PROCESS_ONCE)
                .map_with_model(_Shape(), lambda rec, m: (rec[0], m.run(rec[1])))
                .run_in_processes().collect_into())
        TRANSPORT_STATS.clear()
        t0 = time.perf_counter()
        env.execute("read-file-bench")
        el = time.perf_counter() - t0
        out = sink.results()
        st = [v for k, v in TRANSPORT_STATS.items() if k[0] == "map-with-model"]
        n = sum(v["records"] for v in st) or 1
        print(json.dumps({"files": a.files, "hw": a.hw, "parallelism": a.parallelism,
                          "readers": "coordinator" if a.unchained else "chained into the workers",
                          "records": len(out), "seconds": round(el, 3), "records_per_s": round(len(out) / el, 1),
                          "ring_bytes_per_record": round(sum(v["ring_bytes"] for v in st) / n, 1),
                          "slab_bytes_per_record": round(sum(v["slab_bytes"] for v in st) / n, 1)}), flush=True)
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
