#!/usr/bin/env python3
"""The reference's own workload end to end on the GPU: a directory of JPEG
files -> ``env.read_file(ImageInputFormat)`` -> the compiled ResNet-50 operator
(``map_with_model_batched``, one GPU subtask, the fused resize + normalise preprocess in the
plan) -> discarding sink.  Reference pipeline: ``inception.scala:33-46``
(``readFile(ImageInputFormat, dir, PROCESS_ONCE)`` -> ``mapWithModel``),
``ImageInputFormat.scala:63-80`` (decode per file), ``ImageNormalization.scala:42-77``.

Decode placements (``--decode``): ``staged`` (default) — the reader emits the compressed
bytes (``ImageInputFormat(defer_decode=True)``) and the model's host stage decodes them with
the native baseline decoder on its thread pool straight into the pinned staging slot
(``csrc/jpeg.cpp``); the reader runs in the model's worker, with the directory listing too
under ``--monitor partitioned`` (``sources.PartitionedFileSource``).  ``reader`` — Pillow
decode in R reader worker processes, the reference's placement (``ImageInputFormat.scala``).

Reports, as one JSON line:
* records/s of the timed window on the model operator (W + K micro-batches,
  ``batching/timed.py``) and of the whole job;
* single-thread decode cost per record (the same ``ImageInputFormat.read_record`` on the
  same files, one process);
* the GPU's idle share against the GPU-bound rate (``--gpu-rate``, the SPMD bench's
  records/s: ``1 - rate / gpu_rate``).

    python bench/jpeg_e2e.py [--files 20000] [--readers 12] [--hw 256]
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

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def make_jpegs(d: str, n: int, hw: int, distinct: int = 64, quality: int = 90) -> float:
    """``n`` JPEG files of ``distinct`` photo-like synthetic images (a smooth random field +
    mild noise: compresses like a photo, ~20-40 KB at 256 x 256, not like white noise).
    Returns the mean file size."""
    from PIL import Image

    rng = np.random.default_rng(0)
    blobs = []
    for _ in range(distinct):
        low = rng.integers(0, 256, (8, 8, 3), dtype=np.uint8)
        img = np.asarray(Image.fromarray(low).resize((hw, hw), Image.BICUBIC), np.float32)
        img = np.clip(img + rng.normal(0, 6, img.shape), 0, 255).astype(np.uint8)
        buf = io.BytesIO()
        Image.fromarray(img).save(buf, format="JPEG", quality=quality)
        blobs.append(buf.getvalue())
    for i in range(n):
        with open(os.path.join(d, f"img{i:06d}.jpg"), "wb") as f:
            f.write(blobs[i % distinct])
    return float(np.mean([len(b) for b in blobs]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=20000)
    ap.add_argument("--hw", type=int, default=256)
    ap.add_argument("--readers", type=int, default=12, help="reader (decode) subtasks, each a worker process")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--warmup", type=int, default=4, help="untimed micro-batches")
    ap.add_argument("--lanes", type=int, default=0, help="compute lanes (0: 2 for resnet50, 3 for inception_v3)")
    ap.add_argument("--gpu-rate", type=float, default=0.0,
                    help="GPU-bound records/s (SPMD bench; 0: 77.5k ResNet-50, 84.5k Inception-v3)")
    ap.add_argument("--max-delay-ms", type=float, default=20.0)
    ap.add_argument("--decode", default="staged", choices=["staged", "reader"],
                    help="staged: the reader emits the JPEG bytes and the model's host stage decodes them with the "
                         "native pool into the pinned slot (reader chained into the model worker); reader: Pillow "
                         "decode in --readers reader processes (the reference's placement)")
    ap.add_argument("--decode-threads", type=int, default=32)
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "inception_v3"],
                    help="resnet50: bf16, 2 lanes, 256x256 files (the headline model); inception_v3: the reference "
                         "example's model, fp8, 3 lanes, 299x299 files")
    ap.add_argument("--monitor", default="partitioned", choices=["partitioned", "coordinator"],
                    help="partitioned: the listing + reading source runs inside the model's worker (nothing crosses "
                         "the coordinator); coordinator: Flink's monitor in the coordinator forwarding paths")
    a = ap.parse_args()

    from flink_tensorflow_amd.batching.timed import TimedWindow
    from flink_tensorflow_amd.models.zoo.image_classifier import InceptionV3Model, ResNet50Model
    from flink_tensorflow_amd.models.zoo.inception import ImageInputFormat
    from flink_tensorflow_amd.runtime import PROCESS_ONCE, StreamExecutionEnvironment
    from flink_tensorflow_amd.runtime.sources import DiscardingSink

    inc = a.model == "inception_v3"
    if inc and a.hw == 256:
        a.hw = 299

    class TimedModel(TimedWindow, InceptionV3Model if inc else ResNet50Model):
        pass

    d = tempfile.mkdtemp(prefix="ftm-jpeg-")
    out_dir = tempfile.mkdtemp(prefix="ftm-jpeg-out-")
    try:
        t0 = time.perf_counter()
        mean_bytes = make_jpegs(d, a.files, a.hw)
        gen_s = time.perf_counter() - t0
        # single-thread decode cost of the format's read_record (Pillow)
        fmt = ImageInputFormat()
        files = sorted(os.listdir(d))[:400]
        datas = [open(os.path.join(d, f), "rb").read() for f in files]
        fmt.read_record(files[0], datas[0])
        t0 = time.perf_counter()
        for f, b in zip(files, datas):
            fmt.read_record(f, b)
        decode_ms = (time.perf_counter() - t0) / len(files) * 1e3

        # native decode capacity in this process: 256 images into one buffer, 1 thread and
        # --decode-threads threads, in 64-image pieces as the runner stages them
        from flink_tensorflow_amd import _ext

        nat = _ext.native()
        blobs = (datas * (256 // len(datas) + 1))[:256]
        buf = np.empty((256, a.hw, a.hw, 3), np.uint8)
        rb = a.hw * a.hw * 3
        native_ms = {}
        for th in (1, a.decode_threads):
            nat.jpeg_decode_into(buf.ctypes.data, buf.nbytes, blobs[:64], rb, a.hw, a.hw, th)
            t0 = time.perf_counter()
            reps = 2 if th == 1 else 10
            for _ in range(reps):
                for lo in range(0, 256, 64):
                    nat.jpeg_decode_into(buf.ctypes.data + lo * rb, buf.nbytes - lo * rb, blobs[lo:lo + 64], rb,
                                         a.hw, a.hw, th)
            native_ms[th] = (time.perf_counter() - t0) / reps * 1e3

        B = a.batch
        K = a.files // B - a.warmup - 1  # the last, partial batch is not timed
        extra = {}
        if inc:  # fp8 scales from the bench's own images (decoded once here)
            from flink_tensorflow_amd.graph.ops_io import decode_jpegs

            extra["calibration_images"] = decode_jpegs(datas[:64], a.hw, a.hw)
        model = TimedModel(image_hw=(a.hw, a.hw), buckets=(B,), lanes=a.lanes or (3 if inc else 2), depth=3,
                           lane_offset_us=1500.0, **extra).timed_window(a.warmup, K, out_dir)
        env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(1)
        staged = a.decode == "staged"
        model.decode_threads = a.decode_threads
        fmt_job = ImageInputFormat(defer_decode=staged)
        if staged:  # one reader in the model's worker process (partitioned: the listing too)
            readers = env.read_file(fmt_job, d, PROCESS_ONCE, parallelism=1, monitor=a.monitor)
        else:
            readers = env.read_file(fmt_job, d, PROCESS_ONCE, parallelism=a.readers).run_in_processes()
        readers.map_with_model_batched(model, None, max_batch=B, max_delay_ms=a.max_delay_ms, name="resnet50",
                                       parallelism=1).run_in_processes() \
            .add_sink(DiscardingSink()).run_in_processes()
        if not a.gpu_rate:
            a.gpu_rate = 84500.0 if inc else 77500.0
        t0 = time.perf_counter()
        res = env.execute("jpeg-e2e")
        wall = time.perf_counter() - t0
        with open(os.path.join(out_dir, "rank0.json")) as f:
            r0 = json.load(f)
        rate = r0["records"] / r0["elapsed_s"]
        lat = np.asarray(r0["latencies_s"])
        print(json.dumps({
            "bench": "jpeg_e2e", "files": a.files, "hw": a.hw, "mean_jpeg_bytes": round(mean_bytes),
            "decode": ("native baseline decoder on the model's host pool, into the pinned slot "
                       f"({a.decode_threads} threads)" if staged else f"Pillow in {a.readers} reader processes"),
            "readers": 1 if staged else a.readers, "monitor": a.monitor if staged else "coordinator", "gpus": 1,
            "model": "Inception-v3 (fp8, compiled plan)" if inc else "ResNet-50 v1.5 (bf16, compiled plan)",
            "records_per_s": round(rate, 1), "job_records_per_s": round(a.files / wall, 1),
            "job_wall_s": round(wall, 2), "timed_batches": K, "timed_records": r0["records"],
            "decode_ms_per_record_1thread": round(decode_ms, 3),
            "native_decode_ms_per_record_1thread": round(native_ms[1] / 256, 3),
            f"native_decode_ms_per_256_batch_{a.decode_threads}threads": round(native_ms[a.decode_threads], 3),
            "pillow_decode_bound_records_per_s": round(a.readers * 1e3 / decode_ms, 1),
            "gpu_rate_records_per_s": a.gpu_rate, "gpu_idle_share": round(max(0.0, 1 - rate / a.gpu_rate), 3),
            "p50_latency_ms": round(float(np.percentile(lat, 50)) * 1e3, 2) if lat.size else None,
            "host_ms_per_batch": r0.get("host_ms_per_batch"),
            "batch_interval_ms": round(r0["elapsed_s"] / max(1, K) * 1e3, 3),
            "allowed_cpus": len(os.sched_getaffinity(0)), "generate_s": round(gen_s, 1),
            "attempts": res.attempts}), flush=True)
    finally:
        shutil.rmtree(d, ignore_errors=True)
        shutil.rmtree(out_dir, ignore_errors=True)


if __name__ == "__main__":
    main()
