"""``env.read_file`` as Flink builds it (``EX/inception/inception.scala:33-34``): a
parallelism-1 monitor that forwards paths, parallel readers that read and decode, the
readers chained into the worker processes of the GPU operator they feed, checkpointed
monitor/reader state, and the Johnny / Inception pipelines under PROCESS_CONTINUOUSLY."""
import io
import os
import sys
import threading
import time

import numpy as np
from PIL import Image

from flink_tensorflow_amd.models.zoo.inception import ImageInputFormat, InceptionModel
from flink_tensorflow_amd.runtime import (PROCESS_CONTINUOUSLY, PROCESS_ONCE, RestartStrategy,
                                          StreamExecutionEnvironment)
from flink_tensorflow_amd.runtime.executor import LocalExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _jpeg(h=64, w=48, seed=0, color=None) -> bytes:
    if color is None:
        img = np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)
    else:
        img = np.zeros((h, w, 3), np.uint8)
        img[..., color] = 220
    buf = io.BytesIO()
    Image.fromarray(img).save(buf, format="JPEG")
    return buf.getvalue()


class _ColorModel:
    """Labels an image by its dominant channel: red cheeseburger, green ladybug, blue llama."""
    NAMES = ("cheeseburger", "ladybug", "llama")

    def label(self, imgs):
        return [[(0.9, self.NAMES[int(np.argmax(np.asarray(im).reshape(-1, 3).mean(0)))])] for im in imgs]


def test_read_file_readers_chain_into_model_workers(tmp_path):
    """Monitor (p=1, coordinator) → 4 readers chained into the 4 worker processes of a
    ``map_with_model`` operator: each worker reads and decodes its files, and what crosses
    from the coordinator to a worker per record is the path (plus pickle framing), never
    the decoded image — nothing goes through the tensor slab."""
    from flink_tensorflow_amd.runtime.remote import TRANSPORT_STATS

    imgs = tmp_path / "imgs"
    imgs.mkdir()
    for i in range(16):
        (imgs / f"img{i:02d}.jpg").write_bytes(_jpeg(seed=i))
    (imgs / "partial.crdownload").write_bytes(b"junk")
    TRANSPORT_STATS.clear()
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(4)
    model = InceptionModel(str(tmp_path), image_hw=(64, 48), device="cpu")
    sink = (env.read_file(ImageInputFormat(), str(imgs), PROCESS_ONCE)
            .map_with_model(model, lambda rec, m: (rec[0], os.getpid(), tuple(rec[1].shape), m.label([rec[1]])[0][0][1]))
            .run_in_processes().collect_into())
    ex = LocalExecutor(env, "read-file-p4")
    ex.execute()
    out = sink.results()
    assert sorted(n for n, *_ in out) == [f"img{i:02d}.jpg" for i in range(16)]
    assert all(shape == (64, 48, 3) and lbl.startswith("class_") for _, _, shape, lbl in out)
    pids = {p for _, p, _, _ in out}
    assert len(pids) == 4 and os.getpid() not in pids  # decoded and labelled in 4 workers
    names = {n.name for n in env.nodes if getattr(n, "merged_into", None) is not None}
    assert names == {"file-reader"}  # the readers run inside the model workers
    stats = {k: v for k, v in TRANSPORT_STATS.items() if k[0] == "map-with-model"}
    assert len(stats) == 4
    recs = sum(v["records"] for v in stats.values())
    ring = sum(v["ring_bytes"] for v in stats.values())
    assert recs == 16 and sum(v["slab_bytes"] for v in stats.values()) == 0
    longest = max(len(str(p)) for p in imgs.iterdir())
    assert ring / recs <= longest + 32, (ring, recs, longest)  # a path per record
    assert ring / recs < 64 * 48 * 3 / 50  # vs the decoded image the old source shipped


def test_read_file_restart_reads_every_file_once(tmp_path):
    """A failure after some files were read: the restarted job resumes from the monitor's
    seen set and the readers' pending splits — each file is emitted exactly once across
    the committed output (no replays of forwarded-and-read files)."""
    from flink_tensorflow_amd.runtime.sources import BytesInputFormat
    from flink_tensorflow_amd.utils.fault import FailAfter

    d = tmp_path / "in"
    d.mkdir()
    for i in range(40):
        (d / f"f{i:02d}.bin").write_bytes(bytes([i]) * (i + 1))
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(2)
    env.enable_checkpointing(0.02, str(tmp_path / "chk"))
    env.set_restart_strategy(RestartStrategy.fixed_delay(2, 0.0))
    src = env.read_file(BytesInputFormat(), str(d), PROCESS_CONTINUOUSLY, 0.05, max_polls=40)
    sink = src.map(lambda v: (os.path.basename(v[0]), len(v[1]))).map(FailAfter(15, attempts=(0,))) \
        .key_by(lambda v: v[0]).process(_DedupLast()).collect_into()
    res = env.execute("read-file-restart")
    assert res.attempts == 1
    got = {}
    for name, n, count in sink.results():
        got[name] = max(got.get(name, 0), count)
    assert sorted(got) == [f"f{i:02d}.bin" for i in range(40)]
    assert set(got.values()) == {1}  # keyed count restored from the checkpoint: read once


from flink_tensorflow_amd.runtime import ProcessFunction, ValueStateDescriptor  # noqa: E402


class _DedupLast(ProcessFunction):
    def open(self, config=None):
        self.count = self.get_runtime_context().get_state(ValueStateDescriptor("count", 0))

    def process_element(self, value, ctx, out):
        self.count.update(self.count.value() + 1)
        out.collect((value[0], value[1], self.count.value()))


def _johnny_job(tmp_path, workers: bool, parallelism: int = 1):
    sys.path.insert(0, os.path.join(ROOT, "examples"))
    import johnny

    d = tmp_path / "cam"
    d.mkdir()
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(parallelism)
    sink = johnny.build_job(env, _ColorModel(), str(d), polls=12, interval_s=0.25, image_hw=(32, 32),
                            workers=workers).collect_into()

    def camera():  # one picture per poll interval, in the order Johnny shows them
        time.sleep(0.3)
        for i, color in enumerate((0, 1, 2)):
            (d / f"shot{i}.tmp").write_bytes(_jpeg(color=color))
            os.replace(d / f"shot{i}.tmp", d / f"shot{i}.jpg")  # appears atomically
            time.sleep(0.6)

    t = threading.Thread(target=camera)
    t.start()
    env.execute("johnny")
    t.join()
    return sink.results()


def test_johnny_process_continuously(tmp_path):
    """``EX/inception/johnny.scala``: images appear one by one in a continuously monitored
    directory; cheeseburger → ladybug → llama within 60 s grants access."""
    out = _johnny_job(tmp_path, workers=False)
    assert ("AccessGranted", ["shot0.jpg", "shot1.jpg", "shot2.jpg"]) in out


def test_johnny_process_continuously_in_a_worker(tmp_path):
    """The same job with the labelling operator in a worker process: the reader is
    chained into it, the monitor stays in the coordinator."""
    out = _johnny_job(tmp_path, workers=True)
    assert ("AccessGranted", ["shot0.jpg", "shot1.jpg", "shot2.jpg"]) in out


def test_inception_process_continuously_picks_up_new_files(tmp_path):
    """The Inception labelling job on a continuously monitored directory at parallelism 2:
    files present at start and files added between polls are each labelled once."""
    d = tmp_path / "imgs"
    d.mkdir()
    for i in range(3):
        (d / f"a{i}.jpg").write_bytes(_jpeg(seed=i))
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(2)
    model = InceptionModel(str(tmp_path), image_hw=(64, 48), device="cpu")
    sink = (env.read_file(ImageInputFormat(), str(d), PROCESS_CONTINUOUSLY, 0.2, max_polls=8)
            .map_with_model(model, lambda rec, m: (rec[0], m.label([rec[1]])[0][0])).collect_into())

    def later():
        time.sleep(0.5)
        for i in range(3):
            (d / f"b{i}.tmp").write_bytes(_jpeg(seed=10 + i))
            os.replace(d / f"b{i}.tmp", d / f"b{i}.jpg")

    t = threading.Thread(target=later)
    t.start()
    env.execute("inception-continuous")
    t.join()
    out = sink.results()
    assert sorted(n for n, _ in out) == ["a0.jpg", "a1.jpg", "a2.jpg", "b0.jpg", "b1.jpg", "b2.jpg"]
    assert all(0.0 <= p <= 1.0 and lbl.startswith("class_") for _, (p, lbl) in out)


def test_read_file_rebalance_then_workers_still_chains(tmp_path):
    """``read_file(...).rebalance().map_with_model(...)`` (the reference's shape with an
    explicit repartition): the repartition has nothing to move once the readers run in the
    model workers, so the readers still chain into them and only paths cross."""
    from flink_tensorflow_amd.runtime.remote import TRANSPORT_STATS

    imgs = tmp_path / "imgs"
    imgs.mkdir()
    for i in range(6):
        (imgs / f"img{i}.jpg").write_bytes(_jpeg(seed=i))
    TRANSPORT_STATS.clear()
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(2)
    sink = (env.read_file(ImageInputFormat(), str(imgs), PROCESS_ONCE).rebalance()
            .map_with_model(_ColorModel(), lambda rec, m: (rec[0], os.getpid(), m.label([rec[1]])[0][0][1]))
            .run_in_processes().collect_into())
    env.execute("read-file-rebalance")
    out = sink.results()
    assert sorted(n for n, _, _ in out) == [f"img{i}.jpg" for i in range(6)]
    assert os.getpid() not in {p for _, p, _ in out}
    stats = [v for k, v in TRANSPORT_STATS.items() if k[0] == "map-with-model"]
    recs = sum(v["records"] for v in stats)
    longest = max(len(str(p)) for p in imgs.iterdir())
    assert recs == 6 and sum(v["ring_bytes"] for v in stats) / recs <= longest + 32


def test_partitioned_monitor_runs_inside_the_workers(tmp_path):
    """``read_file(..., monitor="partitioned")``: each of the 3 model workers lists the
    directory itself and takes its hash share of the files — every file labelled exactly
    once, in the worker that read it, and nothing crosses the coordinator on the way in."""
    from flink_tensorflow_amd.runtime.remote import TRANSPORT_STATS

    imgs = tmp_path / "imgs"
    imgs.mkdir()
    for i in range(24):
        (imgs / f"img{i:02d}.jpg").write_bytes(_jpeg(seed=i))
    (imgs / "partial.crdownload").write_bytes(b"junk")
    TRANSPORT_STATS.clear()
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(3)
    sink = (env.read_file(ImageInputFormat(), str(imgs), PROCESS_ONCE, monitor="partitioned")
            .map_with_model(_ColorModel(), lambda rec, m: (rec[0], os.getpid(), m.label([rec[1]])[0][0][1]))
            .run_in_processes().collect_into())
    env.execute("read-file-partitioned")
    out = sink.results()
    assert sorted(n for n, _, _ in out) == [f"img{i:02d}.jpg" for i in range(24)]
    pids = {p for _, p, _ in out}
    assert len(pids) == 3 and os.getpid() not in pids
    inbound = [v for k, v in TRANSPORT_STATS.items() if k[0] == "map-with-model"]
    assert sum(v.get("records", 0) for v in inbound) == 0  # the sources ran in the workers


def test_partitioned_source_splits_files_disjointly(tmp_path):
    """The hash split: subtasks of one ``PartitionedFileSource`` see disjoint file sets
    that together cover the directory, each emitted in runs (``collect_many``)."""
    import zlib

    from flink_tensorflow_amd.runtime.sources import BytesInputFormat, PartitionedFileSource

    d = tmp_path / "in"
    d.mkdir()
    for i in range(50):
        (d / f"f{i:02d}.bin").write_bytes(bytes([i]) * 3)

    class Ctx:
        def __init__(self, idx, par):
            self.subtask_index, self.parallelism = idx, par
            self.runs = []
            self.checkpoint_lock = threading.RLock()

        def collect_many(self, values, timestamp=None):
            self.runs.append(list(values))

    got = []
    for idx in range(3):
        src = PartitionedFileSource(BytesInputFormat(), str(d), PROCESS_ONCE, run=8)
        ctx = Ctx(idx, 3)
        src.set_runtime_context(ctx)
        src.open()
        src.run(ctx)
        names = [os.path.basename(p) for r in ctx.runs for p, _ in r]
        assert all(len(r) <= 8 for r in ctx.runs)
        assert all(zlib.crc32(str(d / n).encode()) % 3 == idx for n in names)
        assert all(data == bytes([int(n[1:3])]) * 3 for r in ctx.runs for p, data in r for n in [os.path.basename(p)])
        got += names
    assert sorted(got) == [f"f{i:02d}.bin" for i in range(50)]


def test_partitioned_monitor_restart_reads_every_file_once(tmp_path):
    """The partitioned source's checkpointed seen set: after a failure the restarted job
    resumes each subtask's share where its last checkpoint left it — every file counted
    exactly once in the restored keyed state."""
    from flink_tensorflow_amd.runtime.sources import BytesInputFormat
    from flink_tensorflow_amd.utils.fault import FailAfter

    d = tmp_path / "in"
    d.mkdir()
    for i in range(40):
        (d / f"f{i:02d}.bin").write_bytes(bytes([i]) * (i + 1))
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(2)
    env.enable_checkpointing(0.02, str(tmp_path / "chk"))
    env.set_restart_strategy(RestartStrategy.fixed_delay(2, 0.0))
    src = env.read_file(BytesInputFormat(), str(d), PROCESS_CONTINUOUSLY, 0.05, max_polls=40, monitor="partitioned")
    sink = src.map(lambda v: (os.path.basename(v[0]), len(v[1]))).map(FailAfter(15, attempts=(0,))) \
        .key_by(lambda v: v[0]).process(_DedupLast()).collect_into()
    res = env.execute("read-file-partitioned-restart")
    assert res.attempts == 1
    got = {}
    for name, n, count in sink.results():
        got[name] = max(got.get(name, 0), count)
    assert sorted(got) == [f"f{i:02d}.bin" for i in range(40)]
    assert set(got.values()) == {1}


def test_partitioned_source_reads_non_local_filesystems():
    """A ``mem://`` directory: the partitioned source lists and reads through the file-system
    registry (no native bulk read), same split rule."""
    from flink_tensorflow_amd.runtime.sources import BytesInputFormat, PartitionedFileSource
    from flink_tensorflow_amd.utils import fs

    for i in range(12):
        fs.write_bytes(f"mem://ptest/in/f{i:02d}.bin", bytes([i]) * 2)

    class Ctx:
        def __init__(self, idx, par):
            self.subtask_index, self.parallelism = idx, par
            self.checkpoint_lock = threading.RLock()
            self.got = []

        def collect_many(self, values, timestamp=None):
            self.got += values

    got = []
    for idx in range(2):
        src = PartitionedFileSource(BytesInputFormat(), "mem://ptest/in", PROCESS_ONCE, run=5)
        ctx = Ctx(idx, 2)
        src.set_runtime_context(ctx)
        src.open()
        src.run(ctx)
        got += [(p.rsplit("/", 1)[1], d) for p, d in ctx.got]
    assert sorted(got) == [(f"f{i:02d}.bin", bytes([i]) * 2) for i in range(12)]
