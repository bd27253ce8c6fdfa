"""Worker-process subtasks over native shared-memory rings: ring protocol across
processes, remote operators with keyed state, checkpoints/restarts and error propagation,
and (GPU) a micro-batched ResNet operator whose subtasks are worker processes."""
import multiprocessing as mp
import os

import pytest

from flink_tensorflow_amd import _ext
from flink_tensorflow_amd.runtime import (JobExecutionException, ListStateDescriptor, ProcessFunction,
                                          RestartStrategy, StreamExecutionEnvironment, ValueStateDescriptor)
from flink_tensorflow_amd.runtime.remote import ShmChannel
from flink_tensorflow_amd.utils.fault import FailAfter


def _echo_worker(a, b):
    inp, out = ShmChannel(a, False), ShmChannel(b, False)
    while True:
        m = inp.recv(10.0)
        if m is None or m == "stop":
            break
        out.send(m)
    out.close()


def test_shm_channel_across_processes():
    tag = f"/ftm-t-{os.getpid()}"
    a, b = ShmChannel(tag + "a", True, 1 << 16), ShmChannel(tag + "b", True, 1 << 16)
    p = mp.get_context("spawn").Process(target=_echo_worker, args=(a.name, b.name))
    p.start()
    try:
        msgs = [("small", i) for i in range(500)] + [bytes(100_000), list(range(50_000))]  # > ring: fragmented
        for m in msgs:
            a.send(m)
            assert b.recv(10.0) == m
        a.send("stop")
        assert b.recv(10.0) is None  # producer closed its ring
    finally:
        p.join(10)
        a.unlink()
        b.unlink()
    with pytest.raises(RuntimeError):
        _ext.native().ShmRing(tag + "a", 0, False)  # unlinked


def test_remote_map_runs_in_worker_processes():
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(2)
    out = env.from_collection(list(range(300))).rebalance() \
        .map(lambda v: (os.getpid(), v * 2)).run_in_processes().execute_and_collect()
    pids = {p for p, _ in out}
    assert sorted(v for _, v in out) == [2 * i for i in range(300)]
    assert len(pids) == 2 and os.getpid() not in pids


def test_worker_operator_is_not_chained():
    """A worker-process operator's proxy keeps its own coordinator thread: chained behind
    its upstream, producing records and scattering them into the slab would serialise on
    one thread (profiles/r03_transport).  Operators around it still chain."""
    from flink_tensorflow_amd.runtime.executor import LocalExecutor

    env = StreamExecutionEnvironment.get_execution_environment()
    s = env.from_collection(list(range(500))).map(lambda v: v + 1).name("inc")
    s = s.map(lambda v: (os.getpid(), v)).name("remote").run_in_processes()
    sink = s.map(lambda pv: pv).name("after").collect_into()
    ex = LocalExecutor(env, "remote-alone")
    ex.execute()
    assert ex.chains == [["collection", "inc"], ["after", "collect"]]
    out = sink.results()
    assert sorted(v for _, v in out) == list(range(1, 501))
    assert {p for p, _ in out} != {os.getpid()} and len({p for p, _ in out}) == 1


def test_remote_batched_operator_metrics():
    """A micro-batching operator in a worker: its batch-size histogram (recorded in the
    worker) reaches the job result."""
    env = StreamExecutionEnvironment.get_execution_environment()
    res_sink = env.from_collection(list(range(100))).map_with_model_batched(
        object(), lambda m, vals: [v + 1 for v in vals], max_batch=16, max_delay_ms=2).run_in_processes().collect_into()
    res = env.execute("remote-batched")
    assert sorted(res_sink.results()) == list(range(1, 101))
    m = [v for k, v in res.metrics.items() if k.startswith("batched-model")][0]
    assert m["histograms"]["batch_size"]["max"] == 16


class _RunningSum(ProcessFunction):
    def open(self, config=None):
        self.total = self.get_runtime_context().get_state(ValueStateDescriptor("total", 0))

    def process_element(self, value, ctx, out):
        self.total.update(self.total.value() + value)
        out.collect((ctx.get_current_key(), self.total.value()))


def test_remote_keyed_state_survives_failure_and_restart(tmp_path):
    """A worker-process keyed operator snapshots through the ring; after an injected
    failure the restarted workers resume from the checkpoint consistently."""
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(2)
    env.enable_checkpointing(0.05, str(tmp_path / "chk"))
    env.set_restart_strategy(RestartStrategy.fixed_delay(2, 0.0))
    from flink_tensorflow_amd.runtime.sources import CollectionSource

    src = env.add_source(CollectionSource(list(range(1, 301)), delay_s=0.002), "numbers")
    res_sink = src.map(FailAfter(100, attempts=(0,))).key_by(lambda v: v % 3).process(_RunningSum()) \
        .run_in_processes().collect_into()
    res = env.execute("remote-recover")
    assert res.attempts == 1 and len(res.checkpoints) >= 1
    final = {}
    for k, t in res_sink.results():
        final[k] = max(final.get(k, 0), t)
    assert final == {k: sum(v for v in range(1, 301) if v % 3 == k) for k in range(3)}


def test_killed_worker_process_restarts_from_checkpoint(tmp_path):
    """A worker process dies mid-stream (os._exit, no error message): the coordinator
    notices the dead process, fails the attempt, and the restart resumes every keyed sum
    consistently from the last completed checkpoint."""
    from flink_tensorflow_amd.runtime.sources import CollectionSource
    from flink_tensorflow_amd.utils.fault import KillProcessAfter

    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(2)
    env.enable_checkpointing(0.05, str(tmp_path / "chk"))
    env.set_restart_strategy(RestartStrategy.fixed_delay(2, 0.0))
    src = env.add_source(CollectionSource(list(range(1, 301)), delay_s=0.002), "numbers")
    sink = src.map(KillProcessAfter(80)).run_in_processes().key_by(lambda v: v % 3).process(_RunningSum()) \
        .collect_into()
    res = env.execute("worker-crash")
    assert res.attempts == 1 and len(res.checkpoints) >= 1
    final = {}
    for k, t in sink.results():
        final[k] = max(final.get(k, 0), t)
    assert final == {k: sum(v for v in range(1, 301) if v % 3 == k) for k in range(3)}


def _boom(v):
    if v == 7:
        raise ValueError("bad record 7")
    return v


def test_remote_error_propagates():
    env = StreamExecutionEnvironment.get_execution_environment()
    env.from_collection(list(range(20))).map(_boom).run_in_processes().collect_into()
    with pytest.raises(JobExecutionException, match="bad record 7"):
        env.execute("remote-boom")


def _two_gpu_subtasks_resnet():
    """Body of ``test_remote_batched_resnet_gpu`` (runs in its own process)."""
    import numpy as np

    from flink_tensorflow_amd.models.zoo.image_classifier import ResNet50Model

    rng = np.random.default_rng(0)
    imgs = [rng.integers(0, 256, (64, 64, 3), dtype=np.uint8) for _ in range(40)]
    model = ResNet50Model(image_hw=(64, 64), buckets=(8, 16), top_k=3, depth_layers=26)

    def run(remote):
        env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(2)
        s = env.from_collection(imgs).rebalance() \
            .map_with_model_batched(model, None, max_batch=16, max_delay_ms=5, emit_batches=False)
        if remote:
            s = s.run_in_processes()
        return s.execute_and_collect()

    local, remote = run(False), run(True)
    assert len(remote) == len(local) == 40
    # numerics: the fp32 interpreter on the host over the same images (results arrive in
    # any order: compare the sorted top-1 probabilities and the multiset of top-1 labels)
    ref = ResNet50Model(image_hw=(64, 64), buckets=(8, 16), top_k=3, depth_layers=26, device="cpu")
    ref.open()
    want = ref.label(imgs)
    ref.close()
    for got in (local, remote):
        p_got = np.sort([r[0][0] for r in got])
        p_want = np.sort([r[0][0] for r in want])
        assert np.abs(p_got - p_want).max() < 0.01, (p_got, p_want)
        lab_got = sorted(r[0][1] for r in got)
        lab_want = sorted(r[0][1] for r in want)
        common = sum(min(lab_got.count(x), lab_want.count(x)) for x in set(lab_want))
        assert common >= 36, (lab_got, lab_want)
    top1 = lambda res: sorted(r[0][1] for r in res)  # noqa: E731 - each result: top-k (prob, label)
    assert top1(remote) == top1(local)


@pytest.mark.gpu
def test_remote_batched_resnet_gpu():
    """Two ResNet subtasks, first as two threads of one process (each with its own runner,
    arena and captured plans: the start barrier keeps every capture ahead of the first
    replay), then as worker processes sharing the box's GPU (one per GPU on a node); both
    checked against the fp32 interpreter.  Runs in a child process (a native abort fails
    this test with every thread's stack, not the suite)."""
    from _helpers import run_isolated

    run_isolated("test_remote:_two_gpu_subtasks_resnet", timeout=300)


def _digest(v):
    import numpy as np
    import torch

    from flink_tensorflow_amd.types.tensor_value import TensorValue

    if isinstance(v, TensorValue):
        return ("tv", int(np.asarray(v.to_numpy()).astype(np.int64).sum()), v.shape())
    if isinstance(v, torch.Tensor):
        return ("torch", int(v.to(torch.int64).sum()), tuple(v.shape))
    root = v
    while isinstance(root, np.ndarray) and root.base is not None:
        root = root.base
    return ("np", int(v.astype(np.int64).sum()), tuple(v.shape), type(root).__name__)


def test_tensor_slab_transport_round_trip(monkeypatch):
    """Large ndarray / CPU-tensor / TensorValue records cross to worker processes through the
    shared-memory tensor slab (written once, zero-copy views in the worker) and arrive
    intact; small records ride in the pickle."""
    import numpy as np
    import torch

    from flink_tensorflow_amd.types.tensor_value import TensorValue

    rng = np.random.default_rng(0)
    vals = []
    for i in range(60):
        k = i % 4
        if k == 0:
            vals.append(rng.integers(0, 256, (64, 64, 3), dtype=np.uint8))
        elif k == 1:
            vals.append(torch.from_numpy(rng.standard_normal((32, 64)).astype(np.float32)))
        elif k == 2:
            a = rng.integers(0, 100, (40, 40), dtype=np.int32)
            vals.append(TensorValue("INT32", a.shape, a))
        else:
            vals.append(np.arange(8, dtype=np.int64))  # below the slab threshold
    want = sorted(map(repr, (_digest(v)[:3] for v in vals)))
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(2)
    got = env.from_collection(vals).map(_digest).run_in_processes().execute_and_collect()
    assert sorted(map(repr, (g[:3] for g in got))) == want
    # worker-side ndarrays of slab records are views of the shared mapping (zero copy)
    assert any(g[0] == "np" and g[3] == "memoryview" for g in got)


def _window_sum(vals):
    return int(sum(int(v.astype("int64").sum()) for v in vals))


class _WinSum:
    def apply(self, window, inputs, out):
        out.collect(_window_sum(inputs))


def test_tensor_slab_full_falls_back_to_pickle(monkeypatch):
    """A worker operator that holds more payload than the slab (a count window of 40 x
    196 KB records over a 4 MB slab) still gets every record: the coordinator waits briefly,
    then pickles."""
    import numpy as np

    from flink_tensorflow_amd.runtime import remote

    monkeypatch.setattr(remote, "_SLAB_BYTES", 4 << 20)
    rng = np.random.default_rng(1)
    vals = [rng.integers(0, 256, (256, 256, 3), dtype=np.uint8) for _ in range(40)]
    env = StreamExecutionEnvironment.get_execution_environment()
    got = env.from_collection(vals).count_window_all(40).apply(_WinSum()).run_in_processes().execute_and_collect()
    assert got == [sum(int(v.astype(np.int64).sum()) for v in vals)]


class _KeepDerived:
    """Keeps only DERIVED views of every record (``reshape(-1)``, a column slice) and,
    every 25th record, returns the checksum over everything kept so far."""

    def __init__(self):
        self.kept = []

    def __call__(self, v):
        self.kept.append(v.reshape(-1))
        self.kept.append(v[:, 0])
        if len(self.kept) % 50:
            return None
        return int(sum(int(k.astype("int64").sum()) for k in self.kept))


def test_tensor_slab_keeps_records_alive_through_derived_views(monkeypatch):
    """An operator that stores only views derived from slab records (not the records
    themselves) must still see their bytes intact after later batches wrap the slab."""
    import numpy as np

    from flink_tensorflow_amd.runtime import remote

    monkeypatch.setattr(remote, "_SLAB_BYTES", 4 << 20)
    rng = np.random.default_rng(2)
    vals = [rng.integers(0, 256, (64, 64, 4), dtype=np.uint8) for _ in range(400)]  # 16 KB: 6.4 MB in all
    want, acc = [], 0
    for i, v in enumerate(vals):
        acc += int(v.astype(np.int64).sum()) + int(v[:, 0].astype(np.int64).sum())
        want.append(acc if (i + 1) % 25 == 0 else None)
    env = StreamExecutionEnvironment.get_execution_environment()
    got = env.from_collection(vals).map(_KeepDerived()).run_in_processes().execute_and_collect()
    assert got == want


def _own_partition(n, delay_s=0.0):
    def gen(idx, par, start):
        import time as _t

        for v in [i for i in range(1, n + 1) if i % par == idx][start:]:
            if delay_s:
                _t.sleep(delay_s)
            yield v
    return gen


def test_remote_source_chain_runs_in_workers():
    """A worker-process source with its worker-process map chained into the same process:
    records are produced and mapped in the workers (never through the coordinator); only
    the map's output comes back."""
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(2)
    out = env.generate(_own_partition(400)).run_in_processes() \
        .map(lambda v: (os.getpid(), v * 3)).run_in_processes().execute_and_collect()
    assert sorted(v for _, v in out) == [3 * i for i in range(1, 401)]
    pids = {p for p, _ in out}
    assert len(pids) == 2 and os.getpid() not in pids


def test_remote_source_chain_checkpoint_restart(tmp_path):
    """Checkpoints of a worker-process source chain: triggers reach the worker, which
    snapshots the source offset and the chained operators between two records and sends
    the barrier inline; after a failure inside the chain the job restarts from the last
    checkpoint and every keyed running sum downstream is exact (no record lost or
    duplicated)."""
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(2)
    env.enable_checkpointing(0.05, str(tmp_path / "chk"))
    env.set_restart_strategy(RestartStrategy.fixed_delay(2, 0.0))
    sink = env.generate(_own_partition(300, delay_s=0.002)).run_in_processes() \
        .map(FailAfter(100, attempts=(0,))).run_in_processes() \
        .key_by(lambda v: v % 3).process(_RunningSum()).collect_into()
    res = env.execute("remote-source-recover")
    assert res.attempts == 1 and len(res.checkpoints) >= 1
    final = {}
    for k, t in sink.results():
        final[k] = max(final.get(k, 0), t)
    assert final == {k: sum(v for v in range(1, 301) if v % 3 == k) for k in range(3)}


def test_tensor_slab_view_batch_releases_with_the_last_view():
    """The worker maps a message's slab records as slices of one base array: contents and
    dtypes round-trip, a surviving derived view of ANY record holds the whole span, and the
    span is released (header advanced) once the last view is gone."""
    import gc

    import numpy as np

    from flink_tensorflow_amd.runtime.remote import TensorSlab

    tag = f"/ftm-vb-{os.getpid()}"
    co = TensorSlab(tag, True, 1 << 22)
    wk = TensorSlab(tag, False)
    try:
        rng = np.random.default_rng(3)
        vals = [rng.integers(0, 256, (64, 96), dtype=np.uint8), rng.standard_normal((33, 65)).astype(np.float32),
                rng.integers(-999, 999, (7, 301), dtype=np.int16)]
        out = co.put_batch([(v, None, 0) for v in vals])
        arrs = wk.view_batch([r for r, _, _ in out])
        for a, v in zip(arrs, vals):
            assert a.dtype == v.dtype and a.shape == v.shape and np.array_equal(a, v)
        keep = arrs[2][3:, ::2]  # a view derived from the LAST record only
        del a, arrs
        gc.collect()
        assert int(wk.hdr[0]) == 0  # still held by the derived view
        del keep
        gc.collect()
        assert int(wk.hdr[0]) == out[-1][0][3]  # the whole span released
    finally:
        wk.close()
        co.unlink()
        co.close()


def _slow_stamped(n, gap_s):
    def gen(idx, par, start):
        import time as _t

        for i in [i for i in range(n) if i % par == idx][start:]:
            _t.sleep(gap_s)
            yield (i, _t.time())
    return gen


def _stamp_batch(model, vals):
    import time as _t

    now = _t.time()
    return [(i, now - t) for i, t in vals]


def test_worker_source_chain_timer_fires_deadlines(tmp_path):
    """A worker-process source that blocks between records (longer than the micro-batch
    ``max_delay``): the worker's chain timer still flushes every partial batch on its
    deadline (latency ~ max_delay, not the source's gap) and checkpoints still complete
    while the source sleeps."""
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(1)
    env.enable_checkpointing(0.05, str(tmp_path / "chk"))
    sink = env.generate(_slow_stamped(8, 0.25)).run_in_processes() \
        .map_with_model_batched(object(), _stamp_batch, max_batch=64, max_delay_ms=5).run_in_processes() \
        .collect_into()
    res = env.execute("slow-worker-source")
    out = sorted(sink.results())
    assert [i for i, _ in out] == list(range(8))
    assert max(lat for _, lat in out) < 0.15, out  # without the timer: ~0.25 s (the next record)
    assert len(res.checkpoints) >= 2


class _DeviceProbe:
    """A model that is a RichFunction: the batched operator hands it the runtime context."""

    def set_runtime_context(self, ctx):
        self.ctx = ctx


def _device_of(model, vals):
    import torch

    c = model.ctx
    want = torch.device("cuda", c.subtask_index % torch.cuda.device_count())
    return [(c.subtask_index, str(c.device), str(want), str(torch.cuda.current_device())) for _ in vals]


@pytest.mark.gpu
def test_worker_source_chain_binds_gpu_member_device():
    """In a worker-process source chain the source node itself uses no GPU: the chained GPU
    operator still gets ``ctx.device = cuda:(subtask % gpus)`` and the worker's current
    device is set to it (the device used to come from the source's spec)."""
    from flink_tensorflow_amd.runtime import functions as F

    class Probe(_DeviceProbe, F.RichFunction):
        pass

    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(2)
    out = env.generate(_own_partition(20)).run_in_processes() \
        .map_with_model_batched(Probe(), _device_of, max_batch=4, max_delay_ms=2).run_in_processes() \
        .execute_and_collect()
    assert len(out) == 20
    for sub, dev, want, cur in out:
        assert dev == want and dev.endswith(":" + cur), (sub, dev, want, cur)


def _pid_records(n):
    def gen(idx, par, start):
        import os as _os

        for i in [i for i in range(n) if i % par == idx][start:]:
            yield (_os.getpid(), i)
    return gen


def test_splittable_source_relocates_into_its_worker_consumer():
    """A generator source feeding (rebalance) a worker-process map of equal parallelism runs
    inside the workers, chained with the map: every record is produced in the process that
    maps it, none crosses the coordinator.  ``relocate_sources = False`` keeps the old
    layout (produced in the coordinator, shipped to the workers)."""
    from flink_tensorflow_amd.runtime.executor import LocalExecutor

    for relocate in (True, False):
        env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(2)
        env.relocate_sources = relocate
        sink = env.generate(_pid_records(300)).rebalance().map(lambda r: (r[0], os.getpid(), r[1])) \
            .run_in_processes().collect_into()
        ex = LocalExecutor(env, "relocate")
        ex.execute()
        out = sink.results()
        assert sorted(v for _, _, v in out) == list(range(300))
        if relocate:
            assert ex.relocated == ["generator"]
            assert all(src == mapper != os.getpid() for src, mapper, _ in out)
        else:
            assert ex.relocated == [] and {src for src, _, _ in out} == {os.getpid()}
