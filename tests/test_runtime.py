"""Streaming runtime: the reference's ITCases ported onto the local executor, plus the
function kinds, windows, keyed state, co-processing, checkpoints and restarts that the
reference declares but never tests."""
import os
import time

import pytest
import torch

from flink_tensorflow_amd.models import RegressionMethod, TensorFlowModel
from flink_tensorflow_amd.runtime import (PROCESS_ONCE, BytesInputFormat, CheckpointedFunction, CountWindows,
                                          ListStateDescriptor, MemorySink, ModelAllWindowFunction,
                                          ModelCoProcessFunction, ModelFlatMapFunction, ModelProcessFunction,
                                          ModelWindowFunction, OutputTag, ProcessFunction, RestartStrategy,
                                          RichFlatMapFunction, StreamExecutionEnvironment, ValueStateDescriptor,
                                          register_types)
from flink_tensorflow_amd.types import example, feature
from flink_tensorflow_amd.utils.fault import FailAfter


class HalfPlusTwo(TensorFlowModel):
    def __init__(self, path):
        super().__init__(device="cpu")
        self._loader = TensorFlowModel.load(path, "serve")

    @property
    def loader(self):
        return self._loader

    def regress_x_to_y(self, exs):
        return self.function("regress_x_to_y", RegressionMethod()).apply(exs)


def examples():
    return [(example(("x", feature(float(v)))), 0.5 * v + 2.0) for v in range(4)]


class _RegressFlatMap(RichFlatMapFunction):
    """RegressITCase's in-operator check (``TST/.../ml/RegressITCase.scala:46-62``)."""

    def __init__(self, model):
        super().__init__()
        self.model = model

    def open(self, config=None):
        self.model.open()

    def close(self):
        self.model.close()

    def flat_map(self, value, out):
        ex, expected = value
        y = self.model.regress_x_to_y([ex]).reshape(-1).tolist()
        assert y == [expected], (y, expected)
        out.collect(y[0])


@pytest.mark.parametrize("parallelism", [1, 4])
def test_regress_itcase(half_plus_two, parallelism):
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(parallelism)
    register_types(env.get_config())
    sink = env.from_collection(examples()).rebalance().flat_map(_RegressFlatMap(HalfPlusTwo(half_plus_two))) \
        .collect_into()
    res = env.execute("regress")
    assert sorted(sink.results()) == [2.0, 2.5, 3.0, 3.5]
    assert res.attempts == 0


def test_map_with_model(half_plus_two):
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(2)
    out = env.from_collection(examples()).rebalance() \
        .map_with_model(HalfPlusTwo(half_plus_two), lambda v, m: m.regress_x_to_y([v[0]]).item()) \
        .execute_and_collect()
    assert sorted(out) == [2.0, 2.5, 3.0, 3.5]
    with pytest.raises(ValueError):
        env.from_collection([1]).map_with_model(None, lambda v, m: v)


class _Proc(ModelProcessFunction):
    def process_element(self, value, ctx, out):
        out.collect(self.model.regress_x_to_y([value[0]]).item())


class _Co(ModelCoProcessFunction):
    def process_element1(self, value, ctx, out):
        out.collect(("data", self.model.regress_x_to_y([value[0]]).item()))

    def process_element2(self, value, ctx, out):
        out.collect(("control", value))


class _Win(ModelWindowFunction):
    def apply(self, key, window, inputs, out):
        ys = self.model.regress_x_to_y([v[0] for v in inputs]).reshape(-1).tolist()
        out.collect((key, sorted(ys)))


class _AllWin(ModelAllWindowFunction):
    def apply(self, window, inputs, out):
        out.collect(sorted(self.model.regress_x_to_y([v[0] for v in inputs]).reshape(-1).tolist()))


class _FM(ModelFlatMapFunction):
    def flat_map(self, value, out):
        out.collect(self.model.regress_x_to_y([value[0]]).item())


def test_all_six_model_function_kinds(half_plus_two):
    """The reference's Abstract{Process,CoProcess,Window,AllWindow}Function crash with
    MatchError for non-CheckpointedModels (B6); here all six kinds run."""
    m = HalfPlusTwo(half_plus_two)
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(2)
    s = env.from_collection(examples())
    checkpoint_dir = None
    del checkpoint_dir
    r_map = s.map_with_model(m, lambda v, mm: mm.regress_x_to_y([v[0]]).item()).collect_into()
    r_fm = s.flat_map(_FM(m)).collect_into()
    r_proc = s.process(_Proc(m)).collect_into()
    r_co = s.connect(env.from_collection(["reload"])).process(_Co(m)).collect_into()
    r_win = s.key_by(lambda v: int(v[1] * 2) % 2).count_window(2).apply(_Win(m)).collect_into()
    r_all = s.count_window_all(4).apply(_AllWin(m)).collect_into()
    env.execute("six-kinds")
    want = [2.0, 2.5, 3.0, 3.5]
    assert sorted(r_map.results()) == want
    assert sorted(r_fm.results()) == want
    assert sorted(r_proc.results()) == want
    co = r_co.results()
    assert sorted(v for k, v in co if k == "data") == want and ("control", "reload") in co
    assert sorted(r_win.results()) == [(0, [2.0, 3.0]), (1, [2.5, 3.5])]
    assert r_all.results() == [want]


class _CountPerKey(ProcessFunction):
    def open(self, config=None):
        self.count = self.get_runtime_context().get_state(ValueStateDescriptor("n", 0))

    def process_element(self, value, ctx, out):
        self.count.update(self.count.value() + 1)
        out.collect((ctx.get_current_key(), self.count.value()))
        if value % 5 == 0:
            ctx.output(OutputTag("fives"), value)


def test_keyed_state_and_side_output():
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(3)
    main = env.from_collection(list(range(30))).key_by(lambda v: v % 3).process(_CountPerKey())
    side = main.get_side_output(OutputTag("fives")).collect_into()
    res = main.collect_into()
    env.execute("keyed")
    last = {}
    for k, c in res.results():
        last[k] = max(last.get(k, 0), c)
    assert last == {0: 10, 1: 10, 2: 10}
    assert sorted(side.results()) == [0, 5, 10, 15, 20, 25]


def test_event_time_windows_and_watermarks():
    from flink_tensorflow_amd.runtime import WindowFunction

    class Sum(WindowFunction):
        def apply(self, key, window, inputs, out):
            out.collect((key, window.start, sum(v[1] for v in inputs)))

    data = [("a", 1, 0.5), ("a", 2, 1.5), ("b", 3, 0.7), ("a", 4, 2.2), ("b", 5, 2.9), ("a", 6, 1.9)]
    env = StreamExecutionEnvironment.get_execution_environment()
    res = (env.from_collection(data).assign_timestamps_and_watermarks(lambda v: v[2], 1.0)
           .key_by(lambda v: v[0]).time_window(1.0, event_time=True).apply(Sum()).execute_and_collect())
    assert sorted(res) == [("a", 0.0, 1), ("a", 1.0, 8), ("a", 2.0, 4), ("b", 0.0, 3), ("b", 2.0, 5)]


def test_file_source_zero_length_and_filters(tmp_path):
    for name, data in [("a.jpg", b"x" * 10), ("b.jpeg", b""), ("c.crdownload", b"y"), ("d.txt", b"z")]:
        (tmp_path / name).write_bytes(data)
    fmt = BytesInputFormat(include=["*.jpg"]).configure(include=["*.jpeg"], exclude=["*.crdownload"])
    env = StreamExecutionEnvironment.get_execution_environment()
    out = env.read_file(fmt, str(tmp_path), PROCESS_ONCE).map(lambda v: (os.path.basename(v[0]), len(v[1]))) \
        .execute_and_collect()
    assert sorted(out) == [("a.jpg", 10), ("b.jpeg", 0)]  # zero-length file emitted exactly once (B5)


class _Summer(ProcessFunction, CheckpointedFunction):
    def __init__(self):
        super().__init__()
        self.total = 0

    def initialize_state(self, ctx):
        self.st = ctx.operator_state.get_list_state(ListStateDescriptor("total"))
        if ctx.is_restored():
            self.total = sum(self.st.get())

    def snapshot_state(self, ctx):
        self.st.update([self.total])

    def process_element(self, value, ctx, out):
        self.total += value
        out.collect(self.total)


def test_checkpoint_and_restart_from_latest(tmp_path):
    """Fail on the first attempt after a checkpoint completed; the restarted job rewinds
    the source to the checkpointed offset and restores operator state."""
    env = StreamExecutionEnvironment.get_execution_environment()
    env.enable_checkpointing(0.05, str(tmp_path / "chk"))
    env.set_restart_strategy(RestartStrategy.fixed_delay(2, 0.0))
    from flink_tensorflow_amd.runtime.sources import CollectionSource

    src = env.add_source(CollectionSource(list(range(1, 201)), delay_s=0.002), "numbers")
    sink = src.map(FailAfter(150, attempts=(0,))).process(_Summer()).collect_into()
    res = env.execute("recover")
    assert res.attempts == 1
    assert len(res.checkpoints) >= 1
    assert max(sink.results()) == sum(range(1, 201))  # state + offsets restored consistently
    from flink_tensorflow_amd.runtime.checkpoint import CheckpointStorage

    assert CheckpointStorage(str(tmp_path / "chk")).latest() is not None


def test_failure_without_restart_raises():
    from flink_tensorflow_amd.runtime import JobExecutionException

    env = StreamExecutionEnvironment.get_execution_environment()
    env.from_collection(list(range(10))).map(FailAfter(3)).collect_into()
    with pytest.raises(JobExecutionException):
        env.execute("boom")


def test_batched_model_operator(half_plus_two):
    env = StreamExecutionEnvironment.get_execution_environment()

    def run_batch(model, values):
        return model.regress_x_to_y([v[0] for v in values]).reshape(-1).tolist()

    sink = env.from_collection(examples() * 25).map_with_model_batched(HalfPlusTwo(half_plus_two), run_batch,
                                                                       max_batch=16, max_delay_ms=2).collect_into()
    res = env.execute("batched")
    out = sink.results()
    assert len(out) == 100 and sorted(set(out)) == [2.0, 2.5, 3.0, 3.5]
    hist = [m for k, m in res.metrics.items() if k.startswith("batched-model")][0]["histograms"]["batch_size"]
    assert hist["max"] == 16


class _OnlineA(ModelCoProcessFunction):
    """Data stream: y = a*x + b through the regress signature.  Update stream: assigns a
    new value to the SavedModel variable ``a`` with the graph's own ``a/Assign`` op."""

    def process_element1(self, x, ctx, out):
        y = self.model.regress_x_to_y([example(("x", feature(float(x))))]).item()
        out.collect((x, y))

    def process_element2(self, a, ctx, out):
        self.model.session().run(targets=["a/Assign"], feed_dict={"a/initial_value:0": torch.tensor(a)})


class _UncheckpointedHalfPlusTwo(HalfPlusTwo):
    def snapshot_state(self, ctx):  # control: variables are NOT part of the checkpoint
        pass


@pytest.mark.parametrize("checkpointed", [True, False])
def test_savedmodel_variables_survive_worker_kill(half_plus_two, tmp_path, checkpointed):
    """TensorFlowModel is a CheckpointedModel (``CheckpointedModel.scala:24-46``):
    an update stream assigns ``a = 3`` once; a worker process is killed mid-stream; after the
    restart (the update record is not replayed — its source offset was checkpointed) the
    late records are still computed with the restored ``a``.  The control run, whose model
    does not snapshot its variables, falls back to the SavedModel's ``a = 0.5``."""
    from flink_tensorflow_amd.runtime.sources import CollectionSource
    from flink_tensorflow_amd.utils.fault import KillProcessAfter

    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(1)
    env.enable_checkpointing(0.05, str(tmp_path / "chk"))
    env.set_restart_strategy(RestartStrategy.fixed_delay(2, 0.0))
    data = env.add_source(CollectionSource(list(range(1, 201)), delay_s=0.004), "xs")
    updates = env.add_source(CollectionSource([3.0]), "updates")
    m = (HalfPlusTwo if checkpointed else _UncheckpointedHalfPlusTwo)(half_plus_two)
    sink = data.map(KillProcessAfter(120)).run_in_processes().connect(updates).process(_OnlineA(m)).collect_into()
    res = env.execute("online-a")
    assert res.attempts == 1 and len(res.checkpoints) >= 1
    late = {x: y for x, y in sink.results() if x >= 150}   # only computed after the restart
    assert sorted(late) == list(range(150, 201))
    a = 3.0 if checkpointed else 0.5
    assert all(y == pytest.approx(a * x + 2.0) for x, y in late.items()), sorted(late.items())[:3]


# ------------------------------------------------------------------ operator chaining
def _chain_job(**marks):
    env = StreamExecutionEnvironment.get_execution_environment()
    s = env.from_collection(list(range(1000))).map(lambda x: x + 1).name("inc")
    s = s.filter(lambda x: x % 2 == 0).name("even")
    if marks.get("new_chain"):
        s = s.start_new_chain()
    if marks.get("no_chain"):
        s = s.disable_chaining()
    s = s.map(lambda x: x * 10).name("x10")
    return env, s.collect_into()


def test_operator_chaining_forms_chains_and_keeps_per_operator_metrics():
    """Forward-connected operators with equal parallelism run in one subtask thread (Flink's
    operator chaining); each keeps its own metrics, and the result is unchanged."""
    from flink_tensorflow_amd.runtime.executor import LocalExecutor

    env, sink = _chain_job()
    ex = LocalExecutor(env, "chained")
    res = ex.execute()
    assert ex.chains == [["collection", "inc", "even", "x10", "collect"]]  # the source heads the chain
    assert sum(t.thread is not None for t in ex.tasks) == 1   # one thread runs the whole job
    assert sink.results() == [10 * x for x in range(2, 1001, 2)]
    assert res.metrics["x10[0]"]["counters"]["records_in"] == 500


@pytest.mark.parametrize("mark,chains", [("new_chain", [["collection", "inc"], ["even", "x10", "collect"]]),
                                         ("no_chain", [["collection", "inc"], ["x10", "collect"]]),  # "even" alone
                                         ("env_off", [])])
def test_chaining_controls(mark, chains):
    from flink_tensorflow_amd.runtime.executor import LocalExecutor

    env, sink = _chain_job(**{mark: True})
    if mark == "env_off":
        env.disable_operator_chaining()
    ex = LocalExecutor(env, mark)
    ex.execute()
    assert ex.chains == chains
    assert sink.results() == [10 * x for x in range(2, 1001, 2)]


def test_source_chain_flushes_micro_batches_while_the_source_is_idle():
    """A micro-batching operator chained into its source still honours ``max_delay_ms``
    while the source function sleeps between records (the chain timer flushes it), and a
    checkpoint taken mid-stream acks the source and every chain member."""
    from flink_tensorflow_amd.runtime.executor import LocalExecutor
    from flink_tensorflow_amd.runtime.functions import SourceFunction

    class Bursty(SourceFunction):
        def run(self, ctx):
            for burst in range(3):
                with ctx.checkpoint_lock:
                    for i in range(3):
                        ctx.collect(burst * 3 + i)
                time.sleep(0.25)  # far longer than max_delay: the batch must not wait for this

    def run_batch(model, vals):  # (value, batch contents, flush time); the function is cloned
        t = time.perf_counter()
        return [(v * 2, tuple(vals), t) for v in vals]

    env = StreamExecutionEnvironment.get_execution_environment()
    sink = env.add_source(Bursty(), "bursty").map_with_model_batched(
        object(), run_batch, max_batch=64, max_delay_ms=5, name="batched").collect_into()
    ex = LocalExecutor(env, "idle-flush")
    t0 = time.perf_counter()
    ex.execute()
    assert ex.chains == [["bursty", "batched", "collect"]]
    out = sink.results()
    assert sorted(v for v, _, _ in out) == [2 * i for i in range(9)]
    batches = sorted({(t, b) for _, b, t in out})
    assert [b for _, b in batches] == [(0, 1, 2), (3, 4, 5), (6, 7, 8)]
    # each burst was flushed by the timer long before the next burst arrived
    assert batches[0][0] - t0 < 0.2 and batches[1][0] - batches[0][0] < 0.45


def test_key_by_and_fan_out_break_chains():
    from flink_tensorflow_amd.runtime.executor import LocalExecutor

    env = StreamExecutionEnvironment.get_execution_environment()
    base = env.from_collection(list(range(100))).map(lambda x: x).name("id")
    a = base.map(lambda x: x + 1).name("a").collect_into()          # fan-out: "id" has two consumers
    b = base.key_by(lambda x: x % 3).map(lambda x: x).name("k").collect_into()
    ex = LocalExecutor(env, "fanout")
    ex.execute()
    assert ["id", "a"] not in ex.chains and all(c[0] != "id" for c in ex.chains)
    assert len(a.results()) == 100 and len(b.results()) == 100


def test_bulk_generator_feeds_a_chained_micro_batcher_in_order():
    """``env.generate(factory, bulk=True)``: the factory yields runs of records; a chained
    micro-batching operator in the worker takes each run at once (``process_many``) and
    forms the same batches, in the same order, as record-at-a-time emission; ``limit``
    counts records, not runs."""
    from flink_tensorflow_amd.runtime import StreamExecutionEnvironment

    def gen(idx, par, start):
        for i in range(start, 100, 7):
            yield list(range(i, min(i + 7, 100)))

    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(1)
    out = env.generate(gen, bulk=True, limit=90).run_in_processes() \
        .map_with_model_batched(object(), lambda m, recs: [r * 2 for r in recs], max_batch=16, max_delay_ms=50,
                                name="x2").run_in_processes().execute_and_collect()
    assert out == [2 * i for i in range(90)]
