"""Data parallelism inside ONE streaming job (SURVEY §2.12 "one subtask per GPU, rank 0
loads, RCCL broadcast"): the P worker-process subtasks of a GPU operator form one
communicator (``LocalExecutor.operator_group`` → ``runtime/remote.py::_open_group``).

Reference: parallel subtasks are the reference's execution model
(``flink-tensorflow-examples/.../inception/inception.scala:22-23``); there every subtask
reads the model itself (``DefaultSavedModelLoader.scala:40-56``).  Here only subtask 0
reads the variables and the others receive them; CPU tests inject the loopback
communicator, the GPU test runs through RCCL."""
import os

import pytest
import torch

from flink_tensorflow_amd.models.savedmodel import DefaultSavedModelLoader, TensorFlowModel
from flink_tensorflow_amd.runtime import StreamExecutionEnvironment


class _RecordingLoader(DefaultSavedModelLoader):
    """Marks, per process, whether it read the variables from the bundle."""

    def __init__(self, path, marks):
        super().__init__(path, ("serve",))
        self.marks = marks

    def load(self, device=None, read_variables: bool = True):
        if read_variables:
            open(os.path.join(self.marks, f"read-{os.getpid()}"), "w").close()
        return super().load(device=device, read_variables=read_variables)


class _HalfPlusTwo(TensorFlowModel):
    def __init__(self, path, marks, distributed=True):
        super().__init__(None, distributed_weights=distributed)
        self._loader = _RecordingLoader(path, marks)

    @property
    def loader(self):
        return self._loader


def _variables_of(value, model):
    from flink_tensorflow_amd.parallel import comm

    vs = model.session().variables
    return (os.getpid(), comm.rank_size(), {k: float(vs[k].reshape(-1)[0]) for k in ("a", "b", "c")}, value)


def test_p4_job_reads_once_and_broadcasts(tmp_path, half_plus_two):
    """A P=4 job of worker-process model subtasks: only subtask 0 reads the bundle's
    variables; all four serve bit-identical values after the in-job broadcast."""
    from flink_tensorflow_amd.parallel.fake import FakeCommunicator

    marks = tmp_path / "marks"
    marks.mkdir()
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(4)
    env.enable_job_communicator(True, communicator=FakeCommunicator)
    model = _HalfPlusTwo(half_plus_two, str(marks))
    out = env.from_collection(list(range(40))).rebalance().map_with_model(model, _variables_of) \
        .run_in_processes().execute_and_collect()
    assert sorted(o[3] for o in out) == list(range(40))
    pids = {o[0] for o in out}
    assert len(pids) == 4 and os.getpid() not in pids
    assert {o[1] for o in out} == {(r, 4) for r in range(4)}  # every subtask is a rank of one group
    assert {tuple(o[2].items()) for o in out} == {(("a", 0.5), ("b", 2.0), ("c", 3.0))}
    readers = [f for f in os.listdir(marks)]
    assert len(readers) == 1, readers  # subtask 0 only


def test_no_group_without_enough_gpus_or_for_host_operators(tmp_path, half_plus_two):
    """Without an injected communicator the group is formed only when the node has a GPU
    per subtask: on this host the subtasks run without one (each reads its own model)."""
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(2)
    marks = tmp_path / "marks"
    marks.mkdir()
    out = env.from_collection(list(range(10))).rebalance().map_with_model(_HalfPlusTwo(half_plus_two, str(marks)),
                                                                          _variables_of) \
        .run_in_processes().execute_and_collect()
    if torch.cuda.device_count() < 2:
        assert {o[1] for o in out} == {(0, 1)} and len(os.listdir(marks)) == 2


def test_auto_mode_forms_a_group_only_for_collective_operators(tmp_path, half_plus_two):
    """The default "auto" job communicator: a P=2 inference operator without
    ``distributed_weights`` opens no communicator (each subtask reads its model); the same
    operator with ``distributed_weights=True`` forms one group of 2."""
    from flink_tensorflow_amd.parallel.fake import FakeCommunicator

    for distributed, want_ranks, want_reads in ((False, {(0, 1)}, 2), (True, {(0, 2), (1, 2)}, 1)):
        marks = tmp_path / f"marks{int(distributed)}"
        marks.mkdir()
        env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(2)
        env.enable_job_communicator("auto", communicator=FakeCommunicator)
        model = _HalfPlusTwo(half_plus_two, str(marks), distributed=distributed)
        out = env.from_collection(list(range(12))).rebalance().map_with_model(model, _variables_of) \
            .run_in_processes().execute_and_collect()
        assert {o[1] for o in out} == want_ranks, distributed
        assert len(os.listdir(marks)) == want_reads, distributed


def _rccl_probe(value, model):
    from flink_tensorflow_amd.parallel import comm

    c = comm.get()
    t = torch.full((4,), float(c.rank + 1), device=c.device)
    c.all_reduce(t)
    return (type(c).__name__, c.size, str(c.device), float(t[0].item()),
            float(model.session().variables["a"].reshape(-1)[0]))


@pytest.mark.gpu
def test_p1_job_communicator_runs_through_rccl_gpu(tmp_path, half_plus_two):
    """P = 1 with the job communicator on: the worker subtask opens an RCCL communicator on
    its GPU, the distributed-weights open goes through it, and an all-reduce works."""
    marks = tmp_path / "marks"
    marks.mkdir()
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(1)
    env.enable_job_communicator(True)
    model = _HalfPlusTwo(half_plus_two, str(marks))
    model.device = torch.device("cuda", 0)
    out = env.from_collection(list(range(3))).map_with_model(model, _rccl_probe).run_in_processes() \
        .execute_and_collect()
    assert out and all(o == ("RcclCommunicator", 1, "cuda:0", 1.0, 0.5) for o in out), out
    assert len(os.listdir(marks)) == 1


class _DPTrainer:
    """A co-process online trainer (the reference's ``AbstractCoProcessFunction`` home of
    training) run as P worker-process subtasks of one job: full micro-batches only, so every
    subtask takes the same number of steps (each step is collective: dense all-reduce, the
    owner sparse exchange); at the end of input it emits a digest of its replica."""

    @staticmethod
    def make(batch):
        from flink_tensorflow_amd.models.zoo.wide_deep import WideDeepConfig, WideDeepTrainer
        from flink_tensorflow_amd.runtime.model_functions import ModelCoProcessFunction

        class Fn(ModelCoProcessFunction):
            def __init__(self):
                super().__init__(WideDeepTrainer(WideDeepConfig.tiny(), device="cpu", seed=3))
                self.buf, self.steps = [], 0

            def process_element1(self, rec, ctx, out):
                if self.steps == 0 and not self.buf:
                    ctx.timer_service().register_event_time_timer(float("inf"))
                self.buf.append(rec)
                if len(self.buf) == batch:
                    self.model.train_step(self.buf)
                    self.buf, self.steps = [], self.steps + 1

            def process_element2(self, tick, ctx, out):
                pass

            def on_timer(self, ts, ctx, out):
                import hashlib

                from flink_tensorflow_amd.parallel import comm

                m, ex = self.model.model, self.model._exchange
                parts = [p.detach().reshape(-1) for p in m.dense_parameters()]
                for e in (m.emb, m.wide):
                    parts.append((ex.merge_owner_shards(e.table.data) if ex is not None else e.table.data).reshape(-1))
                digest = hashlib.sha256(torch.cat(parts).numpy().tobytes()).hexdigest()[:16]
                out.collect((comm.rank_size(), self.steps, digest))

        return Fn()


def test_online_training_dp_inside_one_job(tmp_path):
    """Wide&Deep online training in a ``ModelCoProcessFunction`` with parallelism 2 in
    worker processes: the subtasks form the job communicator (loopback here, RCCL on a
    node), start from rank 0's weights, all-reduce dense gradients and exchange sparse rows
    by owner — both replicas end bit-identical after training on different records."""
    from flink_tensorflow_amd.models.zoo.wide_deep import WideDeepConfig, synthetic_click_records
    from flink_tensorflow_amd.parallel.fake import FakeCommunicator
    from flink_tensorflow_amd.runtime.sources import CollectionSource

    recs = synthetic_click_records(2 * 4 * 64, WideDeepConfig.tiny(), seed=11)
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(2)
    env.enable_job_communicator(True, communicator=FakeCommunicator)
    clicks = env.add_source(CollectionSource(recs), "clicks", parallelism=1).rebalance()
    ticks = env.add_source(CollectionSource([]), "control", parallelism=1)
    out = clicks.connect(ticks).process(_DPTrainer.make(64)).name("trainer").run_in_processes().execute_and_collect()
    assert sorted(o[0] for o in out) == [(0, 2), (1, 2)]
    assert [o[1] for o in out] == [4, 4]
    assert out[0][2] == out[1][2]
