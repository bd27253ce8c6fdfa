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


def _group_of(value, model):
    from flink_tensorflow_amd.parallel import comm

    return tuple(value) + ((os.getpid(), id(comm.get()), comm.rank_size()),)


def test_two_grouped_operators_chained_in_one_worker_keep_their_own_groups(tmp_path, half_plus_two):
    """A worker-process source chained with TWO ``distributed_weights`` model operators:
    one worker process per subtask runs all three, and each model operator sees its own
    communicator (one group per operator, bound around that operator's calls), both of
    world size 2."""
    from flink_tensorflow_amd.parallel.fake import FakeCommunicator

    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(2)
    env.enable_job_communicator(True, communicator=FakeCommunicator)
    marks = [tmp_path / "m1", tmp_path / "m2"]
    for m in marks:
        m.mkdir()
    src = env.generate(lambda idx, par, start: ((idx, i) for i in range(start, 6))).run_in_processes()
    a = src.map_with_model(_HalfPlusTwo(half_plus_two, str(marks[0])), _group_of, name="first").run_in_processes()
    b = a.map_with_model(_HalfPlusTwo(half_plus_two, str(marks[1])), _group_of, name="second").run_in_processes()
    out = b.execute_and_collect()
    assert len(out) == 12
    for rec in out:
        (pid1, g1, rs1), (pid2, g2, rs2) = rec[-2], rec[-1]
        assert pid1 == pid2 != os.getpid()  # chained into one worker process
        assert g1 != g2  # two communicators in that process
        assert rs1 == rs2 and rs1[1] == 2
    assert {rec[-1][2][0] for rec in out} == {0, 1}
    assert [len(os.listdir(m)) for m in marks] == [1, 1]  # each operator: one rank-0 bundle read


class _RecordingCNN:
    """A ``SignatureBatchedModel`` over a ResNet SavedModel whose loader marks the process
    that reads the variables bundle."""

    @staticmethod
    def make(path, marks, distributed=True):
        from flink_tensorflow_amd.models import SignatureBatchedModel

        class M(SignatureBatchedModel):
            @property
            def loader(self):
                return _RecordingLoader(path, marks)

        return M(path, buckets=(8,), output_keys=["classes", "scores"], distributed_weights=distributed)


def _cnn_batch(m, vals):
    import hashlib

    import numpy as np

    from flink_tensorflow_amd.parallel import comm

    vs = m.session().variables
    h = hashlib.sha256()
    for k in sorted(vs):
        h.update(k.encode())
        h.update(vs[k].detach().cpu().contiguous().numpy().tobytes())
    rows = m.submit(vals, np.zeros(len(vals)), list(range(len(vals))))[0][0]
    return [(os.getpid(), comm.rank_size(), h.hexdigest()[:16], int(r["classes"].reshape(-1)[0])) for r in rows]


def test_p4_distributed_weights_cnn_operator_rehearsal(tmp_path):
    """P = 4 rehearsal of the headline job shape on the host (loopback communicator): a
    ResNet SavedModel served by ``SignatureBatchedModel(distributed_weights=True)`` in 4
    worker processes, fed by a worker-process source chained into them.  Only rank 0 reads
    the variables bundle; all four end with bit-identical weights and classify every
    record the same way the 1-process model does."""
    import numpy as np

    from flink_tensorflow_amd.models import SignatureBatchedModel
    from flink_tensorflow_amd.models.zoo.resnet import export_resnet50_saved_model
    from flink_tensorflow_amd.parallel.fake import FakeCommunicator

    d = export_resnet50_saved_model(str(tmp_path / "rn"), image_hw=(32, 32), depth=26, num_classes=16, seed=4)
    marks = tmp_path / "marks"
    marks.mkdir()
    pool = np.random.default_rng(0).integers(0, 256, (16, 32, 32, 3), dtype=np.uint8)
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(4)
    env.enable_job_communicator(True, communicator=FakeCommunicator)
    src = env.generate(lambda idx, par, start: (pool[(idx + i * par) % 16] for i in range(start, 8))).run_in_processes()
    out = src.map_with_model_batched(_RecordingCNN.make(d, str(marks)), _cnn_batch, max_batch=8, max_delay_ms=50,
                                     name="resnet").run_in_processes().execute_and_collect()
    assert len(out) == 32
    assert {o[1] for o in out} == {(r, 4) for r in range(4)}
    assert len({o[0] for o in out}) == 4 and os.getpid() not in {o[0] for o in out}
    assert len({o[2] for o in out}) == 1  # bit-identical weights on every rank
    assert len(os.listdir(marks)) == 1  # one bundle read (rank 0)
    ref = SignatureBatchedModel(d, buckets=(8,), output_keys=["classes", "scores"], device="cpu")
    ref.open()
    cls = [int(r["classes"].reshape(-1)[0]) for r in ref.submit(list(pool), np.zeros(16), list(range(16)))[0][0]]
    ref.close()
    assert sorted(o[3] for o in out) == sorted(cls[(idx + i * 4) % 16] for idx in range(4) for i in range(8))


def _timed_job(tmp_path, P, communicator=None, device_note=""):
    import json

    import numpy as np

    from flink_tensorflow_amd.batching.timed import TimedWindow
    from flink_tensorflow_amd.models.zoo.image_classifier import ResNet50Model
    from flink_tensorflow_amd.runtime.sources import DiscardingSink

    class TimedResNet(TimedWindow, ResNet50Model):
        pass

    W, K, B, HW = 1, 2, 4, 32
    out_dir = str(tmp_path / "timed")
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(P)
    env.enable_job_communicator(True, communicator=communicator)

    def images(idx, par, start):
        pool = np.random.default_rng(idx).integers(0, 256, (8, HW, HW, 3), dtype=np.uint8)
        for i in range(start, (W + K) * B):
            yield pool[i % 8]

    model = TimedResNet(image_hw=(HW, HW), buckets=(B,), distributed_weights=True, depth_layers=26, lanes=1) \
        .timed_window(W, K, out_dir)
    env.generate(images).run_in_processes() \
        .map_with_model_batched(model, None, max_batch=B, max_delay_ms=60_000.0, name="resnet").run_in_processes() \
        .add_sink(DiscardingSink()).run_in_processes()
    env.execute("timed-job")
    ranks = []
    for r in range(P):
        with open(os.path.join(out_dir, f"rank{r}.json")) as f:
            ranks.append(json.load(f))
    return ranks, K * B


def test_bench_job_shape_rehearsal_p2(tmp_path):
    """The ``bench.py --job`` job shape on the host: 2 worker-process subtasks, each a
    chained source + a ``distributed_weights`` ResNet operator timing its own window
    (``batching/timed.py``): every rank writes its K-batch window, inside a 2-rank group."""
    from flink_tensorflow_amd.parallel.fake import FakeCommunicator

    ranks, per_rank = _timed_job(tmp_path, 2, FakeCommunicator)
    assert [r["rank"] for r in ranks] == [0, 1] and {r["world"] for r in ranks} == {2}
    assert all(r["records"] == per_rank and r["elapsed_s"] > 0 for r in ranks)
    assert all(len(r["latencies_s"]) == per_rank for r in ranks)
    assert len({r["pid"] for r in ranks}) == 2 and os.getpid() not in {r["pid"] for r in ranks}


@pytest.mark.gpu
def test_bench_job_mode_p1_through_rccl_gpu(tmp_path):
    """``bench.py --job`` at P = 1: the operator's communicator is RCCL (world 1) and the
    timed window covers exactly K micro-batches."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--job", "--steps", "4", "--warmup", "2",
                        "--batch", "64"], capture_output=True, text=True, timeout=600, cwd=root)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert out["communicator"] == "RcclCommunicator" and out["comm_world_size"] == 1
    assert out["n_gpus"] == 1 and out["steps"] == 4 and out["value"] > 0


def _bert_batch(m, vals):
    import hashlib

    import numpy as np

    from flink_tensorflow_amd.parallel import comm

    vs = m.session().variables
    h = hashlib.sha256()
    for k in sorted(vs):
        h.update(k.encode())
        h.update(vs[k].detach().cpu().contiguous().numpy().tobytes())
    rows = m.submit(vals, np.zeros(len(vals)), list(range(len(vals))))[0][0]
    return [(os.getpid(), comm.rank_size(), h.hexdigest()[:16], r["logits"].reshape(-1).tolist()) for r in rows]


def test_p4_distributed_weights_bert_savedmodel_rehearsal(tmp_path):
    """VERDICT r5 #3, BASELINE config 3 as a job: a BERT classifier exported as a TF
    SavedModel (``modeling.py`` GraphDef, mask computed from the ids) served by
    ``SignatureBatchedModel(distributed_weights=True)`` in 4 worker processes fed by chained
    sources of token-id records.  Only rank 0 reads the variables bundle, all four ranks end
    with bit-identical weights, and every record's logits equal the 1-process model's."""
    import numpy as np

    from flink_tensorflow_amd.models import SignatureBatchedModel
    from flink_tensorflow_amd.models.zoo.bert import BertConfig
    from flink_tensorflow_amd.models.zoo.bert_graph import export_bert_saved_model
    from flink_tensorflow_amd.parallel.fake import FakeCommunicator

    cfg, S = BertConfig.tiny(), 16
    d = export_bert_saved_model(str(tmp_path / "bert"), cfg, S, seed=5, mask_from_ids=True)
    marks = tmp_path / "marks"
    marks.mkdir()
    rng = np.random.default_rng(0)
    pool = rng.integers(1000 // 2, cfg.vocab_size, (16, S), dtype=np.int32)
    for i, n in enumerate(rng.integers(S // 2, S + 1, 16)):
        pool[i, n:] = 0

    class M(SignatureBatchedModel):
        @property
        def loader(self):
            return _RecordingLoader(d, str(marks))

    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(4)
    env.enable_job_communicator(True, communicator=FakeCommunicator)
    src = env.generate(lambda idx, par, start: (pool[(idx + i * par) % 16] for i in range(start, 4))).run_in_processes()
    out = src.map_with_model_batched(M(d, buckets=(4,), output_keys=["logits"], distributed_weights=True),
                                     _bert_batch, max_batch=4, max_delay_ms=50, name="bert") \
        .run_in_processes().execute_and_collect()
    assert len(out) == 16
    assert {o[1] for o in out} == {(r, 4) for r in range(4)}
    assert len({o[2] for o in out}) == 1  # bit-identical weights on every rank
    assert len(os.listdir(marks)) == 1  # one bundle read (rank 0)
    ref = SignatureBatchedModel(d, buckets=(4,), output_keys=["logits"], device="cpu")
    ref.open()
    want = {}
    for s in range(0, 16, 4):
        for i, r in zip(range(s, s + 4), ref.submit(list(pool[s:s + 4]), np.zeros(4), list(range(4)))[0][0]):
            want[i] = r["logits"].reshape(-1).tolist()
    ref.close()
    got = sorted(o[3] for o in out)
    assert got == sorted(want[(idx + i * 4) % 16] for idx in range(4) for i in range(4))
