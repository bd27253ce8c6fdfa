"""Collective layer on CPU processes (loopback fake communicator, world_size 2 — no RCCL,
no gloo): weight broadcast, bucketed
overlapped gradient all-reduce, metric reduction, and a distributed stream whose sources
are partitioned by rank (the one-process-per-GPU DP layout, rehearsed on the host)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp
from _helpers import torchrun_smoke as _torchrun


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        from flink_tensorflow_amd.parallel import comm
        from flink_tensorflow_amd.parallel.fake import FakeCommunicator

        comm.init_distributed(communicator=FakeCommunicator)
        # tensors cross the queue as numpy: torch's fd-sharing pickler needs the child alive
        # until the parent unpickles, which races with the child's exit
        q.put((rank, _to_numpy(fn(rank, world))))
        comm.destroy()
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, f"ERROR {e}\n{traceback.format_exc()}"))


def _to_numpy(v):
    if isinstance(v, torch.Tensor):
        return v.numpy()
    if isinstance(v, (list, tuple)):
        return type(v)(_to_numpy(x) for x in v)
    if isinstance(v, dict):
        return {k: _to_numpy(x) for k, x in v.items()}
    return v


def _run(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, fn, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for r, v in out.items():
        assert not (isinstance(v, str) and v.startswith("ERROR")), v
    return out


def _broadcast(rank, world):
    from flink_tensorflow_amd.parallel import comm

    ts = [torch.full((3, 4), float(rank)), torch.arange(5, dtype=torch.int64) * (rank + 1),
          torch.full((7,), float(rank + 10))]
    n = comm.broadcast_tensors(ts, src=0)
    return [t.tolist() for t in ts], n


def test_broadcast_tensors():
    out = _run(_broadcast)
    assert out[0][0] == out[1][0]
    assert out[1][0][0] == [[0.0] * 4] * 3 and out[1][0][1] == [0, 1, 2, 3, 4]
    assert out[1][1] == (12 + 7) * 4 + 5 * 8


def _grads(rank, world):
    from flink_tensorflow_amd.parallel import comm

    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 3))
    bucketer = comm.GradBucketer(list(model.parameters()), bucket_bytes=256)
    x = torch.randn(4, 8) + rank
    model(x).pow(2).sum().backward()
    bucketer.synchronize()
    total = comm.all_reduce_scalar(float(rank + 1), "sum")
    return [p.grad.clone() for p in model.parameters()], len(bucketer.buckets), total


def test_grad_bucketer_averages():
    out = _run(_grads)
    g0, nb, total = out[0]
    g1, _, _ = out[1]
    assert nb > 1 and total == 3.0
    g0, g1 = [torch.from_numpy(a) for a in g0], [torch.from_numpy(b) for b in g1]
    for a, b in zip(g0, g1):
        torch.testing.assert_close(a, b)
    # compare with the single-process average of both ranks' gradients
    ref = None
    for r in range(2):  # replay each rank's RNG sequence: seed → model init → input
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 3))
        x = torch.randn(4, 8) + r
        model(x).pow(2).sum().backward()
        if ref is None:
            ref = [torch.zeros_like(p) for p in model.parameters()]
        for acc, p in zip(ref, model.parameters()):
            acc += p.grad / 2
    for a, b in zip(g0, ref):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def _stream(rank, world):
    from flink_tensorflow_amd.runtime import StreamExecutionEnvironment

    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(2)
    return sorted(env.from_collection(list(range(40)), parallelism=2).map(lambda v: v * 10).execute_and_collect())


def _widedeep(rank, world):
    from flink_tensorflow_amd.models.zoo.wide_deep import WideDeepConfig, WideDeepTrainer, synthetic_click_records

    t = WideDeepTrainer(WideDeepConfig.tiny(), device="cpu", seed=rank)  # different seeds: broadcast fixes
    t.open()
    recs = synthetic_click_records(256, t.cfg, seed=100 + rank)  # different data per rank
    for i in range(4):
        t.train_step(recs[i * 64:(i + 1) * 64])
    sd = dict(t.model.state_dict())
    if t._exchange is not None:  # owner exchange: rows / Adagrad state are authoritative at their owner
        for name in ("emb", "wide"):
            e = getattr(t.model, name)
            sd[f"{name}.table"] = t._exchange.merge_owner_shards(e.table.data)
            sd[f"{name}.accum"] = t._exchange.merge_owner_shards(e.accum)
    sd = {k: v.detach().numpy().copy() for k, v in sd.items()}  # plain arrays over the queue
    t.close()
    return sd


def test_widedeep_dp_replicas_stay_identical():
    out = _run(_widedeep)
    a, b = out[0], out[1]
    assert a.keys() == b.keys()
    for k in a:
        assert (a[k] == b[k]).all(), k


def test_distributed_stream_partitions_sources():
    out = _run(_stream)
    allv = sorted(out[0] + out[1])
    assert allv == [v * 10 for v in range(40)]
    assert set(out[0]).isdisjoint(out[1])


def _bert_weights(rank, world):
    import numpy as np

    from flink_tensorflow_amd.models.zoo.bert import BertClassifierModel, BertConfig

    m = BertClassifierModel(BertConfig.tiny(), seq_len=16, buckets=(4,), seed=rank, device="cpu",
                            distributed_weights=True)
    m.open()
    p = m.predict(["streaming inference", "on every rank", "same weights"])
    m.close()
    return np.asarray(p)


def test_model_weights_broadcast_at_open():
    """Ranks initialise different weights (seed = rank); with distributed_weights every rank
    serves rank 0's model after open."""
    out = _run(_bert_weights)
    assert out[0].shape == (3, 2)
    assert (out[0] == out[1]).all()


@pytest.mark.gpu
def test_numa_binding_gpu():
    """Best-effort NUMA pinning of a DP rank: either nothing to do, or a non-empty subset
    of the CPUs this process may use; the mask is restored afterwards."""
    from flink_tensorflow_amd.parallel import comm

    before = os.sched_getaffinity(0)
    try:
        r = comm.bind_to_gpu_numa(torch.device("cuda", 0))
        after = os.sched_getaffinity(0)
        if r is None:
            assert after == before
        else:
            assert after and after <= before and r["cpus"] == len(after)
    finally:
        os.sched_setaffinity(0, before)


def _metrics(rank, world):
    import numpy as np

    from flink_tensorflow_amd.parallel import comm
    from flink_tensorflow_amd.utils.metrics import MetricGroup

    g = MetricGroup("op")
    g.inc("records_in", 100 * (rank + 1))
    # rank 0: 1..100 ms, rank 1: 101..300 ms -> node-level p50 is ~150 ms, not median(p50s)
    lo, hi = (1, 100) if rank == 0 else (101, 300)
    g.histogram("latency_s").update_many(np.arange(lo, hi + 1) * 1e-3)
    if rank == 1:
        g.histogram("only_rank1").update_many([0.5])
    return comm.allgather_metrics(g)


def test_allgather_metrics_merges_histograms_across_ranks():
    out = _run(_metrics)
    m = out[0]
    assert m == out[1]
    assert m["world_size"] == 2 and m["counters"]["records_in"] == 300
    h = m["histograms"]["latency_s"]
    assert h["count"] == 300
    assert abs(h["p50"] - 0.150) / 0.150 < 0.01          # true node-level median of 1..300 ms
    assert abs(h["p99"] - 0.297) / 0.297 < 0.01
    assert m["histograms"]["only_rank1"]["count"] == 1


def test_bucket_histogram_percentiles_match_numpy():
    import numpy as np

    from flink_tensorflow_amd.utils.metrics import BucketHistogram, Histogram, histogram_buckets

    rng = np.random.default_rng(0)
    v = rng.lognormal(-5, 1, 20000)
    b = BucketHistogram()
    b.update_many(v)
    for q in (50, 90, 99):
        ref = np.percentile(v, q)
        assert abs(b.percentile(q) - ref) / ref < 0.01
    h = Histogram(cap=1000)
    h.update_many(v)                                     # decimated to <= cap samples
    hb = histogram_buckets(h)
    assert hb.count == pytest.approx(20000, rel=0.01)
    assert abs(hb.percentile(50) - np.percentile(v, 50)) / np.percentile(v, 50) < 0.05


def test_torchrun_agent_store_rendezvous():
    """bench.py's launch path: ``torch.distributed.run`` workers find the job's store (the
    agent's, on MASTER_PORT) and exchange through the communicator."""
    out = _torchrun(2, "--fake")
    assert [o["rank"] for o in out] == [0, 1]
    for o in out:
        assert o["bcast"] == [1.0] * 4 and o["sum"] == [3.0] * 3 and o["objs"] == [0, 1]


def _savedmodel_rank0_broadcast(paths, dist_weights, rank, world):
    from flink_tensorflow_amd.models import RegressionMethod, SavedModelModel
    from flink_tensorflow_amd.types import example, feature

    m = SavedModelModel(paths[rank], device="cpu", distributed_weights=dist_weights)
    m.open()
    y = m.function("regress_x_to_y", RegressionMethod()).apply([example(("x", feature(1.0)))])
    a = float(m.session().variables["a"])
    m.close()
    return [float(y.reshape(-1)[0]), a]


def test_savedmodel_variables_read_by_rank0_and_broadcast(half_plus_two, tmp_path):
    """``distributed_weights=True``: rank 0 reads the SavedModel's variables, the other
    ranks only allocate them from the checkpoint index and receive rank 0's values — rank 1
    here points at a copy whose ``a`` was re-saved as 3 and still computes 0.5 x + 2."""
    import functools
    import shutil

    from flink_tensorflow_amd.io.saver import VariableSaver
    from flink_tensorflow_amd.models import SavedModelModel

    other = str(tmp_path / "hpt_a3")
    shutil.copytree(half_plus_two, other)
    m = SavedModelModel(other, device="cpu")
    m.open()
    m.session().variables["a"].fill_(3.0)
    VariableSaver().save(m.session(), os.path.join(other, "variables", "variables"))
    m.close()
    out = _run(functools.partial(_savedmodel_rank0_broadcast, [half_plus_two, other], True))
    assert out[0] == [2.5, 0.5] and out[1] == [2.5, 0.5], out
    ctrl = _run(functools.partial(_savedmodel_rank0_broadcast, [half_plus_two, other], False))
    assert ctrl[1] == [5.0, 3.0], ctrl  # without it, rank 1 serves its own copy


def test_restore_targets_map_variables_to_checkpoint_keys(half_plus_two):
    """A receiving rank allocates exactly the variables rank 0's SaverDef restore assigns,
    under the same names (not the raw index keys)."""
    from flink_tensorflow_amd.graph.graph import Graph
    from flink_tensorflow_amd.models.savedmodel import read_saved_model, restore_targets, select_meta_graph

    mg = select_meta_graph(read_saved_model(half_plus_two), ["serve"])
    t = restore_targets(Graph.from_graph_def(mg.graph_def), mg.saver_def.restore_op_name)
    assert t == {"a": ("a", ""), "b": ("b", ""), "c": ("c", "")}


class _ExtraVarLoader:
    """Loads half_plus_two; on rank 1 the session gains a variable rank 0 does not have."""

    def __init__(self, path):
        from flink_tensorflow_amd.models.savedmodel import DefaultSavedModelLoader

        self.inner = DefaultSavedModelLoader(path)

    @property
    def metagraph(self):
        return self.inner.metagraph

    def load(self, device=None, read_variables=True):
        import torch

        from flink_tensorflow_amd.parallel import comm

        b = self.inner.load(device=device, read_variables=read_variables)
        if comm.rank_size()[0] == 1:
            b.session.variables["extra"] = torch.zeros(2)
        return b


def _mismatched_open(path, rank, world):
    from flink_tensorflow_amd.models.savedmodel import TensorFlowModel

    class M(TensorFlowModel):
        loader = _ExtraVarLoader(path)

    m = M(device="cpu", distributed_weights=True)
    try:
        m.open()
    except RuntimeError as e:
        return "refused" if "refusing a mismatched broadcast" in str(e) else f"other: {e}"
    return "opened"


def test_distributed_weights_refuse_mismatched_variable_sets(half_plus_two):
    """Ranks whose sessions hold different variable lists raise before any broadcast
    (instead of issuing mismatched RCCL broadcasts that hang or corrupt)."""
    import functools

    out = _run(functools.partial(_mismatched_open, half_plus_two))
    assert out == {0: "refused", 1: "refused"}, out
