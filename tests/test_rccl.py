"""Direct RCCL binding (``_rccl``) on device tensors at world size 1.

The communicator is created exactly as a DP rank creates it (``ncclGetUniqueId`` →
``ncclCommInitRank`` on the rank's GPU) and every collective of the framework runs through
it on HBM tensors: broadcast (in place and through the staging bucket), all-reduce
(sync and async on the comm stream), all-gather, reduce-scatter, the bucketed gradient
all-reduce driven by autograd hooks, and the metric all-gather.  Multi-rank semantics are
covered on the CPU by the loopback communicator (``tests/test_dist.py``)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rccl_comm():
    from flink_tensorflow_amd import _ext
    from flink_tensorflow_amd.parallel import comm

    lib = _ext.rccl()
    assert lib.version() >= 22000
    c = comm.RcclCommunicator(0, 1, torch.device("cuda", 0), unique_id=lib.unique_id())
    comm.set_communicator(c)
    yield c
    comm.destroy()


def test_collectives_on_device(rccl_comm):
    c = rccl_comm
    dev = c.device
    x = torch.arange(1000, dtype=torch.float32, device=dev)
    ref = x.clone()
    c.broadcast(x, 0)
    c.all_reduce(x, "sum")
    c.all_reduce(x, "max")
    torch.testing.assert_close(x, ref)
    for dt in (torch.bfloat16, torch.float16, torch.int64, torch.uint8, torch.float64):
        y = (torch.arange(257, device=dev) % 100).to(dt)
        y0 = y.clone()
        c.all_reduce(y)
        assert torch.equal(y, y0), dt
    out = torch.empty(1000, dtype=torch.float32, device=dev)
    c.all_gather(out, ref)
    torch.testing.assert_close(out, ref)
    rs = torch.empty(1000, dtype=torch.float32, device=dev)
    c.reduce_scatter(rs, ref)
    torch.testing.assert_close(rs, ref)
    w = c.all_reduce_async(x)
    w.wait()
    torch.cuda.synchronize()
    torch.testing.assert_close(x, ref)
    assert c.async_error() == ""
    with pytest.raises(ValueError):
        c.all_reduce(torch.zeros(4, 4, device=dev).t())  # non-contiguous
    with pytest.raises(ValueError):
        c.all_reduce(torch.zeros(4))  # host tensor


def test_broadcast_tensors_bucketed(rccl_comm):
    from flink_tensorflow_amd.parallel import comm

    dev = rccl_comm.device
    big = torch.randn(1 << 20, device=dev)                      # in place (>= bucket/4)
    small = [torch.randn(3, 5, device=dev).to(torch.bfloat16) for _ in range(7)]
    strided = torch.randn(8, 8, device=dev).t()                 # non-contiguous: staged
    before = [t.clone() for t in [big, *small, strided]]
    n = comm.broadcast_tensors([big, *small, strided], src=0, bucket_bytes=1 << 16)
    assert n == big.numel() * 4 + 7 * 15 * 2 + 64 * 4
    for a, b in zip([big, *small, strided], before):
        assert torch.equal(a, b)


def test_grad_bucketer_through_rccl(rccl_comm):
    from flink_tensorflow_amd.parallel import comm

    dev = rccl_comm.device
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.ReLU(), torch.nn.Linear(128, 8)).to(dev)
    b = comm.GradBucketer(list(model.parameters()), bucket_bytes=4096)
    assert b.active and len(b.buckets) > 1
    x = torch.randn(32, 64, device=dev)
    model(x).pow(2).sum().backward()
    got = [p.grad.clone() for p in model.parameters()]
    b.synchronize()  # world size 1: the averaged all-reduce returns each gradient unchanged
    for p, g in zip(model.parameters(), got):
        torch.testing.assert_close(p.grad, g)
    b.remove()


def test_metrics_allgather_through_rccl(rccl_comm):
    import numpy as np

    from flink_tensorflow_amd.parallel import comm
    from flink_tensorflow_amd.utils.metrics import MetricGroup

    g = MetricGroup("op")
    g.inc("records_in", 42)
    g.histogram("latency_s").update_many(np.arange(1, 101) * 1e-3)
    m = comm.allgather_metrics(g)
    assert m["world_size"] == 1 and m["counters"]["records_in"] == 42
    assert abs(m["histograms"]["latency_s"]["p50"] - 0.050) < 0.002
    assert comm.all_gather_object({"rank": 0}) == [{"rank": 0}]
    assert comm.all_reduce_scalar(2.5, "max") == 2.5
    comm.barrier()


def test_torchrun_rccl_rendezvous():
    """bench.py's N-GPU launch path at N=1: ``torch.distributed.run`` → agent store →
    ``ncclGetUniqueId`` / ``ncclCommInitRank`` → collectives, in a child process."""
    from _helpers import torchrun_smoke

    out = torchrun_smoke(1)
    assert out == [{"rank": 0, "ws": 1, "bcast": [1.0] * 4, "sum": [1.0] * 3, "objs": [0]}]


def test_widedeep_dp_step_captured_with_rccl(rccl_comm):
    """The data-parallel Wide&Deep step — bucketed dense all-reduce on the comm stream and
    row-sparse all-gathers, all through RCCL — captured as ONE hipGraph equals the eager DP
    step (world size 1: the collectives run, the values are unchanged), and batches staged
    from packed binary rows equal the Python collation."""
    from flink_tensorflow_amd.models.zoo.wide_deep import (PackedBatchStager, WideDeepConfig, WideDeepTrainer,
                                                           pack_click_records, synthetic_click_records)

    dev = rccl_comm.device
    cfg = WideDeepConfig.tiny()
    nx = min(8, cfg.num_fields - 1)
    recs = synthetic_click_records(64 * 8, cfg, seed=5)
    rows = list(pack_click_records(recs, cfg, nx))
    stager = PackedBatchStager(cfg, 64, dev, n_cross=nx)
    # the autograd DP step (the fused step has its own chunked all-reduce: test_widedeep.py)
    a, b = WideDeepTrainer(cfg, device=dev, seed=1, fused=False), WideDeepTrainer(cfg, device=dev, seed=1, fused=False)
    a.open()
    b.open()
    assert a._bucketer.active and b._bucketer.active  # the RCCL communicator is installed
    batches = [tuple(t.clone() for t in stager.stage(rows[i * 64:(i + 1) * 64])) for i in range(8)]
    ref = a.collate(recs[:64])
    for x, y in zip(batches[0], ref):
        assert torch.equal(x, y.to(x.dtype))
    for _ in range(2):
        a.train_step(batch=batches[0])
    b.capture(batches[0])
    assert b._graph is not None
    la = [float(a.train_step(batch=bt)) for bt in batches[2:]]
    lb = [float(b.train_step(batch=bt)) for bt in batches[2:]]
    torch.testing.assert_close(torch.tensor(lb), torch.tensor(la), rtol=1e-4, atol=1e-5)
    for (k, va), vb in zip(a.model.state_dict().items(), b.model.state_dict().values()):
        torch.testing.assert_close(vb, va, rtol=1e-4, atol=1e-5, msg=k)
    a.close()
    b.close()


def test_widedeep_bucketed_owner_step_captured_with_rccl(rccl_comm):
    """The fused Wide&Deep DP step with the fixed-capacity owner exchange
    (``BucketedOwnerExchange``: static unique ids from the in-tree radix sort, per-peer
    buckets, equal-split RCCL all-to-alls, row gather / scatter kernels) is host-sync free:
    it captures as ONE hipGraph (capacities calibrated on the warm-up steps), and replays
    track the eager step with the same exchange.  World size 1: every row is owned here,
    the all-to-alls run through RCCL with the values unchanged."""
    from flink_tensorflow_amd.models.zoo.wide_deep import WideDeepConfig, WideDeepTrainer, synthetic_click_records
    from flink_tensorflow_amd.parallel.sparse_exchange import BucketedOwnerExchange

    dev = rccl_comm.device
    cfg = WideDeepConfig.tiny()
    recs = synthetic_click_records(64 * 8, cfg, seed=6)
    tr = []
    for _ in range(2):
        t = WideDeepTrainer(cfg, device=dev, seed=2)
        t.open()
        assert t._fused is not None
        ex = BucketedOwnerExchange(rccl_comm)
        t._exchange = t._fused.exchange = ex
        tr.append(t)
    a, b = tr
    batches = [a.collate(recs[i * 64:(i + 1) * 64]) for i in range(8)]
    for _ in range(3):  # b's capture runs 3 real steps (2 warm-up + 1 calibrated)
        a.train_step(batch=batches[0])
    a._exchange.calibrate()
    b.capture(batches[0])
    assert b._graph is not None  # a host sync inside the step would have failed the capture
    torch.cuda.set_sync_debug_mode("error")  # the eager bucketed DP step never syncs with the host
    try:
        la = [a.train_step(batch=bt).clone() for bt in batches[2:]]
    finally:
        torch.cuda.set_sync_debug_mode(0)
    la = [float(x) for x in la]
    lb = [float(b.train_step(batch=bt)) for bt in batches[2:]]
    torch.testing.assert_close(torch.tensor(lb), torch.tensor(la), rtol=1e-4, atol=1e-5)
    for (k, va), vb in zip(a.model.state_dict().items(), b.model.state_dict().values()):
        torch.testing.assert_close(vb, va, rtol=1e-4, atol=1e-5, msg=k)
    a._exchange.check()
    b._exchange.check()
    assert b._exchange.capacity(64 * cfg.num_fields, cfg.num_fields * cfg.vocab_per_field) <= 64 * cfg.num_fields
    a.close()
    b.close()
