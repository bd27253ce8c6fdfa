"""Wide&Deep online training: embedding kernels, loss going down, streaming checkpoints."""
import numpy as np
import pytest
import torch

from flink_tensorflow_amd.models.zoo.wide_deep import (WideDeepConfig, WideDeepTrainer, synthetic_click_records)
from flink_tensorflow_amd.ops import embedding as E
from flink_tensorflow_amd.runtime import RestartStrategy, StreamExecutionEnvironment


def test_embedding_ops_host():
    table = torch.randn(50, 8)
    ids = torch.tensor([[1, 2], [2, -1], [49, 1]], dtype=torch.int32)
    out = E.embedding_bag(ids, table)
    torch.testing.assert_close(out, torch.stack([table[1] + table[2], table[2], table[49] + table[1]]))
    g = torch.randn(3, 8)
    uids, rows = E.embedding_bag_backward(ids, g, 50)
    assert uids.tolist() == [1, 2, 49]
    torch.testing.assert_close(rows, torch.stack([g[0] + g[2], g[0] + g[1], g[2]]))


def _train(device, steps=60):
    t = WideDeepTrainer(WideDeepConfig.tiny(), device=device)
    t.open()
    recs = synthetic_click_records(steps * 64, t.cfg, seed=1)
    losses = [float(t.train_step(recs[i * 64:(i + 1) * 64])) for i in range(steps)]
    t.close()
    return losses


def test_training_reduces_loss_host():
    losses = _train("cpu")
    assert np.mean(losses[-10:]) < np.mean(losses[:10])


def test_online_training_stream_with_checkpoint(tmp_path):
    cfg = WideDeepConfig.tiny()
    recs = synthetic_click_records(2048, cfg, seed=3)
    env = StreamExecutionEnvironment.get_execution_environment()
    env.enable_checkpointing(0.05, str(tmp_path / "chk"))
    env.set_restart_strategy(RestartStrategy.fixed_delay(1))
    from flink_tensorflow_amd.runtime.sources import CollectionSource

    out = (env.add_source(CollectionSource(recs, delay_s=0.0005), "clicks")
           .map_with_model_batched(WideDeepTrainer(cfg, device="cpu"), lambda m, b: float(m.train_step(b)),
                                   max_batch=64, max_delay_ms=50, emit_batches=True, name="trainer")
           .collect_into())
    res = env.execute("online-training")
    losses = out.results()
    assert len(losses) >= 2048 // 64
    assert res.checkpoints, "no checkpoint completed"
    import glob

    assert glob.glob(str(tmp_path / "chk" / "chk-*" / "models" / "widedeep-0" / "variables.index"))


@pytest.mark.gpu
def test_embedding_kernels_gpu():
    dev = torch.device("cuda", 0)
    table = torch.randn(1000, 32)
    ids = torch.randint(-1, 1000, (512, 3), dtype=torch.int32)
    ref = E.embedding_bag(ids, table)
    got = E.embedding_bag(ids.to(dev), table.to(dev))
    torch.testing.assert_close(got.float().cpu(), ref, rtol=1e-2, atol=1e-2)
    g = torch.randn(512, 32).to(torch.bfloat16)
    u_ref, r_ref = E.embedding_bag_backward(ids, g.float(), 1000)
    u, r = E.embedding_bag_backward(ids.to(dev), g.to(dev), 1000)
    assert torch.equal(u.cpu(), u_ref)
    torch.testing.assert_close(r.cpu(), r_ref, rtol=1e-4, atol=1e-4)
    # determinism: identical bits on repeat
    u2, r2 = E.embedding_bag_backward(ids.to(dev), g.to(dev), 1000)
    assert torch.equal(r2, r)
    acc_ref, tab_ref = torch.full((1000, 32), 0.1), table.clone()
    E.sparse_adagrad(tab_ref, acc_ref, u_ref, r_ref, 0.05)
    tab, acc = table.to(dev), torch.full((1000, 32), 0.1, device=dev)
    E.sparse_adagrad(tab, acc, u, r, 0.05)
    torch.testing.assert_close(tab.cpu(), tab_ref, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_training_reduces_loss_gpu():
    losses = _train(torch.device("cuda", 0))
    assert np.mean(losses[-10:]) < np.mean(losses[:10])


@pytest.mark.gpu
def test_static_segment_sum_gpu():
    """Sync-free static-shape segment sum == the compact host result (plus padding)."""
    dev = torch.device("cuda", 0)
    ids = torch.randint(-1, 300, (1024, 2), dtype=torch.int32)
    g = torch.randn(1024, 16)
    u_ref, r_ref = E.embedding_bag_backward(ids, g, 300)
    u, r = E.embedding_bag_backward(ids.to(dev), g.to(dev), 300, static=True)
    u, r = u.cpu(), r.cpu()
    assert u.numel() == ids.numel() and (u[u_ref.numel():] == -1).all()
    assert torch.equal(u[: u_ref.numel()], u_ref)
    torch.testing.assert_close(r[: u_ref.numel()], r_ref, rtol=1e-5, atol=1e-5)
    # slots past the unique ids (incl. the dropped invalid-id bucket) are inert: uid -1


@pytest.mark.gpu
def test_captured_train_step_matches_eager_gpu():
    """The hipGraph-captured training step == the eager step (same updates, same loss)."""
    dev = torch.device("cuda", 0)
    cfg = WideDeepConfig.tiny()
    recs = synthetic_click_records(64 * 8, cfg, seed=5)
    a, b = WideDeepTrainer(cfg, device=dev, seed=1), WideDeepTrainer(cfg, device=dev, seed=1)
    a.open()
    b.open()
    batches = [a.collate(recs[i * 64:(i + 1) * 64]) for i in range(8)]
    for bt in batches[:2]:  # b's capture warm-up runs two real steps on batch 0
        a.train_step(batch=batches[0])
    b.capture(batches[0])
    la = [float(a.train_step(batch=bt)) for bt in batches[2:]]
    lb = [float(b.train_step(batch=bt)) for bt in batches[2:]]
    torch.testing.assert_close(torch.tensor(lb), torch.tensor(la), rtol=1e-4, atol=1e-5)
    for (k, va), vb in zip(a.model.state_dict().items(), b.model.state_dict().values()):
        torch.testing.assert_close(vb, va, rtol=1e-4, atol=1e-5, msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize("D", [8, 32, 64, 128])
def test_embedding_lane_groups_and_hot_ids_gpu(D):
    """Lane-group kernels (D/8 lanes per row) for every row width, and a hot id (600
    occurrences) that sends its wave down the whole-wave path: sums == the host reference,
    bit-identical on repeat."""
    dev = torch.device("cuda", 0)
    g0 = torch.Generator().manual_seed(D)
    table = torch.randn(5000, D, generator=g0)
    ids = torch.randint(-1, 5000, (3000, 2), generator=g0, dtype=torch.int32)
    ids[::5, 0] = 7                                          # hot id
    torch.testing.assert_close(E.embedding_bag(ids.to(dev), table.to(dev)).float().cpu(),
                               E.embedding_bag(ids, table), rtol=1e-2, atol=1e-2)
    g = torch.randn(3000, D, generator=g0).to(torch.bfloat16)
    u_ref, r_ref = E.embedding_bag_backward(ids, g.float(), 5000)
    u, r = E.embedding_bag_backward(ids.to(dev), g.to(dev), 5000, static=True)
    n = u_ref.numel()
    assert torch.equal(u[:n].cpu(), u_ref)
    torch.testing.assert_close(r[:n].cpu(), r_ref, rtol=1e-4, atol=1e-4)
    _, r2 = E.embedding_bag_backward(ids.to(dev), g.to(dev), 5000, static=True)
    assert torch.equal(r2, r)
    acc_ref, tab_ref = torch.full((5000, D), 0.1), table.clone()
    E.sparse_adagrad(tab_ref, acc_ref, u_ref, r_ref, 0.05)
    tab, acc = table.to(dev), torch.full((5000, D), 0.1, device=dev)
    E.sparse_adagrad(tab, acc, u.contiguous(), r.contiguous(), 0.05)
    torch.testing.assert_close(tab.cpu(), tab_ref, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_fused_step_matches_autograd_gpu():
    """The hand-fused GPU step (gather, MFMA GEMMs, drelu-masked dX, library dW, fused
    loss / head / Adam kernels) == the autograd step with torch Adam, step by step, within
    bf16 rounding; also under hipGraph capture."""
    dev = torch.device("cuda", 0)
    cfg = WideDeepConfig.tiny(hidden=(128, 64), embed_dim=16)
    recs = synthetic_click_records(256 * 8, cfg, seed=9)
    ref = WideDeepTrainer(cfg, device=dev, seed=3, fused=False)
    fus = WideDeepTrainer(cfg, device=dev, seed=3, fused=True)
    ref.open()
    fus.open()
    assert fus._fused is not None and ref._fused is None
    batches = [ref.collate(recs[i * 256:(i + 1) * 256]) for i in range(8)]
    la = [float(ref.train_step(batch=b)) for b in batches]
    lb = [float(fus.train_step(batch=b)) for b in batches]
    torch.testing.assert_close(torch.tensor(lb), torch.tensor(la), rtol=2e-2, atol=2e-3)
    for (k, va), vb in zip(ref.model.state_dict().items(), fus.model.state_dict().values()):
        torch.testing.assert_close(vb, va, rtol=2e-2, atol=3e-3, msg=k)
    cap = WideDeepTrainer(cfg, device=dev, seed=3, fused=True)
    cap.open()
    for b in batches[:2]:
        cap.train_step(batch=batches[0])
    cap.capture(batches[0])
    eager = WideDeepTrainer(cfg, device=dev, seed=3, fused=True)
    eager.open()
    for _ in range(4):  # the capture ran 2 warm-up steps on batch 0
        eager.train_step(batch=batches[0])
    lc = [float(cap.train_step(batch=b)) for b in batches[2:]]
    le = [float(eager.train_step(batch=b)) for b in batches[2:]]
    torch.testing.assert_close(torch.tensor(lc), torch.tensor(le), rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_fused_step_on_packed_rows_captured_gpu():
    """The bench path: batches are strided views of one packed device buffer (no split
    copies), the captured fused step re-binds a batch with one copy, and matches the eager
    fused step on the same batches."""
    from flink_tensorflow_amd.models.zoo.wide_deep import PackedBatchStager, pack_click_records

    dev = torch.device("cuda", 0)
    cfg = WideDeepConfig.tiny(hidden=(128, 64), embed_dim=16)
    nx = min(8, cfg.num_fields - 1)
    rows = list(pack_click_records(synthetic_click_records(128 * 6, cfg, seed=4), cfg, n_cross=nx))
    stager = PackedBatchStager(cfg, 128, dev, n_cross=nx, depth=6)
    batches = [stager.stage(rows[i * 128:(i + 1) * 128]) for i in range(6)]
    assert all(getattr(b, "packed", None) is not None and b[2].stride(0) != b[2].shape[1] for b in batches)
    cap = WideDeepTrainer(cfg, device=dev, seed=2, fused=True)
    eag = WideDeepTrainer(cfg, device=dev, seed=2, fused=True)
    cap.open()
    eag.open()
    cap.capture(batches[0])          # two warm-up steps on batch 0
    for _ in range(2):
        eag.train_step(batch=batches[0])
    lc = [float(cap.train_step(batch=b)) for b in batches[1:]]
    le = [float(eag.train_step(batch=b)) for b in batches[1:]]
    torch.testing.assert_close(torch.tensor(lc), torch.tensor(le), rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_fused_dp_replicas_stay_identical_gpu():
    """Two ranks (loopback communicator, both on this GPU) train the fused step on different
    records: after broadcast init, dense all-reduce and the merged row-sparse updates, every
    parameter and both embedding tables are bit-identical across the replicas."""
    from _helpers import torchrun_smoke

    out = torchrun_smoke(2, "--fake", script="wd_dp_check.py", timeout=300)
    assert [o["rank"] for o in out] == [0, 1] and all(o["fused"] for o in out)
    assert out[0]["sums"] == out[1]["sums"]
    assert out[0]["losses"] != out[1]["losses"]  # the ranks did see different data


def test_sparse_adagrad_offset_host():
    """Two tables in one key space: each table's update takes only its own ids."""
    ta, tb = torch.zeros(10, 8), torch.zeros(6, 8)
    aa, ab = torch.full((10, 8), 0.1), torch.full((6, 8), 0.1)
    uids = torch.tensor([3, 12, -1, 15], dtype=torch.int32)   # 3 -> table a; 12, 15 -> table b rows 2, 5
    g = torch.ones(4, 8)
    E.sparse_adagrad(ta, aa, uids, g, 0.5)
    E.sparse_adagrad(tb, ab, uids, g, 0.5, offset=10)
    assert ta[3].ne(0).all() and ta.abs().sum(1).ne(0).sum() == 1
    assert tb[2].ne(0).all() and tb[5].ne(0).all() and tb.abs().sum(1).ne(0).sum() == 2


@pytest.mark.gpu
def test_group_keys_and_grouped_sums_gpu():
    """``group_keys`` (radix sort over the used bits + runs) == a stable torch sort, invalid
    keys in one dropped bucket; ``segment_sum_grouped`` with index ranges sums two tables
    that share the key space from one grouping."""
    dev = torch.device("cuda", 0)
    g0 = torch.Generator().manual_seed(3)
    ka = torch.randint(-2, 500, (3000,), generator=g0, dtype=torch.int32)
    ka[::7] = 11                                              # hot key
    kb = torch.randint(0, 300, (1000,), generator=g0, dtype=torch.int32) + 500
    keys = torch.cat([ka, kb]).to(dev)
    perm, seg_id, seg, uids = E.group_keys(keys, 800)
    k = keys.cpu().long()
    kk = torch.where((k >= 0) & (k < 800), k, torch.full_like(k, 800))
    sk, sp = torch.sort(kk, stable=True)
    assert torch.equal(perm.cpu().long(), sp)
    runs = torch.unique_consecutive(sk)
    nr = runs.numel()
    want = torch.where(runs < 800, runs, torch.full_like(runs, -1)).to(torch.int32)
    assert torch.equal(uids[:nr].cpu(), want) and (uids[nr:] == -1).all()
    ra = torch.randn(3000, 16, generator=g0).to(torch.bfloat16)
    rb = torch.randn(1000, 8, generator=g0)
    sa = E.segment_sum_grouped((perm, seg_id, seg, uids), ra.to(dev), 1, 0, 3000).cpu()
    sb = E.segment_sum_grouped((perm, seg_id, seg, uids), rb.to(dev), 1, 3000, 4000).cpu()
    for i in range(nr):
        key = int(runs[i])
        ia = [j for j in range(3000) if int(kk[j]) == key]
        ib = [j - 3000 for j in range(3000, 4000) if int(kk[j]) == key]
        torch.testing.assert_close(sa[i], ra.float()[ia].sum(0) if ia else torch.zeros(16), rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(sb[i], rb[ib].sum(0) if ib else torch.zeros(8), rtol=1e-4, atol=1e-4)
    assert sa[nr:].abs().sum() == 0 and sb[nr:].abs().sum() == 0


@pytest.mark.gpu
def test_fused_step_checkpoint_roundtrip_gpu(tmp_path):
    """CheckpointedModel on the fused path: weights, tables and the flat Adam state go into
    the checkpoint bundle; a fresh trainer restored from it continues exactly like the
    uninterrupted one."""
    from flink_tensorflow_amd.runtime.functions import InitializationContext, SnapshotContext
    from flink_tensorflow_amd.runtime.state import OperatorStateStore

    dev = torch.device("cuda", 0)
    cfg = WideDeepConfig.tiny(hidden=(128, 64), embed_dim=16)
    recs = synthetic_click_records(256 * 6, cfg, seed=12)
    a = WideDeepTrainer(cfg, device=dev, seed=4, fused=True)
    a.open()
    batches = [a.collate(recs[i * 256:(i + 1) * 256]) for i in range(6)]
    for b in batches[:3]:
        a.train_step(batch=b)
    ops = OperatorStateStore()
    a.snapshot_state(SnapshotContext(1, 0.0, ops, str(tmp_path), 0))
    r = WideDeepTrainer(cfg, device=dev, seed=99, fused=True)  # different init: all of it must come back
    r.open()
    r.initialize_state(InitializationContext(ops, True, str(tmp_path), 0))
    la = [float(a.train_step(batch=b)) for b in batches[3:]]
    lr = [float(r.train_step(batch=b)) for b in batches[3:]]
    torch.testing.assert_close(torch.tensor(lr), torch.tensor(la), rtol=1e-5, atol=1e-6)
    for (k, va), vb in zip(a.model.state_dict().items(), r.model.state_dict().values()):
        torch.testing.assert_close(vb, va, rtol=1e-5, atol=1e-6, msg=k)
    assert r.steps == a.steps == 6  # the step counter came back too


@pytest.mark.gpu
def test_group_keys_int64_out_of_range_ids_are_dropped_gpu():
    """int64 ids at or above 2^31 (or negative) land in the dropped bucket; before the fix
    they wrapped on the int32 cast and could alias valid rows."""
    dev = torch.device("cuda", 0)
    keys = torch.tensor([5, (1 << 32) + 5, 7, -(1 << 33) + 7, 5, (1 << 31)], dtype=torch.int64, device=dev)
    perm, seg_id, seg, uids = E.group_keys(keys, 100)
    assert uids[:3].cpu().tolist() == [5, 7, -1]  # runs: 5 (x2), 7 (x1), dropped (x3)
    assert perm[:3].cpu().tolist() == [0, 4, 2]


@pytest.mark.gpu
def test_fused_step_tracks_fp32_host_trainer_gpu():
    """Training numerics pinned against fp32: 8 fused GPU steps (hand-written gather, MFMA
    forward / dX / dW GEMMs, loss, head backward, sort-based sparse Adagrad, flat Adam) vs
    the fp32 autograd trainer on the host, same seed and data.  Per-step losses agree to
    bf16 precision and the parameter updates (p8 - p0) point the same way with the same size."""
    dev = torch.device("cuda", 0)
    cfg = WideDeepConfig.tiny(num_fields=8, vocab_per_field=500, embed_dim=16, hidden=(256, 128, 64),
                              wide_buckets=4099)
    recs = synthetic_click_records(512 * 8, cfg, seed=21)
    gpu = WideDeepTrainer(cfg, device=dev, seed=5, fused=True)
    cpu = WideDeepTrainer(cfg, device="cpu", seed=5, fused=False)
    gpu.open()
    cpu.open()
    assert gpu._fused is not None
    p0 = {k: v.detach().float().cpu().clone() for k, v in cpu.model.state_dict().items()}
    for i in range(8):
        chunk = recs[i * 512:(i + 1) * 512]
        lg = float(gpu.train_step(chunk))
        lc = float(cpu.train_step(chunk))
        assert abs(lg - lc) <= 2e-2 * abs(lc) + 2e-3, (i, lg, lc)
    torch.cuda.synchronize()
    sg = {k: v.detach().float().cpu() for k, v in gpu.model.state_dict().items()}
    sc = {k: v.detach().float().cpu() for k, v in cpu.model.state_dict().items()}
    for k in sc:
        if k.endswith("accum") or k.endswith("anchor"):
            continue
        dg, dc = (sg[k] - p0[k]).reshape(-1), (sc[k] - p0[k]).reshape(-1)
        if dc.norm() == 0:
            assert dg.norm() <= 1e-6, k
            continue
        cos = float(torch.dot(dg, dc) / (dg.norm() * dc.norm() + 1e-30))
        ratio = float(dg.norm() / dc.norm())
        assert cos > 0.98 and 0.9 < ratio < 1.1, (k, cos, ratio)
    gpu.close()
    cpu.close()


@pytest.mark.gpu
def test_autograd_linear_matches_torch_fp32_gpu():
    """``ops.autograd.Linear`` (forward, dX, dW, db all on gemm_train) vs torch.nn.Linear in
    fp32 on the same (bf16-representable) data."""
    from flink_tensorflow_amd.ops.autograd import Linear

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    lin = Linear(256, 192, "relu", device=dev)
    ref = torch.nn.Linear(256, 192).to(dev)
    with torch.no_grad():
        w16 = lin.weight.to(torch.bfloat16).float()
        lin.weight.copy_(w16)
        ref.weight.copy_(w16)
        ref.bias.copy_(lin.bias)
    x = torch.randn(1000, 256, device=dev).to(torch.bfloat16)
    xr = x.float().clone().requires_grad_(True)
    xg = x.clone().requires_grad_(True)
    y = lin(xg)
    yr = torch.relu(ref(xr))
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
    gy = torch.randn_like(yr).to(torch.bfloat16)
    y.backward(gy)
    yr.backward(gy.float())
    for a, b, nm in ((xg.grad, xr.grad, "dx"), (lin.weight.grad, ref.weight.grad, "dW"), (lin.bias.grad, ref.bias.grad, "db")):
        err = (a.float() - b).abs().max().item() / b.abs().max().item()
        assert err < 2e-2, (nm, err)


@pytest.mark.gpu
def test_group_keys_three_pass_radix_gpu():
    """The in-tree radix sort over a Wide&Deep-sized key space (3.6M rows: 22 bits, three
    8-bit passes; 139k keys, not a multiple of the 2048-key tile, hot keys) is stable and
    its runs match a torch stable sort."""
    dev = torch.device("cuda", 0)
    g0 = torch.Generator().manual_seed(9)
    n, rows = 4096 * 34 - 77, 3_600_003
    keys = torch.randint(0, rows, (n,), generator=g0, dtype=torch.int32)
    keys[::5] = 1234567
    keys[::97] = -3
    keys[1::113] = rows + 5
    perm, seg_id, seg, uids = E.group_keys(keys.to(dev), rows)
    k = keys.long()
    kk = torch.where((k >= 0) & (k < rows), k, torch.full_like(k, rows))
    sk, sp = torch.sort(kk, stable=True)
    assert torch.equal(perm.cpu().long(), sp)
    runs, counts = torch.unique_consecutive(sk, return_counts=True)
    nr = runs.numel()
    want = torch.where(runs < rows, runs, torch.full_like(runs, -1)).to(torch.int32)
    assert torch.equal(uids[:nr].cpu(), want) and (uids[nr:] == -1).all()
    starts = torch.cat([torch.zeros(1, dtype=torch.long), counts.cumsum(0)])
    assert torch.equal(seg[:nr + 1].cpu().long(), starts) and (seg[nr:] == n).all()
    assert torch.equal(seg_id.cpu().long(), torch.repeat_interleave(torch.arange(nr), counts))


@pytest.mark.gpu
def test_fused_step_partial_batch_gpu():
    """A micro-batch that is not a multiple of the training GEMM's 8-row granule (a
    deadline-flushed or agreed partial piece): the fused step pads it with rows that look
    up nothing and get zero loss / gradient; the loss matches the host trainer."""
    from flink_tensorflow_amd.models.zoo.wide_deep import WideDeepConfig, WideDeepTrainer, synthetic_click_records

    cfg = WideDeepConfig.tiny()
    recs = synthetic_click_records(37, cfg, seed=9)
    g = WideDeepTrainer(cfg, device="cuda", seed=4)
    h = WideDeepTrainer(cfg, device="cpu", seed=4, fused=False)
    g.open()
    h.open()
    assert g._fused is not None
    lg, lh = float(g.train_step(recs)), float(h.train_step(recs))
    assert abs(lg - lh) <= 2e-2 * abs(lh) + 2e-3, (lg, lh)
    lg2 = float(g.train_step(recs, counts=[37]))  # the agreed form of the same piece
    lh2 = float(h.train_step(recs))
    assert abs(lg2 - lh2) <= 3e-2 * abs(lh2) + 3e-3, (lg2, lh2)
