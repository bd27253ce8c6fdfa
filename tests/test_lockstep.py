"""Collective online training over uneven streams (``parallel/step_agreement.py``,
``runtime/lockstep.py``): P = 2 worker-process ranks of one Wide&Deep trainer fed 5 : 3,
with a rebalance remainder, across checkpoints and a restart — no hang, and both replicas
bit-identical to a 1-rank reference trained on the same pieces in the same step order
(``WideDeepTrainer.train_pieces``)."""
import hashlib

import pytest
import torch

from flink_tensorflow_amd.parallel.step_agreement import RoundPlan, StepAgreement
from flink_tensorflow_amd.runtime import RestartStrategy, StreamExecutionEnvironment
from flink_tensorflow_amd.runtime.lockstep import LockstepTrainer
from flink_tensorflow_amd.runtime.sources import CollectionSource

BATCH = 64


def _digest(model, exchange=None) -> str:
    parts = [p.detach().reshape(-1).float() for p in model.dense_parameters()]
    for e in (model.emb, model.wide):
        for t in (e.table.data, e.accum):
            parts.append((exchange.merge_owner_shards(t) if exchange is not None else t).reshape(-1).float())
    return hashlib.sha256(torch.cat([p.cpu() for p in parts]).numpy().tobytes()).hexdigest()[:16]


class _Logged(LockstepTrainer):
    """Emits every step's piece (record ids) and, once all ranks finished, a digest of the
    replica (a collective: safe in ``on_finished``)."""

    def __init__(self, batch=BATCH, max_delay_ms=15.0, device="cpu"):
        from flink_tensorflow_amd.models.zoo.wide_deep import WideDeepConfig, WideDeepTrainer

        super().__init__(WideDeepTrainer(WideDeepConfig.tiny(), device=device, seed=3), batch, max_delay_ms)

    def on_step(self, plan, piece, loss, out, counts=None):
        out.collect(("piece", self.get_runtime_context().attempt, self.steps, self.rank, [r[4] for r in piece],
                     counts))

    def on_finished(self, out):
        out.collect(("digest", self.rank, self.steps, _digest(self.model.model, self.model._exchange)))


def _records(n, seed=11):
    from flink_tensorflow_amd.models.zoo.wide_deep import WideDeepConfig, synthetic_click_records

    recs = synthetic_click_records(n, WideDeepConfig.tiny(), seed=seed)
    return [tuple(r) + (i,) for i, r in enumerate(recs)]


def _reference(recs, pieces_by_step) -> str:
    """1-rank reference: the same pieces, same step order, one process, no communicator."""
    from flink_tensorflow_amd.models.zoo.wide_deep import WideDeepConfig, WideDeepTrainer

    t = WideDeepTrainer(WideDeepConfig.tiny(), device="cpu", seed=3)
    t.open()
    for s in sorted(pieces_by_step):
        ranks = pieces_by_step[s]
        t.train_pieces([[recs[i] for i in ranks.get(r, [])] for r in range(2)])
    return _digest(t.model)


def _run(recs, partition, checkpoint_dir=None, fail_after=None, device="cpu"):
    from flink_tensorflow_amd.parallel.fake import FakeCommunicator

    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(2)
    env.enable_job_communicator(True, communicator=FakeCommunicator)
    if checkpoint_dir is not None:
        env.enable_checkpointing(0.05, checkpoint_dir)
        env.set_restart_strategy(RestartStrategy.fixed_delay(2, 0.0))
    clicks = env.add_source(CollectionSource(recs, delay_s=0.0005), "clicks", parallelism=1)
    if fail_after is not None:
        from flink_tensorflow_amd.utils.fault import FailAfter

        clicks = clicks.map(FailAfter(fail_after, attempts=(0,))).name("fault").set_parallelism(1)
    clicks = partition(clicks)
    ticks = env.add_source(CollectionSource([]), "control", parallelism=1)
    sink = clicks.connect(ticks).process(_Logged(device=device)).name("trainer").run_in_processes().collect_into()
    res = env.execute("lockstep")
    return res, sink.results()


def _check(recs, out, final_attempt=0):
    digests = [o for o in out if o[0] == "digest"]
    assert sorted(d[1] for d in digests) == [0, 1], digests
    assert digests[0][2] == digests[1][2] and digests[0][3] == digests[1][3]  # replicas bit-identical
    pieces = [o for o in out if o[0] == "piece"]
    final = [p for p in pieces if p[1] == final_attempt]
    first_final = min(p[2] for p in final)
    by_step: dict = {}
    for _, att, step, rank, ids, counts in pieces:
        if (att == final_attempt and step >= first_final) or (att < final_attempt and step < first_final):
            by_step.setdefault(step, {})[rank] = ids
    assert sorted(by_step) == list(range(1, digests[0][2] + 1))  # every step accounted for, once
    trained = sorted(i for s in by_step.values() for ids in s.values() for i in ids)
    assert trained == list(range(len(recs)))  # every record trained exactly once
    assert _reference(recs, by_step) == digests[0][3]
    return by_step


def test_step_agreement_plan_local():
    a = StepAgreement()
    p = a.round(5, ended=False, barrier=-1)
    assert p == RoundPlan(((5,),), (False,), (-1,), (0,), 0) and p.step and not p.finished
    assert a.round(0, ended=True).finished
    assert RoundPlan(((), ()), (True, False), (3, 3), (0, 0)).snapshot_barrier == 3
    assert RoundPlan(((), ()), (False, False), (3, -1), (0, 0)).snapshot_barrier is None
    # k steps per round: the busiest rank sets k, the others bring empty pieces
    q = a.round(7, full=3, batch=64)
    assert q.pieces == ((64, 64, 64, 7),) and q.k == 4 and q.total == 199
    r = RoundPlan(((64, 64, 64), (), (64, 10)), (False,) * 3, (-1,) * 3, (0,) * 3)
    assert r.k == 3 and [r.counts_at(j) for j in range(3)] == [(64, 0, 64), (64, 0, 10), (64, 0, 0)]


def test_uneven_5_to_3_split_matches_one_rank_reference():
    """Rank 0 gets 5 micro-batches' worth of records, rank 1 gets 3 (custom partitioner):
    the ranks agree on every step (rank 1 joins the last ones with empty pieces), the job
    ends without a hang, both replicas are bit-identical to each other and to the 1-rank
    reference trained on the same pieces in the same order."""
    recs = _records(8 * BATCH)
    res, out = _run(recs, lambda s: s.partition_custom(lambda k, n: k, lambda r: 0 if r[4] % 8 < 5 else 1))
    by_step = _check(recs, out)
    per_rank = [sum(len(s.get(r, [])) for s in by_step.values()) for r in range(2)]
    assert per_rank == [5 * BATCH, 3 * BATCH]
    assert any(len(s.get(1, [])) == 0 for s in by_step.values())  # rank 1 stepped with an empty piece


def test_rebalance_remainder_matches_one_rank_reference():
    """A record count that is not a multiple of P x batch: the remainders are trained in
    agreed partial steps at end of input."""
    recs = _records(4 * BATCH + 37)
    res, out = _run(recs, lambda s: s.rebalance())
    by_step = _check(recs, out)
    assert any(sum(len(v) for v in s.values()) < 2 * BATCH for s in by_step.values())


def test_checkpoint_and_restart_stay_in_lockstep(tmp_path):
    """Checkpoints every 50 ms snapshot both ranks after the same agreed step (collective-
    free, owner shards); a failure restarts the job from the last one and the result is
    still bit-identical to the reference over (pre-checkpoint pieces + replayed pieces)."""
    import os

    recs = _records(6 * BATCH + 11)
    res, out = _run(recs, lambda s: s.partition_custom(lambda k, n: k, lambda r: 0 if r[4] % 8 < 5 else 1),
                    str(tmp_path / "chk"), fail_after=4 * BATCH)
    assert res.attempts == 1 and res.checkpoints, res
    _check(recs, out, final_attempt=1)
    # the trainer's checkpoints: rank 0's dense state + one owner shard per rank
    dirs = [os.path.join(str(tmp_path / "chk"), f"chk-{c}", "models", "widedeep-0") for c in res.checkpoints]
    dirs = [d for d in dirs if os.path.isdir(d)]
    assert dirs
    for d in dirs:
        files = sorted(os.listdir(d))
        assert "variables.index" in files and "shard-0-of-2.index" in files and "shard-1-of-2.index" in files


class _Eval(_Logged):
    def __init__(self, heldout):
        super().__init__()
        self.eval_records = heldout

    def on_eval(self, probs, out):
        out.collect(("eval", self.steps, self.rank, list(probs)))


def test_eval_requests_are_served_in_agreed_rounds():
    """``predict`` is collective-free; an eval command reaching one rank refreshes its
    rows from their owners in an agreed round (the peers take part with none).  Every eval
    scores exactly what the 1-rank reference predicts after the same number of steps."""
    from flink_tensorflow_amd.models.zoo.wide_deep import WideDeepConfig, WideDeepTrainer
    from flink_tensorflow_amd.parallel.fake import FakeCommunicator

    recs = _records(6 * BATCH)
    heldout = _records(32, seed=99)
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(2)
    env.enable_job_communicator(True, communicator=FakeCommunicator)
    clicks = env.add_source(CollectionSource(recs, delay_s=0.002), "clicks", parallelism=1).rebalance()
    ticks = env.add_source(CollectionSource(["eval"] * 4, delay_s=0.1), "control", parallelism=1)
    sink = clicks.connect(ticks).process(_Eval(heldout)).name("trainer").run_in_processes().collect_into()
    env.execute("lockstep-eval")
    out = sink.results()
    evals = [o for o in out if o[0] == "eval"]
    assert len(evals) >= 4  # (the control stream may reach both ranks)
    by_step = _check(recs, out)
    t = WideDeepTrainer(WideDeepConfig.tiny(), device="cpu", seed=3)
    t.open()
    done = 0
    for _, steps, rank, probs in sorted(evals, key=lambda e: e[1]):
        while done < steps:
            done += 1
            t.train_pieces([[recs[i] for i in by_step[done].get(r, [])] for r in range(2)])
        assert t.predict(heldout) == probs, (steps, rank)


@pytest.mark.gpu
def test_fused_agreed_step_gpu():
    """The fused GPU step under the agreement: ``counts=[B]`` is bitwise the plain step
    (the loss normaliser is the batch), and two ranks sharing the GPU (loopback
    communicator) fed 5 : 3 — one of them stepping with empty pieces (``empty_step``) —
    finish without a hang with bit-identical replicas."""
    from flink_tensorflow_amd.models.zoo.wide_deep import WideDeepConfig, WideDeepTrainer

    recs = _records(8 * BATCH)
    a = WideDeepTrainer(WideDeepConfig.tiny(), device="cuda", seed=3)
    b = WideDeepTrainer(WideDeepConfig.tiny(), device="cuda", seed=3)
    a.open()
    b.open()
    assert a._fused is not None
    for i in range(3):
        piece = recs[i * BATCH:(i + 1) * BATCH]
        la, lb = a.train_step(piece), b.train_step(piece, counts=[BATCH])
        assert float(la) == float(lb)
    assert _digest(a.model) == _digest(b.model)
    res, out = _run(recs, lambda s: s.partition_custom(lambda k, n: k, lambda r: 0 if r[4] % 8 < 5 else 1),
                    device=None)
    digests = [o for o in out if o[0] == "digest"]
    assert sorted(d[1] for d in digests) == [0, 1] and digests[0][2:] == digests[1][2:], digests
    pieces = [o for o in out if o[0] == "piece"]
    assert any(len(p[4]) == 0 for p in pieces if p[3] == 1)  # rank 1 ran empty steps
    assert sorted(i for p in pieces for i in p[4]) == list(range(len(recs)))


def _reference_p(recs, pieces_by_step, P) -> str:
    from flink_tensorflow_amd.models.zoo.wide_deep import WideDeepConfig, WideDeepTrainer

    t = WideDeepTrainer(WideDeepConfig.tiny(), device="cpu", seed=3)
    t.open()
    for s in sorted(pieces_by_step):
        t.train_pieces([[recs[i] for i in pieces_by_step[s].get(r, [])] for r in range(P)])
    return _digest(t.model)


def test_idle_rank_and_three_ranks_match_reference():
    """P = 3 with a keyed skew that starves rank 2 completely (it never receives a record:
    it only heartbeats and joins every step with an empty piece) and gives rank 0 twice
    rank 1's share: no hang, all three replicas bit-identical to the 1-rank reference."""
    from flink_tensorflow_amd.parallel.fake import FakeCommunicator

    P = 3
    recs = _records(6 * BATCH + 5)
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(P)
    env.enable_job_communicator(True, communicator=FakeCommunicator)
    clicks = env.add_source(CollectionSource(recs, delay_s=0.0005), "clicks", parallelism=1) \
        .partition_custom(lambda k, n: k, lambda r: 0 if r[4] % 3 else 1)
    ticks = env.add_source(CollectionSource([]), "control", parallelism=1)
    sink = clicks.connect(ticks).process(_Logged()).name("trainer").run_in_processes().collect_into()
    env.execute("lockstep-p3")
    out = sink.results()
    digests = [o for o in out if o[0] == "digest"]
    assert sorted(d[1] for d in digests) == [0, 1, 2]
    assert len({(d[2], d[3]) for d in digests}) == 1  # three bit-identical replicas, same step count
    by_step: dict = {}
    for _, att, step, rank, ids, counts in (o for o in out if o[0] == "piece"):
        by_step.setdefault(step, {})[rank] = ids
    assert sorted(by_step) == list(range(1, digests[0][2] + 1))
    assert all(len(s.get(2, [])) == 0 for s in by_step.values())  # rank 2 never had data
    assert sorted(i for s in by_step.values() for ids in s.values() for i in ids) == list(range(len(recs)))
    assert _reference_p(recs, by_step, P) == digests[0][3]


class _SleepStep:
    """A stand-in trainer whose step is one small collective plus 4 ms of "GPU" work: the
    skew test measures the agreement protocol, not a model."""

    def train_step(self, piece, counts=None):
        import time

        import torch

        from flink_tensorflow_amd.parallel import comm

        if comm.is_dist():
            comm.get().all_reduce(torch.ones(1))
        time.sleep(0.004)
        return 0.0


class _Timed(LockstepTrainer):
    """Records each step's wall time and piece size."""

    def __init__(self, **kw):
        super().__init__(_SleepStep(), BATCH, **kw)

    def on_step(self, plan, piece, loss, out, counts=None):
        import time

        from flink_tensorflow_amd.runtime.lockstep import piece_len

        out.collect(("step", self.rank, time.perf_counter(), piece_len(piece)))


def _busy_rank_rate(skew: bool, **kw) -> tuple[float, int]:
    """P = 2; rank 0's generator yields 40 micro-batches of packed rows in blocks of 3
    batches; rank 1's the same (unskewed), or nothing for 3 s (skewed: its source is alive
    but idle, so it only heartbeats): rank 0's steps per second between its first and last
    step, and the records it trained."""
    import time

    import numpy as np

    from flink_tensorflow_amd.parallel.fake import FakeCommunicator

    rows = np.zeros((40 * BATCH, 64), np.uint8)

    def gen(idx, par, start):
        if skew and idx == 1:
            t_end = time.time() + 3.0
            while time.time() < t_end:
                time.sleep(0.01)
            return
        for b in range(0, len(rows), 3 * BATCH):
            yield rows[b:b + 3 * BATCH]

    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(2)
    env.enable_job_communicator(True, communicator=FakeCommunicator)
    sink = env.generate(gen).run_in_processes().process(_Timed(**kw)).name("trainer").run_in_processes() \
        .collect_into()
    env.execute("lockstep-skew")
    st = sorted((t, n) for kind, r, t, n in (o for o in sink.results() if o[0] == "step") if r == 0)
    busy = [t for t, n in st if n]
    return (len(busy) - 1) / (busy[-1] - busy[0]), sum(n for _, n in st)


def test_idle_rank_does_not_gate_the_busy_rank():
    """with one rank starved (its source alive but idle) the busy rank
    must keep stepping at >= 80 % of its unskewed rate — the idle rank follows the busy
    one round after round (``busy_poll_ms``) instead of joining once per ``max_delay_ms``
    heartbeat (which capped it at 1000 / max_delay_ms = 20 steps/s here), and each round
    carries every full batch the busy rank holds.  Both sources are chained into their
    trainer in the worker and hand over packed-row blocks (the bench job's record form)."""
    kw = dict(max_delay_ms=50.0, steps_per_round=2)
    even, n_even = _busy_rank_rate(False, **kw)
    skew, n_skew = _busy_rank_rate(True, **kw)
    assert n_even == n_skew == 40 * BATCH  # every record of rank 0 trained exactly once
    print(f"[lockstep] busy-rank step rate: unskewed {even:.1f}/s, skewed {skew:.1f}/s ({skew / even:.2f})")
    assert skew >= 0.8 * even, (skew, even)
    assert skew > 2 * 1000 / 50.0  # far above the one-step-per-heartbeat bound


@pytest.mark.gpu
def test_agreed_step_captured_tracks_exact_step_gpu():
    """The captured agreed step (pieces padded to the fixed micro-batch with look-up-nothing
    rows, ``{nvalid, norm}`` in the staged header, ONE hipGraph for every piece size) tracks
    the exact uneven-piece step, capturing trains nothing (the first step equals the exact
    first step), and the replays never synchronise with the host."""
    import numpy as np

    from flink_tensorflow_amd.models.zoo.wide_deep import WideDeepConfig, WideDeepTrainer, pack_click_records

    cfg = WideDeepConfig.tiny()
    recs = [r[:4] for r in _records(6 * BATCH)]
    a = WideDeepTrainer(cfg, device="cuda", seed=3)
    b = WideDeepTrainer(cfg, device="cuda", seed=3)
    a.micro_batch = BATCH
    a.open()
    b.open()
    sizes = [BATCH, 40, BATCH, 17, BATCH, 3]
    pieces, o = [], 0
    for n in sizes:
        pieces.append(recs[o:o + n])
        o += n
    # packed-row blocks for a (the job's record form), tuples for b
    blocks = [[np.ascontiguousarray(pack_click_records(p, cfg, 3))] for p in pieces]
    la = [a.train_step(blocks[0], counts=[sizes[0]]).clone()]
    assert a._ag is not None and a._ag.graph is not None  # captured on the first piece
    lb = [b.train_step(pieces[0], counts=[sizes[0]]).clone()]
    torch.cuda.set_sync_debug_mode("error")
    try:
        for p, n in zip(blocks[1:], sizes[1:]):
            la.append(a.train_step(p, counts=[n]).clone())
    finally:
        torch.cuda.set_sync_debug_mode(0)
    for p, n in zip(pieces[1:], sizes[1:]):
        lb.append(b.train_step(p, counts=[n]).clone())
    torch.testing.assert_close(torch.stack(la), torch.stack(lb), rtol=2e-3, atol=2e-4)
    for (k, va), vb in zip(b.model.state_dict().items(), a.model.state_dict().values()):
        torch.testing.assert_close(vb.float(), va.float(), rtol=2e-2, atol=2e-3, msg=k)
    assert a.steps == b.steps == len(sizes)
    a.close()
    b.close()


class _BlockLogged(LockstepTrainer):
    """Packed-row blocks in, the ids (dense[0]) of every step's piece out, a digest at the end."""

    def __init__(self, **kw):
        from flink_tensorflow_amd.models.zoo.wide_deep import WideDeepConfig, WideDeepTrainer

        super().__init__(WideDeepTrainer(WideDeepConfig.tiny(), device="cpu", seed=3), BATCH, **kw)

    def on_step(self, plan, piece, loss, out, counts=None):
        from flink_tensorflow_amd.models.zoo.wide_deep import WideDeepConfig, unpack_click_rows

        ids = []
        for blk in piece:
            ids += [int(v) for v in unpack_click_rows(blk, WideDeepConfig.tiny())[1][:, 0].tolist()]
        out.collect(("piece", self.steps, self.rank, ids, counts))

    def on_finished(self, out):
        out.collect(("digest", self.rank, self.steps, _digest(self.model.model, self.model._exchange)))


def test_packed_blocks_k_steps_per_round_p3_match_reference():
    """The bench job's shape on the CPU: P = 3 generator sources chained into their
    trainers hand over packed-row BLOCKS (uneven: 7, 3 and 0 micro-batches' worth plus
    remainders; block cuts fall inside micro-batches), rounds carry up to 4 full batches
    each (``steps_per_round=2``), rank 2 only heartbeats — all three replicas end
    bit-identical to the 1-rank reference trained on the same pieces in the same order."""
    import numpy as np

    from flink_tensorflow_amd.models.zoo.wide_deep import WideDeepConfig, pack_click_records
    from flink_tensorflow_amd.parallel.fake import FakeCommunicator

    P = 3
    cfg = WideDeepConfig.tiny()
    recs = [(r[0], np.concatenate([[float(r[4])], r[1][1:]]).astype(np.float32), r[2], r[3])
            for r in _records(10 * BATCH + 29)]
    per = {0: recs[:7 * BATCH + 20], 1: recs[7 * BATCH + 20:], 2: []}

    def gen(idx, par, start):
        rows = pack_click_records(per[idx], cfg, 3) if per[idx] else None
        for b in range(0, len(per[idx]), 45):
            yield np.ascontiguousarray(rows[b:b + 45])

    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(P)
    env.enable_job_communicator(True, communicator=FakeCommunicator)
    sink = env.generate(gen).run_in_processes().process(_BlockLogged(max_delay_ms=15.0, steps_per_round=2,
                                                                     max_steps_per_round=4)) \
        .name("trainer").run_in_processes().collect_into()
    env.execute("lockstep-blocks")
    out = sink.results()
    digests = [o for o in out if o[0] == "digest"]
    assert sorted(d[1] for d in digests) == [0, 1, 2] and len({d[2:] for d in digests}) == 1
    by_step: dict = {}
    for _, step, rank, ids, counts in (o for o in out if o[0] == "piece"):
        by_step.setdefault(step, {})[rank] = ids
    assert sorted(by_step) == list(range(1, digests[0][2] + 1))
    assert sorted(i for s in by_step.values() for ids in s.values() for i in ids) == list(range(len(recs)))
    assert all(len(s.get(2, [])) == 0 for s in by_step.values())
    assert _reference_p(recs, by_step, P) == digests[0][3]
