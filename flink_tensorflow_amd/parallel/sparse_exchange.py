"""Row-sparse embedding updates across data-parallel ranks by row OWNER.

The reference has no training at all; the online-training operator this
serves lives in a ``ModelCoProcessFunction`` (``AbstractCoProcessFunction.scala:11-16``).

Every row of an embedding table has one owner, ``row % world``; only the owner's copy of a
row is authoritative and only the owner runs its optimizer.  Each rank keeps a full-size
table, but the rows it does not own are a cache that is refreshed right before it reads
them:

1. ``pull`` (before the forward): the step's unique ids go to their owners, the owners
   answer with the current fp32 rows, which are written into the local table, so the
   forward reads exactly what a replicated table would hold;
2. ``apply`` (after the backward): the rank's deduplicated gradient rows (one summed fp32
   row per unique id: the trainer's static segment sum) go to their owners with one
   ``all_to_all_v`` (per-peer counts exchanged first by one small all-gather); the owner
   merges all ranks' contributions — stable by (id, source rank), summed in rank order,
   the same association as the padded all-gather it replaces — and applies sparse
   Adagrad to its rows.  The Adagrad accumulator lives only at the owner.
3. ``merge_owner_shards`` rebuilds the full table / accumulator from the owner shards (one
   all-reduce) for checkpoints and checks.

Against the padded all-gather of one row per lookup (``models/zoo/wide_deep.py:
_sparse_sync``: ≈107 MB received per rank per step at DP=8 for the 26-field, 32-wide table
at micro-batch 4096) a rank receives its own unique rows twice (fresh rows in, gradient
contributions for its owned rows in): ≈5 MB on the benchmark's Zipf ids
(``tests/test_sparse_exchange.py``).  The counts make the step synchronise with the host,
so a step using this exchange is not captured in a hipGraph.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from ..ops.embedding import segment_sum, sparse_adagrad, unique_static


@dataclass
class ExchangeStats:
    """Bytes this rank sent / received in the last ``apply`` (payload, counts included)."""

    sent: int = 0
    received: int = 0
    rows_out: int = 0      # unique rows this rank sent to owners
    rows_owned: int = 0    # unique rows this rank updated as their owner


class OwnerSparseExchange:
    def __init__(self, comm):
        self.comm = comm
        self.stats = ExchangeStats()  # this step's totals (``begin_step`` resets them)

    def begin_step(self) -> None:
        self.stats = ExchangeStats()

    def _add(self, st: ExchangeStats) -> ExchangeStats:
        t = self.stats
        self.stats = ExchangeStats(t.sent + st.sent, t.received + st.received, t.rows_out + st.rows_out,
                                   t.rows_owned + st.rows_owned)
        return st

    def pull_lookups(self, table: torch.Tensor, ids: torch.Tensor, offset: int = 0) -> ExchangeStats:
        """``pull`` of the unique values of ``ids`` (any shape, duplicates allowed)."""
        return self.pull(table, torch.unique(ids.reshape(-1)), offset)

    def owned_mask(self, num_rows: int, device) -> torch.Tensor:
        c = self.comm
        return torch.arange(num_rows, device=device) % c.size == c.rank

    def apply(self, table: torch.Tensor, accum: torch.Tensor, uids: torch.Tensor, rows: torch.Tensor, lr: float,
              eps: float = 1e-8, offset: int = 0) -> ExchangeStats:
        """One step's sparse update of ``table`` (rows ``uids - offset``; -1 and ids outside
        the table are padding) with this rank's deduplicated gradient ``rows``."""
        c = self.comm
        ws, me = c.size, c.rank
        dev = table.device
        V, D = table.shape
        st = ExchangeStats()
        ids = uids.reshape(-1).to(torch.int64) - offset
        keep = (uids.reshape(-1) >= 0) & (ids >= 0) & (ids < V)
        ids, g = ids[keep], rows.reshape(-1, D)[keep].float()
        # 1. to the owners: stable by owner keeps every rank's id order inside a destination
        owner = ids % ws
        order = torch.sort(owner, stable=True).indices
        ids, g, owner = ids[order], g[order], owner[order]
        send_n = torch.bincount(owner, minlength=ws).to(torch.int64)
        allc = torch.empty(ws * ws, dtype=torch.int64, device=c.device)
        c.all_gather(allc, send_n.to(c.device))
        mat = allc.view(ws, ws).cpu()  # mat[src, dst]: rows src sends to dst (host sync)
        in_splits = mat[me].tolist()
        out_splits = mat[:, me].tolist()
        n_in = int(sum(out_splits))
        r_ids = torch.empty(n_in, dtype=torch.int32, device=dev)
        r_g = torch.empty((n_in, D), dtype=torch.float32, device=dev)
        with c.group():  # int32 ids + fp32 rows on the wire
            c.all_to_all_v(r_ids, out_splits, ids.to(torch.int32).contiguous(), in_splits)
            c.all_to_all_v(r_g, out_splits, g.contiguous(), in_splits)
        row_b = 4 + 4 * D
        st.rows_out = int(ids.numel())
        st.sent = 8 * ws + sum(n for r, n in enumerate(in_splits) if r != me) * row_b
        st.received = 8 * ws * (ws - 1) + sum(n for r, n in enumerate(out_splits) if r != me) * row_b
        # 2. the owner's merged update (rank order within an id: the stable sort keeps the
        # concatenation order of the sources)
        own_u, own_g = segment_sum(r_ids, r_g, V)
        sparse_adagrad(table, accum, own_u.to(torch.int32).contiguous(), own_g.contiguous(), lr, eps)
        st.rows_owned = int(own_u.numel())
        return self._add(st)

    def pull(self, table: torch.Tensor, uids: torch.Tensor, offset: int = 0) -> ExchangeStats:
        """Refreshes the rows ``uids - offset`` (unique; -1 / out-of-table ids ignored) of
        the local ``table`` from their owners."""
        c = self.comm
        ws, me = c.size, c.rank
        dev = table.device
        V, D = table.shape
        ids = uids.reshape(-1).to(torch.int64) - offset
        keep = (uids.reshape(-1) >= 0) & (ids >= 0) & (ids < V)
        ids = ids[keep]
        owner = ids % ws
        order = torch.sort(owner, stable=True).indices
        ids, owner = ids[order], owner[order]
        send_n = torch.bincount(owner, minlength=ws).to(torch.int64)
        allc = torch.empty(ws * ws, dtype=torch.int64, device=c.device)
        c.all_gather(allc, send_n.to(c.device))
        mat = allc.view(ws, ws).cpu()
        ask = mat[me].tolist()            # ids I ask of each owner
        asked = mat[:, me].tolist()       # ids each rank asks of me
        q = torch.empty(int(sum(asked)), dtype=torch.int32, device=dev)
        c.all_to_all_v(q, asked, ids.to(torch.int32).contiguous(), ask)
        ans = table[q.long()].contiguous()  # my authoritative rows, in the askers' order
        got = torch.empty((ids.numel(), D), dtype=table.dtype, device=dev)
        c.all_to_all_v(got, ask, ans, asked)
        table[ids] = got
        row_b = D * table.element_size()
        st = ExchangeStats(sent=8 * ws + sum(n for r, n in enumerate(ask) if r != me) * 4
                           + sum(n for r, n in enumerate(asked) if r != me) * row_b,
                           received=8 * ws * (ws - 1) + sum(n for r, n in enumerate(asked) if r != me) * 4
                           + sum(n for r, n in enumerate(ask) if r != me) * row_b)
        return self._add(st)

    def merge_owner_shards(self, accum: torch.Tensor) -> torch.Tensor:
        """The full table / optimizer state from the owner shards (checkpoints, checks):
        every rank's rows of the ids it owns, summed across ranks (each row has one owner)."""
        mask = self.owned_mask(accum.shape[0], accum.device).unsqueeze(-1)
        full = torch.where(mask, accum, torch.zeros((), dtype=accum.dtype, device=accum.device)).contiguous()
        # summed as integers of the same width: bit-exact (a float sum would turn an owner's
        # -0.0 into +0.0)
        ity = {4: torch.int32, 8: torch.int64}.get(full.element_size())
        if ity is None:
            self.comm.all_reduce(full)
            return full
        bits = full.view(ity)
        self.comm.all_reduce(bits)
        return bits.view(full.dtype)


class CapacityExceeded(RuntimeError):
    """A bucketed exchange dropped rows: some owner's bucket needed more slots than its
    capacity.  Raised at the next check, BEFORE the state is checkpointed, so the job
    restarts from a checkpoint that never saw a dropped update — and the restarted
    trainer opens its exchange with the slack doubled per attempt (``WideDeepTrainer``),
    so the replay does not overflow the same way again."""


class BucketedOwnerExchange(OwnerSparseExchange):
    """The owner exchange with FIXED-CAPACITY per-peer buckets: static shapes end to end,
    no host synchronisation, so a data-parallel step using it is captured in a hipGraph.

    Every exchange sends each peer a bucket of ``cap`` slots (table-local ids, -1 padding;
    rows for the gradient direction) with one equal-split ``all_to_all`` — RCCL's grouped
    send/recv with sizes fixed at capture time.  On the GPU every data movement is an
    in-tree kernel: ids are deduplicated by the radix sort (``kernels/sort_segments.hip``),
    ``owner_buckets`` (``kernels/embedding.hip``) places each id in its owner's bucket (a
    count pass and a place pass over 4096-id segments x owners: wave ballots + an LDS
    prefix, input order kept), rows move
    with ``rows_gather`` / ``rows_scatter`` and the owner merges with the static segment sum
    in (id, source rank) order — no ``torch.unique`` / ``sort`` / ``bincount``, no fancy
    indexing, and the merge association of the exact exchange.

    Capacity: before ``calibrate`` ``min(n, ceil(slack * n / world) + 64)`` for n candidate
    slots (ids spread over owners by ``id % world``: a bucket holds about U / world ≤ n /
    world distinct ids); ``calibrate`` (once, after the warm-up steps, before the capture)
    sizes every call site at ``slack x`` the largest demand its steps showed, agreed across
    ranks — Zipf click ids have far fewer distinct ids than lookups.  Slots beyond a
    bucket's capacity cannot travel: the kernel keeps the largest excess in a device
    counter (``over``) and ``check()`` raises ``CapacityExceeded`` — the trainer checks
    before every snapshot and every ``check_every`` steps (one step late, from a pinned
    copy: no sync in the step), so a dropped update never reaches a checkpoint and the
    restart replays it.

    ``exact = True`` switches to the parent's exact, host-synced exchange (the agreed steps
    of ``runtime/lockstep.py``, whose pieces differ in size across ranks)."""

    capturable = True

    def __init__(self, comm, slack: float = 2.0, check_every: int = 64):
        super().__init__(comm)
        self.slack = float(slack)
        self.check_every = int(check_every)
        self.exact = False
        self.over = torch.zeros(1, dtype=torch.int32, device=comm.device)  # largest demand beyond capacity
        self._site_need: dict = {}   # (rows, slots) -> device max demand of that call site
        self._caps: dict = {}        # (rows, slots) -> calibrated per-peer capacity
        self._pinned = None
        self._pending = None
        self._steps = 0

    @property
    def need(self) -> torch.Tensor:
        """The largest bucket demand any call site showed (device scalar)."""
        if not self._site_need:
            return torch.zeros(1, dtype=torch.int32, device=self.over.device)
        return torch.stack([v.reshape(()) for v in self._site_need.values()]).max().reshape(1)

    def capacity(self, n: int, rows: int | None = None) -> int:
        """Per-peer slots for an exchange of ``n`` candidate ids of a ``rows``-row table:
        calibrated (``calibrate``) or the a-priori ``slack x n / world + 64``."""
        c = self._caps.get((rows, n))
        if c is not None:
            return c
        ws = self.comm.size
        return max(1, min(n, -(-int(self.slack * n) // ws) + 64))

    def calibrate(self) -> dict:
        """Sizes every call site's buckets from the demand its steps so far showed
        (``slack x`` the largest, + 64, at most the slot count), agreed across ranks (max).
        One host sync: the trainer calls it once, after its warm-up steps and before it
        captures the step (``WideDeepTrainer.capture``)."""
        keys = sorted(self._site_need, key=str)
        if not keys:
            return {}
        d = torch.cat([self._site_need[k].reshape(1) for k in keys]).to(self.comm.device)
        self.comm.all_reduce(d, "max")
        ws = self.comm.size
        for k, v in zip(keys, d.cpu().tolist()):
            n = k[1]
            self._caps[k] = max(1, min(n, int(self.slack * v) + 64, -(-int(self.slack * n) // ws) + 64))
        return dict(self._caps)

    # ---- overflow accounting
    def check(self) -> None:
        """Raises ``CapacityExceeded`` if any bucket overflowed so far (host sync)."""
        over = int(self.over.item())
        if over:
            raise CapacityExceeded(f"owner bucket overflow: a bucket needed {over} slots beyond its capacity "
                                   f"(slack {self.slack}); raise EngineConfig.wd_bucket_slack")

    def step_done(self) -> None:
        """Once per training step: every ``check_every`` steps the overflow counter is copied
        to pinned memory without a sync, and the previous copy (long landed) is checked."""
        self._steps += 1
        if self.check_every <= 0 or self._steps % self.check_every:
            return
        if self._pending is not None:
            ev, host = self._pending
            ev.synchronize()
            if int(host[0]):
                raise CapacityExceeded(f"owner bucket overflow by {int(host[0])} slots (slack {self.slack})")
        if self.over.is_cuda:
            if self._pinned is None:
                self._pinned = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            self._pinned.copy_(self.over, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._pending = (ev, self._pinned)
        else:
            self._pending = (_Done(), self.over.clone())

    # ---- buckets
    def _bucket(self, uids: torch.Tensor, off: int, V: int):
        """``uids`` int32 [n] (distinct keys; -1 / outside [off, off + V) = none) ->
        (send_ids int32 [world * cap]: table-local ids by owner bucket, -1 padding;
        src int32 [world * cap]: each slot's position in ``uids``, -1 padding; cap)."""
        ws = self.comm.size
        ids = uids.reshape(-1)
        n = ids.numel()
        dev = ids.device
        site = (V, n)
        cap = self.capacity(n, V)
        need = self._site_need.get(site)
        if need is None:
            need = self._site_need[site] = torch.zeros(1, dtype=torch.int32, device=dev)
        send = torch.empty(ws * cap, dtype=torch.int32, device=dev)
        src = torch.empty(ws * cap, dtype=torch.int32, device=dev)
        if ids.is_cuda:
            from .. import _ext

            H = _ext.hip()
            ids = ids if ids.dtype == torch.int32 else ids.to(torch.int32)
            counts = torch.empty(ws * H.owner_buckets_segments(n), dtype=torch.int32, device=dev)
            H.owner_buckets(ids.contiguous().data_ptr(), n, off, V, ws, cap, send.data_ptr(), src.data_ptr(),
                            need.data_ptr(), self.over.data_ptr(), counts.data_ptr(),
                            torch.cuda.current_stream().cuda_stream)
            return send, src, cap
        # host: the same placement with torch ops (tests; the loopback communicator)
        loc = ids.long() - off
        valid = (ids >= 0) & (loc >= 0) & (loc < V)
        owner = torch.where(valid, loc.remainder(ws), torch.full_like(loc, ws))
        send.fill_(-1)
        src.fill_(-1)
        for o in range(ws):
            idx = torch.nonzero(owner == o).reshape(-1)
            k = min(idx.numel(), cap)
            send[o * cap:o * cap + k] = loc[idx[:k]].to(torch.int32)
            src[o * cap:o * cap + k] = idx[:k].to(torch.int32)
            need.copy_(torch.maximum(need, torch.tensor([idx.numel()], dtype=torch.int32)))
            if idx.numel() > cap:
                self.over.copy_(torch.maximum(self.over, torch.tensor([idx.numel() - cap], dtype=torch.int32)))
        return send, src, cap

    def _a2a(self, out, inp, cap):
        ws = self.comm.size
        self.comm.all_to_all_v(out, [cap] * ws, inp, [cap] * ws)

    def pull_lookups(self, table: torch.Tensor, ids: torch.Tensor, offset: int = 0) -> ExchangeStats:
        if self.exact:
            return super().pull_lookups(table, ids, offset)
        V = table.shape[0]
        flat = ids.reshape(-1)
        loc = torch.where((flat >= offset) & (flat < offset + V), flat - offset, torch.full_like(flat, -1))
        return self.pull(table, unique_static(loc, V), 0)

    def pull(self, table: torch.Tensor, uids: torch.Tensor, offset: int = 0) -> ExchangeStats:
        if self.exact:
            return super().pull(table, uids, offset)
        from ..ops.embedding import rows_gather, rows_scatter

        ws = self.comm.size
        V, D = table.shape
        ask, _, cap = self._bucket(uids, offset, V)
        asked = torch.empty_like(ask)
        self._a2a(asked, ask, cap)            # ids each rank asks of me (rank-major buckets)
        ans = rows_gather(table, asked)       # my authoritative rows (zeros for padding)
        got = torch.empty_like(ans)
        self._a2a(got, ans, cap)              # answers, aligned with my buckets
        rows_scatter(table, ask, got)
        row_b = D * table.element_size()
        return self._add(ExchangeStats(sent=(ws - 1) * cap * (4 + row_b), received=(ws - 1) * cap * (4 + row_b)))

    def apply(self, table: torch.Tensor, accum: torch.Tensor, uids: torch.Tensor, rows: torch.Tensor, lr: float,
              eps: float = 1e-8, offset: int = 0) -> ExchangeStats:
        if self.exact:
            return super().apply(table, accum, uids, rows, lr, eps, offset)
        from ..ops.embedding import rows_gather

        ws = self.comm.size
        V, D = table.shape
        send_ids, src, cap = self._bucket(uids, offset, V)
        send_rows = rows_gather(rows.reshape(-1, D).float().contiguous(), src)  # zeros for padding
        r_ids = torch.empty_like(send_ids)
        r_g = torch.empty_like(send_rows)
        with self.comm.group():
            self._a2a(r_ids, send_ids, cap)
            self._a2a(r_g, send_rows, cap)
        # the owner's merged update: static segment sum in (id, source rank) order
        own_u, own_g = segment_sum(r_ids, r_g, V, static=True)
        sparse_adagrad(table, accum, own_u, own_g, lr, eps)
        row_b = 4 + 4 * D
        return self._add(ExchangeStats(sent=(ws - 1) * cap * row_b, received=(ws - 1) * cap * row_b))


class _Done:
    def synchronize(self):
        pass
