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

from ..ops.embedding import segment_sum, sparse_adagrad


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
