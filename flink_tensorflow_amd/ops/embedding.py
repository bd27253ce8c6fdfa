"""Embedding ops for online training: bag lookup (fwd), row-sparse gradient (bwd) and a
sparse Adagrad update, on the HIP kernels for HBM tensors and PyTorch fp32 references on
the host.  The backward is deterministic: gradient rows are sorted by destination on the
GPU (``torch.sort``) and every destination row is summed by one wave in a fixed order."""
from __future__ import annotations

import torch

from .kernels import _check, _hip, _stream


def embedding_bag(ids: torch.Tensor, table: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """``ids`` [R, L] int32 (−1 = empty slot), ``table`` fp32 [V, D] → bf16 [R, D] (sum over L)."""
    R, L = ids.shape
    V, D = table.shape
    if out is None:
        out = torch.empty((R, D), dtype=torch.bfloat16 if table.is_cuda else torch.float32, device=table.device)
    if table.is_cuda:
        _check(ids, "ids", torch.int32, table.device)
        _check(table, "table", torch.float32, table.device)
        _check(out, "out", device=table.device)
        _hip().embedding_bag_fwd(ids.data_ptr(), table.data_ptr(), out.data_ptr(), R, L, D, V, _stream())
        return out
    idx = ids.long()
    valid = (idx >= 0) & (idx < V)
    rows = table[idx.clamp(0, V - 1)] * valid.unsqueeze(-1)
    out.copy_(rows.sum(1).to(out.dtype))
    return out


_SLICE = 8  # sorted rows per lane group in the static segment sum (one batch of 8 loads)


def group_keys(keys: torch.Tensor, num_rows: int):
    """Static-shape grouping of int32 keys on the GPU (``kernels/sort_segments.hip``: radix
    sort over the key bits in use + run boundaries; keys outside [0, num_rows) form one
    dropped bucket).  Returns ``(perm, seg_id, seg, uids)``: the stable sorted order, the
    run of every sorted position, the run starts (n past the last run) and the run keys
    (-1 past the runs / for the dropped bucket) — one slot per key, no host sync."""
    n = keys.numel()
    dev = keys.device
    H = _hip()
    if num_rows >= (1 << 30):
        raise ValueError(f"group_keys: tables of 2^30 rows or more are not supported (got {num_rows})")
    flat = keys.reshape(-1)
    if flat.dtype != torch.int32:
        # out-of-range wide ids go to the dropped bucket BEFORE narrowing: an int64 id at or
        # above 2^31 must not wrap into [0, num_rows) and update a valid row
        flat = torch.where((flat >= 0) & (flat < num_rows), flat, num_rows).to(torch.int32)
    flat = flat.contiguous()
    i32 = dict(dtype=torch.int32, device=dev)
    sorted_k, perm, seg_id, uids = (torch.empty(n, **i32) for _ in range(4))
    seg = torch.empty(n + 1, **i32)
    work = torch.empty(3 * n, **i32)
    tb = H.sort_segments_temp_bytes(n, num_rows)
    temp = torch.empty(tb, dtype=torch.uint8, device=dev)
    H.sort_segments(flat.data_ptr(), n, num_rows, sorted_k.data_ptr(), perm.data_ptr(), seg_id.data_ptr(),
                    seg.data_ptr(), uids.data_ptr(), work.data_ptr(), temp.data_ptr(), tb, _stream())
    return perm, seg_id, seg, uids


def segment_sum_grouped(groups, rows: torch.Tensor, L: int = 1, lo: int = 0, hi: int | None = None) -> torch.Tensor:
    """Per-run sums (fp32 [n, D], one row per run slot, zero for empty slots) of ``rows``
    under a ``group_keys`` grouping; only sorted positions whose original index lies in
    [lo, hi) contribute (row (index - lo) // L): tables sharing one key space share one
    sort.  Reduce-by-key over fixed slices + a fix-up pass for runs spanning slices (hot
    ids), all in fixed order (``kernels/embedding.hip``)."""
    perm, seg_id, seg, _ = groups
    n = perm.numel()
    D = rows.shape[1]
    hi = n if hi is None else hi
    out = torch.empty((n, D), dtype=torch.float32, device=rows.device)
    g = rows.contiguous()
    fp32 = g.dtype == torch.float32
    if not fp32 and g.dtype != torch.bfloat16:
        g = g.to(torch.bfloat16)
    ws = torch.empty(2 * (-(-n // _SLICE)) * D, dtype=torch.float32, device=rows.device)
    _hip().segment_sum_sorted(g.data_ptr(), perm.data_ptr(), seg_id.data_ptr(), seg.data_ptr(), out.data_ptr(),
                              ws.data_ptr(), n, n, D, L, _SLICE, int(fp32), lo, hi, _stream())
    return out


def _segment_sum_static(keys: torch.Tensor, rows: torch.Tensor, num_rows: int, L: int):
    """Sync-free, static-shape segment sum on the GPU: outputs are sized by the number of
    keys n (an upper bound of the unique count); unused slots carry uid -1 and zero rows.
    No ``.item()`` / ``unique`` host round trip, so a training step stays asynchronous
    (and capturable)."""
    groups = group_keys(keys, num_rows)
    return groups[3], segment_sum_grouped(groups, rows, L)


def segment_sum(keys: torch.Tensor, rows: torch.Tensor, num_rows: int, L: int = 1, static: bool = False):
    """Deterministic sum of ``rows[i // L]`` grouped by ``keys[i]`` (keys outside
    ``[0, num_rows)`` dropped).  Returns ``(unique keys int32 [U], sums fp32 [U, D])``;
    with ``static=True`` the outputs have one slot per key (padding uid -1, zero rows) and
    the GPU path never synchronises with the host."""
    D = rows.shape[1]
    if static:
        if keys.is_cuda and keys.numel():
            return _segment_sum_static(keys, rows, num_rows, L)
        u, r = segment_sum(keys, rows, num_rows, L)
        n = keys.numel()
        up = torch.full((n,), -1, dtype=torch.int32, device=keys.device)
        rp = torch.zeros((n, D), dtype=torch.float32, device=rows.device)
        up[: u.numel()] = u
        rp[: r.shape[0]] = r
        return up, rp
    flat = keys.reshape(-1).long()
    valid = (flat >= 0) & (flat < num_rows)
    key = torch.where(valid, flat, torch.full_like(flat, num_rows))
    sorted_ids, perm = torch.sort(key, stable=True)
    uids, counts = torch.unique_consecutive(sorted_ids, return_counts=True)
    if uids.numel() and uids[-1].item() == num_rows:  # drop the invalid bucket
        uids, counts = uids[:-1], counts[:-1]
    U = uids.numel()
    seg = torch.zeros(U + 1, dtype=torch.int64, device=keys.device)
    seg[1:] = torch.cumsum(counts, 0)
    out = torch.empty((U, D), dtype=torch.float32, device=rows.device)
    if rows.is_cuda:
        g = rows.contiguous()
        fp32 = g.dtype == torch.float32
        if not fp32 and g.dtype != torch.bfloat16:
            g = g.to(torch.bfloat16)
        # keep the int32 copies referenced until the launch is enqueued: a temporary freed
        # back to the caching allocator mid-call would let the next one reuse its block
        perm32 = perm.to(torch.int32)
        seg32 = seg.to(torch.int32)
        _hip().segment_sum_rows(g.data_ptr(), perm32.data_ptr(), seg32.data_ptr(), out.data_ptr(), U, D, L, int(fp32),
                                _stream())
        return uids.to(torch.int32), out
    src = perm[: int(seg[-1])] // L
    dst = torch.repeat_interleave(torch.arange(U), counts)
    out.zero_()
    out.index_add_(0, dst, rows.float()[src])
    return uids.to(torch.int32), out


def unique_static(keys: torch.Tensor, num_rows: int) -> torch.Tensor:
    """The distinct keys in [0, num_rows) of ``keys``, one int32 slot per key (ascending,
    -1 past the last): static shape and, on the GPU, the in-tree radix sort — no host
    sync (a capturable replacement of ``torch.unique``)."""
    flat = keys.reshape(-1)
    if flat.is_cuda and flat.numel():
        return group_keys(flat, num_rows)[3]
    f = flat.long()
    u = torch.unique(f[(f >= 0) & (f < num_rows)])
    out = torch.full((flat.numel(),), -1, dtype=torch.int32, device=flat.device)
    out[: u.numel()] = u.to(torch.int32)
    return out


def rows_gather(table: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
    """fp32 [n, D]: ``table[ids[k]]`` per slot, zeros where ``ids[k]`` is outside the table."""
    n, (V, D) = ids.numel(), table.shape
    out = torch.empty((n, D), dtype=torch.float32, device=table.device)
    if table.is_cuda:
        ids = ids.reshape(-1).to(torch.int32).contiguous()
        _hip().rows_gather(table.data_ptr(), ids.data_ptr(), out.data_ptr(), n, D, V, _stream())
        return out
    i = ids.reshape(-1).long()
    ok = (i >= 0) & (i < V)
    out.copy_(table[i.clamp(0, V - 1)] * ok.unsqueeze(-1))
    return out


def rows_scatter(table: torch.Tensor, ids: torch.Tensor, rows: torch.Tensor) -> None:
    """``table[ids[k]] = rows[k]`` for the slots whose id lies in the table (ids unique)."""
    n, (V, D) = ids.numel(), table.shape
    if table.is_cuda:
        ids = ids.reshape(-1).to(torch.int32).contiguous()
        rows = rows.contiguous()
        _hip().rows_scatter(table.data_ptr(), ids.data_ptr(), rows.data_ptr(), n, D, V, _stream())
        return
    i = ids.reshape(-1).long()
    ok = (i >= 0) & (i < V)
    table[i[ok]] = rows[ok].to(table.dtype)


def embedding_bag_backward(ids: torch.Tensor, grad_out: torch.Tensor, num_rows: int, static: bool = False):
    """Row-sparse gradient of ``embedding_bag``: returns ``(uids int32 [U], rows fp32 [U, D])``."""
    return segment_sum(ids, grad_out, num_rows, ids.shape[1], static=static)


def sparse_adagrad(table: torch.Tensor, accum: torch.Tensor, uids: torch.Tensor, grads: torch.Tensor, lr: float,
                   eps: float = 1e-8, offset: int = 0) -> None:
    """Adagrad on the rows ``uids - offset`` (``offset``: the table's base in a key space
    shared with other tables; ids outside the table, and -1, are skipped)."""
    U, D = grads.shape
    if table.is_cuda:
        _check(table, "table", torch.float32, table.device)
        _check(accum, "accum", torch.float32, table.device)
        _check(grads, "grads", torch.float32, table.device)
        _check(uids, "uids", torch.int32, table.device)
        _hip().sparse_adagrad(table.data_ptr(), accum.data_ptr(), uids.data_ptr(), grads.data_ptr(), U, D,
                              table.shape[0], float(lr), float(eps), int(offset), _stream())
        return
    uids = torch.where(uids >= 0, uids - offset, -1)
    keep = (uids >= 0) & (uids < table.shape[0])  # static-shape padding slots / other tables
    uids, grads = uids[keep], grads[keep]
    idx = uids.long()
    a = accum[idx] + grads * grads
    accum[idx] = a
    table[idx] -= lr * grads / (a.sqrt() + eps)


class EmbeddingBagFunction(torch.autograd.Function):
    """Autograd node whose table gradient is delivered row-sparse to ``table_holder``
    (dense table gradients would cost V x D per step)."""

    @staticmethod
    def forward(ctx, ids, table, anchor, holder):
        ctx.save_for_backward(ids)
        ctx.holder = holder
        ctx.V = table.shape[0]
        return embedding_bag(ids, table)

    @staticmethod
    def backward(ctx, grad):
        (ids,) = ctx.saved_tensors
        ctx.holder.sparse_grads.append(embedding_bag_backward(ids, grad, ctx.V, static=True))
        return None, None, torch.zeros_like(ctx.holder.anchor), None


class SparseEmbedding(torch.nn.Module):
    """fp32 master table + Adagrad accumulator; bf16 lookups; row-sparse updates."""

    def __init__(self, num_rows: int, dim: int, device=None, init_std: float = 0.01, seed: int = 0):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.table = torch.nn.Parameter((torch.randn(num_rows, dim, generator=g) * init_std).to(device),
                                        requires_grad=False)
        self.register_buffer("accum", torch.full((num_rows, dim), 0.1, device=device))
        # a scalar leaf that makes the lookup part of the autograd graph
        self.anchor = torch.nn.Parameter(torch.zeros((), device=device))
        self.sparse_grads: list = []

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        return EmbeddingBagFunction.apply(ids, self.table, self.anchor, self)

    def apply_updates(self, lr: float, sync=None, exchange=None, merge: bool = False):
        """Applies the step's sparse gradients (optionally synchronised across ranks:
        ``sync`` all-gathers them for every replica to apply; ``exchange`` — an
        ``parallel.sparse_exchange.OwnerSparseExchange`` — sends them to the rows' owners).
        ``merge``: always pass the rows through the segment sum, as the synchronised paths
        do (bitwise the same rows, signed zeros included, for single-process references)."""
        if not self.sparse_grads:
            return 0
        several = len(self.sparse_grads) > 1
        uids = torch.cat([u for u, _ in self.sparse_grads])
        rows = torch.cat([r for _, r in self.sparse_grads])
        self.sparse_grads.clear()
        if exchange is not None:
            if several:  # one row per id on this rank before the exchange
                uids, rows = segment_sum(uids, rows, self.table.shape[0], static=True)
            exchange.apply(self.table.data, self.accum, uids, rows, lr)
            return int(uids.numel())
        if sync is not None:
            uids, rows = sync(uids, rows)
        # merge duplicate rows (several lookups, several ranks) with the deterministic
        # segment sum so every replica applies bit-identical updates (one lookup on one
        # rank is already unique); static shapes keep the step free of host syncs
        if several or sync is not None or merge:
            uids, rows = segment_sum(uids, rows, self.table.shape[0], static=True)
        sparse_adagrad(self.table.data, self.accum, uids.to(torch.int32).contiguous(), rows.contiguous(), lr)
        return int(uids.numel())
