"""Wide & Deep recommender with online training (BASELINE config 4: RCCL all-reduce of
gradients across the GPUs of a node).

Model (Criteo-shaped synthetic data: 13 dense features, 26 categorical fields):

* wide:  Σ_f w[cross_id_f] + b           (row-sparse linear part, Adagrad)
* deep:  concat(embedding_bag(ids_f) for f, dense) → MLP 1024 → 512 → 256 → 1 (ReLU)
         embeddings: fp32 master table in HBM, bf16 lookups (HIP gather kernel), row-sparse
         deterministic backward + sparse Adagrad (HIP kernels); MLP: MFMA GEMMs with fused
         bias+ReLU epilogues forward and backward (``ops.autograd.Linear``).
* loss:  sigmoid cross-entropy; dense params: Adam.

Data parallel across ranks (one process per GPU): dense gradients are bucket-all-reduced
by ``GradBucketer`` from autograd hooks, overlapping backward; embedding gradients are
row-sparse, so ranks all-gather ``(row ids, rows)`` and every replica applies the same
deterministic merged update (tables stay bit-identical without a dense V×D all-reduce).

``WideDeepTrainer`` is a ``RichModel`` + ``CheckpointedModel``: streaming checkpoints
write all weights and optimizer state as a TensorBundle V2 into the checkpoint dir.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F

from ...io import bundle
from ...ops.autograd import Linear
from ...utils.tracing import capture_lock, graph_capture
from ...ops.embedding import SparseEmbedding
from ...parallel import comm
from ...runtime.model_functions import CheckpointedModel
from ..core import RichModel, default_device


@dataclass
class WideDeepConfig:
    num_dense: int = 13
    num_fields: int = 26
    vocab_per_field: int = 100_000
    embed_dim: int = 32
    hidden: tuple = (1024, 512, 256)
    wide_buckets: int = 1_000_003
    lr_dense: float = 1e-3
    lr_sparse: float = 0.05

    @staticmethod
    def tiny(**kw):
        d = dict(num_dense=5, num_fields=4, vocab_per_field=100, embed_dim=8, hidden=(32, 16), wide_buckets=1009)
        d.update(kw)
        return WideDeepConfig(**d)


class WideDeep(torch.nn.Module):
    def __init__(self, cfg: WideDeepConfig, device=None, seed: int = 0):
        super().__init__()
        torch.manual_seed(seed)
        self.cfg = cfg
        dev = torch.device(device) if device is not None else torch.device("cpu")
        self.emb = SparseEmbedding(cfg.num_fields * cfg.vocab_per_field, cfg.embed_dim, dev, seed=seed)
        self.wide = SparseEmbedding(cfg.wide_buckets, 8, dev, init_std=0.0, seed=seed + 1)  # col 0 used
        width = cfg.num_fields * cfg.embed_dim + cfg.num_dense
        self.in_pad = -(-width // 8) * 8
        layers = []
        w = self.in_pad
        for h in cfg.hidden:
            layers.append(Linear(w, h, "relu", device=dev, dtype=torch.bfloat16 if dev.type == "cuda" else torch.float32))
            w = h
        self.mlp = torch.nn.ModuleList(layers)
        self.head = Linear(w, 8, None, device=dev, dtype=torch.bfloat16 if dev.type == "cuda" else torch.float32)
        self.wide_bias = torch.nn.Parameter(torch.zeros((), device=dev))
        self.device = dev

    def forward(self, dense: torch.Tensor, cats: torch.Tensor, cross: torch.Tensor) -> torch.Tensor:
        """dense [B, num_dense] float, cats [B, F] int32 (field-local ids), cross [B, C] int32 → logits [B]."""
        cfg = self.cfg
        B = dense.shape[0]
        offs = (torch.arange(cfg.num_fields, device=cats.device, dtype=torch.int32) * cfg.vocab_per_field)
        ids = (cats + offs).reshape(B * cfg.num_fields, 1)
        e = self.emb(ids).reshape(B, cfg.num_fields * cfg.embed_dim)
        x = torch.cat([e, dense.to(e.dtype)], 1)
        if x.shape[1] != self.in_pad:
            x = F.pad(x, (0, self.in_pad - x.shape[1]))
        for l in self.mlp:
            x = l(x)
        deep = self.head(x)[:, 0].float()
        wide = self.wide(cross.reshape(-1, 1)).reshape(B, -1, 8)[:, :, 0].float().sum(1)
        return deep + wide + self.wide_bias

    def dense_parameters(self):
        return [p for n, p in self.named_parameters() if p.requires_grad and not n.endswith("table")]

    def state(self) -> dict[str, torch.Tensor]:
        return {k: v.detach() for k, v in self.state_dict().items()}


def _rebase_view(t: torch.Tensor, base: torch.Tensor, new_base: torch.Tensor) -> torch.Tensor:
    """The view of ``new_base`` (a same-shape copy of ``base``) that ``t`` is of ``base``."""
    nb = new_base.view(torch.uint8).reshape(-1)
    off = t.data_ptr() - base.data_ptr()
    es = t.element_size()
    if off % es:
        raise ValueError("misaligned view")
    flat = nb[off:].view(t.dtype) if off else nb.view(t.dtype)
    return flat.as_strided(t.shape, t.stride())


def _sparse_sync(uids: torch.Tensor, rows: torch.Tensor):
    """All-gather row-sparse gradients.  The static-shape sparse pipeline pads every rank's
    (uids, rows) to the same length (one slot per looked-up id, uid -1 = empty), so the
    exchange is two fixed-size all-gathers with no size round trip or host sync."""
    if not comm.is_dist():
        return uids, rows
    c = comm.get()
    ws = c.size
    gu = torch.empty((ws * uids.numel(),), dtype=uids.dtype, device=uids.device)
    gr = torch.empty((ws * rows.shape[0], rows.shape[1]), dtype=rows.dtype, device=rows.device)
    with c.group():  # both gathers in one RCCL launch
        c.all_gather(gu, uids.contiguous())
        c.all_gather(gr, rows.contiguous())
    return gu, gr  # -1 ids are dropped by the merge


def _sparse_sync_var(uids: torch.Tensor, rows: torch.Tensor):
    """``_sparse_sync`` for pieces of different sizes (an agreed step over uneven inputs,
    ``parallel/step_agreement.py``): the slot counts are all-gathered first and every rank
    pads its slots (uid -1, zero rows) to the largest."""
    if not comm.is_dist():
        return uids, rows
    c = comm.get()
    n = torch.tensor([uids.numel()], dtype=torch.int64, device=c.device)
    sizes = torch.empty(c.size, dtype=torch.int64, device=c.device)
    c.all_gather(sizes, n)
    cap = int(sizes.max().item())
    if cap > uids.numel():
        pad = cap - uids.numel()
        uids = torch.cat([uids.reshape(-1), torch.full((pad,), -1, dtype=uids.dtype, device=uids.device)])
        rows = torch.cat([rows, torch.zeros((pad, rows.shape[1]), dtype=rows.dtype, device=rows.device)])
    return _sparse_sync(uids, rows)


class WideDeepTrainer(RichModel, CheckpointedModel):
    """Online trainer: ``train_step(records)`` on micro-batches of
    ``(label, dense[13], cats[26], cross[C])`` records; ``predict(records)``."""

    restart_attempt = 0  # the job attempt this replica was opened in (set by the operator)
    restart_budget: int | None = None  # the job's restart attempts (None: not run by a job operator)
    micro_batch: int | None = None  # fixed piece size of captured agreed steps (set by LockstepTrainer)
    capture_agreed = True  # agreed fused-GPU steps replay one hipGraph (False: the same padded step, eager)

    _TRANSIENT = ("_model", "_opt", "_bucketer", "_graph", "_static", "_static_loss", "_fused", "_exchange",
                  "_ag")
    uses_collectives = True  # under DP every step all-reduces / exchanges: the job forms a communicator

    def __init__(self, cfg: WideDeepConfig | None = None, device=None, seed: int = 0, fused: bool | None = None):
        self.cfg = cfg or WideDeepConfig()
        self.device = device
        self.seed = seed
        # fused: the hand-fused GPU step (models/zoo/wide_deep_fused.py); None = on a GPU
        # unless EngineConfig.wd_fused_step is off.  False: autograd forward/backward + torch Adam.
        self.fused = fused
        self._exchange = None  # owner-based sparse exchange under DP (parallel/sparse_exchange.py)
        self._model = self._opt = self._bucketer = self._fused = None
        self._graph = self._static = self._static_loss = None
        self._ag = None  # the captured agreed step (``_AgreedStep``)
        self.steps = 0

    def open(self):
        dev = torch.device(self.device) if self.device is not None else default_device()
        self._model = WideDeep(self.cfg, dev, self.seed)
        if comm.is_dist():  # identical initial replicas: rank 0's weights to everyone
            comm.broadcast_tensors([p.data for p in self._model.parameters()] + list(self._model.buffers()), 0)
        from ...config import current

        use_fused = self.fused if self.fused is not None else current().wd_fused_step
        mode = current().wd_sparse_exchange
        if comm.is_dist() and comm.get().size > 1 and mode in ("owner", "bucketed"):
            from ...parallel.sparse_exchange import BucketedOwnerExchange, OwnerSparseExchange

            if mode == "bucketed" and self.restart_budget == 0:
                # a bucket overflow is recovered by restarting from the last checkpoint with
                # doubled slack: a job without restarts would just fail on it
                raise ValueError("wd_sparse_exchange='bucketed' needs a restart strategy (set restart_attempts "
                                 "> 0 / env.set_restart_strategy) or use the exact 'owner' exchange")

            # each restart doubles the bucket slack (up to 16x): a job that failed on a bucket
            # overflow (CapacityExceeded, raised before any checkpoint saw a dropped row)
            # replays its input with larger buckets instead of overflowing again
            slack = current().wd_bucket_slack * 2.0 ** min(int(self.restart_attempt), 4)
            self._exchange = (BucketedOwnerExchange(comm.get(), slack) if mode == "bucketed"
                              else OwnerSparseExchange(comm.get()))
        from .wide_deep_fused import FusedWideDeepStep

        if dev.type == "cuda" and use_fused and FusedWideDeepStep.supports(self.cfg):
            self._fused = FusedWideDeepStep(self._model, self.cfg.lr_dense, self.cfg.lr_sparse, exchange=self._exchange)
            return
        fused = dev.type == "cuda"  # one multi-tensor Adam launch instead of one per parameter tensor
        self._opt = torch.optim.Adam(self._model.dense_parameters(), lr=self.cfg.lr_dense, fused=fused,
                                     capturable=fused)
        self._bucketer = comm.GradBucketer(self._model.dense_parameters())

    def finish_training(self) -> None:
        """End of training (``LockstepTrainer`` at agreed end of input, a bounded loop's
        end): the bucketed exchange's last overflow check — a dropped row in the final
        steps raises ``CapacityExceeded`` here instead of being published."""
        ex = self._exchange
        if ex is not None and hasattr(ex, "check"):
            ex.check()

    def close(self):
        ex = self._exchange
        try:
            if ex is not None and hasattr(ex, "check") and self._model is not None:
                ex.check()  # never release a replica whose last window dropped rows unnoticed
        finally:
            if self._bucketer is not None:
                self._bucketer.remove()
            self._model = self._opt = self._bucketer = self._fused = self._exchange = None
            self._graph = self._static = self._static_loss = None
            self._ag = None

    @property
    def exchange_stats(self):
        """Bytes sent / received by the last step's owner exchange (None without one)."""
        return self._exchange.stats if self._exchange is not None else None

    @property
    def is_open(self):
        return self._model is not None

    @property
    def model(self) -> WideDeep:
        return self._model

    # ---- batches
    def collate(self, records):
        if records and isinstance(records[0], np.ndarray):  # blocks of packed click rows
            rows = np.concatenate([r.reshape(-1, r.shape[-1]) for r in records])
            return unpack_click_rows(rows, self.cfg, self._model.device)
        labels = torch.tensor([r[0] for r in records], dtype=torch.float32)
        dense = torch.from_numpy(np.stack([np.asarray(r[1], np.float32) for r in records]))
        cats = torch.from_numpy(np.stack([np.asarray(r[2], np.int32) for r in records]))
        cross = torch.from_numpy(np.stack([np.asarray(r[3], np.int32) for r in records]))
        d = self._model.device
        nb = d.type == "cuda"
        return (labels.to(d, non_blocking=nb), dense.to(d, non_blocking=nb), cats.to(d, non_blocking=nb),
                cross.to(d, non_blocking=nb))

    def train_step(self, records=None, batch=None, counts=None) -> float:
        """One training step on a micro-batch (``records`` or a collated ``batch``).

        ``counts``: the per-rank record counts of an AGREED step (``parallel/step_agreement.py``,
        driven by ``runtime/lockstep.py``): this rank's piece may be empty or smaller than
        its peers'; the loss is the piece's sum over ``sum(counts)`` and the dense gradients
        are summed across ranks, so the update is the gradient of the mean over the union
        of the pieces, and every rank issues the same collectives in the same order."""
        if counts is not None and self._fused is not None and self.micro_batch and batch is None:
            return self._agreed_step(records or [], counts)
        if counts is not None:
            n = int(batch[0].shape[0]) if batch is not None else sum(_piece_rows(r) for r in (records or ()))
            if n:
                batch = batch if batch is not None else self.collate(records)
            ex = self._exchange
            if ex is not None and hasattr(ex, "exact"):
                ex.exact = True  # pieces differ in size across ranks: exact, host-sized exchange
            try:
                return self._step(batch if n else None, norm=int(sum(counts)))
            finally:
                if ex is not None and hasattr(ex, "exact"):
                    ex.exact = False
        batch = batch if batch is not None else self.collate(records)
        if self._graph is not None and all(a.shape == b.shape for a, b in zip(batch, self._static)):
            sp, bp = getattr(self._static, "packed", None), getattr(batch, "packed", None)
            if sp is not None and bp is not None and sp.shape == bp.shape:
                sp.copy_(bp, non_blocking=True)  # one copy re-binds all four views
            else:
                for dst, src in zip(self._static, batch):  # new micro-batch into the captured inputs
                    dst.copy_(src, non_blocking=True)
            self._graph.replay()
            self.steps += 1
            self._after_step()
            return self._static_loss
        loss = self._step(batch)
        self._after_step()
        return loss

    def _agreed_step(self, piece, counts) -> torch.Tensor:
        """An agreed step on the fused GPU path: the piece (tuples or packed-row blocks, 0 to
        ``micro_batch`` records) is staged into the fixed-size packed batch, padded with
        look-up-nothing rows, with ``{nvalid, norm}`` in the header row; ONE captured step
        replays for every piece size — empty pieces included — so the agreed stream runs at
        the captured step's rate with no host sync inside the step."""
        total = int(sum(counts))
        if self._ag is None:
            self._ag = _AgreedStep(self, piece)
        return self._ag.run(piece, total)

    def _after_step(self) -> None:
        if self._exchange is not None and hasattr(self._exchange, "step_done"):
            self._exchange.step_done()  # bucket overflow check, one step late and sync-free

    def capture(self, batch) -> None:
        """Captures one whole training step (forward, backward, fused Adam, sparse Adagrad
        row updates) as a hipGraph for micro-batches shaped like ``batch``; later
        ``train_step`` calls with that shape replay it (one launch instead of ~190).  The
        sparse pipeline is static-shape and sync-free, which is what makes this possible.
        Under data parallelism the RCCL collectives are captured too: the bucketed dense
        all-reduce forks onto the communicator's stream and joins back through events, and
        the row-sparse exchange — the fixed-capacity owner buckets (``wd_sparse_exchange =
        "bucketed"``, calibrated on the warm-up steps) or the padded all-gathers — runs on
        the capturing stream, so one replay is one whole DP step."""
        dev = self._model.device
        if self._exchange is not None and not getattr(self._exchange, "capturable", False):
            return  # the exact owner exchange sizes its messages on the host: steps run uncaptured
        packed = getattr(batch, "packed", None)
        if packed is not None:  # static copy of the packed buffer + the same views into it
            sp = packed.to(dev).clone()
            self._static = PackedBatch(tuple(_rebase_view(t, packed, sp) for t in batch), sp)
        else:
            self._static = tuple(t.to(dev).clone() for t in batch)
        with capture_lock():
            s = torch.cuda.Stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                for _ in range(2):  # warm-up (real steps): allocator pools, optimizer state
                    self._step(self._static)
                if self._exchange is not None and hasattr(self._exchange, "calibrate"):
                    self._exchange.calibrate()  # bucket capacities from the warm-up demand (one sync)
                    self._step(self._static)    # ... and one step on the calibrated buckets
            torch.cuda.current_stream(dev).wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with graph_capture(g):
                self._static_loss = self._step(self._static)
            self._graph = g

    def _step(self, batch, norm: int | None = None):
        """``norm`` None: a plain step (batch mean, gradients averaged over ranks).  Else an
        agreed step: ``batch`` None when this rank brings no records."""
        m = self._model
        agreed = norm is not None
        if self._fused is not None:
            loss = self._fused.step(*batch, norm=norm) if batch is not None else self._fused.empty_step()
            self.steps += 1
            return loss
        if batch is None:
            batch = self._empty_batch()
        labels, dense, cats, cross = batch
        if self._exchange is not None:
            self._exchange.begin_step()
            self.pull_rows(cats, cross)
        self._opt.zero_grad(set_to_none=True)
        # agreed steps launch the buckets in index order at synchronize(): a rank without
        # records has no backward to launch them from, and the order must match its peers'
        self._bucketer.deferred = agreed
        self._bucketer.average = not agreed
        if labels.numel():
            logits = m(dense, cats, cross)
            if agreed:
                loss = F.binary_cross_entropy_with_logits(logits, labels, reduction="sum") / norm
            else:
                loss = F.binary_cross_entropy_with_logits(logits, labels)
            loss.backward()
        else:  # no rows to send, but the sparse exchange is collective: take part with none
            loss = torch.zeros((), device=m.device)
            for e in (m.emb, m.wide):
                e.sparse_grads.append((torch.empty(0, dtype=torch.int32, device=m.device),
                                       torch.empty((0, e.table.shape[1]), dtype=torch.float32, device=m.device)))
        self._bucketer.synchronize()  # dense grads: bucketed all-reduce (launched during backward unless deferred)
        self._opt.step()
        sync = (_sparse_sync_var if agreed else _sparse_sync) if comm.is_dist() else None
        m.emb.apply_updates(self.cfg.lr_sparse, sync, self._exchange)
        m.wide.apply_updates(self.cfg.lr_sparse, sync, self._exchange)
        self.steps += 1
        return loss.detach()

    def _empty_batch(self):
        cfg, dev = self.cfg, self._model.device
        return (torch.empty(0, device=dev), torch.empty((0, cfg.num_dense), device=dev),
                torch.empty((0, cfg.num_fields), dtype=torch.int32, device=dev),
                torch.empty((0, 1), dtype=torch.int32, device=dev))

    def train_pieces(self, pieces) -> torch.Tensor:
        """The 1-rank reference of an agreed data-parallel step: the pieces ``P`` ranks
        bring to one round (rank order, empty ones included), trained in ONE process with
        the arithmetic of the P-rank step — each piece's gradients of its loss sum over the
        round's record count, summed in rank order starting from rank 0's (zeros for an
        empty piece), as the loopback / 2-rank all-reduce sums them; the sparse rows merged
        in (id, piece) order, as the owner exchange and the padded all-gather merge them.
        Host autograd path only (tests pin DP replicas to it bit for bit)."""
        if comm.is_dist() or self._fused is not None:
            raise RuntimeError("train_pieces is the single-process host reference")
        m = self._model
        norm = sum(len(p) for p in pieces)
        params = [p for p in self._opt.param_groups[0]["params"]]
        acc = None
        total = torch.zeros(())
        for recs in pieces:
            self._opt.zero_grad(set_to_none=True)
            if recs:
                labels, dense, cats, cross = self.collate(recs)
                loss = F.binary_cross_entropy_with_logits(m(dense, cats, cross), labels, reduction="sum") / norm
                loss.backward()
                total = total + loss.detach()
            g = [p.grad.detach().clone() if p.grad is not None else torch.zeros_like(p) for p in params]
            acc = g if acc is None else [a + b for a, b in zip(acc, g)]
        for p, a in zip(params, acc):
            p.grad = a
        self._opt.step()
        m.emb.apply_updates(self.cfg.lr_sparse, merge=True)
        m.wide.apply_updates(self.cfg.lr_sparse, merge=True)
        self.steps += 1
        return total

    def pull_rows(self, cats, cross) -> None:
        """Owner exchange: refreshes the embedding / wide rows this batch looks up from their
        owners (the rows a rank does not own are a cache, ``parallel/sparse_exchange.py``)."""
        m, cfg = self._model, self.cfg
        offs = torch.arange(cfg.num_fields, device=cats.device, dtype=torch.int64) * cfg.vocab_per_field
        self._exchange.pull_lookups(m.emb.table.data, cats.to(torch.int64) + offs)
        self._exchange.pull_lookups(m.wide.table.data, cross)

    @torch.no_grad()
    def refresh_rows(self, records) -> None:
        """Under the owner exchange: refreshes the rows ``records`` look up from their owners
        (COLLECTIVE — every rank calls it at the same point, with its own records or none;
        ``runtime/lockstep.py`` does so in an agreed round).  No-op otherwise."""
        if self._exchange is None:
            return
        if records:
            _, _, cats, cross = self.collate(records)
        else:
            _, _, cats, cross = self._empty_batch()
        ex = self._exchange
        exact = getattr(ex, "exact", None)
        if exact is not None:
            ex.exact = True  # one rank asks, the others ask nothing: exact, host-sized exchange
        try:
            self.pull_rows(cats, cross)
        finally:
            if exact is not None:
                ex.exact = exact

    @torch.no_grad()
    def predict(self, records) -> list[float]:
        """Scores ``records`` with this replica's tables — collective-free, so it is safe
        anywhere in a stream.  Under the owner exchange the rows this rank does not own are
        its cache, current as of the last step or ``refresh_rows`` that read them: call
        ``refresh_rows`` in an agreed round first for owner-fresh rows."""
        _, dense, cats, cross = self.collate(records)
        return torch.sigmoid(self._model(dense, cats, cross)).tolist()

    # ---- CheckpointedModel
    _SHARDED = ("emb.table", "emb.accum", "wide.table", "wide.accum")

    def snapshot_state(self, ctx):
        """Collective-free (a barrier reaches the ranks at different points of
        their step sequences, so a collective here could pair with a peer's step).  The
        dense weights and optimizer state are identical on every replica: rank 0 writes
        them.  Under the owner exchange only the owner's copy of a row (and its Adagrad
        state) is authoritative: every rank writes the rows it owns (``row % world ==
        rank``) as its own shard file, and a restore assembles the tables from all shards.
        With ``runtime/lockstep.py`` the ranks snapshot after the same agreed step."""
        if self._exchange is not None and hasattr(self._exchange, "check"):
            self._exchange.check()  # a dropped bucket slot must never reach a checkpoint
        rank, ws = comm.rank_size()
        sharded = self._exchange is not None
        st, shard = {}, {}
        for k, v in self._model.state().items():
            if sharded and k in self._SHARDED:
                shard[f"shard/{k}"] = v[rank::ws].contiguous()
            elif rank == 0:
                st[f"model/{k}"] = v
        if rank == 0:
            if self._fused is not None:
                st.update(self._fused.state())
            else:
                for i, s in enumerate(self._opt.state_dict()["state"].values()):
                    for k, v in s.items():
                        if torch.is_tensor(v):
                            st[f"adam/{i}/{k}"] = v.detach().reshape(v.shape)
        d = self._state_dir(ctx)
        if d is not None:
            if st:
                bundle.save_tensors(os.path.join(d, "variables"), st)
            if shard:
                bundle.save_tensors(os.path.join(d, f"shard-{rank}-of-{ws}"), shard)
        ctx.operator_state.blobs["widedeep_steps"] = self.steps

    @staticmethod
    def _state_dir(ctx) -> str | None:
        """One directory for the whole group (rank 0's dense state + every rank's shard)."""
        if ctx.checkpoint_dir is None:
            return None
        d = os.path.join(ctx.checkpoint_dir, "models", "widedeep-0")
        os.makedirs(d, exist_ok=True)
        return d

    def initialize_state(self, ctx):
        if not ctx.is_restored() or ctx.checkpoint_dir is None:
            return
        d = os.path.join(ctx.checkpoint_dir, "models", "widedeep-0")
        prefix = os.path.join(d, "variables")
        if not os.path.exists(prefix + ".index"):
            return
        if self._model is None:
            self.open()
        with bundle.BundleReader(prefix) as r:
            sd = {k[len("model/"):]: r.read(k) for k in r.keys() if k.startswith("model/")}
            adam = {k: r.read(k) for k in r.keys() if k.startswith("adam/")}
        shards = sorted(f[:-len(".index")] for f in os.listdir(d) if f.startswith("shard-") and f.endswith(".index"))
        if shards:  # owner shards: rows r::world of every sharded tensor come from rank r's file
            world = int(shards[0].rsplit("-of-", 1)[1])
            if len(shards) != world:
                raise RuntimeError(f"checkpoint {d} holds {len(shards)} of {world} owner shards")
            cur = self._model.state()
            for k in self._SHARDED:
                sd[k] = torch.empty_like(cur[k], device="cpu")
            for f in shards:
                rank = int(f.split("-")[1])
                with bundle.BundleReader(os.path.join(d, f)) as r:
                    for k in self._SHARDED:
                        sd[k][rank::world] = r.read(f"shard/{k}").reshape(sd[k][rank::world].shape)
        with torch.no_grad():  # in place: the fused step's parameters are views of its flat buffer
            for k, v in self._model.state_dict().items():
                if k in sd:
                    v.copy_(sd[k].to(v.device).reshape(v.shape))
        if self._fused is not None:
            self._fused.load_state(adam)
        else:
            self._load_adam(adam)
        self.steps = ctx.operator_state.blobs.get("widedeep_steps", 0)

    def _load_adam(self, adam: dict) -> None:
        """Restores torch Adam's per-parameter state (``adam/<i>/<key>``) of the autograd path."""
        if not adam:
            return
        sd = self._opt.state_dict()
        ids = list(sd["state"].keys()) or [i for g in sd["param_groups"] for i in g["params"]]
        state = {}
        for i, pid in enumerate(ids):
            ent = {k.split("/", 2)[2]: v for k, v in adam.items() if k.startswith(f"adam/{i}/")}
            if ent:
                state[pid] = ent
        sd["state"] = state
        self._opt.load_state_dict(sd)


def click_record_layout(cfg: WideDeepConfig, n_cross: int = 8) -> np.dtype:
    """Fixed-size binary row of one labelled click record (little-endian):
    ``label f32 | dense f32[num_dense] | cats i32[num_fields] | cross i32[n_cross]`` —
    the TensorValue-style wire row a Criteo stream carries (192 B for the default
    config), so a micro-batch is staged by one native gather of rows into pinned memory
    and split into tensors on the device (no per-record Python work)."""
    return np.dtype([("label", "<f4"), ("dense", "<f4", (cfg.num_dense,)), ("cats", "<i4", (cfg.num_fields,)),
                     ("cross", "<i4", (n_cross,))])


def pack_click_records(records, cfg: WideDeepConfig, n_cross: int | None = None) -> np.ndarray:
    """``(label, dense, cats, cross)`` tuples -> uint8 rows ``[n, row_bytes]`` (``n_cross``
    defaults to the first record's crossed-feature count, 8 for an empty list)."""
    if n_cross is None:
        n_cross = len(records[0][3]) if len(records) else 8
    lay = click_record_layout(cfg, n_cross)
    arr = np.zeros(len(records), lay)
    for i, r in enumerate(records):  # (label, dense, cats, cross[, anything else])
        arr[i] = tuple(r[:4])
    return arr.view(np.uint8).reshape(len(records), lay.itemsize)


def _piece_rows(x) -> int:
    return int(x.shape[0]) if isinstance(x, np.ndarray) and x.ndim == 2 else 1


def n_cross_of_row(cfg: WideDeepConfig, row_bytes: int) -> int:
    """Crossed-id count of a packed click row of ``row_bytes`` bytes."""
    c, r = divmod(row_bytes - 4 - 4 * cfg.num_dense - 4 * cfg.num_fields, 4)
    if r or c <= 0:
        raise ValueError(f"{row_bytes}-byte rows are not click rows of this config")
    return c


def unpack_click_rows(rows: np.ndarray, cfg: WideDeepConfig, device=None) -> tuple:
    """uint8 packed rows ``[n, row]`` -> ``(labels, dense, cats, cross)`` tensors."""
    lay = click_record_layout(cfg, n_cross_of_row(cfg, rows.shape[1]))
    a = np.ascontiguousarray(rows).view(lay).reshape(-1)
    out = (torch.from_numpy(a["label"].copy()), torch.from_numpy(a["dense"].copy()),
           torch.from_numpy(a["cats"].copy()), torch.from_numpy(a["cross"].copy()))
    return tuple(t.to(device) for t in out) if device is not None else out


def pad_click_row(cfg: WideDeepConfig, n_cross: int = 8) -> np.ndarray:
    """A packed row that looks up nothing (ids < 0: no embedding row, no wide row, no key)
    with label 0: the padding of a fixed-size agreed-step piece."""
    lay = click_record_layout(cfg, n_cross)
    a = np.zeros(1, lay)
    a["cats"] = -(1 << 30)
    a["cross"] = -1
    return a.view(np.uint8).reshape(lay.itemsize)


class _AgreedStep:
    """The captured agreed step of a fused-GPU ``WideDeepTrainer``: a header-carrying
    ``PackedBatchStager`` H2Ds each piece straight into the static packed batch (pinned
    slots double-buffered), and one hipGraph replays the whole step.  The graph is captured
    on the first piece: its warm-up steps (and the bucketed exchange's calibration on real
    demand) run on it, then every tensor a step mutates is handed back unchanged, so
    capturing trains nothing.  Under the exact owner exchange (not capturable) the same
    padded step runs eagerly."""

    def __init__(self, trainer: "WideDeepTrainer", first_piece):
        t = trainer
        self.t = t
        B = -(-int(t.micro_batch) // 8) * 8
        dev = t._model.device
        x = next((r for r in first_piece if isinstance(r, np.ndarray)), None)
        if x is not None:
            n_cross = n_cross_of_row(t.cfg, x.shape[-1])
        elif first_piece:
            n_cross = len(first_piece[0][3])
        else:
            n_cross = 8
        self.stager = PackedBatchStager(t.cfg, B, dev, n_cross=n_cross, header=True)
        self.static = torch.zeros((B + 1, self.stager.row), dtype=torch.uint8, device=dev)
        self.B = B
        self.graph = None
        self.loss = None
        ex = t._exchange
        c = comm.get() if comm.is_dist() else None
        # a host-staged test communicator (parallel/fake.py) or the exact owner exchange
        # cannot run inside a capture: the same padded step then runs eagerly
        self.capturable = (ex is None or getattr(ex, "capturable", False)) and getattr(c, "capturable", True)

    def run(self, piece, total: int) -> torch.Tensor:
        t = self.t
        batch = self.stager.stage_piece(piece, total, into=self.static)
        if not self.capturable or not t.capture_agreed:
            loss = t._fused.step(*batch, args=batch.args)
        else:
            if self.graph is None:
                self._capture(batch)
            self.graph.replay()
            loss = self.loss
        t.steps += 1
        t._after_step()
        return loss

    def _capture(self, batch) -> None:
        t, f = self.t, self.t._fused
        dev = t._model.device
        keep = [x.clone() for x in f.mutable_tensors()]
        with capture_lock():
            s = torch.cuda.Stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                for _ in range(2):  # warm-up: allocator pools, exchange demand
                    f.step(*batch, args=batch.args)
                ex = t._exchange
                if ex is not None and hasattr(ex, "calibrate"):
                    ex.calibrate()
                    f.step(*batch, args=batch.args)
            torch.cuda.current_stream(dev).wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with graph_capture(g):
                self.loss = f.step(*batch, args=batch.args)
            self.graph = g
            for x, k in zip(f.mutable_tensors(), keep):  # the warm-ups trained nothing
                x.copy_(k)
            f.refresh()
            if ex is not None and hasattr(ex, "over"):
                ex.over.zero_()


class PackedBatch(tuple):
    """``(labels, dense, cats, cross)`` as views of ONE device buffer of packed rows
    (``.packed``): a captured training step re-binds a batch with a single copy.  ``args``:
    the header row's device ``{nvalid, norm}`` of an agreed-step piece (else None)."""

    def __new__(cls, parts, packed):
        t = super().__new__(cls, parts)
        t.packed = packed
        t.args = None
        return t


class PackedBatchStager:
    """Micro-batch staging of packed click rows: native multithreaded gather into a pinned
    slot, async H2D on the current stream, and device-side views split into (labels,
    dense, cats, cross).  ``depth`` slots rotate; a slot is reused only after the H2D
    that read it completed (event), so the host can stage batch i+1 while batch i trains."""

    def __init__(self, cfg: WideDeepConfig, batch: int, device, n_cross: int = 8, depth: int = 2,
                 header: bool = False):
        from ... import _ext

        self.lay = click_record_layout(cfg, n_cross)
        self.row = self.lay.itemsize
        self.batch = batch
        self.cfg, self.n_cross = cfg, n_cross
        self.device = torch.device(device)
        self._native = _ext.native()
        pin = self.device.type == "cuda"
        # header: one more row after the batch carrying the piece's {nvalid, norm} (int32,
        # float32 bits) for the fused step's device arguments (``stage_piece``)
        rows = batch + (1 if header else 0)
        self.header = header
        self.pinned = [torch.zeros((rows, self.row), dtype=torch.uint8, pin_memory=pin) for _ in range(depth)]
        self.dev = [torch.empty((rows, self.row), dtype=torch.uint8, device=self.device) for _ in range(depth)]
        self.ev = [torch.cuda.Event() if pin else None for _ in range(depth)]
        self._i = 0
        self.pad = pad_click_row(cfg, n_cross)

    def stage_piece(self, piece, norm: int, into: torch.Tensor | None = None) -> "PackedBatch":
        """A piece of 0..batch records (tuples or packed-row blocks) padded to ``batch``
        rows with look-up-nothing rows; the header row holds ``{len(piece), norm}``.  One
        H2D of the whole slot into ``into`` (the captured step's static batch) or a slot."""
        if not self.header:
            raise ValueError("stage_piece needs a stager built with header=True")
        i = self._i
        self._i = (i + 1) % len(self.pinned)
        if self.ev[i] is not None:
            self.ev[i].synchronize()  # the previous H2D out of this pinned slot is done
        pin = self.pinned[i]
        a = pin.numpy()
        o, tup = 0, []
        for x in piece:
            if isinstance(x, np.ndarray) and x.ndim == 2:
                if tup:
                    a[o:o + len(tup)] = pack_click_records(tup, self.cfg, self.n_cross)
                    o += len(tup)
                    tup = []
                a[o:o + x.shape[0]] = x
                o += x.shape[0]
            else:
                tup.append(x)
        if tup:
            a[o:o + len(tup)] = pack_click_records(tup, self.cfg, self.n_cross)
            o += len(tup)
        if o > self.batch:
            raise ValueError(f"a piece of {o} records does not fit the {self.batch}-row micro-batch")
        a[o:self.batch] = self.pad
        hdr = a[self.batch]
        hdr[0:4] = np.frombuffer(np.int32(o).tobytes(), np.uint8)
        hdr[4:8] = np.frombuffer(np.float32(max(norm, 1)).tobytes(), np.uint8)
        dev = into if into is not None else self.dev[i]
        dev.copy_(pin, non_blocking=True)
        if self.ev[i] is not None:
            self.ev[i].record()
        out = self._views(dev)
        out.args = dev[self.batch, 0:8].view(torch.int32)
        return out

    def _views(self, dev: torch.Tensor) -> "PackedBatch":
        c = self.cfg
        o_d = 4
        o_c = o_d + 4 * c.num_dense
        o_x = o_c + 4 * c.num_fields
        rows = dev[:self.batch]
        labels = rows[:, 0:4].view(torch.float32).reshape(-1)
        dense = rows[:, o_d:o_c].view(torch.float32)
        cats = rows[:, o_c:o_x].view(torch.int32)
        cross = rows[:, o_x:o_x + 4 * self.n_cross].view(torch.int32)
        return PackedBatch((labels, dense, cats, cross), dev)

    def stage(self, rows) -> tuple:
        """``rows``: buffer-protocol rows of ``row`` bytes (exactly ``batch`` of them)."""
        if len(rows) != self.batch:
            raise ValueError(f"expected {self.batch} rows, got {len(rows)}")
        i = self._i
        self._i = (i + 1) % len(self.pinned)
        if self.ev[i] is not None:
            self.ev[i].synchronize()  # the previous H2D out of this pinned slot is done
        pin, dev = self.pinned[i], self.dev[i]
        self._native.gather_into(pin.data_ptr(), self.batch * self.row, list(rows), self.row, 8)
        dev.copy_(pin, non_blocking=True)
        if self.ev[i] is not None:
            self.ev[i].record()
        # strided views of the packed rows (no splitting copies); ``.packed`` is the buffer
        return self._views(dev)


def synthetic_click_records(n: int, cfg: WideDeepConfig, seed: int = 0, n_cross: int = 8):
    """Criteo-shaped synthetic labelled records with a learnable signal."""
    rng = np.random.default_rng(seed)
    dense = rng.standard_normal((n, cfg.num_dense)).astype(np.float32)
    cats = rng.zipf(1.3, (n, cfg.num_fields)).astype(np.int64) % cfg.vocab_per_field
    n_cross = min(n_cross, cfg.num_fields - 1)
    cross =((cats[:, :n_cross] * 1000003 + cats[:, 1:n_cross + 1]) % cfg.wide_buckets).astype(np.int32)
    score = dense[:, 0] - 0.5 * dense[:, 1] + ((cats[:, 0] % 7) == 0) * 1.5 - 0.5
    labels = (rng.random(n) < 1 / (1 + np.exp(-score))).astype(np.float32)
    return [(labels[i], dense[i], cats[i].astype(np.int32), cross[i]) for i in range(n)]


def smoke_train_step(device, steps: int = 2) -> tuple[list[float], dict]:
    """Losses of ``steps`` training steps of the tiny Wide&Deep on fixed records and the
    parameter updates they made (``state - initial state`` per tensor, optimizer state
    excluded): the GPU runs the fused step, the host the autograd trainer in fp32, and the
    smoke test compares the two (as ``tests/test_widedeep.py::
    test_fused_step_tracks_fp32_host_trainer_gpu`` does over 8 steps)."""
    t = WideDeepTrainer(WideDeepConfig.tiny(), device=device, seed=0)
    t.open()
    p0 = {k: v.detach().float().cpu().clone() for k, v in t.model.state_dict().items()}
    recs = synthetic_click_records(256, t.cfg, seed=5)
    out = [float(t.train_step(recs[i * 128:(i + 1) * 128])) for i in range(steps)]
    if t.model.device.type == "cuda":
        torch.cuda.synchronize(t.model.device)
    deltas = {k: (v.detach().float().cpu() - p0[k]).reshape(-1) for k, v in t.model.state_dict().items()
              if not (k.endswith("accum") or k.endswith("anchor"))}
    t.close()
    return out, deltas
