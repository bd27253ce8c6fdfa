"""Fused Wide&Deep training step for the GPU (BASELINE config 4).

The autograd step (``WideDeepTrainer._step``: module forward, ``loss.backward()``, torch
Adam) launches ~140 kernels per micro-batch, most of them framework elementwise kernels
(casts, cat/pad, slices, BCE pieces, bias-grad reductions, the Adam multi-tensor kernel,
bf16 weight copies).  This step computes the same forward, gradients and updates with:

* ``wd_gather`` (``kernels/widedeep.hip``): embedding rows + dense features + zero pad
  straight into the bf16 MLP input, the wide-part sum, the global embedding ids;
* every dense GEMM on the layout-general MFMA training GEMM (``ops.kernels.gemm_train``,
  ``kernels/gemm_train.hip``): the forward with fused bias + ReLU epilogues, per hidden
  layer the weight gradient dW = dA^T . H straight from the row-major activations (both
  operands K-major, hardware transpose reads, split-K with a fixed-order reduction) into
  the flat fp32 gradient buffer, and dX = dA . W with the ReLU mask of the layer input in
  the epilogue and the next bias gradient as per-tile column sums (no transposed copies, no
  library GEMM, no separate mask / column-sum pass);
* ``wd_head_bwd2`` for the 256 -> 1 head: dh, the top bias gradient and the head weight
  gradient in one pass over the activations;
* the deterministic row-sparse pipeline: both tables' lookups in one key space, one radix
  sort, a reduce-by-key per table, sparse Adagrad;
* ``wd_adam`` over ONE flat fp32 buffer holding every dense parameter (the module's
  parameters are views of it), writing the bf16 copies the next forward reads.

Under data parallelism the flat gradient buffer is all-reduced in two chunks on the
communicator's stream while the step goes on: everything but the first layer's weight
gradient as soon as the second layer's backward is done, the first layer's weights right
after its dW GEMM — both overlap the remaining GEMMs and the sparse grouping; Adam waits
for them (the average is folded into Adam).  The sparse rows are all-gathered as before.
The result is the autograd step's update up to bf16 rounding (``tests/test_widedeep.py``).
"""
from __future__ import annotations

import torch

from ... import _ext
from ...ops import kernels as K
from ...ops.embedding import group_keys, segment_sum, segment_sum_grouped, sparse_adagrad
from ...parallel import comm


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


class _Acts:
    """Static activations / gradients of one micro-batch size."""

    def __init__(self, step: "FusedWideDeepStep", B: int):
        dev, m = step.dev, step.m
        bf = dict(dtype=torch.bfloat16, device=dev)
        self.B = B
        self.x = torch.empty(B, step.XP, **bf)
        self.h = [torch.empty(B, l.weight.shape[0], **bf) for l in step.layers]
        self.hd = torch.empty(B, m.head.weight.shape[0], **bf)
        self.da = [torch.empty(B, l.weight.shape[0], **bf) for l in step.layers]
        self.de = torch.empty(B, step.F * step.D, **bf)
        self.wsum = torch.empty(B, dtype=torch.float32, device=dev)
        self.keys = None
        self.dlogit = torch.empty(B, dtype=torch.float32, device=dev)
        self.dlogit16 = torch.empty(B, **bf)
        self.loss = torch.empty((), dtype=torch.float32, device=dev)
        self.part = torch.empty(2 * (-(-B // 256)), dtype=torch.float32, device=dev)
        self.C = None
        self.wgrad = None


class FusedWideDeepStep:
    """``step(labels, dense, cats, cross)`` -> loss (device scalar); activations are kept
    per micro-batch size.  Owns the Adam state; ``state()`` / ``load_state()`` for
    checkpoints."""

    @staticmethod
    def supports(cfg) -> bool:
        """Shapes the kernels take: hidden widths multiples of 8 (GEMM K / N), the top one
        with width / 8 dividing 256 (head backward), embedding rows of 8..512 floats with D/8
        a power of two."""
        d8 = cfg.embed_dim // 8
        top8 = cfg.hidden[-1] // 8
        return (all(h % 8 == 0 for h in cfg.hidden) and 0 < top8 <= 256 and 256 % top8 == 0
                and cfg.embed_dim % 8 == 0 and d8 & (d8 - 1) == 0 and d8 <= 64
                and (cfg.num_fields * cfg.embed_dim) % 8 == 0)

    def __init__(self, model, lr: float, lr_sparse: float, betas=(0.9, 0.999), eps: float = 1e-8, exchange=None):
        dev = model.device
        self.exchange = exchange  # OwnerSparseExchange under DP (else the padded all-gather)
        if dev.type != "cuda":
            raise ValueError("the fused Wide&Deep step runs on a GPU")
        self.m, self.cfg, self.dev = model, model.cfg, dev
        self.lr, self.lr_sparse, self.b1, self.b2, self.eps = lr, lr_sparse, betas[0], betas[1], eps
        self._H = _ext.hip()
        cfg = self.cfg
        # ---- one flat fp32 buffer for every dense parameter; the module's params become views
        named = [(n, p) for n, p in model.named_parameters() if p.requires_grad and not n.endswith("table")]
        al = 64  # every parameter starts on a 256-B boundary (16-B vector access of biases)
        total = sum(-(-p.numel() // al) * al for _, p in named)
        self.flat = torch.zeros(total, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(total, dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros(total, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(total, dtype=torch.float32, device=dev)
        self.t = torch.zeros(1, dtype=torch.float32, device=dev)
        self.g: dict[str, torch.Tensor] = {}
        self.off: dict[str, tuple[int, int]] = {}
        o = 0
        for n, p in named:
            k = p.numel()
            self.flat[o:o + k].copy_(p.data.reshape(-1))
            p.data = self.flat[o:o + k].view_as(p)
            self.g[n] = self.grad[o:o + k].view(p.shape)
            self.off[n] = (o, k)
            o += -(-k // al) * al
        # ---- bf16 operands of every Linear (rewritten by the Adam kernel)
        self.layers = list(model.mlp)
        self.w16 = [l.weight.detach().to(torch.bfloat16) for l in self.layers] + [
            model.head.weight.detach().to(torch.bfloat16)]
        names = [f"mlp.{i}.weight" for i in range(len(self.layers))] + ["head.weight"]
        self.seg = torch.tensor([[self.off[n][0] for n in names], [self.off[n][1] for n in names],
                                 [w.data_ptr() for w in self.w16]], dtype=torch.int64, device=dev)
        # all-reduce chunking: [0, _chunk) = mlp.0.weight (ready last), [_chunk, end) = the rest
        # (another parameter order: one late all-reduce of everything)
        o0, k0 = self.off["mlp.0.weight"]
        self._chunk = min(total, -(-k0 // al) * al) if o0 == 0 else total
        self.F, self.D, self.ND = cfg.num_fields, cfg.embed_dim, cfg.num_dense
        self.XP = model.in_pad
        self._acts: dict[int, _Acts] = {}

    def refresh(self):
        """Re-derives the bf16 operands from the fp32 masters (after a restore)."""
        for w, l in zip(self.w16, self.layers + [self.m.head]):
            w.copy_(l.weight.detach())

    # ------------------------------------------------------------------ the step
    def _bwd_buffers(self, a: "_Acts"):
        """Split-K workspaces of the dW GEMMs, column-sum partials of the dX GEMMs and of the
        head backward (allocated once per micro-batch size)."""
        if getattr(a, "ws", None) is not None:
            return
        dev, B = self.dev, a.B
        a.splits, a.ws = [], []
        for i, l in enumerate(self.layers):
            n_out, k_in = l.weight.shape
            s = K.gemm_train_splits(n_out, k_in, B)
            a.splits.append(s)
            a.ws.append(torch.empty(max(1, s) * n_out * k_in if s > 1 else 1, dtype=torch.float32, device=dev))
        a.colsum = [torch.empty(-(-B // 128), l.weight.shape[1], dtype=torch.float32, device=dev)
                    for l in self.layers[1:]]
        self.head_blocks = 64
        H = a.h[-1].shape[1]
        a.head_part = torch.empty(self.head_blocks, 2 * H, dtype=torch.float32, device=dev)

    def step(self, labels, dense, cats, cross, norm: int | None = None, args: torch.Tensor | None = None
             ) -> torch.Tensor:
        """One step.  ``norm``: an agreed data-parallel step over uneven pieces
        (``parallel/step_agreement.py``) — the loss is this piece's sum over the round's
        global record count and the all-reduced gradients are summed, not averaged.
        ``args``: the same, with the piece's valid-row count and the global count in device
        memory (int32 ``{nvalid, bits of float norm}``, ``PackedBatchStager`` header): the
        batch is a fixed-size piece padded with look-up-nothing rows, so one captured step
        replays for every piece size (``WideDeepTrainer`` agreed steps)."""
        H, m, cfg = self._H, self.m, self.cfg
        nvalid = labels.shape[0]
        if args is not None and nvalid % 8:
            raise ValueError("fused step: a device-argument batch must be a multiple of 8 rows")
        if nvalid % 8:  # the training GEMMs take 8-row granules: pad with rows that look up
            # nothing (ids < 0) and get zero loss and gradient (wd_loss nvalid)
            pad = 8 - nvalid % 8
            dev = labels.device
            labels = torch.cat([labels.reshape(-1).float(), torch.zeros(pad, device=dev)])
            dense = torch.cat([dense.float(), torch.zeros((pad, dense.shape[1]), device=dev)])
            cats = torch.cat([cats.to(torch.int32), torch.full((pad, cats.shape[1]), -(1 << 30), dtype=torch.int32,
                                                                  device=dev)])
            cross = torch.cat([cross.to(torch.int32), torch.full((pad, cross.shape[1]), -1, dtype=torch.int32,
                                                                    device=dev)])
        B = labels.shape[0]
        a = self._acts.get(B)
        if a is None:
            a = self._acts[B] = _Acts(self, B)
        self._bwd_buffers(a)
        C = cross.shape[1]
        WV, WD = m.wide.table.shape
        if a.wgrad is None or a.C != C:
            a.C = C
            a.wgrad = torch.empty(B * C, WD, dtype=torch.float32, device=self.dev)
            a.keys = torch.empty(B * self.F + B * C, dtype=torch.int32, device=self.dev)
        s = _stream()
        # the inputs may be strided views of one packed record buffer (rows of label | dense |
        # cats | cross): the kernels take row strides, no splitting copies
        cats, cross = (t if t.dtype == torch.int32 else t.to(torch.int32) for t in (cats, cross))
        dense, labels = (t if t.dtype == torch.float32 else t.float() for t in (dense, labels))
        cats, dense, cross = (t if t.stride(-1) == 1 else t.contiguous() for t in (cats, dense, cross))
        if labels.dim() != 1:
            labels = labels.reshape(-1)
        dist = comm.is_dist()
        if dist and self.exchange is not None:  # fresh copies of the rows this batch reads
            # the batch's keys in the shared key space (wd_keys: the ones wd_gather will
            # read), deduplicated by the radix sort, refreshed from their owners per table
            self.exchange.begin_step()
            H.wd_keys(cats.data_ptr(), cats.stride(0), cross.data_ptr(), cross.stride(0), a.keys.data_ptr(), B, self.F,
                      cfg.vocab_per_field, C, WV, s)
            pu = group_keys(a.keys, m.emb.table.shape[0] + WV)[3]
            self.exchange.pull(m.emb.table.data, pu, 0)
            self.exchange.pull(m.wide.table.data, pu, m.emb.table.shape[0])
        # forward
        H.wd_gather(cats.data_ptr(), cats.stride(0), dense.data_ptr(), dense.stride(0), cross.data_ptr(),
                    cross.stride(0), m.emb.table.data_ptr(), m.wide.table.data_ptr(), a.x.data_ptr(), a.wsum.data_ptr(),
                    a.keys.data_ptr(), B, self.F, cfg.vocab_per_field, self.D, self.ND, self.XP, C, WV, WD, s)
        h = a.x
        for i, l in enumerate(self.layers):
            h = K.gemm_train(h, self.w16[i], bias=l.bias, act="relu", out=a.h[i])
        K.gemm_train(h, self.w16[-1], bias=m.head.bias, out=a.hd)
        H.wd_loss(a.hd.data_ptr(), a.hd.shape[1], a.wsum.data_ptr(), m.wide_bias.data_ptr(),
                  labels.data_ptr(), labels.stride(0), B, nvalid, float(norm if norm is not None else nvalid),
                  a.dlogit.data_ptr(),
                  a.dlogit16.data_ptr(), a.loss.data_ptr(),
                  self.g["wide_bias"].data_ptr(), self.g["head.bias"].data_ptr(), a.wgrad.data_ptr(), C, WD, a.part.data_ptr(),
                  self.t.data_ptr(), args.data_ptr() if args is not None else 0, s)  # also counts Adam's step
        # backward: head (only logit column 0 is used) -> dh, top bias and head weight gradients
        last = a.h[-1]
        Hl = last.shape[1]
        top = len(self.layers) - 1
        H.wd_head_bwd2(last.data_ptr(), a.dlogit.data_ptr(), m.head.weight.data_ptr(), a.da[-1].data_ptr(),
                       a.head_part.data_ptr(), B, Hl, self.head_blocks, s)
        K.colsum_reduce(a.head_part[:, :Hl], self.g[f"mlp.{top}.bias"])
        K.colsum_reduce(a.head_part[:, Hl:], self.g["head.weight"][0])
        works = []
        for i in range(top, -1, -1):
            da = a.da[i]  # masked; its column sums are already in the bias gradient
            inp = a.h[i - 1] if i else a.x
            K.gemm_train(da, inp, x_t=True, w_t=True, out=self.g[f"mlp.{i}.weight"], splits=a.splits[i], ws=a.ws[i])
            if i:  # dX with the ReLU mask of this layer's input; the next bias gradient from its column sums
                K.gemm_train(da, self.w16[i], w_t=True, mask=inp, out=a.da[i - 1], colsum=a.colsum[i - 1])
                K.colsum_reduce(a.colsum[i - 1], self.g[f"mlp.{i - 1}.bias"])
                if i == 1 and dist and self._chunk < self.grad.numel():
                    # every dense gradient but mlp.0.weight is final: reduce it now
                    works.append(comm.get().all_reduce_async(self.grad[self._chunk:]))
            else:
                if dist:  # mlp.0.weight (and all the rest, unless it went early)
                    works.append(comm.get().all_reduce_async(self.grad[:self._chunk] if works else self.grad))
                # embedding columns of dX only
                K.gemm_train(da, self.w16[0][:, : self.F * self.D], w_t=True, out=a.de)
        # sparse rows: both tables share one key space (wide ids offset by the embedding
        # rows) and one radix sort; each table's sums read only its own lookups
        FV = m.emb.table.shape[0]
        ne = B * self.F
        groups = group_keys(a.keys, FV + WV)
        u = groups[3]
        re = segment_sum_grouped(groups, a.de.view(ne, self.D), 1, 0, ne)
        rw = segment_sum_grouped(groups, a.wgrad, 1, ne, ne + B * C)
        ue = uw = u
        ws = 1
        if dist and self.exchange is not None:
            # deduplicated rows to their owners, owner-side Adagrad, updated rows back
            ws = comm.get().size
            self.exchange.apply(m.emb.table.data, m.emb.accum, u, re, self.lr_sparse)
            self.exchange.apply(m.wide.table.data, m.wide.accum, u, rw, self.lr_sparse, offset=FV)
        elif dist:
            from .wide_deep import _sparse_sync, _sparse_sync_var

            sync = _sparse_sync if norm is None else _sparse_sync_var  # uneven pieces: pad to the largest
            ue, re = segment_sum(*sync(u, re), FV + WV, static=True)
            uw, rw = segment_sum(*sync(u, rw), FV + WV, static=True)
            ws = comm.get().size
        if not (dist and self.exchange is not None):
            sparse_adagrad(m.emb.table.data, m.emb.accum, ue, re, self.lr_sparse)
            sparse_adagrad(m.wide.table.data, m.wide.accum, uw, rw, self.lr_sparse, offset=FV)
        for w in works:  # dense gradients reduced (overlapped with the GEMMs + sparse pipeline)
            w.wait()
        self._adam(1.0 / ws if norm is None and args is None else 1.0, s)
        return a.loss

    def _adam(self, scale: float, s) -> None:
        """Dense Adam over the flat buffer + the bf16 operands of the next step (the step
        count ``t`` was advanced by ``wd_loss``, or by ``empty_step``)."""
        self._H.wd_adam(self.flat.data_ptr(), self.grad.data_ptr(), self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(),
                        self.flat.numel(), self.t.data_ptr(), self.lr, self.b1, self.b2, self.eps, scale,
                        self.seg.data_ptr(), self.seg.shape[1], s)

    def empty_step(self) -> torch.Tensor:
        """This rank's part of an agreed step it brings no records to: zero gradients into
        the same all-reduces, no rows into the same sparse exchange, the same Adam update —
        the collectives are issued in ``step``'s order, so the ranks stay paired."""
        m = self.m
        dev = self.dev
        s = _stream()
        FV, WV = m.emb.table.shape[0], m.wide.table.shape[0]
        none = torch.empty(0, dtype=torch.int64, device=dev)
        dist = comm.is_dist()
        if dist and self.exchange is not None:
            self.exchange.begin_step()
            self.exchange.pull_lookups(m.emb.table.data, none)
            self.exchange.pull_lookups(m.wide.table.data, none)
        self.grad.zero_()
        if dist:
            c = comm.get()
            if len(self.layers) > 1 and self._chunk < self.grad.numel():
                works = [c.all_reduce_async(self.grad[self._chunk:]), c.all_reduce_async(self.grad[:self._chunk])]
            else:
                works = [c.all_reduce_async(self.grad)]
            u = torch.empty(0, dtype=torch.int32, device=dev)
            re = torch.empty(0, self.D, dtype=torch.float32, device=dev)
            rw = torch.empty(0, m.wide.table.shape[1], dtype=torch.float32, device=dev)
            if self.exchange is not None:
                self.exchange.apply(m.emb.table.data, m.emb.accum, u, re, self.lr_sparse)
                self.exchange.apply(m.wide.table.data, m.wide.accum, u, rw, self.lr_sparse, offset=FV)
            else:
                from .wide_deep import _sparse_sync_var

                ue, re = segment_sum(*_sparse_sync_var(u, re), FV + WV, static=True)
                uw, rw = segment_sum(*_sparse_sync_var(u, rw), FV + WV, static=True)
                sparse_adagrad(m.emb.table.data, m.emb.accum, ue, re, self.lr_sparse)
                sparse_adagrad(m.wide.table.data, m.wide.accum, uw, rw, self.lr_sparse, offset=FV)
            for w in works:
                w.wait()
        self.t.add_(1.0)
        self._adam(1.0, s)
        return torch.zeros((), dtype=torch.float32, device=dev)

    def mutable_tensors(self) -> list[torch.Tensor]:
        """Every device tensor a step writes that outlives it (dense masters, Adam state,
        step count, the tables and their Adagrad accumulators): what a capture's warm-up
        steps must hand back unchanged (``WideDeepTrainer._capture_agreed``)."""
        m = self.m
        return [self.flat, self.exp_avg, self.exp_avg_sq, self.t, m.emb.table.data, m.emb.accum, m.wide.table.data,
                m.wide.accum]

    # ------------------------------------------------------------------ checkpoints
    def state(self) -> dict[str, torch.Tensor]:
        return {"adam/exp_avg": self.exp_avg, "adam/exp_avg_sq": self.exp_avg_sq, "adam/step": self.t}

    def load_state(self, st: dict) -> None:
        for k, dst in self.state().items():
            if k in st:
                dst.copy_(st[k].to(dst.device).reshape(dst.shape))
        self.refresh()
