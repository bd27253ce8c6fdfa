"""BERT-base text classification (BASELINE config 3: BERT stream, DP over xGMI).

The encoder runs entirely on the CDNA4 kernels, one hipGraph per (batch bucket, seq):

    embed_ln (gather word/pos/type + LayerNorm, one pass)
    12 x [ gemm(x, Wqkv) + b          -> qkv [T, 2304]     (fused Q|K|V projection)
           attention(qkv, ids)        -> ctx [T, 768]      (flash-style, key-padding mask)
           gemm(ctx, Wo) + b + x      -> y                 (residual fused in the epilogue)
           layernorm(y)               -> x
           gemm(x, W1) + b -> GELU    -> h [T, 3072]       (activation fused)
           gemm(h, W2) + b + x        -> y ; layernorm(y) -> x ]
    pooler: gemm(x[:, 0], Wp) + b -> tanh ; classifier gemm -> softmax (host: 2 logits)

Weights are random-init (no checkpoint download) but use the TF BERT checkpoint variable
names, so ``load_tf_checkpoint`` can read a real ``bert_model.ckpt`` bundle through the
native TensorBundle reader.  Text records are tokenized on the host by a hashing
WordPiece-free tokenizer (no vocab file offline); token-id records bypass it.
"""
from __future__ import annotations

import re
import zlib
from dataclasses import dataclass

import numpy as np
import torch

from ...ops import kernels as K
from ...runtime.model_functions import BatchedGpuModel
from ...utils.tracing import capture_lock, graph_capture
from ..core import RichModel, default_device


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    intermediate: int = 3072
    max_position: int = 512
    type_vocab: int = 2
    num_labels: int = 2
    eps: float = 1e-12

    @staticmethod
    def base(**kw) -> "BertConfig":
        return BertConfig(**kw)

    @staticmethod
    def tiny(**kw) -> "BertConfig":
        d = dict(vocab_size=1000, hidden=128, layers=2, heads=2, intermediate=256, max_position=128)
        d.update(kw)
        return BertConfig(**d)

    def params(self) -> int:
        h, i = self.hidden, self.intermediate
        emb = (self.vocab_size + self.max_position + self.type_vocab) * h + 2 * h
        layer = 4 * h * h + 4 * h + 2 * h * i + i + h + 4 * h
        return emb + self.layers * layer + h * h + h + h * self.num_labels + self.num_labels


class HashingTokenizer:
    """Lower-case word split, crc32-hashed into the vocab; [CLS] ... [SEP], pad 0."""

    CLS, SEP, PAD = 101, 102, 0

    def __init__(self, vocab_size: int, max_len: int):
        self.vocab_size = vocab_size
        self.max_len = max_len

    def __call__(self, text: str) -> np.ndarray:
        ids = [self.CLS]
        lo = min(1000, self.vocab_size // 2)  # ids below `lo` are reserved (special tokens)
        for w in re.findall(r"[a-z0-9]+|[^\sa-z0-9]", text.lower()):
            ids.append(lo + zlib.crc32(w.encode()) % (self.vocab_size - lo))
            if len(ids) >= self.max_len - 1:
                break
        ids.append(self.SEP)
        out = np.zeros(self.max_len, dtype=np.int32)
        out[: len(ids)] = ids
        return out


def init_bert_weights(cfg: BertConfig, seed: int = 0) -> dict[str, torch.Tensor]:
    """Random-init fp32 host weights named like the TF BERT checkpoint."""
    g = torch.Generator().manual_seed(seed)

    def n(*shape):
        return torch.randn(*shape, generator=g) * 0.02

    h, i = cfg.hidden, cfg.intermediate
    w = {
        "bert/embeddings/word_embeddings": n(cfg.vocab_size, h),
        "bert/embeddings/position_embeddings": n(cfg.max_position, h),
        "bert/embeddings/token_type_embeddings": n(cfg.type_vocab, h),
        "bert/embeddings/LayerNorm/gamma": torch.ones(h),
        "bert/embeddings/LayerNorm/beta": torch.zeros(h),
        "bert/pooler/dense/kernel": n(h, h),
        "bert/pooler/dense/bias": torch.zeros(h),
        "output_weights": n(cfg.num_labels, h),
        "output_bias": torch.zeros(cfg.num_labels),
    }
    for l in range(cfg.layers):
        p = f"bert/encoder/layer_{l}/"
        for nm in ("query", "key", "value"):
            w[p + f"attention/self/{nm}/kernel"] = n(h, h)
            w[p + f"attention/self/{nm}/bias"] = torch.zeros(h)
        w[p + "attention/output/dense/kernel"] = n(h, h)
        w[p + "attention/output/dense/bias"] = torch.zeros(h)
        w[p + "attention/output/LayerNorm/gamma"] = torch.ones(h)
        w[p + "attention/output/LayerNorm/beta"] = torch.zeros(h)
        w[p + "intermediate/dense/kernel"] = n(h, i)
        w[p + "intermediate/dense/bias"] = torch.zeros(i)
        w[p + "output/dense/kernel"] = n(i, h)
        w[p + "output/dense/bias"] = torch.zeros(h)
        w[p + "output/LayerNorm/gamma"] = torch.ones(h)
        w[p + "output/LayerNorm/beta"] = torch.zeros(h)
    return w


def load_tf_checkpoint(prefix: str, cfg: BertConfig) -> dict[str, torch.Tensor]:
    """Reads a TF BERT checkpoint (TensorBundle V2) with the native bundle reader."""
    from ...io.bundle import BundleReader

    ref = init_bert_weights(cfg)
    with BundleReader(prefix) as r:
        return {k: r.read(k).float() if k in r else v for k, v in ref.items()}


class BertDeviceWeights:
    """Kernel-layout device weights: bf16 [N, K] matrices (QKV fused), fp32 biases/LN."""

    def __init__(self, host: dict[str, torch.Tensor], cfg: BertConfig, device):
        d = torch.device(device)
        bf = torch.bfloat16 if d.type == "cuda" else torch.float32

        def mat(kernel):  # TF kernels are [in, out]; the GEMM wants [out, in]
            return kernel.t().contiguous().to(d, bf)

        def vec(v):
            return v.float().contiguous().to(d)

        self.cfg = cfg
        self.word = host["bert/embeddings/word_embeddings"].to(d, bf).contiguous()
        self.pos = host["bert/embeddings/position_embeddings"].to(d, bf).contiguous()
        self.type = host["bert/embeddings/token_type_embeddings"].to(d, bf).contiguous()
        self.emb_g = vec(host["bert/embeddings/LayerNorm/gamma"])
        self.emb_b = vec(host["bert/embeddings/LayerNorm/beta"])
        self.layers = []
        for l in range(cfg.layers):
            p = f"bert/encoder/layer_{l}/"
            qkv_w = torch.cat([host[p + f"attention/self/{nm}/kernel"] for nm in ("query", "key", "value")], 1)
            qkv_b = torch.cat([host[p + f"attention/self/{nm}/bias"] for nm in ("query", "key", "value")])
            self.layers.append({
                "qkv_w": mat(qkv_w), "qkv_b": vec(qkv_b),
                "o_w": mat(host[p + "attention/output/dense/kernel"]), "o_b": vec(host[p + "attention/output/dense/bias"]),
                "ln1_g": vec(host[p + "attention/output/LayerNorm/gamma"]),
                "ln1_b": vec(host[p + "attention/output/LayerNorm/beta"]),
                "i_w": mat(host[p + "intermediate/dense/kernel"]), "i_b": vec(host[p + "intermediate/dense/bias"]),
                "f_w": mat(host[p + "output/dense/kernel"]), "f_b": vec(host[p + "output/dense/bias"]),
                "ln2_g": vec(host[p + "output/LayerNorm/gamma"]), "ln2_b": vec(host[p + "output/LayerNorm/beta"]),
            })
        self.pool_w = mat(host["bert/pooler/dense/kernel"])
        self.pool_b = vec(host["bert/pooler/dense/bias"])
        nl = cfg.num_labels
        npad = -(-nl // 8) * 8  # GEMM N must be a multiple of 8: pad the classifier
        cw = torch.zeros(npad, cfg.hidden)
        cw[:nl] = host["output_weights"]
        cb = torch.zeros(npad)
        cb[:nl] = host["output_bias"]
        self.cls_w = cw.to(d, bf).contiguous()
        self.cls_b = cb.to(d)

    def tensors(self) -> list[torch.Tensor]:
        out = [self.word, self.pos, self.type, self.emb_g, self.emb_b, self.pool_w, self.pool_b, self.cls_w, self.cls_b]
        for L in self.layers:
            out += list(L.values())
        return out


class BertBuffers:
    """Activation buffers of one (batch, seq) encoder, sized for ``tokens`` rows; the
    token-capacity plans of a packed encoder share one set (they replay serially)."""

    def __init__(self, cfg: "BertConfig", batch: int, seq: int, tokens: int, device, dtype):
        d, h = device, cfg.hidden
        self.ids = torch.zeros(batch * seq, dtype=torch.int32, device=d)   # padded [B, S] input
        self.pids = torch.zeros(tokens, dtype=torch.int32, device=d)       # packed token ids
        self.ppos = torch.zeros(tokens, dtype=torch.int32, device=d)       # their in-row positions
        self.cu = torch.zeros(batch + 1, dtype=torch.int32, device=d)      # sequence row offsets
        self.cls = torch.zeros(batch, dtype=torch.int32, device=d)         # first-token rows
        self.x = torch.empty(tokens, h, dtype=dtype, device=d)
        self.y = torch.empty(tokens, h, dtype=dtype, device=d)
        self.qkv = torch.empty(tokens, 3 * h, dtype=dtype, device=d)
        self.ctx = torch.zeros(tokens, h, dtype=dtype, device=d)  # rows past the packed tokens stay finite
        self.x2 = torch.empty(tokens, h, dtype=dtype, device=d)
        self.ffn = torch.empty(tokens, cfg.intermediate, dtype=dtype, device=d)
        self.cls_in = torch.empty(batch, h, dtype=dtype, device=d)
        self.pooled = torch.empty(batch, h, dtype=dtype, device=d)
        # final-layer first-token rows (packed classifier: only they feed the pooler)
        self.c_ctx, self.c_y, self.c_x, self.c_x2 = (torch.empty(batch, h, dtype=dtype, device=d) for _ in range(4))
        self.c_ffn = torch.empty(batch, cfg.intermediate, dtype=dtype, device=d)
        # split-K workspace of the final-layer first-token GEMMs (B rows); owned per buffer
        # set because the plans of different compute lanes replay concurrently
        shapes = [(h, h), (cfg.intermediate, h), (h, cfg.intermediate)]
        need = max(K.gemm_pp_splits(batch, n, k) * batch * n for n, k in shapes)
        self.ws = torch.empty(need, dtype=torch.float32, device=d)
        # one hipGraph memory pool for every plan on these buffers (graph temporaries such as
        # the GELU projection output are reused across capacities instead of duplicated)
        self.pool = torch.cuda.graph_pool_handle() if torch.device(d).type == "cuda" else None


class BertEncoderPlan:
    """Preallocated buffers + launch sequence for one (batch, seq); hipGraph-captured.

    Every projection runs on the hand-written ping-pong MFMA GEMM (``kernels/gemm_pp.hip``,
    256x256 tiles, LDS-DMA pipeline) with the bias (+GELU) fused in its epilogue; the
    residual adds are fused into the residual+LayerNorm kernel.  The final-layer
    first-token GEMMs (B rows) run split-K.  Embedding+LN, attention, residual+LN and the
    pooler/classifier are hand-written kernels too — no library GEMM on the path.

    ``tokens=T`` makes the plan padding-free: a packing kernel compacts the batch's
    non-pad tokens into T rows (positions and per-sequence offsets on the device), every
    projection / LayerNorm runs on those T rows, attention runs per packed sequence
    (``cu_seqlens``) and the pooler gathers each sequence's first row — the classifier
    output is that of the padded plan, for the tokens that exist."""

    def __init__(self, w: BertDeviceWeights, batch: int, seq: int, use_graph: bool = True, gemm: str | None = None,
                 tokens: int | None = None, shared: BertBuffers | None = None):
        cfg = w.cfg
        self.w, self.B, self.S = w, batch, seq
        if gemm not in (None, "mfma"):
            raise ValueError("gemm must be 'mfma' (the hand-written MFMA GEMM)")
        self.gemm_impl = "mfma"
        self.packed = tokens is not None
        T = tokens if self.packed else batch * seq
        self.T = T
        d = w.word.device
        dt = w.word.dtype
        b = shared if shared is not None else BertBuffers(cfg, batch, seq, T, d, dt)
        if b.x.shape[0] < T:
            raise ValueError(f"shared buffers hold {b.x.shape[0]} rows, plan needs {T}")
        self.bufs = b
        self.ids = b.ids
        self.pids, self.ppos, self.cu, self.cls_idx = b.pids[:T], b.ppos[:T], b.cu, b.cls
        self.x, self.y, self.qkv, self.ctx, self.x2, self.ffn = (t[:T] for t in (b.x, b.y, b.qkv, b.ctx, b.x2, b.ffn))
        self.cls_in, self.pooled = b.cls_in, b.pooled
        self.c_ctx, self.c_y, self.c_x, self.c_x2, self.c_ffn = b.c_ctx, b.c_y, b.c_x, b.c_x2, b.c_ffn
        if not hasattr(b, "logits"):
            b.logits = torch.empty(batch, w.cls_w.shape[0], dtype=dt, device=d)
        self.logits = b.logits
        self.graph = None
        if use_graph and d.type == "cuda":
            self._capture()

    def _embed(self):
        w, cfg = self.w, self.w.cfg
        if self.packed:
            K.pack_tokens(self.ids.view(self.B, self.S), HashingTokenizer.PAD, self.T, self.pids, self.ppos, self.cu,
                          self.cls_idx)
            K.embed_layernorm(self.pids, None, w.word, w.pos, w.type, w.emb_g, w.emb_b, self.S, cfg.eps, out=self.x,
                              pos_ids=self.ppos)
        else:
            K.embed_layernorm(self.ids, None, w.word, w.pos, w.type, w.emb_g, w.emb_b, self.S, cfg.eps, out=self.x)

    def _attention(self):
        cfg = self.w.cfg
        if self.packed:
            K.attention(self.qkv, None, self.B, self.S, cfg.heads, out=self.ctx, cu_seqlens=self.cu)
        else:
            K.attention(self.qkv, self.ids, self.B, self.S, cfg.heads, out=self.ctx)

    def _pool(self):
        w, B, S = self.w, self.B, self.S
        if self.packed:
            torch.index_select(self.x, 0, self.cls_idx, out=self.cls_in)
        else:
            self.cls_in.copy_(self.x.view(B, S, -1)[:, 0])
        K.gemm(self.cls_in, w.pool_w, w.pool_b, act="tanh", out=self.pooled)
        K.gemm(self.pooled, w.cls_w, w.cls_b, out=self.logits)

    def _run(self):
        w = self.w
        self._embed()
        cfg = w.cfg
        for li, L in enumerate(w.layers):
            K.gemm_pp(self.x, L["qkv_w"], L["qkv_b"], out=self.qkv)
            if self.packed and li == len(w.layers) - 1:
                return self._last_layer_cls(L)
            self._attention()
            K.gemm_pp(self.ctx, L["o_w"], L["o_b"], out=self.y)
            K.layernorm(self.y, L["ln1_g"], L["ln1_b"], residual=self.x, eps=cfg.eps, out=self.x2)
            K.gemm_pp(self.x2, L["i_w"], L["i_b"], act="gelu", out=self.ffn)
            K.gemm_pp(self.ffn, L["f_w"], L["f_b"], out=self.y)
            K.layernorm(self.y, L["ln2_g"], L["ln2_b"], residual=self.x2, eps=cfg.eps, out=self.x)
        self._pool()

    def _last_layer_cls(self, L):
        """Final layer of a packed classifier: only each sequence's first row reaches the
        pooler, so after the (all-token) QKV projection everything runs on B rows —
        first-token attention over the sequence's keys, then output projection, residual
        LayerNorm, FFN and LayerNorm of those rows (the pooler input is unchanged).  The
        B-row GEMMs run split-K through this buffer set's own workspace."""
        w, cfg = self.w, self.w.cfg
        ws = self.bufs.ws
        K.cls_attention(self.qkv, self.cu, self.B, cfg.heads, out=self.c_ctx)
        torch.index_select(self.x, 0, self.cls_idx, out=self.c_x)  # the layer input = residual
        K.gemm_pp(self.c_ctx, L["o_w"], L["o_b"], out=self.c_y, ws=ws)
        K.layernorm(self.c_y, L["ln1_g"], L["ln1_b"], residual=self.c_x, eps=cfg.eps, out=self.c_x2)
        K.gemm_pp(self.c_x2, L["i_w"], L["i_b"], act="gelu", out=self.c_ffn, ws=ws)
        K.gemm_pp(self.c_ffn, L["f_w"], L["f_b"], out=self.c_y, ws=ws)
        K.layernorm(self.c_y, L["ln2_g"], L["ln2_b"], residual=self.c_x2, eps=cfg.eps, out=self.cls_in)
        K.gemm(self.cls_in, w.pool_w, w.pool_b, act="tanh", out=self.pooled)
        K.gemm(self.pooled, w.cls_w, w.cls_b, out=self.logits)

    def _capture(self):
        with capture_lock():  # warm-up + device sync + capture: no sibling capture in between
            s = torch.cuda.Stream(self.ids.device)
            s.wait_stream(torch.cuda.current_stream(self.ids.device))
            with torch.cuda.stream(s):
                for _ in range(2):
                    self._run()
            torch.cuda.current_stream(self.ids.device).wait_stream(s)
            torch.cuda.synchronize(self.ids.device)
            g = torch.cuda.CUDAGraph()
            with graph_capture(g, pool=self.bufs.pool):
                self._run()
            self.graph = g

    # plan protocol used by PipelinedGpuRunner
    def input_buffer(self, feed: str) -> torch.Tensor:
        return self.ids.view(self.B, self.S)

    def replay(self):
        if self.graph is not None:
            self.graph.replay()
        else:
            self._run()

    def output_tensors(self):
        return [self.logits[:, : self.w.cfg.num_labels]]

    def __call__(self, ids: torch.Tensor) -> torch.Tensor:
        self.ids.view(self.B, self.S).copy_(ids)
        self.replay()
        return torch.softmax(self.logits[:, : self.w.cfg.num_labels].float(), -1)

    def flops(self, lengths=None) -> float:
        """Encoder FLOPs of one replay; with ``lengths`` (per-sequence real tokens) the
        useful FLOPs of a padding-free batch."""
        cfg = self.w.cfg
        h, i = cfg.hidden, cfg.intermediate
        lens = np.full(self.B, self.S) if lengths is None else np.asarray(lengths)
        T = float(lens.sum())
        per_layer = 2 * T * (3 * h * h + h * h + 2 * h * i) + 4 * cfg.heads * float((lens ** 2).sum()) * (h // cfg.heads)
        if not self.packed:
            return cfg.layers * per_layer
        # packed classifier: the final layer computes QKV for every token but attention,
        # projection and FFN only for each sequence's first token
        last = 2 * T * 3 * h * h + 4 * cfg.heads * float(lens.sum()) * (h // cfg.heads) + 2 * len(lens) * (h * h + 2 * h * i)
        return (cfg.layers - 1) * per_layer + last


class PackedBertEncoder:
    """Padding-free encoder for a (batch, seq) micro-batch: one captured plan per token
    capacity (multiples of ``granule`` up to batch*seq), all on one shared buffer set.
    ``select(host_ids, n)`` picks the smallest capacity holding the batch's real tokens —
    counted on the host from the pinned staging slot, so no device sync is needed; the
    device-side packing kernel then compacts the same tokens.  Implements the plan
    protocol of ``PipelinedGpuRunner`` (``input_buffer`` / ``replay`` / ``output_tensors``)."""

    def __init__(self, w: BertDeviceWeights, batch: int, seq: int, use_graph: bool = True, gemm: str | None = None,
                 granule: int = 2048):
        self.w, self.B, self.S = w, batch, seq
        full = batch * seq
        granule = max(16, min(granule, full))
        caps = sorted({min(full, g) for g in range(granule, full + granule, granule)})
        self.bufs = BertBuffers(w.cfg, batch, seq, full, w.word.device, w.word.dtype)
        self.plans = {c: BertEncoderPlan(w, batch, seq, use_graph, gemm, tokens=c, shared=self.bufs) for c in caps}
        self.caps = caps
        self.current = self.plans[caps[-1]]
        self.ids = self.bufs.ids
        self.graph = self.current.graph

    def capacity_for(self, n_tokens: int) -> int:
        for c in self.caps:
            if c >= n_tokens:
                return c
        raise ValueError(f"{n_tokens} tokens exceed batch*seq = {self.caps[-1]}")

    def select(self, host_ids, n: int | None = None) -> BertEncoderPlan:
        a = host_ids.numpy() if isinstance(host_ids, torch.Tensor) else np.asarray(host_ids)
        self.current = self.plans[self.capacity_for(int(np.count_nonzero(a != HashingTokenizer.PAD)))]
        return self.current

    # plan protocol
    def input_buffer(self, feed: str) -> torch.Tensor:
        return self.ids.view(self.B, self.S)

    def replay(self):
        self.current.replay()

    def output_tensors(self):
        return self.current.output_tensors()

    def __call__(self, ids: torch.Tensor) -> torch.Tensor:
        self.select(ids.cpu())
        self.ids.view(self.B, self.S).copy_(ids)
        self.current.replay()
        return torch.softmax(self.current.logits[:, : self.w.cfg.num_labels].float(), -1)

    def flops(self, lengths=None) -> float:
        return self.current.flops(lengths)


class BertClassifierModel(RichModel, BatchedGpuModel):
    """Text (or token-id) records → class probabilities; micro-batched on the GPU."""

    _TRANSIENT = ("_w", "_plans", "_runner")

    def __init__(self, cfg: BertConfig | None = None, seq_len: int = 128, buckets=(64, 256), seed: int = 0,
                 device=None, checkpoint: str | None = None, depth: int = 3, use_graph: bool = True,
                 distributed_weights: bool = False, lanes: int = 3):
        self.cfg = cfg or BertConfig.base()
        self.lanes = max(1, int(lanes))  # concurrent encoder instances on their own HIP streams
        # DP over ranks (one process per GPU): rank 0's weights are broadcast to every rank
        # at open (one flattened RCCL broadcast per dtype over xGMI) instead of each rank
        # reading the checkpoint (SURVEY §2.13 model distribution)
        self.distributed_weights = distributed_weights
        self.seq_len = seq_len
        self.buckets = tuple(sorted(buckets))
        self.seed = seed
        self.device = device
        self.checkpoint = checkpoint
        self.depth = depth
        self.use_graph = use_graph
        self.tokenizer = HashingTokenizer(self.cfg.vocab_size, seq_len)
        self._w = self._plans = self._runner = None

    def open(self):
        dev = torch.device(self.device) if self.device is not None else default_device()
        host = load_tf_checkpoint(self.checkpoint, self.cfg) if self.checkpoint else init_bert_weights(self.cfg, self.seed)
        self._w = BertDeviceWeights(host, self.cfg, dev)
        if self.distributed_weights:
            from ...parallel import comm

            comm.broadcast_tensors(self._w.tensors(), src=0)  # before capture: plans read these in place
        # padding-free encoders: each micro-batch runs on the token capacity of its real tokens
        lanes = [{b: PackedBertEncoder(self._w, b, self.seq_len, self.use_graph) for b in self.buckets}
                 for _ in range(self.lanes if dev.type == "cuda" else 1)]
        self._plans = lanes[0]
        if dev.type == "cuda":
            from ...batching.engine import PipelinedGpuRunner

            self._runner = PipelinedGpuRunner(lanes, "ids", lambda p: p.output_tensors(), (self.seq_len,),
                                              torch.int32, depth=self.depth, device=dev)

    def close(self):
        if self._runner is not None:
            self._runner.drain()
        self._w = self._plans = self._runner = None

    @property
    def is_open(self):
        return self._w is not None

    def weights(self) -> BertDeviceWeights:
        return self._w

    def encode(self, record) -> np.ndarray:
        if isinstance(record, str):
            return self.tokenizer(record)
        a = np.asarray(record, dtype=np.int32).reshape(-1)
        out = np.zeros(self.seq_len, dtype=np.int32)
        out[: min(len(a), self.seq_len)] = a[: self.seq_len]
        return out

    def predict(self, records) -> torch.Tensor:
        """Synchronous class probabilities [N, num_labels]."""
        ids = np.stack([self.encode(r) for r in records])
        n = len(ids)
        b = next((bk for bk in self.buckets if bk >= n), None)
        if b is None:
            return torch.cat([self.predict(records[i:i + self.buckets[-1]]) for i in range(0, n, self.buckets[-1])])
        buf = np.zeros((b, self.seq_len), dtype=np.int32)
        buf[:n] = ids
        plan = self._plans[b]
        return plan(torch.from_numpy(buf).to(plan.ids.device))[:n].cpu()

    # BatchedGpuModel
    def _res(self, br):
        probs = torch.softmax(br.outputs[0][: br.n].float(), -1)
        return probs.tolist(), br.tags, br.latencies

    def submit(self, records, ingest_ts, tags):
        if self._runner is None:
            import time

            return [(self.predict(records).tolist(), tags, time.perf_counter() - np.asarray(ingest_ts))]
        arrs = [self.encode(r) for r in records]
        cap = self.buckets[-1]
        out = []
        for s in range(0, len(arrs), cap):
            for br in self._runner.submit(arrs[s:s + cap], np.asarray(ingest_ts[s:s + cap]), list(tags[s:s + cap])):
                out.append(self._res(br))
        return out

    def poll(self):
        return [self._res(b) for b in self._runner.poll()] if self._runner is not None else []

    def drain(self):
        return [self._res(b) for b in self._runner.drain()] if self._runner is not None else []


def reference_forward(host: dict[str, torch.Tensor], cfg: BertConfig, ids: torch.Tensor,
                      return_hidden: bool = False):
    """Plain PyTorch fp32 BERT (numerics oracle): ids [B, S] → logits [B, num_labels]
    (and the final hidden states [B, S, hidden] with ``return_hidden``)."""
    import torch.nn.functional as F

    B, S = ids.shape
    h = cfg.hidden
    x = host["bert/embeddings/word_embeddings"][ids.long()] + host["bert/embeddings/position_embeddings"][:S]
    x = x + host["bert/embeddings/token_type_embeddings"][0]
    x = F.layer_norm(x, (h,), host["bert/embeddings/LayerNorm/gamma"], host["bert/embeddings/LayerNorm/beta"], cfg.eps)
    mask = (ids == 0)[:, None, None, :]
    dh = h // cfg.heads
    for l in range(cfg.layers):
        p = f"bert/encoder/layer_{l}/"

        def lin(t, nm):
            return t @ host[p + nm + "/kernel"] + host[p + nm + "/bias"]

        q = lin(x, "attention/self/query").view(B, S, cfg.heads, dh).transpose(1, 2)
        k = lin(x, "attention/self/key").view(B, S, cfg.heads, dh).transpose(1, 2)
        v = lin(x, "attention/self/value").view(B, S, cfg.heads, dh).transpose(1, 2)
        a = (q @ k.transpose(-1, -2)) / dh ** 0.5
        a = torch.softmax(a.masked_fill(mask, float("-inf")), -1).nan_to_num(0.0)
        ctx = (a @ v).transpose(1, 2).reshape(B, S, h)
        x = F.layer_norm(lin(ctx, "attention/output/dense") + x, (h,), host[p + "attention/output/LayerNorm/gamma"],
                         host[p + "attention/output/LayerNorm/beta"], cfg.eps)
        f = F.gelu(lin(x, "intermediate/dense"), approximate="tanh")
        x = F.layer_norm(lin(f, "output/dense") + x, (h,), host[p + "output/LayerNorm/gamma"],
                         host[p + "output/LayerNorm/beta"], cfg.eps)
    pooled = torch.tanh(x[:, 0] @ host["bert/pooler/dense/kernel"] + host["bert/pooler/dense/bias"])
    logits = pooled @ host["output_weights"].t() + host["output_bias"]
    return (logits, x) if return_hidden else logits
