"""BERT as a TensorFlow 1.x GraphDef / SavedModel — the layout ``modeling.py`` of Google's
BERT produces — so the text-classification config runs through the same
SavedModel / GraphDef loader, ``Session.run`` interpreter and graph compiler as the CNNs.

The graph keeps TF's decomposed ops (no custom fused ops), exactly what a user's frozen
BERT contains:

* embeddings: ``GatherV2(word_embeddings, input_ids)`` + position rows (``Slice`` of the
  table) + token-type row 0, then ``layer_norm``;
* ``layer_norm`` as ``tf.contrib.layers.layer_norm`` emits it: ``moments`` (``Mean``,
  ``SquaredDifference``, ``Mean``), ``batchnorm`` (``add`` eps, ``Rsqrt``, ``mul`` gamma,
  ``mul_1`` x, ``mul_2`` mean, ``sub`` beta, ``add_1``);
* attention: per-head ``Reshape``/``Transpose`` of the query/key/value ``MatMul``+
  ``BiasAdd``, ``BatchMatMulV2(adj_y)``, ``Mul`` by 1/sqrt(d), ``Add`` of the
  ``(1 - mask) * -10000`` adder built from ``input_mask``, ``Softmax``,
  ``BatchMatMulV2``, ``Transpose``/``Reshape`` back;
* GELU (tanh form): ``0.5 * x * (1 + tanh(sqrt(2/pi) * (x + 0.044715 * x^3)))``;
* pooler: ``StridedSlice`` of the first token, ``Squeeze``, ``MatMul``+``BiasAdd``+``Tanh``;
  classifier ``MatMul(transpose_b)``+``BiasAdd``, ``Softmax``.

The graph compiler recognises these patterns and lowers them onto the same hand-written
kernels as the hand-built encoder (``gemm_pp`` with fused bias / GELU / residual, fused
QKV projection, flash-style ``attention``, ``layernorm``, ``embed_layernorm``).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ...graph.builder import GraphBuilder
from ...proto.messages import GraphDef, SignatureDef
from ...types.dtypes import DataType
from .bert import BertConfig, init_bert_weights


def _c(b: GraphBuilder, name: str, v) -> str:
    return b.constant(name, np.asarray(v))


def layer_norm(b: GraphBuilder, x: str, gamma: str, beta: str, eps: float, scope: str) -> str:
    """``tf.contrib.layers.layer_norm(begin_norm_axis=-1)`` node for node."""
    with b.name_scope(scope):
        axes = _c(b, "moments/mean/reduction_indices", np.asarray([-1], np.int32))
        mean = b.op("Mean", [x, axes], name="moments/mean", keep_dims=True, T=DataType.FLOAT, Tidx=DataType.INT32)
        sg = b.op("StopGradient", [mean], name="moments/StopGradient", T=DataType.FLOAT)
        sq = b.op("SquaredDifference", [x, sg], name="moments/SquaredDifference", T=DataType.FLOAT)
        axes2 = _c(b, "moments/variance/reduction_indices", np.asarray([-1], np.int32))
        var = b.op("Mean", [sq, axes2], name="moments/variance", keep_dims=True, T=DataType.FLOAT,
                   Tidx=DataType.INT32)
        e = _c(b, "batchnorm/add/y", np.float32(eps))
        ve = b.add(var, e, name="batchnorm/add")
        rs = b.op("Rsqrt", [ve], name="batchnorm/Rsqrt", T=DataType.FLOAT)
        inv = b.mul(rs, gamma, name="batchnorm/mul")
        xm = b.mul(x, inv, name="batchnorm/mul_1")
        mm = b.mul(mean, inv, name="batchnorm/mul_2")
        sh = b.sub(beta, mm, name="batchnorm/sub")
        return b.add(xm, sh, name="batchnorm/add_1")


def gelu(b: GraphBuilder, x: str, scope: str) -> str:
    """BERT's tanh-approximate GELU."""
    with b.name_scope(scope):
        p3 = b.op("Pow", [x, _c(b, "Pow/y", np.float32(3.0))], name="Pow", T=DataType.FLOAT)
        m1 = b.mul(_c(b, "mul/x", np.float32(0.044715)), p3, name="mul")
        a1 = b.add(x, m1, name="add")
        m2 = b.mul(_c(b, "mul_1/x", np.float32(math.sqrt(2 / math.pi))), a1, name="mul_1")
        t = b.op("Tanh", [m2], name="Tanh", T=DataType.FLOAT)
        a2 = b.add(_c(b, "add_1/x", np.float32(1.0)), t, name="add_1")
        cdf = b.mul(_c(b, "mul_2/x", np.float32(0.5)), a2, name="mul_2")
        return b.mul(x, cdf, name="mul_3")


def bert_graph_def(cfg: BertConfig, seq_len: int, weights: dict | None = None, seed: int = 0,
                   mask_from_ids: bool = False) -> tuple[GraphDef, dict]:
    """(GraphDef, weights) for a BERT sequence classifier on [B, seq_len] inputs (B dynamic).

    Feeds ``input_ids`` / ``input_mask`` (int32 [B, S]); with ``mask_from_ids`` the mask is
    computed in the graph as ``NotEqual(input_ids, 0)`` and ``input_ids`` is the only feed
    (what a stream of token-id records carries).  Fetches ``probs`` [B, labels] and
    ``logits``.  Weights are ``init_bert_weights(cfg, seed)`` unless given; they are Consts
    (frozen graph) — ``export_bert_saved_model`` turns them into variables."""
    w = weights if weights is not None else init_bert_weights(cfg, seed)
    H, S, nh = cfg.hidden, seq_len, cfg.heads
    dh = H // nh
    b = GraphBuilder()

    def W(name):
        return b.constant(name, w[name].float().numpy())

    ids = b.placeholder("input_ids", "INT32", [None, S])
    if mask_from_ids:
        mask = b.op("NotEqual", [ids, _c(b, "bert/NotEqual/y", np.int32(0))], name="bert/NotEqual", T=DataType.INT32,
                    incompatible_shape_error=True)
    else:
        mask = b.placeholder("input_mask", "INT32", [None, S])
    shape_bs = b.op("Shape", [ids], name="bert/Shape", T=DataType.INT32, out_type=DataType.INT32)
    bsz = b.op("StridedSlice", [shape_bs, _c(b, "bert/strided_slice/stack", np.asarray([0], np.int32)),
                                _c(b, "bert/strided_slice/stack_1", np.asarray([1], np.int32)),
                                _c(b, "bert/strided_slice/stack_2", np.asarray([1], np.int32))],
               name="bert/strided_slice", T=DataType.INT32, Index=DataType.INT32, begin_mask=0, end_mask=0,
               ellipsis_mask=0, new_axis_mask=0, shrink_axis_mask=1)
    # ---- embeddings
    word = W("bert/embeddings/word_embeddings")
    emb = b.op("GatherV2", [word, ids, _c(b, "bert/embeddings/GatherV2/axis", np.int32(0))],
               name="bert/embeddings/GatherV2", Tparams=DataType.FLOAT, Tindices=DataType.INT32,
               Taxis=DataType.INT32, batch_dims=0)
    pos_tab = W("bert/embeddings/position_embeddings")
    pos = b.op("Slice", [pos_tab, _c(b, "bert/embeddings/Slice/begin", np.asarray([0, 0], np.int32)),
                         _c(b, "bert/embeddings/Slice/size", np.asarray([S, -1], np.int32))],
               name="bert/embeddings/Slice", T=DataType.FLOAT, Index=DataType.INT32)
    pos = b.reshape(pos, [1, S, H], name="bert/embeddings/Reshape")
    x = b.add(emb, pos, name="bert/embeddings/add")
    typ = b.op("StridedSlice", [W("bert/embeddings/token_type_embeddings"),
                                _c(b, "bert/embeddings/strided_slice/stack", np.asarray([0], np.int32)),
                                _c(b, "bert/embeddings/strided_slice/stack_1", np.asarray([1], np.int32)),
                                _c(b, "bert/embeddings/strided_slice/stack_2", np.asarray([1], np.int32))],
               name="bert/embeddings/strided_slice", T=DataType.FLOAT, Index=DataType.INT32, begin_mask=0,
               end_mask=0, ellipsis_mask=0, new_axis_mask=0, shrink_axis_mask=1)
    x = b.add(x, typ, name="bert/embeddings/add_1")
    x = layer_norm(b, x, W("bert/embeddings/LayerNorm/gamma"), W("bert/embeddings/LayerNorm/beta"), cfg.eps,
                   "bert/embeddings/LayerNorm")
    # ---- attention mask adder [B, 1, 1, S]
    mf = b.cast(mask, "FLOAT", name="bert/encoder/Cast")
    m4 = b.op("ExpandDims", [b.op("ExpandDims", [mf, _c(b, "bert/encoder/ExpandDims/dim", np.int32(1))],
                                  name="bert/encoder/ExpandDims", T=DataType.FLOAT, Tdim=DataType.INT32),
                             _c(b, "bert/encoder/ExpandDims_1/dim", np.int32(1))],
              name="bert/encoder/ExpandDims_1", T=DataType.FLOAT, Tdim=DataType.INT32)
    one_minus = b.sub(_c(b, "bert/encoder/sub/x", np.float32(1.0)), m4, name="bert/encoder/sub")
    adder = b.mul(one_minus, _c(b, "bert/encoder/mul/y", np.float32(-10000.0)), name="bert/encoder/mul")
    x2 = b.reshape(x, [-1, H], name="bert/encoder/Reshape")
    shp4 = [-1, S, nh, dh]
    perm = _c(b, "bert/encoder/perm", np.asarray([0, 2, 1, 3], np.int32))
    for l in range(cfg.layers):
        p = f"bert/encoder/layer_{l}/"

        def dense(t, nm, k_name, act_scope=None):
            y = b.bias_add(b.matmul(t, W(p + k_name + "/kernel"), name=p + k_name + "/MatMul"),
                           W(p + k_name + "/bias"), name=p + k_name + "/BiasAdd")
            return y

        heads = []
        for nm in ("query", "key", "value"):
            t = dense(x2, nm, f"attention/self/{nm}")
            t = b.reshape(t, shp4, name=p + f"attention/self/Reshape_{nm}")
            heads.append(b.op("Transpose", [t, perm], name=p + f"attention/self/transpose_{nm}", T=DataType.FLOAT,
                              Tperm=DataType.INT32))
        q, k, v = heads
        sc = b.op("BatchMatMulV2", [q, k], name=p + "attention/self/MatMul", T=DataType.FLOAT, adj_x=False,
                  adj_y=True)
        sc = b.mul(sc, _c(b, p + "attention/self/Mul/y", np.float32(1.0 / math.sqrt(dh))),
                   name=p + "attention/self/Mul")
        sc = b.add(sc, adder, name=p + "attention/self/add")
        pr = b.softmax(sc, name=p + "attention/self/Softmax")
        ctx = b.op("BatchMatMulV2", [pr, v], name=p + "attention/self/MatMul_1", T=DataType.FLOAT, adj_x=False,
                   adj_y=False)
        ctx = b.op("Transpose", [ctx, perm], name=p + "attention/self/transpose_3", T=DataType.FLOAT,
                   Tperm=DataType.INT32)
        ctx = b.reshape(ctx, [-1, H], name=p + "attention/self/Reshape_3")
        o = dense(ctx, "o", "attention/output/dense")
        o = b.add(o, x2, name=p + "attention/output/add")
        x2 = layer_norm(b, o, W(p + "attention/output/LayerNorm/gamma"), W(p + "attention/output/LayerNorm/beta"),
                        cfg.eps, p + "attention/output/LayerNorm")
        f = gelu(b, dense(x2, "i", "intermediate/dense"), p + "intermediate/dense/gelu")
        f = dense(f, "f", "output/dense")
        f = b.add(f, x2, name=p + "output/add")
        x2 = layer_norm(b, f, W(p + "output/LayerNorm/gamma"), W(p + "output/LayerNorm/beta"), cfg.eps,
                        p + "output/LayerNorm")
    seq = b.reshape(x2, [-1, S, H], name="bert/encoder/Reshape_out")
    first = b.op("StridedSlice", [seq, _c(b, "bert/pooler/strided_slice/stack", np.asarray([0, 0, 0], np.int32)),
                                  _c(b, "bert/pooler/strided_slice/stack_1", np.asarray([0, 1, 0], np.int32)),
                                  _c(b, "bert/pooler/strided_slice/stack_2", np.asarray([1, 1, 1], np.int32))],
                 name="bert/pooler/strided_slice", T=DataType.FLOAT, Index=DataType.INT32, begin_mask=5, end_mask=5,
                 ellipsis_mask=0, new_axis_mask=0, shrink_axis_mask=0)
    first = b.op("Squeeze", [first], name="bert/pooler/Squeeze", T=DataType.FLOAT, squeeze_dims=[1])
    pooled = b.op("Tanh", [b.bias_add(b.matmul(first, W("bert/pooler/dense/kernel"), name="bert/pooler/dense/MatMul"),
                                      W("bert/pooler/dense/bias"), name="bert/pooler/dense/BiasAdd")],
                  name="bert/pooler/dense/Tanh", T=DataType.FLOAT)
    logits = b.bias_add(b.matmul(pooled, W("output_weights"), transpose_b=True, name="loss/MatMul"),
                        W("output_bias"), name="logits")
    b.softmax(logits, name="probs")
    del bsz
    return b.build_graph_def(), w


def bert_signature(cfg: BertConfig, seq_len: int, mask_from_ids: bool = False) -> SignatureDef:
    from ..export import tensor_info

    ins = {"input_ids": tensor_info("input_ids:0", "INT32", [-1, seq_len])}
    if not mask_from_ids:
        ins["input_mask"] = tensor_info("input_mask:0", "INT32", [-1, seq_len])
    return SignatureDef(inputs=ins,
                        outputs={"probabilities": tensor_info("probs:0", "FLOAT", [-1, cfg.num_labels]),
                                 "logits": tensor_info("logits:0", "FLOAT", [-1, cfg.num_labels])},
                        method_name="tensorflow/serving/predict")


def export_bert_saved_model(export_dir: str, cfg: BertConfig, seq_len: int, seed: int = 0,
                            mask_from_ids: bool = False) -> str:
    """BERT classifier (random init) as a TF 1.x SavedModel: weights in ``variables/``,
    ``serving_default`` predict signature over ``input_ids`` (/ ``input_mask``)."""
    from ..export import graph_def_to_saved_model

    gd, _ = bert_graph_def(cfg, seq_len, seed=seed, mask_from_ids=mask_from_ids)
    return graph_def_to_saved_model(export_dir, gd,
                                    {"serving_default": bert_signature(cfg, seq_len, mask_from_ids)})


def ids_and_mask(ids: torch.Tensor) -> dict:
    """Feeds of the graph for padded ids (pad id 0)."""
    ids = ids.to(torch.int32)
    return {"input_ids:0": ids, "input_mask:0": (ids != 0).to(torch.int32)}
