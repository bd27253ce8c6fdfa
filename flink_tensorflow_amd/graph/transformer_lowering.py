"""Transformer patterns of TF 1.x graphs for the graph compiler (BERT-style encoders).

A frozen / SavedModel BERT (``models/zoo/bert_graph.py`` builds one node for node like
Google's ``modeling.py``) arrives as decomposed ops.  Before lowering, the compiler matches:

* ``layer_norm`` — ``tf.contrib.layers.layer_norm``'s moments + batchnorm subgraph (11
  nodes) -> one ``layernorm`` kernel launch;
* embeddings — ``GatherV2(word, ids) + position rows + token-type row -> layer_norm`` ->
  one ``embed_layernorm`` launch (position and type rows are folded constants);
* self-attention — the query/key/value ``MatMul+BiasAdd -> Reshape -> Transpose`` of one
  input, ``BatchMatMul(adj_y) -> Mul(scale) -> Add(mask adder) -> Softmax -> BatchMatMul
  -> Transpose -> Reshape`` -> ONE fused QKV projection on the ping-pong MFMA GEMM (weights
  concatenated at compile time) + ONE flash-style ``attention`` launch; the
  ``(1 - mask) * -10000`` adder is replaced by the kernel's key mask (the int32
  ``input_mask``), and its subgraph disappears when nothing else reads it;
* GELU — BERT's tanh form after a ``MatMul+BiasAdd`` -> the GEMM's GELU epilogue;
* ``StridedSlice`` with constant bounds (the pooler's first token) -> one strided device
  copy; ``Squeeze`` / ``ExpandDims`` -> reshape aliases.

Every match is structural (op types, single-consumer chains, constant operands) and is
re-validated at lowering time against the folded constants; anything that does not match
lowers op by op as before.

**Token packing** (``CompiledFunction(token_capacity=T)``, driven by ``graph/packed.py``):
when the attention masks are ``NotEqual(input_ids, 0)`` of the fed ids (the mask-from-ids
layout) the plan runs padding-free — the embedding group becomes ``pack_tokens`` (real
tokens compacted into T rows, their in-sequence positions and per-sequence offsets on the
device) + ``embed_layernorm`` at those positions; every row-wise op (projections with their
fused bias / GELU / residual epilogues, LayerNorms, reshapes) runs on the T packed rows;
attention runs per packed sequence (``cu_seqlens``).  The pooler's first-token
``StridedSlice`` marks a **first-token-only region**: every node whose values reach the
fetches only through that slice (the final layer after its QKV projection) runs on one row
per sequence — ``cls_attention`` (first query over the sequence's keys), then the output
projection, residual LayerNorm, FFN and LayerNorm on B rows, with each packed operand read
through a first-row gather.  The reference product path this accelerates is
``ModelFunction`` over a loaded signature (``ModelFunction.scala:34-79``).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..ops import kernels as K

_ADDS = ("Add", "AddV2")
_BMM = ("BatchMatMul", "BatchMatMulV2", "BatchMatMulV3")


class TransformerLowering:
    """Mixin of ``CompiledFunction`` (uses its graph, ``cons``, ``vals`` and emitters)."""

    # ------------------------------------------------------------------ helpers
    def _node(self, src):
        return self.graph.nodes.get(src[0] if isinstance(src, tuple) else src)

    def _consumers(self, name):
        return list(self.cons.get(name, []))

    def _only_consumer(self, name, op_types):
        c = self._consumers(name)
        if len(c) != 1 or self._fetched(name):
            return None
        n = self.graph[c[0]]
        return n if n.op in op_types else None

    def _fetched(self, name):
        from ..types.names import TensorName

        return any(TensorName.parse(f).name == name for f in self.fetch_names)

    def _is_const_node(self, src) -> bool:
        """True when ``src`` depends only on constants (checked structurally)."""
        n = self._node(src)
        seen = set()
        stack = [n]
        while stack:
            m = stack.pop()
            if m is None or m.name in seen:
                continue
            seen.add(m.name)
            if m.op in ("Placeholder", "PlaceholderV2"):
                return False
            if m.op in ("VariableV2", "Variable", "VarHandleOp", "Const"):
                continue
            stack.extend(self._node(s) for s in m.inputs)
        return True

    def _const_of(self, src):
        v = self._const_val(src)
        return None if v is None else v.const

    # ------------------------------------------------------------------ matching
    def _prematch_transformer(self):
        self._groups: dict[str, dict] = {}
        g = self.graph
        for name in self.order:
            if g[name].op == "Rsqrt":
                self._match_ln(g[name])
        for name in self.order:
            if g[name].op == "Softmax":
                self._match_attention(g[name])
        for name in self.order:
            if g[name].op in ("GatherV2", "Gather"):
                self._match_embedding(g[name])
        self._drop_dead_mask_chains()

    def _add_group(self, grp):
        if any(m in self._groups for m in grp["members"]):
            return
        grp["done"] = False
        for m in grp["members"]:
            self._groups[m] = grp

    def _match_ln(self, rs):
        ve = self._node(rs.inputs[0])
        if ve is None or ve.op not in _ADDS:
            return
        var = next((self._node(s) for s in ve.inputs if self._node(s).op == "Mean"), None)
        if var is None:
            return
        eps_src = next(s for s in ve.inputs if s[0] != var.name)
        sq = self._node(var.inputs[0])
        if sq is None or sq.op != "SquaredDifference":
            return
        x_src = sq.inputs[0]
        sg = self._node(sq.inputs[1])
        mean = sg if sg.op == "Mean" else (self._node(sg.inputs[0]) if sg.op in ("StopGradient", "Identity") else None)
        if mean is None or mean.op != "Mean" or mean.inputs[0] != x_src:
            return
        inv = self._only_consumer(rs.name, ("Mul",))
        if inv is None:
            return
        gamma_src = next((s for s in inv.inputs if s[0] != rs.name), None)
        ic = [self.graph[c] for c in self._consumers(inv.name)]
        if len(ic) != 2 or any(c.op != "Mul" for c in ic) or self._fetched(inv.name):
            return
        mul1 = next((c for c in ic if x_src in c.inputs), None)
        mul2 = next((c for c in ic if (mean.name, 0) in c.inputs), None)
        if mul1 is None or mul2 is None or mul1 is mul2:
            return
        sub = self._only_consumer(mul2.name, ("Sub",))
        if sub is None or sub.inputs[1] != (mul2.name, 0):
            return
        beta_src = sub.inputs[0]
        add1 = self._only_consumer(mul1.name, _ADDS)
        if add1 is None or self._only_consumer(sub.name, _ADDS) is not add1:
            return
        members = {mean.name, sq.name, var.name, ve.name, rs.name, inv.name, mul1.name, mul2.name, sub.name,
                   add1.name}
        if sg is not mean:
            members.add(sg.name)
        if not set(self._consumers(mean.name)) <= members or not set(self._consumers(var.name)) <= members:
            return
        if not all(self._is_const_node(s) for s in (gamma_src, beta_src, eps_src, mean.inputs[1], var.inputs[1])):
            return
        self._add_group({"kind": "ln", "x": x_src, "gamma": gamma_src, "beta": beta_src, "eps": eps_src,
                         "axes": (mean.inputs[1], var.inputs[1]), "out": add1.name, "members": members})

    def _qkv_branch(self, src, bmm_name):
        """``src`` = Transpose(Reshape(BiasAdd(MatMul(x, W), b), [-1,S,nh,dh]), [0,2,1,3]) ->
        (x_src, matmul, biasadd, reshape, transpose) or None."""
        tr = self._node(src)
        if tr is None or tr.op != "Transpose" or self._consumers(tr.name) != [bmm_name]:
            return None
        rs = self._node(tr.inputs[0])
        if rs is None or rs.op != "Reshape" or self._consumers(rs.name) != [tr.name]:
            return None
        ba = self._node(rs.inputs[0])
        if ba is None or ba.op not in ("BiasAdd",) + _ADDS or self._consumers(ba.name) != [rs.name]:
            return None
        mm = self._node(ba.inputs[0])
        if mm is None or mm.op != "MatMul" or self._consumers(mm.name) != [ba.name] or mm.attr("transpose_a", False):
            return None
        if not (self._is_const_node(mm.inputs[1]) and self._is_const_node(ba.inputs[1])
                and self._is_const_node(rs.inputs[1]) and self._is_const_node(tr.inputs[1])):
            return None
        return mm.inputs[0], mm, ba, rs, tr

    def _match_attention(self, sm):
        add = self._node(sm.inputs[0])
        if add is None or add.op not in _ADDS or self._consumers(add.name) != [sm.name]:
            return
        mul = next((self._node(s) for s in add.inputs if self._node(s).op == "Mul"), None)
        if mul is None or self._consumers(mul.name) != [add.name]:
            return
        adder_src = next(s for s in add.inputs if s[0] != mul.name)
        bmm1 = next((self._node(s) for s in mul.inputs if self._node(s).op in _BMM), None)
        if bmm1 is None or not bmm1.attr("adj_y", False) or bmm1.attr("adj_x", False):
            return
        if self._consumers(bmm1.name) != [mul.name]:
            return
        scale_src = next(s for s in mul.inputs if s[0] != bmm1.name)
        if not self._is_const_node(scale_src):
            return
        bmm2 = self._only_consumer(sm.name, _BMM)
        if bmm2 is None or bmm2.inputs[0] != (sm.name, 0) or bmm2.attr("adj_x", False) or bmm2.attr("adj_y", False):
            return
        tr_o = self._only_consumer(bmm2.name, ("Transpose",))
        rs_o = self._only_consumer(tr_o.name, ("Reshape",)) if tr_o is not None else None
        if rs_o is None:
            return
        br = [self._qkv_branch(bmm1.inputs[0], bmm1.name), self._qkv_branch(bmm1.inputs[1], bmm1.name),
              self._qkv_branch(bmm2.inputs[1], bmm2.name)]
        if any(b is None for b in br) or len({b[0] for b in br}) != 1:
            return
        # the mask adder: a chain of unary / constant-operand ops over ONE non-constant leaf
        mask_src, chain = self._mask_leaf(adder_src)
        if mask_src is None:
            return
        members = {add.name, mul.name, bmm1.name, sm.name, bmm2.name, tr_o.name, rs_o.name}
        for _, mm, ba, rs, tr in br:
            members |= {mm.name, ba.name, rs.name, tr.name}
        self._add_group({"kind": "attn", "x": br[0][0], "branches": [b[1:] for b in br], "scale": scale_src,
                         "mask": mask_src, "mask_chain": chain, "perm": tr_o.inputs[1], "out": rs_o.name,
                         "members": members})

    def _mask_leaf(self, src):
        """(leaf tensor, chain node names) of ``(1 - Cast(m)[:, None, None, :]) * c`` where
        ``m`` is a fed int mask (1 = keep) or ``NotEqual(ids, 0)`` of the fed ids — in both
        cases "key j is padding" is ``leaf[b, j] == 0``, the attention kernel's pad test."""
        chain, cur = [], self._node(src)
        for i in range(7):
            if cur is None:
                return None, None
            if i == 0 and cur.op != "Mul" or i == 1 and cur.op != "Sub":
                return None, None
            if i >= 2 and cur.op not in ("ExpandDims", "Reshape", "Cast", "NotEqual"):
                return None, None
            chain.append(cur.name)
            nonconst = [s for s in cur.inputs if not self._is_const_node(s)]
            if len(nonconst) != 1:
                return None, None
            if cur.op == "NotEqual":
                c = self._const_of(next(s for s in cur.inputs if s != nonconst[0]))
                if c is None or c.numel() != 1 or float(c.reshape(-1)[0]) != 0.0:
                    return None, None
            nxt = self._node(nonconst[0])
            if nxt.op in ("Placeholder", "PlaceholderV2"):
                return nonconst[0], chain
            cur = nxt
        return None, None

    def _match_embedding(self, ga):
        if len(ga.inputs) < 2 or not self._is_const_node(ga.inputs[0]) or self._is_const_node(ga.inputs[1]):
            return
        if len(ga.inputs) > 2 and not self._is_const_node(ga.inputs[2]):
            return
        a0 = self._only_consumer(ga.name, _ADDS)
        a1 = self._only_consumer(a0.name, _ADDS) if a0 is not None else None
        if a1 is None:
            return
        pos_src = next(s for s in a0.inputs if s[0] != ga.name)
        typ_src = next(s for s in a1.inputs if s[0] != a0.name)
        if not (self._is_const_node(pos_src) and self._is_const_node(typ_src)):
            return
        ln = next((g for g in self._groups.values() if g["kind"] == "ln" and g["x"] == (a1.name, 0)), None)
        if ln is None or not set(self._consumers(a1.name)) <= ln["members"]:
            return
        members = {ga.name, a0.name, a1.name} | ln["members"]
        grp = {"kind": "emb", "ids": ga.inputs[1], "word": ga.inputs[0], "axis": ga.inputs[2] if len(ga.inputs) > 2
               else None, "pos": pos_src, "type": typ_src, "ln": ln, "out": ln["out"], "members": members}
        for m in ln["members"]:
            self._groups.pop(m, None)
        grp["done"] = False
        for m in members:
            self._groups[m] = grp

    def _drop_dead_mask_chains(self):
        """Mask-adder nodes read only by fused attention groups are never lowered."""
        chains = {n for g in self._groups.values() if g["kind"] == "attn" for n in g["mask_chain"]}
        changed = True
        while changed:
            changed = False
            for n in list(chains):
                if n in self._groups:
                    continue
                if all(c in self._groups or c in chains for c in self._consumers(n)) and not self._fetched(n):
                    self._groups[n] = {"kind": "dead", "members": {n}, "done": True}
                    self._fused.add(n)
                    changed = True

    # ------------------------------------------------------------------ token packing
    _ROWWISE = ("MatMul", "BiasAdd", "Add", "AddV2", "Sub", "Mul", "Pow", "Tanh", "Identity", "Reshape",
                "RealDiv", "Relu", "Sigmoid")

    def _setup_packing(self):
        """Validates that the graph can run token-packed and finds the first-token-only region
        (``self._cls_nodes``); raises ``CompileError`` otherwise."""
        from ..types.names import TensorName
        from .compiler import CompileError

        grps = list({id(g): g for g in self._groups.values()}.values())
        embs = [g for g in grps if g["kind"] == "emb"]
        attns = [g for g in grps if g["kind"] == "attn"]
        if len(embs) != 1 or not attns:
            raise CompileError("token packing needs one embedding group and fused attention")
        ids_src = embs[0]["ids"]
        feed = next((f for f in self.feed_names if (TensorName.parse(f).name, TensorName.parse(f).index) == ids_src),
                    None)
        if feed is None:
            raise CompileError("token packing needs the embedding ids to be a feed")
        shape, _ = self.feed_specs[feed]
        if len(shape) != 2:
            raise CompileError("token packing needs [batch, seq] ids")
        B, S = (int(v) for v in shape)
        for g in attns:  # every attention mask must be "id != 0" of these ids
            if g["mask"] != ids_src or not any(self.graph[n].op == "NotEqual" for n in g["mask_chain"]):
                raise CompileError("token packing needs attention masks computed from the ids (NotEqual(ids, 0))")
        T = int(self.token_cap)
        if not 0 < T <= B * S:
            raise CompileError(f"token capacity {T} outside (0, {B * S}]")
        self._pack = {"ids": ids_src, "feed": feed, "B": B, "S": S, "T": T, "pad": 0, "cu": None, "cls": None}
        # first-token-only region: nodes whose every consumer is in the region or is the
        # pooler's first-token slice (reverse topological order: consumers first)
        starts = {n for n in self.order if self.graph[n].op == "StridedSlice" and self._first_token_spec(self.graph[n])}
        if not starts:
            return
        attn_out = {g["out"]: g for g in attns}
        fed = {TensorName.parse(f).name for f in self.feed_names}
        region: set[str] = set()
        barrier: set[str] = set()
        for n in reversed(self.order):
            if n in region or n in fed or n in starts or self._fetched(n):
                continue
            cons = self._consumers(n)
            if not cons or any(c in barrier for c in cons) or not all(c in region or c in starts for c in cons):
                continue
            grp = self._groups.get(n)
            if n in attn_out:  # the attention itself: first query only, over all keys
                g = attn_out[n]
                g["cls"] = True
                region |= g["members"]
                barrier |= g["members"]  # its input keeps every row (keys / values)
                continue
            if grp is not None and grp["kind"] == "attn":
                continue
            op = self.graph[n].op
            in_ln = grp is not None and grp["kind"] == "ln"
            if op not in self._ROWWISE and not (in_ln and op in ("Mean", "SquaredDifference", "Rsqrt",
                                                                  "StopGradient")):
                continue
            if self._is_const_node((n, 0)):
                continue
            region.add(n)
        self._cls_nodes = region

    def _first_token_spec(self, node) -> bool:
        """``x[:, 0:1, :]`` / ``x[:, 0, :]`` of a rank-3 tensor (constant bounds, unit strides)."""
        if len(node.inputs) != 4 or node.attr("ellipsis_mask", 0) or node.attr("new_axis_mask", 0):
            return False
        if self._is_const_node(node.inputs[0]):
            return False
        b, e, s = (self._const_of(node.inputs[i]) for i in (1, 2, 3))
        if b is None or e is None or s is None:
            return False
        b, e, s = (t.reshape(-1).tolist() for t in (b, e, s))
        if len(b) != 3 or any(v != 1 for v in s):
            return False
        bm, em, shrink = node.attr("begin_mask", 0), node.attr("end_mask", 0), node.attr("shrink_axis_mask", 0)
        full = all((bm >> d & 1 or b[d] == 0) and em >> d & 1 and not shrink >> d & 1 for d in (0, 2))
        first = not bm >> 1 & 1 and b[1] == 0 and (shrink >> 1 & 1 or (not em >> 1 & 1 and e[1] == 1))
        return full and first

    def _cls_gather(self, v):
        """(B, D) rows of each sequence's first token of the packed ``v`` (one gather step,
        cached per value)."""
        from .compiler import _view

        hit = self._cls_cache.get(id(v))
        if hit is not None:
            return hit
        pk = self._pack
        out = self._new((pk["B"], v.shape[-1]), v.dtype)
        out.rows, out.lshape = "cls", v.lshape
        cls = pk["cls"]

        from ..ops import kernels as K

        def run(v=v, out=out, cls=cls):
            src = _view(v)
            K.gather_rows(src.reshape(-1, src.shape[-1]), cls.buf, out=out.buf)

        self._emit(f"first_token_gather/{len(self._cls_cache)}", "gather", run, [v, cls], [out])
        self._cls_cache[id(v)] = out
        return out

    def _reshape_rows(self, node, x, shape):
        """Reshape of packed / first-token rows: only the row split ([B*S, D] <-> [B, S, D])
        may change; the physical rows stay."""
        from .compiler import CompileError, Val

        pk = self._pack
        D = x.shape[-1]
        n = pk["B"] * pk["S"] * D
        if -1 in shape:
            i = shape.index(-1)
            rest = int(np.prod([v for j, v in enumerate(shape) if j != i]))
            shape[i] = n // max(rest, 1)
        if shape[-1] != D or int(np.prod(shape)) != n or list(shape[:-1]) not in ([pk["B"] * pk["S"]],
                                                                                   [pk["B"], pk["S"]]):
            raise CompileError(f"reshape {node.name} of packed token rows to {shape}")
        self.vals[(node.name, 0)] = Val(tuple(x.shape), x.dtype, alias_of=x, rows=x.rows, lshape=tuple(shape))

    def _slice_first_token(self, node, x) -> bool:
        from .compiler import CompileError, Val

        if not self._first_token_spec(node) or x.lshape is None or len(x.lshape) != 3:
            raise CompileError(f"StridedSlice {node.name} of packed token rows is not a first-token slice")
        if x.rows == "packed":
            x = self._cls_gather(x)
        B, D = self._pack["B"], x.shape[-1]
        shp = (B, D) if node.attr("shrink_axis_mask", 0) >> 1 & 1 else (B, 1, D)
        self.vals[(node.name, 0)] = Val(shp, x.dtype, alias_of=x)
        return True

    # ------------------------------------------------------------------ lowering
    def _lower_group(self, grp) -> bool:
        """Lowers a matched group (False: its constants do not validate -> op by op)."""
        kind = grp["kind"]
        ok = {"ln": self._lower_ln_group, "attn": self._lower_attn_group, "emb": self._lower_emb_group}[kind](grp)
        if ok:
            grp["done"] = True
            for m in grp["members"]:
                self._fused.add(m)
        else:
            for m in grp["members"]:
                self._groups.pop(m, None)
        return ok

    def _ln_params(self, grp):
        gamma, beta, eps = (self._const_of(grp[k]) for k in ("gamma", "beta", "eps"))
        axes = [self._const_of(a) for a in grp["axes"]]
        if any(t is None for t in (gamma, beta, eps, *axes)):
            return None
        if any(int(a.reshape(-1)[0]) not in (-1,) and a.numel() != 1 for a in axes):
            return None
        return gamma.float().reshape(-1), beta.float().reshape(-1), float(eps.float().reshape(-1)[0])

    def _lower_ln_group(self, grp) -> bool:
        x = self._get(grp["x"])
        p = self._ln_params(grp)
        if x is None or x.is_const or p is None:
            return False
        gamma, beta, eps = p
        D = x.shape[-1]
        axes = [int(self._const_of(a).reshape(-1)[0]) for a in grp["axes"]]
        if any(a not in (-1, len(x.shape) - 1) for a in axes) or gamma.numel() != D or beta.numel() != D:
            return False
        xin = self._as_bf16(x, grp["out"])
        g_dev, b_dev = self._dev(gamma, torch.float32), self._dev(beta, torch.float32)
        self.params += [g_dev, b_dev]
        out = self._new(x.shape)
        out.rows, out.lshape = x.rows, x.lshape

        def run(xin=xin, out=out, g=g_dev, b=b_dev, eps=eps, D=D):
            K.layernorm(_rows(xin, D), g, b, eps=eps, out=out.buf.view(-1, D))

        self._emit(grp["out"], "layernorm", run, [xin], [out])
        self.vals[(grp["out"], 0)] = out
        return True

    def _lower_emb_group(self, grp) -> bool:
        ids = self._get(grp["ids"])
        word, pos, typ = (self._const_of(grp[k]) for k in ("word", "pos", "type"))
        p = self._ln_params(grp["ln"])
        if ids is None or ids.is_const or word is None or pos is None or typ is None or p is None:
            return False
        if grp["axis"] is not None and int(self._const_of(grp["axis"]).reshape(-1)[0]) != 0:
            return False
        if len(ids.shape) != 2 or ids.dtype not in (torch.int32, torch.int64):
            return False
        B, S = ids.shape
        V, D = word.shape
        pos = pos.float().reshape(-1, D)
        typ = typ.float().reshape(-1, D)
        if pos.shape[0] != S or typ.shape[0] != 1:
            return False
        gamma, beta, eps = p
        w_dev = self._dev(word.float(), torch.bfloat16)
        pos_dev = self._dev(pos, torch.bfloat16)
        typ_dev = self._dev(typ, torch.bfloat16)
        g_dev, b_dev = self._dev(gamma, torch.float32), self._dev(beta, torch.float32)
        self.params += [w_dev, pos_dev, typ_dev, g_dev, b_dev]
        ids32 = ids
        if ids.dtype != torch.int32:
            return False
        pk = self._pack
        if pk is not None and (grp["ids"] == pk["ids"]):
            if (B, S) != (pk["B"], pk["S"]):
                return False
            T = pk["T"]
            pids, ppos = self._new((T,), torch.int32), self._new((T,), torch.int32)
            cu, cls = self._new((B + 1,), torch.int32), self._new((B,), torch.int32)
            pk["cu"], pk["cls"] = cu, cls

            def run_pack(ids=ids32, pids=pids, ppos=ppos, cu=cu, cls=cls):
                K.pack_tokens(_view_(ids).reshape(B, S), pk["pad"], T, pids.buf, ppos.buf, cu.buf, cls.buf)

            self._emit(grp["out"] + "/pack_tokens", "pack", run_pack, [ids32], [pids, ppos, cu, cls])
            out = self._new((T, D))
            out.rows, out.lshape = "packed", (B, S, D)

            def run_p(pids=pids, ppos=ppos, out=out):
                K.embed_layernorm(pids.buf, None, w_dev, pos_dev, typ_dev, g_dev, b_dev, S, eps, out=out.buf,
                                  pos_ids=ppos.buf)

            self._emit(grp["out"], "embed_ln", run_p, [pids, ppos], [out])
            self.vals[(grp["out"], 0)] = out
            return True
        out = self._new((B, S, D))

        def run(ids=ids32, out=out):
            K.embed_layernorm(_view_(ids).reshape(-1), None, w_dev, pos_dev, typ_dev, g_dev, b_dev, S, eps,
                              out=out.buf.view(-1, D))

        self._emit(grp["out"], "embed_ln", run, [ids32], [out])
        self.vals[(grp["out"], 0)] = out
        return True

    def _lower_attn_group(self, grp) -> bool:
        x = self.vals.get(grp["x"])  # never first-token gathered: keys / values need every row
        mask = self._get(grp["mask"])
        if x is None or x.is_const or len(x.shape) != 2 or mask is None or mask.is_const:
            return False
        if x.rows is not None and x.rows != "packed":
            return False
        if mask.dtype != torch.int32 or len(mask.shape) != 2:
            return False
        ws, bs = [], []
        shp = None
        for mm, ba, rs, tr in grp["branches"]:
            w = self._const_of(mm.inputs[1])
            b = self._const_of(ba.inputs[1])
            s = self._const_of(rs.inputs[1])
            pm = self._const_of(tr.inputs[1])
            if w is None or b is None or s is None or pm is None or pm.reshape(-1).tolist() != [0, 2, 1, 3]:
                return False
            w = w.float()
            ws.append(w.t() if not mm.attr("transpose_b", False) else w)
            bs.append(b.float().reshape(-1))
            s = [int(v) for v in s.reshape(-1).tolist()]
            if shp is not None and s != shp:
                return False
            shp = s
        perm = self._const_of(grp["perm"])
        scale = self._const_of(grp["scale"])
        if perm is None or perm.reshape(-1).tolist() != [0, 2, 1, 3] or scale is None or len(shp) != 4:
            return False
        T, Din = x.shape
        _, S, nh, dh = shp
        H = nh * dh
        pk = self._pack if x.rows == "packed" else None
        B = pk["B"] if pk is not None else T // S
        if pk is not None and (S != pk["S"] or pk["cu"] is None):
            return False
        if dh != 64 or (pk is None and B * S != T) or tuple(mask.shape) != (B, S) or \
                any(w.shape != (H, Din) for w in ws):
            return False
        w_qkv = self._dev(torch.cat(ws, 0), torch.bfloat16)
        b_qkv = self._dev(torch.cat(bs, 0), torch.float32)
        self.params += [w_qkv, b_qkv]
        xin = self._as_bf16(x, grp["out"])
        qkv = self._new((T, 3 * H))
        cls_only = pk is not None and grp.get("cls", False)
        ctx = self._new((B, H) if cls_only else (T, H))
        if pk is not None:
            qkv.rows = "packed"
            ctx.rows, ctx.lshape = ("cls" if cls_only else "packed"), (B * S, H)
        sc = float(scale.float().reshape(-1)[0])
        gpu = self.device.type == "cuda"
        splits = K.gemm_pp_splits(T, 3 * H, Din) if gpu and Din % 64 == 0 else 1
        wsp = torch.empty(splits * T * 3 * H, dtype=torch.float32, device=self.device) if splits > 1 else None

        def run_qkv(xin=xin, qkv=qkv):
            if gpu and Din % 64 == 0:
                K.gemm_pp(_rows(xin, Din), w_qkv, b_qkv, out=qkv.buf, splits=splits, ws=wsp)
            else:
                K.gemm(_rows(xin, Din), w_qkv, b_qkv, out=qkv.buf)

        def run_attn(qkv=qkv, ctx=ctx, mask=mask):
            K.attention(qkv.buf, _view_(mask).reshape(-1), B, S, nh, pad_id=0, scale=sc, out=ctx.buf)

        if pk is not None:
            cu = pk["cu"]

            def run_attn(qkv=qkv, ctx=ctx, cu=cu):  # noqa: F811
                if cls_only:  # first query of each sequence only (the pooler reads nothing else)
                    K.cls_attention(qkv.buf, cu.buf, B, nh, scale=sc, out=ctx.buf)
                else:
                    K.attention(qkv.buf, None, B, S, nh, scale=sc, out=ctx.buf, cu_seqlens=cu.buf)

            mask = cu
        self._emit(grp["out"] + "/qkv", "gemm", run_qkv, [xin], [qkv], {"impl": "gemm_pp", "fused": "qkv"})
        self._emit(grp["out"], "cls_attention" if cls_only else "attention", run_attn, [qkv, mask], [ctx])
        self.vals[(grp["out"], 0)] = ctx
        return True

    # ---- GELU epilogue after MatMul + BiasAdd
    def _match_gelu(self, xnode):
        """``x * 0.5 * (1 + tanh(sqrt(2/pi) * (x + 0.044715 x^3)))`` over ``xnode``'s output
        -> (final node, member nodes) or None."""
        xs = (xnode.name, 0)
        cs = [self.graph[c] for c in self._consumers(xnode.name)]
        if len(cs) != 3 or self._fetched(xnode.name):
            return None
        pw = next((c for c in cs if c.op == "Pow"), None)
        ad = next((c for c in cs if c.op in _ADDS), None)
        fin = next((c for c in cs if c.op == "Mul"), None)
        if pw is None or ad is None or fin is None:
            return None

        def const_is(src, val):
            c = self._const_of(src) if self._is_const_node(src) else None
            return c is not None and c.numel() == 1 and abs(float(c.float().reshape(-1)[0]) - val) < 1e-4 * max(1, val)

        def other(n, s):
            o = [i for i in n.inputs if i != s]
            return o[0] if len(o) == 1 else None

        if pw.inputs[0] != xs or not const_is(pw.inputs[1], 3.0):
            return None
        m1 = self._only_consumer(pw.name, ("Mul",))
        if m1 is None or not const_is(other(m1, (pw.name, 0)), 0.044715):
            return None
        if self._only_consumer(m1.name, _ADDS) is not ad or other(ad, (m1.name, 0)) != xs:
            return None
        m2 = self._only_consumer(ad.name, ("Mul",))
        if m2 is None or not const_is(other(m2, (ad.name, 0)), math.sqrt(2 / math.pi)):
            return None
        th = self._only_consumer(m2.name, ("Tanh",))
        a2 = self._only_consumer(th.name, _ADDS) if th is not None else None
        if a2 is None or not const_is(other(a2, (th.name, 0)), 1.0):
            return None
        cdf = self._only_consumer(a2.name, ("Mul",))
        if cdf is None or not const_is(other(cdf, (a2.name, 0)), 0.5):
            return None
        if self._only_consumer(cdf.name, ("Mul",)) is not fin or other(fin, (cdf.name, 0)) != xs:
            return None
        return fin, [pw, m1, ad, m2, th, a2, cdf, fin]

    # ---- StridedSlice / Squeeze / ExpandDims
    def _lower_strided_slice(self, node) -> bool:
        x = self.vals.get(node.inputs[0])
        if x is not None and x.rows is not None:
            return self._slice_first_token(node, x)
        x = self._get(node.inputs[0])
        if x is None or x.is_const or x.phys_c or x.qscale is not None:
            return False
        b, e, s = (self._const_of(node.inputs[i]) for i in (1, 2, 3))
        if b is None or e is None or s is None:
            return False
        if node.attr("ellipsis_mask", 0) or node.attr("new_axis_mask", 0):
            return False
        b, e, s = (t.reshape(-1).tolist() for t in (b, e, s))
        bm, em, shrink = node.attr("begin_mask", 0), node.attr("end_mask", 0), node.attr("shrink_axis_mask", 0)
        sl, shape = [], []
        for d in range(len(x.shape)):
            if d >= len(b):
                sl.append(slice(None))
                shape.append(x.shape[d])
                continue
            if s[d] != 1:
                return False
            n = x.shape[d]
            lo = 0 if bm >> d & 1 else (b[d] + n if b[d] < 0 else b[d])
            if shrink >> d & 1:
                sl.append(lo)
                continue
            hi = n if em >> d & 1 else (e[d] + n if e[d] < 0 else min(e[d], n))
            sl.append(slice(lo, hi))
            shape.append(max(0, hi - lo))
        out = self._new(tuple(shape), x.dtype)
        sl = tuple(sl)

        def run(x=x, out=out, sl=sl):
            out.buf.copy_(_view_(x)[sl].reshape(out.buf.shape))

        self._emit(node.name, "copy", run, [x], [out])
        self.vals[(node.name, 0)] = out
        return True

    def _lower_squeeze_like(self, node) -> bool:
        from .graph import Node  # noqa: F401

        x = self._get(node.inputs[0])
        if x is None or x.is_const or x.phys_c:
            return False
        shape = list(x.shape)
        if node.op == "Squeeze":
            dims = node.attr("squeeze_dims", []) or [i for i, d in enumerate(shape) if d == 1]
            dims = sorted(d % len(shape) for d in dims)
            if any(shape[d] != 1 for d in dims):
                return False
            shape = [d for i, d in enumerate(shape) if i not in dims]
        else:
            dv = self._const_of(node.inputs[1])
            if dv is None:
                return False
            d = int(dv.reshape(-1)[0])
            d = d + len(shape) + 1 if d < 0 else d
            shape.insert(d, 1)
        from .compiler import Val

        self.vals[(node.name, 0)] = Val(tuple(shape), x.dtype, alias_of=x)
        return True


def _view_(v):
    from .compiler import _view

    return _view(v)


def _rows(v, D):
    return _view_(v).reshape(-1, D)
