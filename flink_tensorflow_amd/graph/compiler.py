"""Graph compiler: lowers a (feeds → fetches) signature of a TF graph onto the CDNA4
kernels for fixed input shapes, plans HBM buffers, and captures the launch sequence in
a hipGraph (``torch.cuda.CUDAGraph`` is HIP graph capture on ROCm).

This is the MI355X replacement of libtensorflow's session executor for the hot path
(SURVEY §2.8 N2/N3, §7.3).  Passes:

1. **prune** to the fetched subgraph, stopping at fed tensors;
2. **constant folding** of everything that depends only on Const/variables (weights are
   frozen into the plan; variables are read from the session at compile time);
3. **fusion** (pattern match, TF semantics preserved):
   * ``Conv2D → [BiasAdd | FusedBatchNorm]* → [Add(residual)] → [Relu|Relu6]`` → one
     implicit-GEMM conv launch with BN folded into the weights and a bias+residual+act
     epilogue;
   * ``MatMul → [BiasAdd] → [Add] → [act]`` → one MFMA GEMM launch;
   * ``uint8 feed → Cast → ResizeBilinear → Sub → Div|Mul`` → the fused preprocess kernel
     (bf16 NHWC, channels padded to 8 for the stem conv);
   * ``Mean(axes=[1,2])`` → global-avg-pool; ``MaxPool``/``AvgPool`` → pool kernel;
   * ``Softmax [→ TopKV2]`` → fused softmax+top-k kernel;
   * ``ConcatV2`` on channels → producers write straight into channel slices of one
     buffer (no copy) when every producer is a kernel that supports it;
   * everything else runs as captured PyTorch glue ops (logged; ``strict=True`` rejects).
4. **memory planning**: every intermediate gets an offset in one activation slab from the
   native liveness planner (``csrc/arena.cpp``); with a subtask ``DeviceArena`` the slab is
   shared by all of the subtask's bucket plans and identical weights are stored once;
5. **capture**: one hipGraph per (signature, batch size).

Activations are bf16 NHWC on device; fetched outputs are cast back to the graph dtype.

``precision="fp8"`` (BASELINE "Inception-v3 fp8 weights"): a bf16 twin of the plan is
first run on calibration inputs to record every activation's absolute maximum; then each
Conv2D chain whose channels are multiples of 16 (and has no residual) is lowered onto the
fp8 MFMA kernel with per-channel e4m3 weights, and its output is stored as e4m3 with a
static per-tensor scale whenever every consumer reads fp8 (convs, pools, concats,
global-average-pool).  Concat branches write with the concat buffer's scale; max/avg
pools requantise on the fly; anything else reads a dequantised bf16 copy.
"""
from __future__ import annotations

import logging
import types
from dataclasses import dataclass, field
from typing import Any, Callable

import numpy as np
import torch

from ..ops import fp8 as F8
from ..ops import kernels as K
from ..types.dtypes import DataType
from ..types.names import TensorName
from ..types.tensor import StringTensor
from ..utils import tracing
from . import ops_core  # noqa: F401
from .graph import Graph, Node
from .op_registry import OpContext, lookup
from .ops_nn import same_pads
from .transformer_lowering import TransformerLowering

LOG = logging.getLogger("flink_tensorflow_amd.compiler")

_ACTS = {"Relu": K.ACT_RELU, "Relu6": K.ACT_RELU6, "Sigmoid": K.ACT_SIGMOID, "Tanh": K.ACT_TANH}
_BINARY = {"Add": "add", "AddV2": "add", "Sub": "sub", "Mul": "mul", "RealDiv": "div", "Div": "div",
           "Maximum": "max", "Minimum": "min"}


def _cfg():
    from ..config import current

    return current()

# conv_lite tiles (kernels/conv_pp.hip): bf16 tile 2 = 128 pixels x 128 channels on 4 waves,
# two LDS-DMA stages; fp8 cfg 11 = the channel tile (192 / 160 / 128 / 96 / 64) staging the
# fewest rows per layer (profiles/r04_af).  Measured slower and removed (numbers in the
# profile READMEs): the 128x256 bf16 tile (r04_ad), the 8-wave DMA / MFMA-split tiles (r04_u,
# r04_w), the halo-staged 3x3 kernel (r04_s-u), the 32-deep tile, the fp8 tile choosers
# 0 / 1 / 3 (r04_ac, r04_ah), conv_lite for the deep-K 1x1 reduces (r03_conv), the streamed
# stage-2 block tail (r01_tail), the persistent dual projection kernel (r02_pw_res2) and the
# probe-selected ping-pong conv_pp tiles (r02_conv_pp).
LITE_TILE = 2
LITE_FP8_CFG = 11


class CompileError(RuntimeError):
    pass


@dataclass
class Val:
    """A symbolic value in the plan."""

    shape: tuple
    dtype: torch.dtype
    const: Any = None          # folded constant (host tensor / StringTensor)
    buf: torch.Tensor | None = None
    phys_c: int | None = None  # physical channel count when padded (stem input)
    alias_of: "Val | None" = None
    last_use: int = -1
    concat_slot: tuple | None = None  # (target Val, channel offset) for concat-by-stride-write
    qscale: float | None = None  # fp8 e4m3 storage (uint8 buffer) with this per-tensor scale
    # token-packed plans (``token_capacity``): "packed" = one row per real token (the plan's
    # token capacity T rows), "cls" = one row per sequence (its first token); ``shape`` is
    # then the physical [rows, D] and ``lshape`` the graph's logical shape ([B*S, D] or
    # [B, S, D]) that Reshape / StridedSlice reason about
    rows: str | None = None
    lshape: tuple | None = None

    @property
    def is_const(self):
        return self.const is not None


@dataclass
class Step:
    name: str
    kind: str
    fn: Callable[[], None]
    inputs: list = field(default_factory=list)
    outputs: list = field(default_factory=list)
    meta: dict = field(default_factory=dict)


class _ConstSession:
    """Minimal session facade for folding constants through interpreter kernels."""

    def __init__(self, variables):
        self.variables = variables
        self._const_cache = {}


class CompiledFunction(TransformerLowering):
    def __init__(self, graph: Graph, feeds: dict[str, tuple[tuple, Any]], fetches: list[str], device,
                 variables: dict | None = None, use_graph: bool = True, strict: bool = False,
                 topk_fetch: bool = True, precision: str = "bf16", calibration: dict | None = None,
                 arena=None, token_capacity: int | None = None):
        if precision not in ("bf16", "fp8"):
            raise ValueError(f"precision must be bf16 or fp8, not {precision!r}")
        from .control_flow import fold_static_control_flow
        from .functions import has_functional_ops, lower_functional_ops

        # function calls / functional If / While inline into plain dataflow first; then TF1
        # conds on compile-time-constant predicates (an exported ``is_training`` switch left
        # at its default) resolve before lowering: the plan is the cond-free one
        if has_functional_ops(graph):
            graph = lower_functional_ops(graph)
        graph = fold_static_control_flow(graph, list(feeds), list(fetches))
        self.graph = graph
        self.arena = arena  # subtask DeviceArena (shared slab + interned weights) or None
        # padding-free transformer plan: token rows packed into this capacity (graph/packed.py)
        self.token_cap = token_capacity
        self._pack: dict | None = None
        self._cls_nodes: set[str] = set()
        self._cur_cls = False
        self._cls_cache: dict[int, Val] = {}
        self.activation_bytes = 0
        self.precision = precision
        self.device = torch.device(device)
        if self.device.type != "cuda":
            use_graph = False  # host plans run the fp32 reference ops (used by CPU tests)
        self.feed_names = [str(TensorName.parse(f)) for f in feeds]
        self.feed_specs = {str(TensorName.parse(f)): v for f, v in feeds.items()}
        self.fetch_names = [str(TensorName.parse(f)) for f in fetches]
        self.variables = variables or {}
        self.strict = strict
        self.steps: list[Step] = []
        self.params: list[torch.Tensor] = []  # device weights/biases baked into the plan
        self.glue_ops: list[str] = []
        self.vals: dict[tuple[str, int], Val] = {}
        self._fused: set[str] = set()
        self._const_sess = _ConstSession(self.variables)
        self._input_bufs: dict[str, torch.Tensor] = {}
        self._outputs: list = []
        self._graph_obj: torch.cuda.CUDAGraph | None = None
        # graph of steps[1:] when steps[0] is the preprocess kernel reading a feed nothing else
        # reads: ``replay_from`` then runs that kernel on the caller's staging buffer
        self._graph_tail: torch.cuda.CUDAGraph | None = None
        self._head: tuple[str, Step] | None = None
        self._amax: dict[str, float] = {}
        self.fp8_layers = 0
        self._debug_sync = tracing.debug_sync()
        self._poison_after: dict[int, list] = {}
        # batch-slice chain (``_find_chain``): (first step, end step, slices, slice size,
        # values whose full buffers are sliced per slice) or None
        self._chain: tuple | None = None
        if self._debug_sync or tracing.debug_poison():
            use_graph = False  # debug modes act between launches: run the plan eagerly
        import contextlib

        if precision == "fp8":  # calibrate activation ranges on a bf16 twin of the plan
            twin = CompiledFunction(graph, feeds, fetches, device, variables, use_graph=False, strict=strict)
            self._amax = twin.calibrate(calibration)
            del twin

        with torch.cuda.device(self.device) if self.device.type == "cuda" else contextlib.nullcontext():
            self._compile()
            self._plan_memory_and_bind()
            if use_graph:
                self._capture()

    # ================================================================== compile
    def _compile(self):
        g = self.graph
        fed = {TensorName.parse(f) for f in self.feed_names}
        fed_nodes = {f.name for f in fed}
        needed, stack = set(), [TensorName.parse(f).name for f in self.fetch_names]
        while stack:
            n = stack.pop()
            if n in needed:
                continue
            needed.add(n)
            if n in fed_nodes:
                continue
            node = g[n]
            stack.extend(s for s, _ in node.inputs)
            stack.extend(node.control_inputs)
        self.order = [n for n in g.topo_order(needed)]
        self.needed = needed
        # consumers restricted to the pruned subgraph
        self.cons: dict[str, list[str]] = {}
        for n in self.order:
            for s, _ in g[n].inputs:
                self.cons.setdefault(s, []).append(n)
        self._groups = {}
        self._prematch_transformer()  # layer_norm / attention / embedding patterns (BERT graphs)
        if self.token_cap is not None:
            self._setup_packing()  # CompileError when the graph cannot run token-packed
        for f in fed:
            shape, dt = self.feed_specs[str(f)]
            dt = DataType.of(dt).torch
            self.vals[(f.name, f.index)] = Val(tuple(shape), dt)
        # Lower in topological order, but defer a Conv2D/MatMul whose fused chain ends in a
        # residual Add until the other Add operand has been lowered (DFS topo order often
        # visits the main path before the shortcut branch).
        pending: list[str] = []

        def ready(n: str, allow_unfused: bool = False) -> bool:
            node = g[n]
            if any(src not in self.vals for src in node.inputs):
                return False
            return allow_unfused or node.op not in ("Conv2D", "MatMul") or self._residual_ready(node)

        def drain(allow_unfused=False):
            progress = True
            while pending and progress:
                progress = False
                for p in list(pending):
                    if p in self._fused:
                        pending.remove(p)
                        progress = True
                    elif ready(p, allow_unfused):
                        pending.remove(p)
                        self._lower(g[p])
                        progress = True

        for name in self.order:
            if name in fed_nodes or name in self._fused:
                continue
            if not ready(name):
                pending.append(name)
                continue
            self._lower(g[name])
            drain()
        while pending:  # residual fusion impossible for what is left: lower unfused
            before = len(pending)
            drain(allow_unfused=True)
            if len(pending) == before:
                raise CompileError(f"cannot schedule nodes {pending[:5]}")
        for f in self.fetch_names:
            tn = TensorName.parse(f)
            if (tn.name, tn.index) not in self.vals:
                raise CompileError(f"fetch {f} was not produced by the plan")
            if self.vals[(tn.name, tn.index)].rows is not None:
                raise CompileError(f"fetch {f} is a token-packed tensor (fetch a per-sequence output)")
        self._decimate_tails()
        self._chain_tails()

    def _chain_tails(self):
        """ResNet stage 1's residual stream by recomputation (kernels/bottleneck_chain.hip):
        a fused tail whose residual is the previous tail's y3, read by nothing else, computes
        that y3 again from the previous tails' 64-channel sources (the 3x3 outputs and the
        stem output, kept alive until it) instead of reading the 256-channel tensor, and the
        previous tail stops storing it.  Chains start at the dual (projection) tail and hold
        up to ``chain_max_links`` links (2: tail 1 -> tail 2, the third tail reads y3 again;
        three links recompute more than the saved traffic buys: 77.6-77.8k vs 79.3-79.6k,
        profiles/r06_chain)."""
        self.chained_tails = 0
        if not _cfg().recompute_tails:
            return
        fetched = {id(_root(self.vals[(TensorName.parse(f).name, TensorName.parse(f).index)]))
                   for f in self.fetch_names}
        links_of: dict[int, list] = {}
        for st in self.steps:
            t = st.meta.get("tail")
            if t is None or t["w3"] is None:
                continue
            if t["xs"] is not None:  # a chain head: the dual tail
                links_of[id(st)] = [(t["x"], t["xs"], t["w3"], t["b3"])]
                continue
            res = t["res"]
            prods = [p for p in self.steps if p.outputs and p.outputs[0] is res and id(p) in links_of]
            if len(prods) != 1:
                continue
            prev = prods[0]
            prev_links = links_of[id(prev)]
            if len(prev_links) >= _cfg().chain_max_links or id(res) in fetched or res.alias_of is not None or res.concat_slot is not None \
                    or getattr(res, "buf_shape", None) is not None \
                    or any(v is not res and _root(v) is res for v in self.vals.values()):
                continue
            readers = [r for r in self.steps if r is not prev and any(_root(i) is res for i in r.inputs)]
            if readers != [st]:
                continue
            links = prev_links + [(t["x"], None, t["w3"], t["b3"])]
            links_of[id(st)] = links
            t["chain"]["links"] = links
            st.meta["impl"] = "bottleneck_chain"
            # the sources of every link are this step's inputs (the planner keeps them alive)
            st.inputs = [v for x, xs, _, _ in links for v in ((x,) if xs is None else (x, xs))]
            # the previous tail no longer writes y3 (it runs as a one-or-more-link chain)
            pt = prev.meta["tail"]
            pt["chain"]["links"] = prev_links
            pt["chain"]["store"] = False
            prev.meta["impl"] = "bottleneck_chain"
            prev.outputs = [o for o in prev.outputs if o is not res]
            self.chained_tails += 1

    def _decimate_tails(self):
        """A fused block tail's wide output y3 whose only other reader is the next stage's
        stride-2 1x1 projection shortcut (fused into that stage's first expand conv) is
        stored decimated: only the even-(h, w) pixels the projection reads, compact — 1/4 of
        the bytes (ResNet v1.5's stage-1 -> stage-2 boundary: 308 MB less HBM write traffic
        per 256 images); the projection then reads it at stride 1."""
        self.decimated_tails = 0
        if not _cfg().decimate_tails:
            return
        fetched = {id(_root(self.vals[(TensorName.parse(f).name, TensorName.parse(f).index)]))
                   for f in self.fetch_names}
        for st in self.steps:
            dec = st.meta.get("dec")
            if dec is None:
                continue
            y3 = st.outputs[0]
            if id(y3) in fetched or y3.alias_of is not None or y3.concat_slot is not None \
                    or getattr(y3, "buf_shape", None) is not None:
                continue
            if any(v is not y3 and _root(v) is y3 for v in self.vals.values()):
                continue  # reshaped / sliced views of y3 read the full layout
            readers = [r for r in self.steps if r is not st and any(_root(i) is y3 for i in r.inputs)]
            if len(readers) != 1:
                continue
            r = readers[0]
            cfg = (r.meta or {}).get("s2cfg")
            N, H, W, C = y3.shape
            if cfg is None or cfg["s2"] != 2 or len(r.inputs) != 2 or r.inputs[1] is not y3 or H % 2 or W % 2 \
                    or tuple(r.outputs[0].shape[1:3]) != (H // 2, W // 2):
                continue
            y3.buf_shape = (N, H // 2, W // 2, C)
            dec["on"] = True
            cfg["s2"] = 1
            self.decimated_tails += 1

    # ------------------------------------------------------------------ calibration
    def synthetic_feeds(self, seed: int = 0) -> dict:
        g = torch.Generator().manual_seed(seed)
        out = {}
        for f in self.feed_names:
            shape, dt = self.feed_specs[f]
            dt = DataType.of(dt).torch
            if dt == torch.uint8:
                out[f] = torch.randint(0, 256, tuple(shape), generator=g, dtype=torch.uint8)
            elif dt.is_floating_point:
                out[f] = torch.randn(tuple(shape), generator=g).to(dt)
            else:
                out[f] = torch.randint(0, 100, tuple(shape), generator=g).to(dt)
        return out

    @torch.no_grad()
    def calibrate(self, feeds: dict | None = None) -> dict[str, float]:
        """Runs the plan step by step on ``feeds`` (synthetic when None) and returns the
        absolute maximum of every computed value, keyed by graph node name."""
        for k, v in (feeds or self.synthetic_feeds()).items():
            self.input_buffer(k).copy_(v)
        by_id: dict[int, float] = {}

        def each(s):  # a batch-slice chain step runs once per slice: max over the slices
            s.fn()
            for o in s.outputs:
                t = _view(o)
                if t.is_floating_point() and t.numel():
                    k = id(_root(o))
                    by_id[k] = max(by_id.get(k, 0.0), float(t.float().abs().max()))

        self._run_range(0, len(self.steps), each)
        for v in self.vals.values():  # concat targets: max over their stride-written children
            kids = getattr(v, "_concat_children", None)
            if kids:
                by_id[id(v)] = max(by_id.get(id(_root(c)), 0.0) for c in kids)
        return {n: by_id[id(_root(v))] for (n, _), v in self.vals.items() if id(_root(v)) in by_id}

    def _qscale(self, name: str) -> float | None:
        a = self._amax.get(name)
        return None if a is None else F8.scale_for(a)

    def _fp8_consumers_ok(self, name: str) -> bool:
        """True when ``name``'s value may be stored as fp8: not fetched, and every consumer
        reads fp8 natively."""
        if any(TensorName.parse(f).name == name for f in self.fetch_names):
            return False
        cons = self.cons.get(name, [])
        return bool(cons) and all(self.graph[c].op in ("Conv2D", "MaxPool", "AvgPool", "ConcatV2", "Mean")
                                  for c in cons)

    # ------------------------------------------------------------------ helpers
    def _in(self, node: Node, i: int) -> Val:
        s, k = node.inputs[i]
        v = self._get((s, k))
        if v is None:
            raise CompileError(f"input {s}:{k} of {node.name} not available")
        return v

    def _get(self, src: tuple[str, int]) -> Val | None:
        v = self.vals.get(src)
        if v is not None and self._cur_cls and v.rows == "packed":
            return self._cls_gather(v)  # first-token-only region: read each sequence's first row
        return v if v is not None else self._const_val(src)

    def _single_consumer(self, name: str) -> Node | None:
        c = self.cons.get(name, [])
        fetched = any(TensorName.parse(f).name == name for f in self.fetch_names)
        if len(c) != 1 or fetched:
            return None
        return self.graph[c[0]]

    def _const_val(self, src: tuple[str, int]) -> Val | None:
        """Value of ``src`` if it is (or can be folded to) a constant, folding on demand
        (DFS topo order may reach a consumer before its constant operands)."""
        v = self.vals.get(src)
        if v is not None:
            return v if v.is_const else None
        node = self.graph.nodes.get(src[0])
        if node is None or node.name not in self.needed:
            return None
        for s in node.inputs:
            if self._const_val(s) is None:
                return None
        if node.op in ("Placeholder", "PlaceholderV2"):
            return None
        try:
            ok = self._fold(node)
        except CompileError:
            return None
        v = self.vals.get(src)
        return v if ok and v is not None and v.is_const else None

    def _residual_ready(self, node: Node) -> bool:
        """True unless ``node``'s fusible chain contains an Add whose other operand is a
        not-yet-lowered (non-constant) value."""
        cur = node
        for _ in range(8):
            nxt = self._single_consumer(cur.name)
            if nxt is None:
                return True
            if nxt.op in ("Add", "AddV2"):
                other = [nxt.inputs[i] for i, (s, _) in enumerate(nxt.inputs) if s != cur.name]
                if len(other) != 1:
                    return True
                src = other[0]
                if src in self.vals:
                    return True
                # constants get folded when reached; only wait for computed values
                return self.graph[src[0]].op in ("Const",)
            if nxt.op in ("BiasAdd",) or nxt.op.startswith("FusedBatchNorm") or nxt.op in _ACTS:
                cur = nxt
                continue
            return True
        return True

    def _fold(self, node: Node) -> bool:
        """Constant-fold ``node`` if all its data inputs are constants."""
        ins = [self.vals.get((s, k)) for s, k in node.inputs]
        if node.op in ("Placeholder", "PlaceholderV2"):
            raise CompileError(f"placeholder {node.name} must be fed")
        if node.op in ("VariableV2", "Variable", "VarHandleOp"):
            name = node.attr("shared_name") or node.name
            v = self.variables.get(name)
            if v is None:
                raise CompileError(f"variable {name} is uninitialized at compile time")
            self.vals[(node.name, 0)] = Val(tuple(v.shape), getattr(v, "dtype", None), const=_host(v))
            return True
        if any(v is None or not v.is_const for v in ins):
            return False
        ctx = OpContext(self._const_sess, torch.device("cpu"))
        outs = lookup(node.op)(ctx, node, *[v.const for v in ins])
        for k, o in enumerate(outs):
            if isinstance(o, ops_core.VarRef):
                o = o.read()
            o = _host(o)
            self.vals[(node.name, k)] = Val(tuple(o.shape), getattr(o, "dtype", None), const=o)
        return True

    def _new(self, shape, dtype=torch.bfloat16, phys_c=None) -> Val:
        return Val(tuple(int(s) for s in shape), dtype, phys_c=phys_c)

    def _emit(self, name, kind, fn, inputs, outputs, meta=None):
        self.steps.append(Step(name, kind, fn, list(inputs), list(outputs), dict(meta or {})))

    # ------------------------------------------------------------------ lowering
    def _lower(self, node: Node):
        if self._fold(node):
            return
        self._cur_cls = node.name in self._cls_nodes
        try:
            self._lower_node(node)
        finally:
            self._cur_cls = False

    _ROW_OPS = ("MatMul", "Reshape", "StridedSlice", "Identity", "StopGradient", "Snapshot", "NoOp")

    def _lower_node(self, node: Node):
        grp = self._groups.get(node.name)
        if grp is not None and not grp["done"] and self._lower_group(grp):
            return
        if self._pack is not None and node.op not in self._ROW_OPS:
            for s in node.inputs:  # packed rows reach only row-wise lowerings
                v = self.vals.get(s)
                if v is not None and v.rows is not None:
                    raise CompileError(f"{node.op} {node.name} reads token-packed rows; no packed lowering")
        op = node.op
        if op == "Conv2D":
            return self._lower_conv(node)
        if op == "MatMul":
            return self._lower_matmul(node)
        if op == "Cast" and self._try_preprocess(node):
            return
        if op in ("MaxPool", "AvgPool"):
            return self._lower_pool(node)
        if op == "Mean":
            if self._lower_mean(node):
                return
        if op == "Softmax":
            return self._lower_softmax(node)
        if op in ("Identity", "StopGradient", "Snapshot"):
            self.vals[(node.name, 0)] = self._in(node, 0)
            return
        if op == "IdentityN":  # e.g. an inlined function call's outputs (graph/functions.py)
            for i in range(len(node.inputs)):
                self.vals[(node.name, i)] = self._in(node, i)
            return
        if op == "Reshape":
            return self._lower_reshape(node)
        if op == "StridedSlice" and self._lower_strided_slice(node):
            return
        if op in ("Squeeze", "ExpandDims") and self._lower_squeeze_like(node):
            return
        if op == "ConcatV2":
            return self._lower_concat(node)
        if op == "NoOp":
            return
        if op == "LRN" and self._lower_lrn(node):
            return
        if op in _BINARY and self._lower_binary(node):
            return
        if op in _ACTS and self._lower_unary_act(node):
            return
        if op == "Cast" and self._lower_float_cast(node):
            return
        return self._lower_glue(node)

    # ---- standalone elementwise / LRN (ops no producer epilogue absorbed)
    def _ew_ok(self, v: Val) -> bool:
        # bf16 activations, fp8 activations (dequantised first) or fed fp32 tensors (cast first)
        return v is not None and not v.is_const and v.dtype in (torch.bfloat16, torch.uint8, torch.float32) and \
            (v.qscale is not None or v.dtype != torch.uint8) and not v.phys_c and int(np.prod(v.shape)) % 8 == 0

    def _lower_binary(self, node: Node) -> bool:
        a, b = self._get(node.inputs[0]), self._get(node.inputs[1])
        op = _BINARY[node.op]
        if a is not None and a.is_const and b is not None and not b.is_const:
            a, b = b, a
            op = {"sub": "rsub", "div": "rdiv"}.get(op, op)
        if not self._ew_ok(a) or b is None:
            return False
        if b.is_const:
            c = b.const.float().reshape(-1) if isinstance(b.const, torch.Tensor) else None
            if c is None:
                return False
            if c.numel() == 1:
                operand, kind = float(c.item()), "scalar"
            elif c.numel() == a.shape[-1] and c.numel() % 8 == 0 and len(b.const.shape) == 1:
                operand, kind = c.to(self.device).contiguous(), "vector"
                self.params.append(operand)
            else:
                return False
        else:
            if not self._ew_ok(b) or tuple(b.shape) != tuple(a.shape):
                return False
            operand, kind = None, "tensor"
        xa = self._as_bf16(a, node.name + "/a")
        xb = self._as_bf16(b, node.name + "/b") if kind == "tensor" else None
        out = self._new(a.shape)

        def run(xa=xa, xb=xb, out=out, operand=operand):
            K.binary(_view(xa), _view(xb) if xb is not None else operand, op, out=out.buf)

        self._emit(node.name, "elementwise", run, [xa] + ([xb] if xb is not None else []), [out])
        self.vals[(node.name, 0)] = out
        return True

    def _lower_unary_act(self, node: Node) -> bool:
        x = self._get(node.inputs[0])
        if not self._ew_ok(x):
            return False
        xa = self._as_bf16(x, node.name)
        out = self._new(x.shape)
        act = _ACTS[node.op]

        def run(xa=xa, out=out):
            K.binary(_view(xa), 0.0, "add", act=act, out=out.buf)

        self._emit(node.name, "elementwise", run, [xa], [out])
        self.vals[(node.name, 0)] = out
        return True

    def _lower_float_cast(self, node: Node) -> bool:
        x = self._get(node.inputs[0])
        dst = node.attr("DstT")
        if x is None or x.is_const or x.dtype != torch.bfloat16 or DataType.of(dst).torch not in (
                torch.float32, torch.bfloat16, torch.float16):
            return False
        self.vals[(node.name, 0)] = x  # device activations are bf16 either way
        return True

    def _lower_lrn(self, node: Node) -> bool:
        x = self._get(node.inputs[0])
        if not self._ew_ok(x) or len(x.shape) != 4 or x.shape[-1] % 8 or node.attr("depth_radius", 5) > 8:
            return False
        xa = self._as_bf16(x, node.name)
        out = self._new(x.shape)
        r, bias = int(node.attr("depth_radius", 5)), float(node.attr("bias", 1.0))
        alpha, beta = float(node.attr("alpha", 1.0)), float(node.attr("beta", 0.5))

        def run(xa=xa, out=out):
            K.lrn(_view(xa), r, bias, alpha, beta, out=out.buf)

        self._emit(node.name, "lrn", run, [xa], [out])
        self.vals[(node.name, 0)] = out
        return True

    # ---- conv chain
    def _conv_chain(self, start: Node):
        """Follows Conv2D/MatMul → BiasAdd/FusedBatchNorm* → Add(res)? → act? ."""
        scale = None
        bias = None
        residual = None
        act = K.ACT_NONE
        cur = start
        absorbed = []
        while True:
            nxt = self._single_consumer(cur.name)
            if nxt is None:
                break
            if nxt.op in ("BiasAdd", "Add", "AddV2") and residual is None and act == K.ACT_NONE:
                other = [i for i, (s, _) in enumerate(nxt.inputs) if s != cur.name]
                if len(other) != 1:
                    break
                ov = self._get(nxt.inputs[other[0]])
                if ov is not None and ov.is_const and ov.const.dim() == 1:
                    b = ov.const.float()
                    bias = b if bias is None else bias + b
                elif nxt.op != "BiasAdd" and ov is not None and not ov.is_const:
                    residual = (nxt, other[0])
                else:
                    break
            elif nxt.op.startswith("FusedBatchNorm") and residual is None and act == K.ACT_NONE:
                if nxt.attr("is_training", False):
                    break
                p = [self._get(nxt.inputs[i]) for i in range(1, 5)]
                if not all(v is not None and v.is_const for v in p):
                    break
                g, b, m, v = (t.const.float() for t in p)
                eps = nxt.attr("epsilon", 1e-3)
                s = g * torch.rsqrt(v + eps)
                shift = b - m * s
                scale = s if scale is None else scale * s
                bias = shift if bias is None else bias * s + shift
                if any(c in self.cons.get(nxt.name, []) for c in []):
                    break
            elif nxt.op in _ACTS and act == K.ACT_NONE:
                act = _ACTS[nxt.op]
            else:
                break
            absorbed.append(nxt)
            cur = nxt
        return cur, scale, bias, residual, act, absorbed

    def _lower_conv(self, node: Node):
        if self.precision == "fp8" and self._lower_sibling_group(node):
            return
        x = self._in(node, 0)
        wv = self._in(node, 1)
        if not wv.is_const:
            return self._lower_glue(node)
        if node.attr("data_format", "NHWC") != "NHWC":
            return self._lower_glue(node)
        strides = node.attr("strides")
        dil = node.attr("dilations") or [1, 1, 1, 1]
        sh, sw = strides[1], strides[2]
        dh, dw = dil[1], dil[2]
        w = wv.const.float()  # HWIO
        KH, KW, Cin, Cout = w.shape
        N, H, W, C = x.shape
        if C != Cin:
            raise CompileError(f"{node.name}: input channels {C} != filter {Cin}")
        padding = node.attr("padding", "SAME")
        if padding == "SAME":
            pt, pb = same_pads(H, KH, sh, dh)
            pl, pr = same_pads(W, KW, sw, dw)
        elif padding == "VALID":
            pt = pb = pl = pr = 0
        else:
            return self._lower_glue(node)
        if Cout % 8:
            return self._lower_glue(node)
        last, scale, bias, residual, act, absorbed = self._conv_chain(node)
        if scale is not None:
            w = w * scale  # fold BN into the output channels
        Ho = (H + pt + pb - ((KH - 1) * dh + 1)) // sh + 1
        Wo = (W + pl + pr - ((KW - 1) * dw + 1)) // sw + 1
        if self.precision == "fp8" and self._conv_fp8_ok(node, x, Cin, Cout, residual, act):
            return self._lower_conv_fp8(node, x, w, bias, act, last, absorbed, (KH, KW, Cin, Cout),
                                        (sh, sw), (pt, pb, pl, pr), (dh, dw), (N, Ho, Wo))
        if self._s2d_ok(x, node, C, sh, sw, dh, dw, pt, pl, H, W):
            # stride-2 RGB stem over the space-to-depth preprocess output (K 392 -> 256)
            w_ohwi, (pt, pb, pl, pr) = K.s2d_stem_weights(w, H, W, (pt, pb, pl, pr))
            x.pre_cfg["s2d"] = True
            x.buf_shape = (N, (H + 1) // 2, (W + 1) // 2, 16)
            x.phys_c = 16
            xin_shape_override = x.buf_shape
            KH, KW = w_ohwi.shape[1], w_ohwi.shape[2]
            sh = sw = 1
            cin_pad = 16
        else:
            xin_shape_override = None
            phys = x.phys_c or C
            cin_pad = -(-phys // 8) * 8
            w_ohwi = w.permute(3, 0, 1, 2).contiguous()
            if cin_pad != Cin:
                w_ohwi = torch.nn.functional.pad(w_ohwi, (0, cin_pad - Cin))
        w_dev = self._dev(w_ohwi, torch.bfloat16)
        b_dev = self._dev(bias, torch.float32) if bias is not None else None
        self.params += [w_dev] + ([b_dev] if b_dev is not None else [])
        out = self._new((N, Ho, Wo, Cout))
        KHe, KWe = w_ohwi.shape[1], w_ohwi.shape[2]
        if (self.precision == "fp8" and residual is None and act in (K.ACT_NONE, K.ACT_RELU) and Cout % 16 == 0
                and self._fp8_consumers_ok(last.name) and self._qscale(last.name) is not None
                and self._use_dconv(cin_pad, KHe, KWe, (sh, sw), (dh, dw), 2, residual, act)):
            # bf16 direct-conv layer (the RGB stem) feeding fp8 consumers: emit e4m3 directly
            # (a wider bf16 layer hands bf16 on; its fp8 successor quantises on load)
            out = self._new((N, Ho, Wo, Cout), torch.uint8)
            out.qscale = self._qscale(last.name)
        res_val = None
        if residual is not None:
            rn, ri = residual
            res_val = self.vals[rn.inputs[ri]]
        xin = x if xin_shape_override is not None else self._ensure_padded(x, cin_pad, node.name)
        for a in absorbed:
            self._fused.add(a.name)
        if self._use_dconv(cin_pad, KHe, KWe, (sh, sw), (dh, dw), 2, residual, act):
            bn = 64 if Cout >= 64 else 32
            w_arr = self._dev(K.dconv_bf16_weight_bytes(w_ohwi, bn))
            if b_dev is None:
                b_dev = torch.zeros(Cout, dtype=torch.float32, device=self.device)
            self.params += [w_arr, b_dev]
            pool = self._fusable_maxpool(last, act, out)
            if pool is not None:
                # ReLU stem + 3x3/s2 max pool in one kernel: the full-resolution stem
                # output never reaches HBM
                pnode, mpad, (Hp, Wp) = pool
                out = self._new((N, Hp, Wp, Cout))
                self._fused.add(pnode.name)
            else:
                mpad = None

            pp = getattr(x, "pre_params", None)
            if (mpad is None and xin_shape_override is not None and pp is not None and not pp["resize"]
                    and _cfg().fuse_preprocess_stem and len(self.steps) == 1 and self.steps[0].kind == "preprocess"
                    and self.steps[0].outputs[0] is x and _root(out) is out and _coff(out) == 0):
                # the plan's head preprocess kernel folds into this stem: the conv builds its s2d
                # patches from the raw uint8 batch (Inception-v3's Conv2d_1a: no resize)
                self.steps.pop()
                xu = pp["x"]
                osc = _eff_scale(out) if out.qscale is not None else None

                def run_u(x=xu, out=out, w_arr=w_arr, b_dev=b_dev, bn=bn, osc=osc, mean=pp["mean"], std=pp["std"],
                          pads=(pt, pb, pl, pr)):
                    K.conv2d_direct_u8s2d(x.buf, w_arr, (KHe, KWe), Cout, b_dev, pads, act, mean, std, out=out.buf,
                                          bn=bn, out_scale=osc)

                # kind "preprocess": still the plan's head, launched per H2D piece by the runner
                self._emit(node.name, "preprocess", run_u, [xu], [out],
                           {"impl": "dconv_u8s2d", "conv_out": (N, Ho, Wo, Cout)})
                self.fused_preprocess = 1
                self.vals[(last.name, 0)] = out
                self._alias_fused_outputs(absorbed, out)
                return

            def run_d(xin=xin, out=out, w_arr=w_arr, b_dev=b_dev, bn=bn, mpad=mpad):
                K.conv2d_direct(xin.buf, w_arr, (KHe, KWe), Cout, b_dev, (sh, sw), (pt, pb, pl, pr), act,
                                out=_target(out), out_channel_offset=_coff(out), bn=bn,
                                out_scale=_eff_scale(out) if out.qscale is not None else None, maxpool_pad=mpad)

            # the MACs of a pool-fused stem are those of its full-resolution (pre-pool) output
            self._emit(node.name, "conv", run_d, [xin], [out], {"conv_out": (N, Ho, Wo, Cout)} if pool else None)
            if pool is not None:
                self.vals[(pool[0].name, 0)] = out
                self.fused_pools = getattr(self, "fused_pools", 0) + 1
                return
            self.vals[(last.name, 0)] = out
            self._alias_fused_outputs(absorbed, out)
            return

        if (res_val is None and out.qscale is None and xin_shape_override is None and (xin.phys_c or Cin) == Cin
                and _cfg().conv3x3c64_kernel
                and K.conv3x3_c64_eligible(tuple(xin.shape), tuple(w_ohwi.shape), (sh, sw), (pt, pb, pl, pr), (dh, dw),
                                           None, act)):
            # 64-channel 3x3 (ResNet stage 1): persistent kernel, filter bank resident in LDS
            bz = b_dev if b_dev is not None else self._dev(torch.zeros(Cout), torch.float32)

            def run_c(xin=xin, out=out, w_dev=w_dev, bz=bz):
                K.conv3x3_c64(xin.buf, w_dev, bz, act, out=_target(out), out_channel_offset=_coff(out))

            self._emit(node.name, "conv", run_c, [xin], [out], {"impl": "conv3x3c64"})
            self.conv3x3c64 = getattr(self, "conv3x3c64", 0) + 1
            self.vals[(last.name, 0)] = out
            self._alias_fused_outputs(absorbed, out)
            return

        pointwise = (KHe, KWe, sh, sw, pt, pb, pl, pr, dh, dw) == (1, 1, 1, 1, 0, 0, 0, 0, 1, 1)
        if (self.device.type == "cuda" and pointwise and res_val is None and act in (K.ACT_NONE, K.ACT_RELU)
                and out.qscale is None and xin_shape_override is None and (xin.phys_c or Cin) == Cin
                and (Cin >= 1024 or (Cin >= _PP_MIN_K and Cout >= 256)) and Cin % 64 == 0 and Cout % 8 == 0
                and _coff(out) % 8 == 0):
            # deep-K 1x1 reduce convs (ResNet stages 3/4: K = 1024 / 2048; the stage-3 entry
            # reduce K = 512 -> 256) are plain GEMMs over the pixel matrix: the ping-pong
            # 256x256 MFMA kernel (kernels/gemm_pp.hip)
            w_nk = w_dev.reshape(Cout, Cin)
            bz = b_dev if b_dev is not None else self._dev(torch.zeros(Cout), torch.float32)
            M = int(np.prod(xin.shape[:-1]))
            splits = K.gemm_pp_splits(M, Cout, Cin)
            ws = torch.empty(splits * M * Cout, dtype=torch.float32, device=self.device) if splits > 1 else None

            def run_pp(xin=xin, out=out, w_nk=w_nk, bz=bz, act=act, splits=splits, ws=ws):
                K.gemm_pp(xin.buf.view(-1, Cin), w_nk, bz, None, act, out=_target(out), out_col=_coff(out),
                          splits=splits, ws=ws)

            self._emit(node.name, "gemm", run_pp, [xin], [out], {"impl": "gemm_pp"})
            self.vals[(last.name, 0)] = out
            self._alias_fused_outputs(absorbed, out)
            return
        if res_val is not None and pointwise and xin_shape_override is None and out.qscale is None \
                and self._fuse_shortcut(node, xin, out, w_ohwi, bias, res_val, residual[0], act, absorbed, last):
            return
        if res_val is not None and pointwise and xin_shape_override is None \
                and self._fuse_block_tail(xin, out, w_ohwi.reshape(w_ohwi.shape[0], -1), w_dev, b_dev, res_val, None, act,
                                      absorbed, last, node.name):
            return
        if (res_val is not None and pointwise and act == K.ACT_RELU and xin_shape_override is None
                and out.qscale is None and out.dtype == torch.bfloat16 and (xin.phys_c or Cin) == Cin
                and K.pw_res_ok(Cin, Cout) and res_val.qscale is None and res_val.concat_slot is None
                and tuple(res_val.shape) == tuple(out.shape) and _cfg().pw_res_kernel):
            # identity-residual expansion conv (ResNet stages 2/3): persistent kernel, resident
            # weight slice, next tile's x / residual prefetched (kernels/pw_res.hip)
            w_nk = w_dev.reshape(Cout, Cin)
            bz = b_dev if b_dev is not None else self._dev(torch.zeros(Cout), torch.float32)

            def run_pw(xin=xin, out=out, res_val=res_val, w_nk=w_nk, bz=bz):
                K.pw_res(xin.buf, w_nk, bz, res_val.buf, out=_target(out), out_channel_offset=_coff(out))

            self._emit(node.name, "conv", run_pw, [xin, res_val], [out], {"impl": "pw_res"})
            self.pw_res_layers = getattr(self, "pw_res_layers", 0) + 1
            self.vals[(last.name, 0)] = out
            self._alias_fused_outputs(absorbed, out)
            return

        def run(xin=xin, out=out, res_val=res_val, w_dev=w_dev, b_dev=b_dev):
            K.conv2d_nhwc(xin.buf, w_dev, b_dev, res_val.buf if res_val is not None else None, (sh, sw),
                          (pt, pb, pl, pr), (dh, dw), act, out=_target(out), out_channel_offset=_coff(out),
                          out_scale=_eff_scale(out) if out.qscale is not None else None)

        lite = (self.device.type == "cuda" and out.qscale is None
                and xin_shape_override is None and (xin.phys_c or Cin) == Cin and Cin % 64 == 0 and Cout % 8 == 0
                and _coff(out) % 8 == 0 and out.dtype == torch.bfloat16 and xin.dtype == torch.bfloat16
                and not pointwise and act in (K.ACT_NONE, K.ACT_RELU)
                and (res_val is None or (res_val.concat_slot is None and res_val.qscale is None
                                         and tuple(res_val.shape) == tuple(out.shape) and res_val.alias_of is None))
                and max(pt, pb) < 1024 and max(pl, pr) < 1024)
        if lite:
            # KxK convs (stage 2-4 3x3): 4-wave 128x128 implicit GEMM on two LDS-DMA stages
            # (kernels/conv_pp.hip conv_lite): 6-24 % faster than the register-staged igemm
            # per layer and 64 KiB of LDS, so it shares a CU with the sibling lane
            cl = K.ConvPP([(tuple(xin.shape), (KHe, KWe), (sh, sw), (pt, pl), (dh, dw))], Cout, tuple(out.shape[1:3]),
                          self.device, tile=LITE_TILE)  # tiles 3 (32-deep K), 256x128 (4 or 8 waves) and 3-stage
            # variants (raw-barrier, counted vmcnt) measured slower: profiles/r03_conv, r04_a, r04_c

            def run(xin=xin, out=out, res_val=res_val, cl=cl, w2=w_dev.reshape(Cout, -1), b_dev=b_dev):  # noqa: F811
                cl([xin.buf], w2, b_dev, res_val.buf if res_val is not None else None, act, out=_target(out),
                   out_channel_offset=_coff(out))

            self.conv_lite_layers = getattr(self, "conv_lite_layers", 0) + 1

        shortcut_ok = (KHe == KWe == 1 and sh == sw and (pt, pb, pl, pr) == (0, 0, 0, 0) and (dh, dw) == (1, 1)
                       and res_val is None and act == K.ACT_NONE and out.qscale is None
                       and xin_shape_override is None and (xin.phys_c or Cin) == Cin)
        meta = {"shortcut": dict(x=xin, w=w_ohwi, bias=bias, stride=sh, params=[w_dev, b_dev])} if shortcut_ok else None
        self._emit(node.name, "conv", run, [xin] + ([res_val] if res_val else []), [out], meta)
        self.vals[(last.name, 0)] = out
        self._alias_fused_outputs(absorbed, out)

    def _fuse_shortcut(self, node, xin, out, w_ohwi, bias, res_val, add_node, act, absorbed, last) -> bool:
        """Pointwise conv whose residual is a 1x1 (strided) projection conv used by nothing
        else: drop the projection's launch and run both as one K loop
        (``conv1x1_dual``) — the projection output never round-trips through HBM."""
        prod = [st for st in self.steps if any(o is res_val for o in st.outputs)]
        if len(prod) != 1 or "shortcut" not in prod[0].meta or res_val.concat_slot is not None:
            return False
        for (n, _), v in self.vals.items():  # the projection feeds only this Add
            if v is res_val:
                if any(TensorName.parse(f).name == n for f in self.fetch_names):
                    return False
                if any(c != add_node.name and c not in self._fused for c in self.cons.get(n, [])):
                    return False
        sc = prod[0].meta["shortcut"]
        x2 = sc["x"]
        s2 = sc["stride"]
        N, Ho, Wo, _ = out.shape
        if x2.shape[0] != N or (Ho - 1) * s2 >= x2.shape[1] or (Wo - 1) * s2 >= x2.shape[2]:
            return False
        Cout, K1 = w_ohwi.shape[0], w_ohwi.shape[3]
        C2 = sc["w"].shape[3]
        if K1 % 8 or C2 % 8:
            return False
        self.steps.remove(prod[0])
        for t in sc["params"]:
            if t is not None:
                self.params = [q for q in self.params if q is not t]
        w_cat = torch.cat([w_ohwi.reshape(Cout, K1), sc["w"].reshape(Cout, C2)], 1)
        b = (bias if bias is not None else torch.zeros(Cout)) + (sc["bias"] if sc["bias"] is not None else 0)
        w_dev = self._dev(w_cat, torch.bfloat16)
        b_dev = self._dev(b, torch.float32)
        self.params += [w_dev, b_dev]
        for a in absorbed:
            self._fused.add(a.name)
        if s2 == 1 and self._fuse_block_tail(xin, out, w_cat, w_dev, b_dev, None, x2, act, absorbed, last, node.name):
            self.fused_shortcuts = getattr(self, "fused_shortcuts", 0) + 1
            return True

        s2cfg = {"s2": s2}  # _decimate_tails: x2 stored already decimated -> stride 1

        def run(xin=xin, x2=x2, out=out, w_dev=w_dev, b_dev=b_dev, s2cfg=s2cfg):
            K.conv1x1_dual(xin.buf, x2.buf, w_dev, b_dev, s2cfg["s2"], act, out=_target(out),
                           out_channel_offset=_coff(out))

        if (self.device.type == "cuda" and K1 % 64 == 0
                and C2 % 64 == 0 and (xin.phys_c or K1) == K1 and (x2.phys_c or C2) == C2
                and act in (K.ACT_NONE, K.ACT_RELU) and out.dtype == torch.bfloat16 and out.qscale is None
                and _coff(out) % 8 == 0 and len(xin.shape) == 4 and N * Ho * Wo <= 65536):
            # expand + projection shortcut as one 4-wave LDS-DMA implicit GEMM over two
            # sources (kernels/conv_pp.hip conv_lite, DUAL); planned for x2 as it is and, when
            # _decimate_tails later stores x2 decimated, for the compact stride-1 layout.
            # Stages 3/4 only (ResNet-50 B=256: 111 / 100 µs vs 114 / 111 on the dual igemm);
            # stage 2's 200k-row GEMM stays on the igemm (141 vs 158 µs, profiles/r03_operating_points)
            xs0 = (tuple(xin.shape), (1, 1), (1, 1), (0, 0), (1, 1))
            lite = {s2: K.ConvPP([xs0, (tuple(x2.shape), (1, 1), (s2, s2), (0, 0), (1, 1))], Cout, (Ho, Wo),
                                 self.device, tile=LITE_TILE)}
            N2, H2, W2, _ = x2.shape
            if s2 == 2 and H2 % 2 == 0 and W2 % 2 == 0:
                lite[1] = K.ConvPP([xs0, ((N2, H2 // 2, W2 // 2, C2), (1, 1), (1, 1), (0, 0), (1, 1))], Cout, (Ho, Wo),
                                   self.device, tile=LITE_TILE)

            def run(xin=xin, x2=x2, out=out, w_dev=w_dev, b_dev=b_dev, s2cfg=s2cfg, lite=lite):  # noqa: F811
                lite[s2cfg["s2"]]([xin.buf, x2.buf], w_dev, b_dev, None, act, out=_target(out),
                                  out_channel_offset=_coff(out))

            self._emit(node.name, "conv", run, [xin, x2], [out], {"s2cfg": s2cfg, "impl": "conv_lite_dual"})
            self.conv_lite_layers = getattr(self, "conv_lite_layers", 0) + 1
            self.vals[(last.name, 0)] = out
            self._alias_fused_outputs(absorbed, out)
            self.fused_shortcuts = getattr(self, "fused_shortcuts", 0) + 1
            return True

        self._emit(node.name, "conv", run, [xin, x2], [out], {"s2cfg": s2cfg})
        self.vals[(last.name, 0)] = out
        self._alias_fused_outputs(absorbed, out)
        self.fused_shortcuts = getattr(self, "fused_shortcuts", 0) + 1
        return True

    def _fuse_block_tail(self, xin, out, w3, w_dev, b_dev, res_val, xs_val, act, absorbed, last, name) -> bool:
        """ResNet bottleneck block boundary: this 1x1 CX -> 4 CX expand conv (+ residual,
        ReLU) and the next block's 1x1 reduce conv (+ ReLU) that reads its output run as one
        persistent kernel (``bottleneck_tail``): the wide output is still stored (it is the
        next residual) but the reduce GEMM reads it from LDS instead of HBM.  Stage 1
        (CX = 64, reduce to 64 or 128) and stage 2 (CX = 128, reduce to 128).  ``w3`` is the
        host [4 CX, K] expand weight; with ``xs_val`` (stage 1's first block) K = 64 + 64
        covers the stride-1 projection shortcut of ``xs_val`` too."""
        if not _cfg().fuse_block_tails or self.precision == "fp8":
            return False
        cx = xin.shape[-1]
        co = 4 * cx
        # (stage 2, its weights streamed through LDS, measured no faster than the two convs
        # it would replace: profiles/r01_tail — stage 1 only)
        widths = {64: (64, 128)}.get(cx, ()) if xs_val is None else ((64,) if cx == 64 else ())

        def plain(v):
            return v.shape[-1] == cx and (v.phys_c or cx) == cx and v.concat_slot is None and v.qscale is None \
                and v.dtype == torch.bfloat16 and tuple(v.shape[:-1]) == tuple(out.shape[:-1])

        if not widths or act != K.ACT_RELU or out.qscale is not None \
                or tuple(w3.shape) != (co, cx if xs_val is None else 2 * cx) or not plain(xin):
            return False
        if res_val is not None and (res_val.shape != out.shape or res_val.qscale is not None
                                    or res_val.concat_slot is not None):
            return False
        if xs_val is not None and not plain(xs_val):
            return False
        cand = [self.graph[c] for c in self.cons.get(last.name, []) if c not in self._fused]

        def reduce_conv(c):  # 1x1 / s1 reduce conv reading this output (not the stage's projection)
            if c.op != "Conv2D" or c.inputs[0] != (last.name, 0) or c.attr("data_format", "NHWC") != "NHWC" \
                    or list(c.attr("strides")) != [1, 1, 1, 1] \
                    or list(c.attr("dilations") or [1, 1, 1, 1]) != [1, 1, 1, 1]:
                return None
            wv = self._get(c.inputs[1])
            if wv is None or not wv.is_const:
                return None
            w = wv.const.float()  # HWIO
            return w if tuple(w.shape[:3]) == (1, 1, co) and w.shape[3] in widths else None

        cand = [(c, w) for c in cand for w in [reduce_conv(c)] if w is not None]
        if len(cand) != 1:
            return False
        c, w2 = cand[0]
        last2, scale2, bias2, residual2, act2, absorbed2 = self._conv_chain(c)
        if residual2 is not None or act2 != K.ACT_RELU:
            return False
        cn = w2.shape[3]
        if scale2 is not None:
            w2 = w2 * scale2
        w3_dev = w_dev  # row-major [4 CX][K] (1x1 OHWI [4 CX, 1, 1, CX], or the dual [W3 | Wsc])
        b3_dev = b_dev if b_dev is not None else self._dev(torch.zeros(co), torch.float32)
        w1_dev = self._dev(w2.reshape(co, cn).t().contiguous(), torch.bfloat16)
        b1_dev = self._dev(bias2 if bias2 is not None else torch.zeros(cn), torch.float32)
        self.params += [b3_dev, w1_dev, b1_dev]
        N, H, W, _ = out.shape
        out2 = self._new((N, H, W, cn))
        for a in absorbed + absorbed2:
            self._fused.add(a.name)
        self._fused.add(c.name)

        second = res_val if xs_val is None else xs_val
        dec = {"on": False}  # set by _decimate_tails when y3's only other reader is a stride-2 projection
        # set by _chain_tails: recompute the residual chain from its narrow sources
        # (``links``) instead of reading y3 of the previous tail; ``store``: y3 is written
        chain = {"links": None, "store": True}

        def run(xin=xin, second=second, out=out, out2=out2, dual=xs_val is not None, dec=dec, chain=chain):
            if chain["links"] is not None:
                K.bottleneck_chain([(x.buf, s.buf if s is not None else None, w, b) for x, s, w, b in chain["links"]],
                                   w1_dev, b1_dev, y1=out2.buf, y3=out.buf if chain["store"] else None,
                                   y3_decimated=dec["on"], store_y3=chain["store"])
                return
            K.bottleneck_tail(xin.buf, None if dual else second.buf, w3_dev, b3_dev, w1_dev, b1_dev, y3=out.buf,
                              y1=out2.buf, xs=second.buf if dual else None, y3_decimated=dec["on"])

        self._emit(name, "conv", run, [xin, second], [out, out2],
                   {"impl": "bottleneck_tail", "dec": dec if xs_val is None and cx == 64 else None,
                    "tail": {"x": xin, "xs": xs_val, "res": res_val, "w3": w3_dev, "b3": b3_dev, "cn": cn,
                             "chain": chain}})
        self.vals[(last.name, 0)] = out
        self._alias_fused_outputs(absorbed, out)
        self.vals[(last2.name, 0)] = out2
        self._alias_fused_outputs(absorbed2, out2)
        self.fused_tails = getattr(self, "fused_tails", 0) + 1
        return True

    def _fusable_maxpool(self, last: Node, act, out: Val, fp8: bool = False):
        """The single consumer of a ReLU conv chain when it is a 3x3 / stride-2 NHWC
        MaxPool whose padding is at most one row/column per side (ResNet's pool1; with
        ``fp8``, Inception's MaxPool_3a after an fp8 -> fp8 direct conv):
        ``(pool node, (top, bottom, left, right), (Hp, Wp))`` or None."""
        if act != K.ACT_RELU:
            return None
        if (out.qscale is not None or out.dtype != torch.bfloat16) if not fp8 else \
                (out.qscale is None or out.dtype != torch.uint8):
            return None
        if any(TensorName.parse(f).name == last.name for f in self.fetch_names):
            return None
        cons = [c for c in self.cons.get(last.name, []) if c not in self._fused]
        if len(cons) != 1 or self.graph[cons[0]].op != "MaxPool":
            return None
        pn = self.graph[cons[0]]
        if pn.attr("data_format", "NHWC") != "NHWC" or list(pn.attr("ksize")) != [1, 3, 3, 1] \
                or list(pn.attr("strides")) != [1, 2, 2, 1]:
            return None
        _, Ho, Wo, _ = out.shape
        if pn.attr("padding", "VALID") == "SAME":
            pt, pb = same_pads(Ho, 3, 2)
            pl, pr = same_pads(Wo, 3, 2)
        else:
            pt = pb = pl = pr = 0
        if max(pt, pb, pl, pr) > 1:
            return None
        return pn, (pt, pb, pl, pr), ((Ho + pt + pb - 3) // 2 + 1, (Wo + pl + pr - 3) // 2 + 1)

    def _use_dconv(self, cin_phys, KH, KW, stride, dil, es, residual, act) -> bool:
        """Direct LDS conv for narrow layers (input row <= 32 B: RGB stems, Inception's
        32-channel fp8 layers); measured faster there by bench/dconv_tune.py, slower for
        wider inputs, which stay on the implicit GEMM."""
        return (self.device.type == "cuda" and residual is None and act in (K.ACT_NONE, K.ACT_RELU)
                and cin_phys * es <= 32 and K.dconv_eligible(cin_phys, KH, KW, stride, dil, es))

    def _conv_fp8_ok(self, node: Node, x: Val, Cin, Cout, residual, act) -> bool:
        if residual is not None or act not in (K.ACT_NONE, K.ACT_RELU) or Cin % 16 or Cout % 16 or x.phys_c:
            return False
        if x.qscale is not None:
            return True
        return x.dtype == torch.bfloat16 and self._qscale(node.inputs[0][0]) is not None

    def _lower_conv_fp8(self, node, x, w, bias, act, last, absorbed, kdims, stride, pads, dil, out_nhw):
        KH, KW, Cin, Cout = kdims
        w_ohwi = w.permute(3, 0, 1, 2).contiguous()
        wq, ws = F8.quantize_weight(w_ohwi)
        x_scale = x.qscale if x.qscale is not None else self._qscale(node.inputs[0][0])
        dev = self.device
        wq_dev = self._dev(wq)
        ws_dev = self._dev(ws)
        cs_dev = self._dev(ws * x_scale, torch.float32)
        b_dev = self._dev(bias, torch.float32) if bias is not None else \
            torch.zeros(Cout, dtype=torch.float32, device=dev)
        self.params += [wq_dev, cs_dev, b_dev]
        o_scale = self._qscale(last.name) if self._fp8_consumers_ok(last.name) else None
        out = self._new((*out_nhw, Cout), torch.uint8 if o_scale is not None else torch.bfloat16)
        out.qscale = o_scale
        for a in absorbed:
            self._fused.add(a.name)
        self.fp8_layers += 1
        if x.qscale is not None and self._use_dconv(Cin, KH, KW, stride, dil, 1, None, act):
            bn = 64 if Cout >= 64 else 32
            w_arr = self._dev(K.dconv_weights(wq, Cout, 1, bn))
            self.params.append(w_arr)
            pool = self._fusable_maxpool(last, act, out, fp8=True) if stride == (1, 1) else None
            if pool is not None:
                # pooled tiles cover 14 x 8 pooled pixels with 8 waves x 64 conv pixels; fuse
                # only when that tiling wastes little conv work (Inception's 73x73 pool rounds to
                # 84 x 80 and costs 1.42x the convs: 445 µs fused vs 236 + 132 µs apart)
                _, Hp_, Wp_ = pool[0], *pool[2]
                waves = K._dconv_waves(None, None, bn)
                pr_ = 14 if waves == 8 else 7
                work = -(-Hp_ // pr_) * -(-Wp_ // 8) * 64 * waves
                if work > 1.15 * out_nhw[1] * out_nhw[2]:
                    pool = None
            mpad = None
            if pool is not None:
                # fp8 ReLU conv + 3x3/s2 max pool in one kernel (Inception's Conv2d_2b ->
                # MaxPool_3a): the pre-pool output never reaches HBM; the pooled values keep
                # the conv output's scale (a max never leaves the input range)
                pnode, mpad, (Hp, Wp) = pool
                q = out.qscale
                out = self._new((out_nhw[0], Hp, Wp, Cout), torch.uint8)
                out.qscale = q
                self._fused.add(pnode.name)

            def run_d(x=x, out=out, w_arr=w_arr, cs=cs_dev, b=b_dev, bn=bn, mpad=mpad):
                K.conv2d_direct(_view(x), w_arr, (KH, KW), Cout, b, stride, pads, act, out=_target(out),
                                out_channel_offset=_coff(out), bn=bn, chan_scale=cs, out_scale=_eff_scale(out),
                                maxpool_pad=mpad)

            self._emit(node.name, "conv_fp8", run_d, [x], [out], {"conv_out": (*out_nhw, Cout)} if pool else None)
            if pool is not None:
                self.vals[(pool[0].name, 0)] = out
                self.fused_pools = getattr(self, "fused_pools", 0) + 1
                return
            self.vals[(last.name, 0)] = out
            self._alias_fused_outputs(absorbed, out)
            return

        # fp8 input: the 4-wave LDS-DMA tile (kernels/fp8.hip conv_lite_fp8, cfg 8); a bf16
        # input (the layer after the stem) is quantised on load by the register-staged kernel
        cfg = LITE_FP8_CFG if x.qscale is not None else -1
        # (an eight-wave 256-pixel tile on three LDS stages measured 5-40 % slower per layer
        # and -2 % in the bench: profiles/r04_d)

        def run(x=x, out=out, wq=wq_dev, ws=ws_dev, cs=cs_dev, b=b_dev, x_scale=x_scale, cfg=cfg):
            F8.conv2d_nhwc_fp8(_view(x), x_scale, wq, (KH, KW), ws, b, stride, pads, dil, act,
                               out_scale=_eff_scale(out), out=_target(out), out_channel_offset=_coff(out), chan_scale=cs,
                               cfg=cfg)

        self._emit(node.name, "conv_fp8", run, [x], [out], {"impl": "conv_lite_fp8"} if cfg in (8, 9, 10, 11, 12) else None)
        if cfg in (8, 9, 10, 11, 12):
            self.conv_lite_layers = getattr(self, "conv_lite_layers", 0) + 1
        self.vals[(last.name, 0)] = out
        self._alias_fused_outputs(absorbed, out)

    def _s2d_ok(self, x: Val, node: Node, C, sh, sw, dh, dw, pt, pl, H, W) -> bool:
        cfg = getattr(x, "pre_cfg", None)
        if cfg is None or C != 3 or (sh, sw) != (2, 2) or (dh, dw) != (1, 1) or pt % 2 or pl % 2:
            return False
        chain = x.pre_chain
        users = set()
        for (n, _), v in self.vals.items():
            if v is x:
                if any(TensorName.parse(f).name == n for f in self.fetch_names):
                    return False
                users.update(c for c in self.cons.get(n, []) if c not in chain)
        return users == {node.name}

    def _alias_fused_outputs(self, absorbed, out):
        for a in absorbed:
            self.vals[(a.name, 0)] = out

    def _ensure_padded(self, x: Val, cin_pad: int, name: str) -> Val:
        if x.qscale is not None:
            x = self._as_bf16(x, name)
        phys = x.phys_c or x.shape[-1]
        if phys == cin_pad and x.dtype == torch.bfloat16:
            return x
        y = self._new((*x.shape[:-1], cin_pad), phys_c=cin_pad)
        c = x.shape[-1]

        def run(x=x, y=y, c=c):
            y.buf.zero_()
            y.buf[..., :c].copy_(x.buf[..., :c])

        self._emit(name + "/pad_cin", "glue", run, [x], [y])
        return y

    # ---- matmul chain
    def _lower_matmul(self, node: Node):
        a = self._in(node, 0)
        b = self._in(node, 1)
        if not b.is_const or node.attr("transpose_a", False) or len(a.shape) != 2:
            return self._lower_glue(node)
        wt = b.const.float()
        w_nk = wt if node.attr("transpose_b", False) else wt.t()
        N, Kd = w_nk.shape
        if Kd % 8:
            return self._lower_glue(node)
        last, scale, bias, residual, act, absorbed = self._conv_chain(node)
        if act == K.ACT_NONE and residual is None:
            gm = self._match_gelu(last)  # BERT's tanh GELU subgraph -> the GEMM's GELU epilogue
            if gm is not None:
                last, extra = gm
                act = K.ACT_GELU
                absorbed = absorbed + extra
        if scale is not None:
            w_nk = w_nk * scale[:, None]
        n_pad = -(-N // 8) * 8  # e.g. 1001 classes: zero rows, output rows strided by n_pad
        if n_pad != N and residual is not None:
            return self._lower_glue(node)
        if n_pad != N:
            w_nk = torch.nn.functional.pad(w_nk, (0, 0, 0, n_pad - N))
            bias = torch.nn.functional.pad(bias if bias is not None else torch.zeros(N), (0, n_pad - N))
        w_dev = self._dev(w_nk, torch.bfloat16)
        b_dev = self._dev(bias, torch.float32) if bias is not None else None
        self.params += [w_dev] + ([b_dev] if b_dev is not None else [])
        out = self._new((a.shape[0], N), phys_c=n_pad if n_pad != N else None)
        out.rows = a.rows
        out.lshape = (*a.lshape[:-1], N) if a.lshape else None
        if n_pad != N:
            out.buf_shape = (a.shape[0], n_pad)
        res_val = self._get(residual[0].inputs[residual[1]]) if residual is not None else None
        if res_val is not None and (res_val.rows != a.rows or tuple(res_val.shape) != tuple(out.shape)):
            if a.rows is not None or res_val.rows is not None:
                raise CompileError(f"{node.name}: residual rows do not match the packed GEMM rows")
        xin = self._as_bf16(a, node.name)
        for n in absorbed:
            self._fused.add(n.name)

        M = a.shape[0]
        if self.device.type == "cuda" and Kd % 64 == 0:
            # ping-pong MFMA GEMM; small-M heads (e.g. the 256 x 2048 -> 1000 classifier)
            # run split-K through this step's own fp32 workspace
            splits = K.gemm_pp_splits(M, n_pad, Kd)
            ws = torch.empty(splits * M * n_pad, dtype=torch.float32, device=self.device) if splits > 1 else None

            def run_pp(xin=xin, out=out, res_val=res_val, w_dev=w_dev, b_dev=b_dev, splits=splits, ws=ws):
                K.gemm_pp(xin.buf, w_dev, b_dev, res_val.buf if res_val is not None else None, act, out=out.buf,
                          splits=splits, ws=ws)

            self._emit(node.name, "gemm", run_pp, [xin] + ([res_val] if res_val else []), [out],
                       {"impl": "gemm_pp", "splits": splits})
            self.vals[(last.name, 0)] = out
            self._alias_fused_outputs(absorbed, out)
            return

        def run(xin=xin, out=out, res_val=res_val, w_dev=w_dev, b_dev=b_dev):
            K.gemm(xin.buf, w_dev, b_dev, res_val.buf if res_val is not None else None, act, out=out.buf)

        self._emit(node.name, "gemm", run, [xin] + ([res_val] if res_val else []), [out])
        self.vals[(last.name, 0)] = out
        self._alias_fused_outputs(absorbed, out)

    def _as_bf16(self, v: Val, name: str) -> Val:
        if v.dtype == torch.bfloat16:
            return v
        y = self._new(v.shape)
        if v.qscale is not None:
            def deq(v=v, y=y):
                F8.dequantize(_view(v), _eff_scale(v), out=y.buf)

            self._emit(name + "/dequant", "dequant", deq, [v], [y])
            return y

        def run(v=v, y=y):
            y.buf.copy_(v.buf)

        self._emit(name + "/to_bf16", "glue", run, [v], [y])
        return y

    # ---- preprocess: uint8 → Cast → ResizeBilinear → Sub → Div|Mul
    def _try_preprocess(self, cast: Node) -> bool:
        x = self._in(cast, 0)
        if x.is_const or x.dtype != torch.uint8 or len(x.shape) != 4 or x.shape[3] != 3:
            return False
        chain = [cast]
        cur = cast
        size = None
        mean = torch.zeros(3)
        std = torch.ones(3)
        align = half = False
        nxt = self._single_consumer(cur.name)
        if nxt is not None and nxt.op == "ResizeBilinear":
            sv = self._get(nxt.inputs[1])
            if sv is None or not sv.is_const:
                return False
            size = tuple(int(v) for v in sv.const.reshape(-1).tolist())
            align = nxt.attr("align_corners", False)
            half = nxt.attr("half_pixel_centers", False)
            chain.append(nxt)
            cur = nxt
            nxt = self._single_consumer(cur.name)
        if nxt is not None and nxt.op == "Sub":
            mv = self._get(nxt.inputs[1])
            if mv is not None and mv.is_const and nxt.inputs[0][0] == cur.name:
                mean = mean + mv.const.float().reshape(-1).expand(3)
                chain.append(nxt)
                cur = nxt
                nxt = self._single_consumer(cur.name)
        if nxt is not None and nxt.op in ("Div", "RealDiv", "Mul"):
            sv2 = self._get(nxt.inputs[1])
            if sv2 is not None and sv2.is_const and nxt.inputs[0][0] == cur.name:
                f = sv2.const.float().reshape(-1).expand(3)
                std = std * f if nxt.op != "Mul" else std / f
                chain.append(nxt)
                cur = nxt
        if size is None:
            size = (x.shape[1], x.shape[2])
        out = self._new((x.shape[0], size[0], size[1], 3), phys_c=8)
        out_buf_shape = (x.shape[0], size[0], size[1], 8)
        out.buf_shape = out_buf_shape
        out.pre_cfg = {"s2d": False}
        out.pre_chain = {n.name for n in chain}
        # what a stem conv needs to absorb this kernel (dconv_u8s2d): no resize, the affine only
        out.pre_params = {"x": x, "mean": tuple(mean.tolist()), "std": tuple(std.tolist()),
                          "resize": size != (x.shape[1], x.shape[2])}
        for n in chain[1:]:
            self._fused.add(n.name)
        mean_t, std_t = tuple(mean.tolist()), tuple(std.tolist())
        cfg = out.pre_cfg

        def run(x=x, out=out):
            K.preprocess_images(x.buf, size, mean_t, std_t, align, half, out=out.buf, s2d=cfg["s2d"])

        self._emit(cast.name + "/preprocess", "preprocess", run, [x], [out])
        for n in chain:
            self.vals[(n.name, 0)] = out
        return True

    # ---- pooling / reductions / softmax
    def _lower_pool(self, node: Node):
        x = self._in(node, 0)
        if node.attr("data_format", "NHWC") != "NHWC" or (x.phys_c or x.shape[-1]) % 8:
            return self._lower_glue(node)
        k = node.attr("ksize")
        s = node.attr("strides")
        kh, kw, sh, sw = k[1], k[2], s[1], s[2]
        N, H, W, C = x.shape
        if node.attr("padding", "VALID") == "SAME":
            pt, pb = same_pads(H, kh, sh)
            pl, pr = same_pads(W, kw, sw)
        else:
            pt = pb = pl = pr = 0
        Ho = (H + pt + pb - kh) // sh + 1
        Wo = (W + pl + pr - kw) // sw + 1
        mode = "max" if node.op == "MaxPool" else "avg"
        if mode == "avg" and self.precision == "fp8" and self._lower_sibling_group(node):
            return
        if mode == "avg" and (sh, sw) == (1, 1) and self._commute_avgpool(node, x, (kh, kw), (pt, pb, pl, pr)):
            return
        if x.qscale is not None and C % 16 == 0:
            # pooled values stay within the input range: keep the input scale, requantise
            # only when written into a concat buffer of another scale
            out = self._new((N, Ho, Wo, C), torch.uint8)
            out.qscale = x.qscale

            def run8(x=x, out=out):
                F8.pool2d_nhwc_fp8(_view(x), (kh, kw), (sh, sw), (pt, pb, pl, pr), mode,
                                   rq=x.qscale / _eff_scale(out), out=_target(out), out_channel_offset=_coff(out))

            self._emit(node.name, "pool_fp8", run8, [x], [out])
            self.vals[(node.name, 0)] = out
            return
        out = self._new((N, Ho, Wo, C))
        xin = self._as_bf16(x, node.name)

        def run(xin=xin, out=out):
            K.pool2d_nhwc(xin.buf, (kh, kw), (sh, sw), (pt, pb, pl, pr), mode, out=_target(out),
                          out_channel_offset=_coff(out))

        self._emit(node.name, "pool", run, [xin], [out])
        self.vals[(node.name, 0)] = out

    # ---- horizontal fusion of sibling pointwise convs (Inception module heads)
    def _pw_member(self, c: Node, x: Val, src, max_cout: int | None = None):
        """``c`` as a member of a sibling group: a 1x1 / stride-1 Conv2D of ``src`` with a
        constant filter and a chain without residual ending in ReLU or nothing."""
        if c.op != "Conv2D" or c.name in self._fused or c.inputs[0] != src or c.attr("data_format", "NHWC") != "NHWC":
            return None
        if list(c.attr("strides") or [1, 1, 1, 1]) != [1, 1, 1, 1] or list(c.attr("dilations") or [1, 1, 1, 1]) != [1, 1, 1, 1]:
            return None
        wv = self._get(c.inputs[1])
        if wv is None or not wv.is_const or tuple(wv.const.shape[:3]) != (1, 1, x.shape[-1]):
            return None
        Cout = int(wv.const.shape[3])
        if Cout % 16 or (max_cout is not None and Cout > max_cout):
            return None
        last, scale, bias, residual, act, absorbed = self._conv_chain(c)
        if residual is not None or act not in (K.ACT_NONE, K.ACT_RELU):
            return None
        w = wv.const.float()
        if scale is not None:
            w = w * scale
        return {"conv": c, "w": w.reshape(-1, Cout).t().contiguous(), "bias": bias, "act": act, "last": last,
                "absorbed": absorbed, "Cout": Cout}

    def _lower_sibling_group(self, entry: Node) -> bool:
        """The 1x1 convs that read one fp8 value — an Inception module's branch heads, and
        its AvgPool(3x3/1) -> 1x1 branch commuted to 1x1 -> pool — run as ONE implicit GEMM
        over their concatenated filters (``conv2d_nhwc_fp8_multi``): the input is read once
        instead of 3-4 times, and the combined channel count tiles better than 32-64-channel
        GEMMs.  Its epilogue sends each branch's channels to that branch's destination (a
        concat slot, an fp8 buffer with its own scale, or the bf16 pre-pool value)."""
        if not _cfg().sibling_conv_fusion:
            return False
        src = entry.inputs[0] if entry.inputs else None
        x = self.vals.get(src) if src is not None else None
        if x is None or x.qscale is None or x.phys_c or x.rows is not None or len(x.shape) != 4 or x.shape[-1] % 16:
            return False
        N, H, W, C = x.shape
        members = []
        for cname in dict.fromkeys(self.cons.get(src[0], [])):
            c = self.graph[cname]
            if c.name in self._fused or not c.inputs or c.inputs[0] != src or any(i == src for i in c.inputs[1:]):
                continue
            if c.op == "Conv2D":
                m = self._pw_member(c, x, src)
                if m is not None:
                    m["kind"], m["entry"] = "conv", c.name
                    members.append(m)
            elif c.op == "AvgPool" and c.attr("data_format", "NHWC") == "NHWC" and list(c.attr("ksize")) == [1, 3, 3, 1] \
                    and list(c.attr("strides")) == [1, 1, 1, 1]:
                pc = self._single_consumer(c.name)
                if pc is None:
                    continue
                m = self._pw_member(pc, x, (c.name, 0), max_cout=C // 2)
                if m is None:
                    continue
                if c.attr("padding", "VALID") == "SAME":
                    pads = (*same_pads(H, 3, 1), *same_pads(W, 3, 1))
                else:
                    continue  # a VALID 3x3/1 pool changes the spatial size: not a sibling of the 1x1s
                m["kind"], m["entry"], m["pool"], m["pads"] = "pool", c.name, c, pads
                members.append(m)
        if len(members) < 2 or entry.name not in {m["entry"] for m in members} or len(members) > 6:
            return False
        xs = x.qscale
        ws_rows, bias_parts, lo_parts, segs, pool_steps = [], [], [], [], []
        c0 = 0
        for m in members:
            Cout = m["Cout"]
            ws_rows.append(m["w"])
            if m["kind"] == "conv":
                last = m["last"]
                o_scale = self._qscale(last.name) if self._fp8_consumers_ok(last.name) else None
                out = self._new((N, H, W, Cout), torch.uint8 if o_scale is not None else torch.bfloat16)
                out.qscale = o_scale
                bias_parts.append(m["bias"] if m["bias"] is not None else torch.zeros(Cout))
                lo_parts.append(torch.full((Cout,), 0.0 if m["act"] == K.ACT_RELU else float("-inf")))
                m["out"] = out
                segs.append((out, c0, c0 + Cout))
            else:
                y = self._new((N, H, W, Cout))  # pre-bias conv output, pooled next
                bias_parts.append(torch.zeros(Cout))
                lo_parts.append(torch.full((Cout,), float("-inf")))
                last = m["last"]
                o_scale = self._qscale(last.name) if self._fp8_consumers_ok(last.name) else None
                out = self._new((N, H, W, Cout), torch.uint8 if o_scale is not None else torch.bfloat16)
                out.qscale = o_scale
                m["y"], m["out"] = y, out
                segs.append((y, c0, c0 + Cout))
            c0 += Cout
        wq, wsc = F8.quantize_weight(torch.cat(ws_rows, 0))
        wq_dev, ws_dev = self._dev(wq), self._dev(wsc)
        cs_dev = self._dev(wsc * xs, torch.float32)
        b_dev = self._dev(torch.cat(bias_parts), torch.float32)
        lo_dev = self._dev(torch.cat(lo_parts), torch.float32)
        self.params += [wq_dev, cs_dev, b_dev, lo_dev]
        self.fp8_layers += len(members)

        def run(x=x, segs=segs, wq=wq_dev, ws=ws_dev, cs=cs_dev, b=b_dev, lo=lo_dev, xs=xs):
            F8.conv2d_nhwc_fp8_multi(_view(x), xs, wq, (1, 1), ws, b, lo,
                                     [(_target(v), a, e, _coff(v), _eff_scale(v) if v.qscale is not None else None)
                                      for v, a, e in segs], chan_scale=cs)

        self._emit("+".join(m["conv"].name for m in members), "conv_fp8", run, [x], [v for v, _, _ in segs],
                   {"impl": "conv_lite_fp8_multi", "multi_out": True})
        for m in members:
            self._fused.add(m["conv"].name)
            for a in m["absorbed"]:
                self._fused.add(a.name)
            if m["kind"] == "pool":
                self._fused.add(m["pool"].name)
                y, out, act = m["y"], m["out"], m["act"]
                bp = self._dev(m["bias"] if m["bias"] is not None else torch.zeros(m["Cout"]), torch.float32)
                self.params.append(bp)

                def run_pool(y=y, out=out, b=bp, act=act, pads=m["pads"]):
                    F8.avgpool_bias_act(y.buf, (3, 3), (1, 1), pads, b, act,
                                        out_scale=_eff_scale(out) if out.qscale is not None else None,
                                        out=_target(out), out_channel_offset=_coff(out))

                self._emit(m["pool"].name, "pool_fp8" if out.qscale is not None else "pool", run_pool, [y], [out],
                           {"impl": "avgpool_bias_act"})
                self.commuted_pools = getattr(self, "commuted_pools", 0) + 1
            self.vals[(m["last"].name, 0)] = m["out"]
            self._alias_fused_outputs(m["absorbed"], m["out"])
        self.sibling_groups = getattr(self, "sibling_groups", 0) + 1
        return True

    def _commute_avgpool(self, node: Node, x: Val, ksize, pads) -> bool:
        """AvgPool(stride 1) -> 1x1 Conv2D (+ BN/bias, ReLU) lowered as 1x1 conv (no bias or
        act, bf16 out) -> avgpool with the bias + act + fp8 quantisation in its epilogue.
        Both operators are linear and the conv is pointwise, so they commute exactly (the
        pool's count-excluding-padding divisor depends on the position only); the pool then
        runs over Cout instead of Cin channels (Inception's pool branches: 32-192 vs
        192-2048), and in fp8 the pooled value is no longer rounded to e4m3 before the
        conv.  Taken when Cout <= Cin / 2 (the extra bf16 round trip of the conv output is
        cheaper than pooling the wide input)."""
        c = self._single_consumer(node.name)
        if c is None or c.op != "Conv2D" or c.inputs[0][0] != node.name or c.attr("data_format", "NHWC") != "NHWC":
            return False
        if list(c.attr("strides") or [1, 1, 1, 1]) != [1, 1, 1, 1] or list(c.attr("dilations") or [1, 1, 1, 1]) != [1, 1, 1, 1]:
            return False
        wv = self._get(c.inputs[1])
        if wv is None or not wv.is_const or tuple(wv.const.shape[:2]) != (1, 1) or x.phys_c or x.concat_slot is not None:
            return False
        N, H, W, C = x.shape
        w = wv.const.float()
        Cin, Cout = w.shape[2], w.shape[3]
        if Cin != C or C % 16 or Cout % 16 or 2 * Cout > C or x.rows is not None:
            return False
        last, scale, bias, residual, act, absorbed = self._conv_chain(c)
        if residual is not None or act not in (K.ACT_NONE, K.ACT_RELU):
            return False
        fp8_in = x.qscale is not None
        if not fp8_in and x.dtype != torch.bfloat16:
            return False
        if scale is not None:
            w = w * scale
        w_ohwi = w.permute(3, 0, 1, 2).contiguous()
        b_dev = self._dev(bias if bias is not None else torch.zeros(Cout), torch.float32)
        y = self._new((N, H, W, Cout))  # the conv's output before bias / act (bf16, real units)
        o_scale = self._qscale(last.name) if (self.precision == "fp8" and self._fp8_consumers_ok(last.name)) else None
        out = self._new((N, H, W, Cout), torch.uint8 if o_scale is not None else torch.bfloat16)
        out.qscale = o_scale
        zero = self._dev(torch.zeros(Cout), torch.float32)
        if fp8_in:
            wq, ws = F8.quantize_weight(w_ohwi)
            wq_dev, ws_dev, cs_dev = self._dev(wq), self._dev(ws), self._dev(ws * x.qscale, torch.float32)
            self.params += [wq_dev, cs_dev, zero, b_dev]
            self.fp8_layers += 1
            cfg = LITE_FP8_CFG if self.device.type == "cuda" else -1

            def run_conv(x=x, y=y, wq=wq_dev, ws=ws_dev, cs=cs_dev, zero=zero, cfg=cfg, xs=x.qscale):
                F8.conv2d_nhwc_fp8(_view(x), xs, wq, (1, 1), ws, zero, act=K.ACT_NONE, out=y.buf, chan_scale=cs,
                                   cfg=cfg)

            self._emit(c.name, "conv_fp8", run_conv, [x], [y], {"impl": "pointwise_before_avgpool"})
        else:
            w_dev = self._dev(w_ohwi, torch.bfloat16)
            self.params += [w_dev, zero, b_dev]

            def run_conv(x=x, y=y, w_dev=w_dev, zero=zero):  # noqa: F811
                K.conv2d_nhwc(x.buf, w_dev, zero, None, (1, 1), (0, 0, 0, 0), (1, 1), K.ACT_NONE, out=y.buf)

            self._emit(c.name, "conv", run_conv, [x], [y], {"impl": "pointwise_before_avgpool"})

        def run_pool(y=y, out=out, b=b_dev, act=act, ksize=tuple(ksize), pads=tuple(pads)):
            F8.avgpool_bias_act(y.buf, ksize, (1, 1), pads, b, act,
                                out_scale=_eff_scale(out) if out.qscale is not None else None, out=_target(out),
                                out_channel_offset=_coff(out))

        self._emit(node.name, "pool_fp8" if o_scale is not None else "pool", run_pool, [y], [out],
                   {"impl": "avgpool_bias_act"})
        self._fused.add(c.name)
        for a in absorbed:
            self._fused.add(a.name)
        self.vals[(last.name, 0)] = out
        self._alias_fused_outputs(absorbed, out)
        self.commuted_pools = getattr(self, "commuted_pools", 0) + 1
        return True

    def _lower_mean(self, node: Node) -> bool:
        x = self._in(node, 0)
        av = self._get(node.inputs[1])
        if av is None or not av.is_const or len(x.shape) != 4:
            return False
        axes = sorted(int(a) % 4 for a in av.const.reshape(-1).tolist())
        if axes != [1, 2] or x.shape[-1] % 8:
            return False
        keep = node.attr("keep_dims", False)
        N, H, W, C = x.shape
        out = self._new((N, 1, 1, C) if keep else (N, C))
        if x.qscale is not None and C % 16 == 0:
            def run8(x=x, out=out):
                F8.global_avgpool_fp8(_view(x), _eff_scale(x), out=out.buf.view(N, C))

            self._emit(node.name, "gap_fp8", run8, [x], [out])
            self.vals[(node.name, 0)] = out
            return True
        xin = self._as_bf16(x, node.name)

        def run(xin=xin, out=out):
            K.global_avgpool(xin.buf, out=out.buf.view(N, C))

        self._emit(node.name, "gap", run, [xin], [out])
        self.vals[(node.name, 0)] = out
        return True

    def _lower_softmax(self, node: Node):
        x = self._in(node, 0)
        if len(x.shape) != 2:
            return self._lower_glue(node)
        R, C = x.shape
        xin = self._as_bf16(x, node.name)
        topk = None
        for c in self.cons.get(node.name, []):
            cn = self.graph[c]
            if cn.op == "TopKV2":
                kv = self._get(cn.inputs[1])
                if kv is not None and kv.is_const:
                    topk = (cn, int(kv.const.item()))
        probs = self._new((R, C))
        k = topk[1] if topk else 1
        vals = self._new((R, k), torch.float32)
        idxs = self._new((R, k), torch.int32)

        def run(xin=xin, probs=probs, vals=vals, idxs=idxs):
            K.softmax_topk(_view(xin), k, want_probs=True, vals=vals.buf, idxs=idxs.buf, probs=probs.buf)

        self._emit(node.name, "softmax_topk", run, [xin], [probs, vals, idxs])
        self.vals[(node.name, 0)] = probs
        if topk is not None:
            self._fused.add(topk[0].name)
            self.vals[(topk[0].name, 0)] = vals
            self.vals[(topk[0].name, 1)] = idxs

    def _lower_reshape(self, node: Node):
        x = self._in(node, 0)
        sv = self._get(node.inputs[1])
        if sv is None or not sv.is_const or x.phys_c:
            return self._lower_glue(node)
        shape = [int(v) for v in sv.const.reshape(-1).tolist()]
        if x.rows is not None:
            return self._reshape_rows(node, x, shape)
        n = int(np.prod(x.shape))
        if -1 in shape:
            i = shape.index(-1)
            rest = int(np.prod([s for j, s in enumerate(shape) if j != i]))
            shape[i] = n // max(rest, 1)
        out = Val(tuple(shape), x.dtype, alias_of=x)
        self.vals[(node.name, 0)] = out

    def _lower_concat(self, node: Node):
        ins = [self._in(node, i) for i in range(len(node.inputs) - 1)]
        av = self._get(node.inputs[-1])
        if av is None or not av.is_const:
            return self._lower_glue(node)
        axis = int(av.const.item()) % len(ins[0].shape)
        shape = list(ins[0].shape)
        shape[axis] = sum(v.shape[axis] for v in ins)
        fp8 = all(v.qscale is not None for v in ins) and self._qscale(node.name) is not None
        out = self._new(tuple(shape), torch.uint8 if fp8 else torch.bfloat16)
        if fp8:
            out.qscale = self._qscale(node.name)
        stride_write = (axis == len(shape) - 1 and len(shape) == 4
                        and all(self._concat_writable(v, node.inputs[i][0], node.name) for i, v in enumerate(ins)))
        if stride_write:
            off = 0
            for v in ins:
                v.concat_slot = (out, off)
                off += v.shape[-1]
            self.vals[(node.name, 0)] = out
            out._concat_children = ins
            return
        if fp8 or any(v.qscale is not None for v in ins):  # mixed scales: concatenate in bf16
            out = self._new(tuple(shape))
            ins = [self._as_bf16(v, f"{node.name}/in{i}") for i, v in enumerate(ins)]

        def run(ins=ins, out=out, axis=axis):
            torch.cat([v.buf for v in ins], dim=axis, out=out.buf)

        self._emit(node.name, "concat", run, ins, [out])
        self.vals[(node.name, 0)] = out

    def _concat_writable(self, v: Val, src_node: str, concat_node: str) -> bool:
        # produced by exactly one conv/pool step (which can write at a channel offset),
        # consumed by nothing but this concat, and not fetched
        prods = [s for s in self.steps if any(o is v for o in s.outputs)]
        if len(prods) != 1 or prods[0].kind not in ("conv", "pool", "conv_fp8", "pool_fp8") or v.concat_slot is not None \
                or (len(prods[0].outputs) != 1 and not prods[0].meta.get("multi_out")):
            return False
        if v.alias_of is not None or v.phys_c:
            return False
        # every graph node that maps to this value must feed only the concat
        for (n, _), val in self.vals.items():
            if val is v and any(c != concat_node and c not in self._fused for c in self.cons.get(n, [])):
                return False
            if val is v and any(TensorName.parse(f).name == n for f in self.fetch_names):
                return False
        if v.qscale is not None:
            return v.shape[-1] % 16 == 0 and src_node in self.cons
        return v.shape[-1] % 8 == 0 and v.dtype == torch.bfloat16 and src_node in self.cons

    def _lower_glue(self, node: Node):
        if any(self.vals.get(s) is not None and self.vals[s].rows is not None for s in node.inputs):
            raise CompileError(f"{node.op} {node.name} reads token-packed rows; no packed lowering")
        if self.strict:
            raise CompileError(f"op {node.op} ({node.name}) has no CDNA4 lowering (strict mode)")
        self.glue_ops.append(node.op)
        LOG.info("glue op %s (%s) runs as a captured PyTorch op", node.op, node.name)
        ins = [self.vals.get((s, k)) for s, k in node.inputs]
        if any(v is None for v in ins):
            raise CompileError(f"inputs of {node.name} not available")
        fn = lookup(node.op)
        # infer output shapes with a meta/CPU dry run on zeros
        ctx = OpContext(self._const_sess, torch.device("cpu"))
        probe = [v.const if v.is_const else torch.zeros(v.shape, dtype=torch.float32 if v.dtype == torch.bfloat16
                                                          else v.dtype) for v in ins]
        outs = fn(ctx, node, *probe)
        outv = [self._new(o.shape, torch.bfloat16 if o.dtype == torch.float32 else o.dtype) for o in outs]
        dev_consts = [None if not v.is_const else (v.const.to(self.device) if isinstance(v.const, torch.Tensor)
                                                    else v.const) for v in ins]
        dctx = OpContext(self._const_sess, self.device)

        def run(node=node, ins=ins, outv=outv, dev_consts=dev_consts):
            args = []
            for v, dc in zip(ins, dev_consts):
                if dc is not None:
                    args.append(dc)
                else:
                    b = _view(v)
                    args.append(b.float() if b.dtype == torch.bfloat16 else b)
            res = fn(dctx, node, *args)
            for o, r in zip(outv, res):
                o.buf.copy_(r.reshape(o.buf.shape))

        self._emit(node.name, "glue", run, [v for v in ins if not v.is_const], outv)
        for k, o in enumerate(outv):
            self.vals[(node.name, k)] = o

    # ================================================================== memory
    def _plan_memory_and_bind(self):
        """Feeds and fetched values get persistent buffers (arena blocks); every other
        produced value lives at a planned offset of one activation slab — lifetimes
        [producing step, last reading step] never overlap in memory (native liveness
        planner, ``batching/arena.py``).  With a subtask arena the slab is shared by all
        of the subtask's plans (they replay serially on one stream)."""
        from ..batching.arena import plan_offsets

        for f in self.feed_names:
            tn = TensorName.parse(f)
            v = self.vals[(tn.name, tn.index)]
            v.buf = self._persistent(v.shape, v.dtype)
            self._input_bufs[f] = v.buf
        fetch_vals = [self.vals[(TensorName.parse(f).name, TensorName.parse(f).index)] for f in self.fetch_names]
        for i, s in enumerate(self.steps):
            for v in s.inputs:
                _root(v).last_use = max(_root(v).last_use, i)
        keep = {id(_root(v)) for v in fetch_vals}
        chain = self._find_chain(keep)
        internal = chain["internal"] if chain else {}
        owners: dict[int, Val] = {}   # buffer-owning values in order of first production
        born: dict[int, int] = {}
        for i, s in enumerate(self.steps):
            for o in s.outputs:
                r = _root(o)
                if r.buf is not None:
                    continue
                tgt = r.concat_slot[0] if r.concat_slot else r  # branches write into their concat
                if tgt.buf is None and id(tgt) not in owners:
                    owners[id(tgt)] = tgt
                    born[id(tgt)] = i
        for t in owners.values():
            t.last_use = max([t.last_use] + [c.last_use for c in getattr(t, "_concat_children", [])])
        transient = []
        for k, t in owners.items():
            if k in internal:
                continue  # slice-sized buffer in the chain's own slab (below)
            if k in keep:
                t.buf = self._persistent(_buf_shape(t), t.dtype)
            else:
                transient.append(t)
        sizes = [_nbytes(_buf_shape(t), t.dtype) for t in transient]
        first = [born[id(t)] for t in transient]
        last = [max(born[id(t)], t.last_use) for t in transient]
        if chain:
            # a tensor the chain writes is written by its first slice pass and one it reads is
            # read by its last: both live across the whole chain
            i0, i1 = chain["range"]
            for j, t in enumerate(transient):
                if id(t) in chain["touched"]:
                    if i0 <= first[j] < i1:
                        first[j] = i0
                    if last[j] >= i0:
                        last[j] = max(last[j], i1 - 1)
            # the slice-sized internals form one region of the same slab, live across the chain
            chain_layout = self._plan_chain(chain, born)
            sizes.append(max(chain_layout[1], 1))
            first.append(i0)
            last.append(i1 - 1)
        offs, total = plan_offsets(sizes, first, last)
        self.activation_bytes = total
        slab = self.arena.shared_slab(total) if self.arena is not None else \
            torch.empty(max(total, 1), dtype=torch.uint8, device=self.device)
        for t, off, nb, lu in zip(transient, offs, sizes, last):
            t.buf = slab[off:off + nb].view(t.dtype).view(tuple(_buf_shape(t)))
            self._poison_after.setdefault(lu, []).append(t.buf)
        if chain:
            self._bind_chain(chain, chain_layout, slab, offs[-1])
        for v in self.vals.values():
            if v.alias_of is not None:
                r = _root(v)
                if r.buf is not None:
                    shape = v.shape if id(r) not in internal else (chain["batch"], *v.shape[1:])
                    v.buf = r.buf.view(shape) if r.buf.is_contiguous() else r.buf.reshape(shape)
        if chain:
            self._chain = (chain["range"][0], chain["range"][1], chain["parts"], chain["batch"],
                           [v for v in chain["vals"] if id(_root(v)) not in internal], chain["n"],
                           [v for v in chain["vals"] if id(_root(v)) in internal and v.buf is not None])
        self._outputs = []
        for fv in fetch_vals:
            if fv.is_const:
                self._outputs.append(fv.const)
            else:
                self._outputs.append(fv)

    # ================================================================== batch-slice chain
    _CHAIN_KINDS = ("conv", "gemm", "pool", "elementwise", "conv_fp8", "pool_fp8")
    # persistent kernels that load a resident weight bank per launch
    _PERSISTENT_IMPLS = ("conv3x3c64", "bottleneck_tail", "bottleneck_chain", "pw_res")

    def _find_chain(self, keep: set) -> dict | None:
        """The leading run of memory-bound layers that executes once per slice of
        ``EngineConfig.chain_batch`` images instead of once over the batch (None when off
        or nothing qualifies).

        Every step of the run is per-image (convs, pools, element-wise) and every tensor it
        touches is NHWC with at least ``chain_min_hw`` pixels per image — ResNet-50's stem
        and 56x56 stage 1, where each tensor is 100-400 MB per 256-image batch and every
        layer streams it from HBM.  Per slice those tensors are 13-51 MB: the values made
        and consumed inside the run ("internal") get slice-sized buffers reused by every
        slice, so a layer reads what the previous one just wrote from the Infinity Cache
        (256 MiB) and a dead intermediate is overwritten there before it is written back.
        Values entering or leaving the run keep their full buffers and are sliced."""
        cfg = _cfg()
        bs = int(getattr(cfg, "chain_batch", 0) or 0)
        auto = bs < 0
        if auto:
            bs = 32
        if bs == 0 or self._pack is not None or not self.steps or not self.feed_names:
            return None
        tn = TensorName.parse(self.feed_names[0])
        N = self.vals[(tn.name, tn.index)].shape[0] if self.vals[(tn.name, tn.index)].shape else 0
        if not N or -(-N // bs) < 2:
            return None
        min_hw = int(getattr(cfg, "chain_min_hw", 3136))

        edge = bool(getattr(cfg, "chain_edge", False))

        def val_ok(v):
            if v is None or v.is_const:
                return True
            r = _root(v)
            if v.rows is not None or v.concat_slot is not None or r.concat_slot is not None or r.is_const:
                return False
            if len(v.shape) != 4 or v.shape[0] != N:
                return False
            return _buf_shape(r)[0] == N

        def step_ok(st):
            vs = [v for v in list(st.inputs) + list(st.outputs) if v is not None and not v.is_const]
            if st.kind not in self._CHAIN_KINDS or not vs or not all(val_ok(v) for v in vs):
                return False
            if auto and st.meta.get("impl") in self._PERSISTENT_IMPLS:
                return False  # its per-launch weight prologue outweighs the cache residency (r04_d)
            big = [v.shape[1] * v.shape[2] >= min_hw for v in vs]
            # chain_edge: a layer reading the large resolution into a smaller one (the next
            # stage's stride-2 conv / projection) joins too, so its large input stays internal
            return any(big) if edge else all(big)

        start = 1 if self.steps[0].kind == "preprocess" else 0  # the head runs per H2D piece
        best, i = None, start
        while i < len(self.steps):
            if not step_ok(self.steps[i]):
                i += 1
                continue
            j = i
            while j < len(self.steps) and step_ok(self.steps[j]):
                j += 1
            if j - i >= 2 and (best is None or j - i > best[1] - best[0]):
                best = (i, j)
            i = j
        if best is None:
            return None
        i0, i1 = best
        vals, touched = [], set()
        for st in self.steps[i0:i1]:
            for v in list(st.inputs) + list(st.outputs):
                while v is not None and not v.is_const:
                    if all(v is not u for u in vals):
                        vals.append(v)
                    touched.add(id(_root(v)))
                    v = v.alias_of
        produced = {id(_root(o)) for st in self.steps[i0:i1] for o in st.outputs}
        used_outside = {id(_root(v)) for k, st in enumerate(self.steps) if not i0 <= k < i1
                        for v in list(st.inputs) + list(st.outputs) if v is not None and not v.is_const}
        feeds = {id(_root(self.vals[(TensorName.parse(f).name, TensorName.parse(f).index)])) for f in self.feed_names}
        internal = {}
        for v in vals:
            r = _root(v)
            k = id(r)
            if k in produced and k not in used_outside and k not in keep and k not in feeds and r.buf is None:
                internal[k] = r
        # a batch that is not a multiple of the slice runs a shorter last slice (the dynamic
        # batch buckets of 8-image steps): its external rows and slice buffers are narrowed
        return {"range": (i0, i1), "batch": bs, "parts": -(-N // bs), "n": N, "vals": vals, "touched": touched,
                "internal": internal}

    def _plan_chain(self, chain: dict, born: dict) -> tuple:
        """Layout of the chain's slice-sized internal values, planned by the same liveness
        planner over the chain's own step range (one slice's lifetime): (offsets, total)."""
        from ..batching.arena import plan_offsets

        i0, i1 = chain["range"]
        bs = chain["batch"]
        ts = list(chain["internal"].values())
        shapes = [(bs, *_buf_shape(t)[1:]) for t in ts]
        sizes = [_nbytes(s, t.dtype) for s, t in zip(shapes, ts)]
        first = [born[id(t)] - i0 for t in ts]
        last = [max(born[id(t)], min(t.last_use, i1 - 1)) - i0 for t in ts]
        offs, total = plan_offsets(sizes, first, last)
        return offs, total

    def _bind_chain(self, chain: dict, layout: tuple, slab: torch.Tensor, base: int):
        """Binds the chain's internal values into their region ``[base, base + total)`` of
        the activation slab (the subtask arena's shared slab when there is one)."""
        i0, i1 = chain["range"]
        bs, parts = chain["batch"], chain["parts"]
        offs, total = layout
        ts = list(chain["internal"].values())
        for t, off in zip(ts, offs):
            s = (bs, *_buf_shape(t)[1:])
            nb = _nbytes(s, t.dtype)
            t.buf = slab[base + off:base + off + nb].view(t.dtype).view(s)
        self.chain_bytes = total
        self.chain_layers = i1 - i0
        LOG.info("batch-slice chain: steps %d-%d (%s .. %s) x %d slices of %d, %d internal values in %.1f MB",
                 i0, i1 - 1, self.steps[i0].name, self.steps[i1 - 1].name, parts, bs, len(ts), total / 1e6)

    def _run_range(self, lo: int, hi: int, each=None):
        """Launches steps[lo:hi] (``each(step)`` instead of ``step.fn()`` if given), the
        batch-slice chain once per slice: the chain's external values are rebound to the
        slice's rows while its steps launch (eager, or into a capture) and restored after.
        A plan is driven by one thread at a time (one lane = one stream)."""
        each = each or (lambda st: st.fn())
        ch = self._chain
        if ch is not None and (ch[0] < lo < ch[1] or ch[0] < hi < ch[1]):
            raise CompileError(f"steps [{lo}, {hi}) cut the batch-slice chain [{ch[0]}, {ch[1]})")
        i = lo
        while i < hi:
            if ch is not None and i == ch[0] and ch[1] <= hi:
                for p in range(ch[2]):
                    self._run_chain_slice(p, each)
                i = ch[1]
                continue
            each(self.steps[i])
            i += 1

    def _run_chain_slice(self, p: int, each=None):
        """The chain's steps for slice ``p`` (images [p*bs, (p+1)*bs)), its external values
        rebound to the slice's rows while they launch."""
        each = each or (lambda st: st.fn())
        i0, i1, parts, bs, ext, n, ints = self._chain
        lo, hi = p * bs, min(n, (p + 1) * bs)
        full = [(v, v.buf, True) for v in ext if v.buf is not None]
        if hi - lo < bs:  # the short last slice: the slice-sized internals' leading rows
            full += [(v, v.buf, False) for v in ints]
        try:
            for v, b, external in full:
                v.buf = b[lo:hi] if external else b[:hi - lo]
            for st in self.steps[i0:i1]:
                each(st)
        finally:
            for v, b, _ in full:
                v.buf = b

    def _persistent(self, shape, dtype) -> torch.Tensor:
        """A buffer outside the shared slab (plan inputs, fetched outputs)."""
        if self.arena is not None:
            return self.arena.alloc(tuple(shape), dtype)
        return torch.empty(tuple(shape), dtype=dtype, device=self.device)

    def _dev(self, t: torch.Tensor, dtype=None) -> torch.Tensor:
        """A baked-in weight on the device; identical weights of a subtask's bucket plans
        are stored once in its arena."""
        t = t.to(dtype) if dtype is not None else t
        if self.arena is not None:
            return self.arena.intern(t.contiguous())
        return t.to(self.device).contiguous()

    # ================================================================== execution
    def _run_steps(self):
        if not (self._debug_sync or self._poison_after and tracing.debug_poison()):
            self._run_range(0, len(self.steps))
            return
        poison = tracing.debug_poison()
        index = {id(s): i for i, s in enumerate(self.steps)}
        ch = self._chain

        def each(s):
            i = index[id(s)]
            s.fn()
            if self._debug_sync and self.device.type == "cuda":
                try:
                    torch.cuda.synchronize(self.device)
                except RuntimeError as e:
                    raise RuntimeError(f"step {i} ({s.kind} {s.name}) failed: {e}") from e
            if poison and not (ch is not None and ch[0] <= i < ch[1]):  # chain buffers: live per slice
                for b in self._poison_after.get(i, ()):
                    b.view(-1).view(torch.uint8).fill_(0xFF)  # NaN in bf16/fp32, 0xFF in e4m3 = NaN

        self._run_range(0, len(self.steps), each)

    def profile(self, feeds: dict | None = None):
        """One eager run with a HIP event pair around every launch: a ``RunMetadata``
        whose ``NodeExecStats`` carry the per-step device time (``timeline_label`` = kind)
        — the compiled counterpart of ``Session.run(run_metadata=True)``."""
        from ..proto.messages import DeviceStepStats, NodeExecStats, RunMetadata, StepStats

        for k, v in (feeds or {}).items():
            self.input_buffer(k).copy_(v)
        stats = []
        index = {id(s): i for i, s in enumerate(self.steps)}
        if self.device.type == "cuda":
            evs = [[] for _ in self.steps]  # a chain step launches once per batch slice

            def each(s):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                s.fn()
                e1.record()
                evs[index[id(s)]].append((e0, e1))

            self._run_range(0, len(self.steps), each)
            torch.cuda.synchronize(self.device)
            times = [sum(e0.elapsed_time(e1) * 1e3 for e0, e1 in ev) for ev in evs]
        else:
            import time

            times = [0.0] * len(self.steps)

            def each(s):
                t0 = time.perf_counter()
                s.fn()
                times[index[id(s)]] += (time.perf_counter() - t0) * 1e6

            self._run_range(0, len(self.steps), each)
        t = 0
        for s, us in zip(self.steps, times):
            stats.append(NodeExecStats(node_name=s.name, all_start_micros=int(t), op_end_rel_micros=int(us),
                                       all_end_rel_micros=int(us), timeline_label=s.kind))
            t += us
        return RunMetadata(step_stats=StepStats(dev_stats=[DeviceStepStats(device=str(self.device),
                                                                           node_stats=stats)]))

    def _capture(self):
        with tracing.capture_lock():  # warm-up + device sync + capture: no sibling capture in between
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                for _ in range(2):
                    self._run_steps()
            torch.cuda.current_stream(self.device).wait_stream(s)
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph()
            with tracing.graph_capture(g):
                self._run_steps()
            self._graph_obj = g
            self._head = self._head_feed_step()
            if self._head is not None:
                # the two graphs of a plan never replay concurrently (one lane = one stream):
                # the tail graph shares the full graph's private memory pool
                gt = torch.cuda.CUDAGraph()
                with tracing.graph_capture(gt, pool=g.pool()):
                    self._run_range(1, len(self.steps))
                self._graph_tail = gt

    def _head_feed_step(self):
        """``(feed, step)`` when the first step is the fused preprocess kernel and its input is
        a feed buffer no other step and no fetch reads; else None."""
        if not self.steps or self.steps[0].kind != "preprocess" or len(self.steps[0].inputs) != 1:
            return None
        st = self.steps[0]
        x = st.inputs[0]
        if x.buf is None:
            return None
        feeds = [k for k, b in self._input_bufs.items() if b.data_ptr() == x.buf.data_ptr()]
        if len(feeds) != 1:
            return None
        # compare alias roots (a Reshape of the feed is an alias Val sharing its buffer) and
        # buffer addresses: any other reader of the raw feed needs the input_buffer copy
        rx, ptr = _root(x), x.buf.data_ptr()

        def reads_feed(v):
            return v is not None and (_root(v) is rx or (v.buf is not None and v.buf.data_ptr() == ptr))

        if any(reads_feed(i) for t in self.steps[1:] for i in t.inputs) or any(reads_feed(o) for o in self._outputs):
            return None
        return feeds[0], st

    def input_buffer(self, feed: str) -> torch.Tensor:
        return self._input_bufs[str(TensorName.parse(feed))]

    def replay_from(self, feed: str, src: torch.Tensor):
        """``input_buffer(feed).copy_(src); replay()`` without the copy when it can: if the
        plan starts with the preprocess kernel on ``feed``, that kernel is launched (outside
        the graph) straight on ``src`` — e.g. the runner's H2D staging slot — and the graph
        of the remaining steps is replayed.  Saves one D2D pass over the raw uint8 batch
        (50 MB for ResNet-50 at B=256) per micro-batch."""
        h = self._head
        buf = self.input_buffer(feed)
        if (h is None or self._graph_tail is None or h[0] != str(TensorName.parse(feed))
                or src.shape != buf.shape or src.dtype != buf.dtype or src.device != buf.device
                or not src.is_contiguous()):
            buf.copy_(src, non_blocking=True)
            self.replay()
            return
        h[1].fn(x=types.SimpleNamespace(buf=src))
        self._graph_tail.replay()

    def replay_from_chunks(self, feed: str, src: torch.Tensor, chunks, wait) -> bool:
        """``replay_from`` for a batch that reaches the device in pieces: the head
        preprocess kernel runs per piece ``chunks[i] = (lo, hi)`` right after ``wait(i)``
        (the current stream waits for that piece's H2D), so the GPU starts on the first
        records while the rest are still being gathered / copied; then the graph of the
        remaining steps.  False (nothing launched) when the plan has no such head."""
        if not self.head_pieces_ok(feed, src):
            return False
        for i, (lo, hi) in enumerate(chunks):
            wait(i)
            self.launch_head_piece(src, lo, hi)
        self.replay_tail()
        return True

    def head_pieces_ok(self, feed: str, src: torch.Tensor) -> bool:
        """The plan starts with a head kernel on ``feed`` that can run per piece of ``src``
        (``launch_head_piece``), the rest of the plan being one captured graph
        (``replay_tail``): the pipelined runner launches each piece's head right after that
        piece's H2D, interleaved with the host gather of the next piece."""
        h = self._head
        buf = self.input_buffer(feed)
        return not (h is None or self._graph_tail is None or h[0] != str(TensorName.parse(feed))
                    or src.shape != buf.shape or src.dtype != buf.dtype or src.device != buf.device
                    or not src.is_contiguous() or len(h[1].outputs) != 1)

    def launch_head_piece(self, src: torch.Tensor, lo: int, hi: int) -> None:
        st = self._head[1]
        out = _root(st.outputs[0]).buf
        st.fn(x=types.SimpleNamespace(buf=src[lo:hi]), out=types.SimpleNamespace(buf=out[lo:hi]))

    def replay_tail(self) -> None:
        self._graph_tail.replay()

    def replay(self):
        """Runs the plan on the current input buffers (no host synchronisation)."""
        if self._graph_obj is not None:
            self._graph_obj.replay()
        else:
            self._run_steps()

    def __call__(self, feeds: dict | None = None, copy_outputs: bool = True, cast_outputs: bool = True):
        for k, v in (feeds or {}).items():
            buf = self.input_buffer(k)
            if isinstance(v, StringTensor):
                raise CompileError("STRING feeds are not supported in compiled plans")
            buf.copy_(v, non_blocking=True)
        self.replay()
        outs = []
        for o in self._outputs:
            if isinstance(o, Val):
                b = _view(o)
                if o.qscale is not None:
                    b = F8.from_fp8_bytes(b) * _eff_scale(o)
                elif cast_outputs and b.dtype == torch.bfloat16:
                    b = b.float()
                elif copy_outputs:
                    b = b.clone()
                outs.append(b)
            else:
                outs.append(o)
        return outs

    def output_tensors(self) -> list:
        """The static device tensors holding the fetched values (valid after replay)."""
        return [_view(o) if isinstance(o, Val) else o for o in self._outputs]

    def param_bytes(self) -> int:
        return sum(p.numel() * p.element_size() for p in self.params)

    def summary(self) -> dict:
        kinds: dict[str, int] = {}
        for s in self.steps:
            kinds[s.kind] = kinds.get(s.kind, 0) + 1
        return {"steps": len(self.steps), "kinds": kinds, "glue_ops": sorted(set(self.glue_ops)),
                "hip_graph": self._graph_obj is not None, "precision": self.precision,
                "fp8_layers": self.fp8_layers, "fused_shortcuts": getattr(self, "fused_shortcuts", 0),
                "fused_tails": getattr(self, "fused_tails", 0), "decimated_tails": getattr(self, "decimated_tails", 0),
                "fused_pools": getattr(self, "fused_pools", 0), "conv3x3c64": getattr(self, "conv3x3c64", 0),
                "pw_res": getattr(self, "pw_res_layers", 0), "chained_tails": getattr(self, "chained_tails", 0),
                "conv_lite": getattr(self, "conv_lite_layers", 0),
                "commuted_pools": getattr(self, "commuted_pools", 0),
                "sibling_groups": getattr(self, "sibling_groups", 0),
                "fused_preprocess": getattr(self, "fused_preprocess", 0),
                "activation_bytes": self.activation_bytes,
                "param_bytes": self.param_bytes(),
                **({"token_capacity": self.token_cap, "first_token_only_nodes": len(self._cls_nodes)}
                   if self._pack is not None else {})}


_PP_MIN_K = 512


def _buf_shape(r: Val) -> tuple:
    """Physical buffer shape of a value (channel-padded / space-to-depth stem inputs,
    decimated block-tail outputs)."""
    bs = getattr(r, "buf_shape", None)
    if bs:
        return tuple(bs)
    if r.phys_c:
        return (*r.shape[:-1], r.phys_c)
    return tuple(r.shape)


def _nbytes(shape, dtype) -> int:
    return int(np.prod(shape, dtype=np.int64)) * torch.empty((), dtype=dtype).element_size()


def _root(v: Val) -> Val:
    while v.alias_of is not None:
        v = v.alias_of
    return v


def _view(v: Val) -> torch.Tensor:
    r = _root(v)
    if r.concat_slot is not None and r.buf is None:
        tgt, off = r.concat_slot
        return tgt.buf[..., off:off + r.shape[-1]]
    b = r.buf
    if r.phys_c and b.shape[-1] != r.shape[-1] and v is r:
        if tuple(b.shape[:-1]) == tuple(r.shape[:-1]):
            return b[..., :r.shape[-1]]  # channel-padded buffer: the logical columns
        return b  # space-to-depth packed stem input
    if v is not r:
        return b.reshape(v.shape)
    return b


def _target(v: Val) -> torch.Tensor:
    r = _root(v)
    if r.concat_slot is not None:
        return r.concat_slot[0].buf
    return r.buf


def _eff_scale(v: Val) -> float | None:
    """Storage scale of an fp8 value: a concat branch is stored with its buffer's scale."""
    r = _root(v)
    if r.concat_slot is not None and r.concat_slot[0].qscale is not None:
        return r.concat_slot[0].qscale
    return r.qscale


def _coff(v: Val) -> int:
    r = _root(v)
    return r.concat_slot[1] if r.concat_slot is not None else 0


def _host(t):
    if isinstance(t, torch.Tensor):
        return t.detach().to("cpu")
    return t


def compile_signature(session, feeds: dict[str, tuple[tuple, Any]], fetches: list[str], use_graph=True,
                      strict=False, precision: str = "bf16", calibration: dict | None = None) -> CompiledFunction:
    """Compiles ``session``'s graph for the given feed shapes on the session's GPU."""
    return CompiledFunction(session.graph, feeds, fetches, session.device, session.variables, use_graph, strict,
                            precision=precision, calibration=calibration)
