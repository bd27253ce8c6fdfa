"""TF1 control flow (``graph/control_flow.py``): ``tf.cond`` / ``tf.while_loop`` graphs as
TF1 emits them (``Switch``/``Merge``/``Enter``/``Exit``/``NextIteration``/``LoopCond``) run
in the interpreter with dead-token propagation, and the compiler folds conds on
compile-time-constant predicates so an ``is_training``-gated CNN compiles to the plan of
its cond-free twin.  No fixture in the reference covers control flow (parity unpinned):
the expected values are computed by hand."""
import numpy as np
import pytest
import torch

from flink_tensorflow_amd.graph.builder import GraphBuilder
from flink_tensorflow_amd.graph.control_flow import fold_static_control_flow
from flink_tensorflow_amd.graph.session import Session


def _cond_graph():
    gb = GraphBuilder()
    p = gb.placeholder("p", "BOOL", [])
    x = gb.placeholder("x", "FLOAT", [3])
    two = gb.constant("two", np.float32(2.0))
    y = gb.cond(p, lambda a, b: gb.mul(a, b, name="twice"),
                lambda a, b: gb.sub(a, gb.constant("ten", np.float32(10.0)), name="minus10"), inputs=[x, two])
    gb.identity(y, name="y")
    return gb.build()


def test_cond_takes_one_branch_and_kills_the_other():
    g = _cond_graph()
    s = Session(g)
    x = torch.tensor([1.0, 2.0, 3.0])
    assert torch.equal(s.run("y:0", {"p:0": torch.tensor(True), "x:0": x}), x * 2)
    assert torch.equal(s.run("y:0", {"p:0": torch.tensor(False), "x:0": x}), x - 10)
    # value_index of the Merge: which branch delivered
    assert int(s.run("cond/Merge:1", {"p:0": torch.tensor(True), "x:0": x})) == 1
    # a tensor of the untaken branch is dead: fetching it is an error, as in TF
    with pytest.raises(RuntimeError, match="dead"):
        s.run("cond/twice:0", {"p:0": torch.tensor(False), "x:0": x})


def _while_graph():
    """i = 0, acc = 1; while i < n: acc = acc * 2 + c; i += 1  (n, c loop invariants)."""
    gb = GraphBuilder()
    n = gb.placeholder("n", "INT32", [])
    c = gb.placeholder("c", "FLOAT", [])
    i0 = gb.constant("i0", np.int32(0))
    a0 = gb.constant("a0", np.float32(1.0))

    def cond(i, acc, n_, c_):
        return gb.op("Less", [i, n_], name="less")

    def body(i, acc, n_, c_):
        one = gb.constant("one", np.int32(1))
        two = gb.constant("two", np.float32(2.0))
        return [gb.add(i, one, name="inc"), gb.add(gb.mul(acc, two), c_, name="step")]

    i_out, acc_out = gb.while_loop(cond, body, [i0, a0], invariants=[n, c])
    gb.identity(acc_out, name="acc")
    gb.identity(i_out, name="iters")
    return gb.build()


@pytest.mark.parametrize("n", [0, 1, 5, 12])
def test_counted_while_loop_matches_python(n):
    s = Session(_while_graph())
    acc, it = s.run(["acc:0", "iters:0"], {"n:0": torch.tensor(n, dtype=torch.int32), "c:0": torch.tensor(0.5)})
    want = 1.0
    for _ in range(n):
        want = want * 2 + 0.5
    assert int(it) == n and float(acc) == want


def test_nested_loops_and_a_loop_inside_an_untaken_branch():
    """An outer loop whose body runs an inner loop (frames nest per outer iteration); then
    the whole loop inside a cond branch that is not taken (every Exit dies, the Merge takes
    the other branch)."""
    gb = GraphBuilder()
    n = gb.placeholder("n", "INT32", [])

    def outer_body(i, tot, n_):
        m = gb.add(i, gb.constant("one_o", np.int32(1)), name="m")  # inner trip count: i + 1

        def inner_body(j, t, m_):
            return [gb.add(j, gb.constant("one_i", np.int32(1))), gb.add(t, j)]

        _, t_out = gb.while_loop(lambda j, t, m_: gb.op("Less", [j, m_]), inner_body,
                                 [gb.constant("j0", np.int32(0)), tot], invariants=[m], name="inner")
        return [gb.add(i, gb.constant("one", np.int32(1))), t_out]

    _, tot = gb.while_loop(lambda i, t, n_: gb.op("Less", [i, n_]), outer_body,
                           [gb.constant("i0", np.int32(0)), gb.constant("t0", np.int32(0))], invariants=[n],
                           name="outer")
    gb.identity(tot, name="tot")
    p = gb.placeholder("p", "BOOL", [])

    def looping(x):
        _, r = gb.while_loop(lambda k, v: gb.op("Less", [k, gb.constant("lim", np.int32(3))]),
                             lambda k, v: [gb.add(k, gb.constant("k1", np.int32(1))), gb.add(v, v)],
                             [gb.constant("k0", np.int32(0)), x], name="w")
        return r

    y = gb.cond(p, looping, lambda x: gb.identity(x, name="same"), inputs=[tot], name="gate")
    gb.identity(y, name="y")
    s = Session(gb.build())
    # sum over i < 4 of sum over j <= i of j = 0 + 1 + 3 + 6
    assert int(s.run("tot:0", {"n:0": torch.tensor(4, dtype=torch.int32)})) == 10
    feeds = {"n:0": torch.tensor(4, dtype=torch.int32)}
    assert int(s.run("y:0", {**feeds, "p:0": torch.tensor(False)})) == 10
    assert int(s.run("y:0", {**feeds, "p:0": torch.tensor(True)})) == 80  # 10 doubled 3 times


def _cnn(cond: bool):
    """conv -> [cond(is_training): dropout-like scale | inference BN] -> relu -> GAP -> fc;
    the twin has the inference BN inline."""
    rng = np.random.default_rng(0)
    gb = GraphBuilder()
    x = gb.placeholder("images", "FLOAT", [None, 16, 16, 8])
    w = gb.constant("w", (rng.standard_normal((3, 3, 8, 16)) * 0.2).astype(np.float32))
    y = gb.conv2d(x, w, name="conv")
    bn = [gb.constant(f"bn_{k}", v.astype(np.float32)) for k, v in
          (("scale", rng.uniform(0.5, 1.5, 16)), ("offset", rng.standard_normal(16) * 0.1),
           ("mean", rng.standard_normal(16) * 0.1), ("var", rng.uniform(0.5, 1.5, 16)))]

    def infer(t, *p):
        return gb.fused_batch_norm(t, *p, epsilon=1e-3, name="bn")

    if cond:
        is_training = gb.placeholder_with_default(gb.constant("false", np.bool_(False)), "is_training", [])
        y = gb.cond(is_training, lambda t, *p: gb.mul(t, gb.constant("keep", np.float32(0.5)), name="drop"),
                    infer, inputs=[y, *bn], name="bn_cond")
    else:
        y = infer(y, *bn)
    y = gb.relu(y, name="relu")
    y = gb.mean(y, [1, 2], name="gap")
    fc = gb.constant("fc_w", (rng.standard_normal((16, 10)) * 0.3).astype(np.float32))
    gb.matmul(y, fc, name="logits")
    return gb.build()


def test_cond_gated_cnn_folds_to_the_cond_free_plan():
    from flink_tensorflow_amd.graph.compiler import CompiledFunction

    g_cond, g_twin = _cnn(True), _cnn(False)
    folded = fold_static_control_flow(g_cond, ["images:0"], ["logits:0"])
    assert not {"Switch", "Merge"} & folded.ops()
    imgs = torch.randn(4, 16, 16, 8)
    # the interpreter runs the cond graph with the default (inference) and a fed is_training
    s = Session(g_cond)
    ref = Session(g_twin).run("logits:0", {"images:0": imgs})
    torch.testing.assert_close(s.run("logits:0", {"images:0": imgs}), ref)
    assert not torch.allclose(s.run("logits:0", {"images:0": imgs, "is_training:0": torch.tensor(True)}), ref)
    spec = {"images:0": ((4, 16, 16, 8), "FLOAT")}
    pc = CompiledFunction(g_cond, spec, ["logits:0"], "cpu")
    pt = CompiledFunction(g_twin, spec, ["logits:0"], "cpu")
    assert pc.summary()["kinds"] == pt.summary()["kinds"] and pc.summary()["steps"] == pt.summary()["steps"]
    got = pc({"images:0": imgs})[0].float()
    assert torch.equal(got, pt({"images:0": imgs})[0].float())  # the same plan: the same numbers
    assert (got - ref).abs().max() <= 0.03 * ref.abs().max() + 1e-3  # host plans round activations to bf16
    # a fed is_training is not a compile-time constant: nothing is folded
    assert {"Switch", "Merge"} <= fold_static_control_flow(g_cond, ["images:0", "is_training:0"], ["logits:0"]).ops()


@pytest.mark.gpu
def test_cond_gated_cnn_compiles_glue_free_gpu():
    from flink_tensorflow_amd.graph.compiler import CompiledFunction

    g_cond, g_twin = _cnn(True), _cnn(False)
    dev = torch.device("cuda", 0)
    imgs = torch.randn(4, 16, 16, 8)
    spec = {"images:0": ((4, 16, 16, 8), "FLOAT")}
    pc = CompiledFunction(g_cond, spec, ["logits:0"], dev, strict=True)
    pt = CompiledFunction(g_twin, spec, ["logits:0"], dev, strict=True)
    sc, st = pc.summary(), pt.summary()
    assert sc["glue_ops"] == [] and sc["kinds"] == st["kinds"] and sc["steps"] == st["steps"], (sc, st)
    got = pc({"images:0": imgs.to(dev)})[0].float().cpu()
    ref = Session(g_twin).run("logits:0", {"images:0": imgs})
    assert (got - ref).abs().max() <= 0.03 * ref.abs().max() + 1e-3


def _cond_in_loop_graph():
    """i = i0, acc = 1; while i < n: acc = cond(i % 2 == 0, acc + 1, acc * 2); i += 1 — a
    cond's Merge inside a loop body, taking a different branch on alternate iterations."""
    gb = GraphBuilder()
    n = gb.placeholder("n", "INT32", [])
    i0 = gb.placeholder("i0", "INT32", [])
    a0 = gb.constant("a0", np.float32(1.0))

    def body(i, acc, n_):
        even = gb.op("Equal", [gb.op("FloorMod", [i, gb.constant("two_i", np.int32(2))]),
                               gb.constant("zero_i", np.int32(0))], name="even")
        acc2 = gb.cond(even, lambda a: gb.add(a, gb.constant("one_f", np.float32(1.0)), name="plus1"),
                       lambda a: gb.mul(a, gb.constant("two_f", np.float32(2.0)), name="times2"),
                       inputs=[acc], name="pick")
        return [gb.add(i, gb.constant("one_i", np.int32(1)), name="inc"), acc2]

    i_out, acc_out = gb.while_loop(lambda i, acc, n_: gb.op("Less", [i, n_], name="less"), body, [i0, a0],
                                   invariants=[n])
    gb.identity(acc_out, name="acc")
    gb.identity(i_out, name="iters")
    return gb.build()


@pytest.mark.parametrize("i0,n", [(0, 5), (1, 6), (0, 1), (3, 3), (1, 9)])
def test_cond_inside_while_body_every_iteration(i0, n):
    """Regression: a non-loop Merge fired DEAD on its first dead input at
    iterations >= 1, before the live branch arrived."""
    s = Session(_cond_in_loop_graph())
    acc, it = s.run(["acc:0", "iters:0"], {"n:0": torch.tensor(n, dtype=torch.int32),
                                           "i0:0": torch.tensor(i0, dtype=torch.int32)})
    want = 1.0
    for i in range(i0, n):
        want = want + 1 if i % 2 == 0 else want * 2
    assert int(it) == max(i0, n) and float(acc) == want
