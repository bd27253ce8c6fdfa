"""Function calls and functional control flow (``graph/functions.py``): GraphDefs with a
``FunctionDefLibrary`` called through ``StatefulPartitionedCall`` / ``PartitionedCall``,
``StatelessIf`` / ``If`` and ``StatelessWhile`` / ``While`` (TF's control flow v2 and TF2
signatures) are lowered to plain dataflow and run in the interpreter; the compiler folds a
lowered ``If`` on a compile-time constant.  No fixture in the reference carries a function
library (parity unpinned): graphs are built from the protos and checked by hand."""
import numpy as np
import torch

from flink_tensorflow_amd.graph.graph import Graph
from flink_tensorflow_amd.graph.session import Session
from flink_tensorflow_amd.graph.tensor_proto import make_tensor_proto
from flink_tensorflow_amd.proto.messages import (ArgDef, AttrValue, FunctionDef, FunctionDefLibrary, GraphDef,
                                                 NameAttrList, NodeDef, OpDef, TensorShapeProto)
from flink_tensorflow_amd.types.dtypes import DataType

F32, I32, BOOL, RES = int(DataType.FLOAT), int(DataType.INT32), int(DataType.BOOL), 20


def _const(name, value, dtype=None):
    t = torch.tensor(value, dtype=dtype)
    tp = make_tensor_proto(t)
    return NodeDef(name=name, op="Const", attr={"value": AttrValue(tensor=tp), "dtype": AttrValue(type=tp.dtype)})


def _fn(name, ins, outs, nodes, ret):
    return FunctionDef(signature=OpDef(name=name, input_arg=[ArgDef(name=n, type=t) for n, t in ins],
                                       output_arg=[ArgDef(name=n, type=t) for n, t in outs]),
                       node_def=nodes, ret=ret)


def _f(name):
    return AttrValue(func=NameAttrList(name=name))


def _ph(name, dtype):
    return NodeDef(name=name, op="Placeholder", attr={"dtype": AttrValue(type=dtype),
                                                      "shape": AttrValue(shape=TensorShapeProto(unknown_rank=True))})


# f(x, y) = 2x + y ; g(x) = f(x, 1) + 1 (a call inside a function)
F = _fn("f", [("x", F32), ("y", F32)], [("out", F32)],
        [_const("two", 2.0), NodeDef(name="mul", op="Mul", input=["x", "two:output:0"]),
         NodeDef(name="add", op="AddV2", input=["mul:z:0", "y"])], {"out": "add:z:0"})
G = _fn("g", [("x", F32)], [("out", F32)],
        [_const("one", 1.0), NodeDef(name="call", op="PartitionedCall", input=["x", "one:output:0"],
                                     attr={"f": _f("f")}),
         NodeDef(name="inc", op="AddV2", input=["call:output:0", "one:output:0"])], {"out": "inc:z:0"})
THEN = _fn("then_fn", [("x", F32)], [("out", F32)], [_const("k", 2.0), NodeDef(name="m", op="Mul", input=["x", "k:output:0"])],
           {"out": "m:z:0"})
ELSE = _fn("else_fn", [("x", F32)], [("out", F32)], [_const("k", 10.0), NodeDef(name="s", op="Sub", input=["x", "k:output:0"])],
           {"out": "s:z:0"})
# while i < n: i += 1; acc *= 2
COND = _fn("cond_fn", [("i", I32), ("acc", F32), ("n", I32)], [("out", BOOL)],
           [NodeDef(name="lt", op="Less", input=["i", "n"])], {"out": "lt:z:0"})
BODY = _fn("body_fn", [("i", I32), ("acc", F32), ("n", I32)], [("i1", I32), ("acc1", F32), ("n1", I32)],
           [_const("one", 1, torch.int32), _const("two", 2.0), NodeDef(name="inc", op="AddV2", input=["i", "one:output:0"]),
            NodeDef(name="dbl", op="Mul", input=["acc", "two:output:0"]), NodeDef(name="n_id", op="Identity", input=["n"])],
           {"i1": "inc:z:0", "acc1": "dbl:z:0", "n1": "n_id:output:0"})
READ = _fn("read_fn", [("v", RES), ("x", F32)], [("out", F32)],
           [NodeDef(name="r", op="ReadVariableOp", input=["v"], attr={"dtype": AttrValue(type=F32)}),
            NodeDef(name="a", op="AddV2", input=["r:value:0", "x"])], {"out": "a:z:0"})
LIB = FunctionDefLibrary(function=[F, G, THEN, ELSE, COND, BODY, READ])


def _graph(nodes):
    return Graph.from_graph_def(GraphDef(node=nodes, library=LIB).encode())  # through the wire codec


def test_partitioned_calls_nested():
    g = _graph([_ph("a", F32), _ph("b", F32),
                NodeDef(name="call", op="StatefulPartitionedCall", input=["a", "b"], attr={"f": _f("f")}),
                NodeDef(name="call2", op="PartitionedCall", input=["a"], attr={"f": _f("g")}),
                NodeDef(name="y", op="Identity", input=["call"])])
    s = Session(g)
    a, b = torch.tensor([1.0, 2.0]), torch.tensor([10.0, 20.0])
    y, c, c2 = s.run(["y:0", "call:0", "call2:0"], {"a:0": a, "b:0": b})
    assert torch.equal(y, 2 * a + b) and torch.equal(c, y) and torch.equal(c2, 2 * a + 2)


def test_stateless_if_both_branches_and_compile_time_fold():
    from flink_tensorflow_amd.graph.control_flow import fold_static_control_flow
    from flink_tensorflow_amd.graph.functions import lower_functional_ops

    nodes = [_ph("p", BOOL), _ph("x", F32),
             NodeDef(name="if", op="StatelessIf", input=["p", "x"],
                     attr={"then_branch": _f("then_fn"), "else_branch": _f("else_fn")}),
             NodeDef(name="y", op="Identity", input=["if:0"])]
    s = Session(_graph(nodes))
    x = torch.tensor([1.0, 4.0])
    assert torch.equal(s.run("y:0", {"p:0": torch.tensor(True), "x:0": x}), x * 2)
    assert torch.equal(s.run("y:0", {"p:0": torch.tensor(False), "x:0": x}), x - 10)
    # is_training-style default: the compiler's fold resolves the lowered If
    nodes[0] = NodeDef(name="p", op="PlaceholderWithDefault", input=["p_default"],
                       attr={"dtype": AttrValue(type=BOOL), "shape": AttrValue(shape=TensorShapeProto())})
    g = _graph([_const("p_default", False)] + nodes)
    folded = fold_static_control_flow(lower_functional_ops(g), ["x:0"], ["y:0"])
    assert not {"Switch", "Merge", "StatelessIf"} & folded.ops()
    assert torch.equal(Session(folded).run("y:0", {"x:0": x}), x - 10)


def test_stateless_while_counts():
    g = _graph([_ph("n", I32), _const("i0", 0, torch.int32), _const("acc0", 1.0),
                NodeDef(name="loop", op="StatelessWhile", input=["i0", "acc0", "n"],
                        attr={"cond": _f("cond_fn"), "body": _f("body_fn")}),
                NodeDef(name="acc", op="Identity", input=["loop:1"])])
    s = Session(g)
    for n in (0, 1, 5):
        acc, i = s.run(["acc:0", "loop:0"], {"n:0": torch.tensor(n, dtype=torch.int32)})
        assert float(acc) == 2.0 ** n and int(i) == n


def test_resource_variable_through_a_call():
    g = _graph([NodeDef(name="v", op="VarHandleOp", attr={"dtype": AttrValue(type=F32), "shape": AttrValue(
        shape=TensorShapeProto.of([2])), "shared_name": AttrValue(s=b"v")}),
                _const("v_init", [3.0, 4.0]),
                NodeDef(name="assign", op="AssignVariableOp", input=["v", "v_init"], attr={"dtype": AttrValue(type=F32)}),
                _ph("x", F32),
                NodeDef(name="call", op="StatefulPartitionedCall", input=["v", "x"], attr={"f": _f("read_fn")})])
    s = Session(g)
    s.run(targets=["assign"])
    assert torch.equal(s.run("call:0", {"x:0": torch.tensor([1.0, 1.0])}), torch.tensor([4.0, 5.0]))


def test_compiled_plan_through_a_call():
    """A CPU compiled plan of a graph whose body is a function call (TF2-style signature)."""
    from flink_tensorflow_amd.graph.compiler import CompiledFunction

    g = _graph([_ph("a", F32), _ph("b", F32),
                NodeDef(name="call", op="StatefulPartitionedCall", input=["a", "b"], attr={"f": _f("f")})])
    plan = CompiledFunction(g, {"a:0": ((4, 8), "FLOAT"), "b:0": ((4, 8), "FLOAT")}, ["call:0"], "cpu")
    a, b = torch.randn(4, 8), torch.randn(4, 8)
    got = plan({"a:0": a, "b:0": b})[0].float()
    assert (got - (2 * a + b)).abs().max() < 0.05
    assert np.isfinite(got.numpy()).all()


def test_stateless_if_inside_stateless_while():
    """A functional If in a While body (lowered to a cond inside a loop frame): the branch
    alternates per iteration — regression for the Merge dead-token rule."""
    then2 = _fn("inc_fn", [("x", F32)], [("out", F32)],
                [_const("k", 1.0), NodeDef(name="a", op="AddV2", input=["x", "k:output:0"])], {"out": "a:z:0"})
    else2 = _fn("dbl_fn", [("x", F32)], [("out", F32)],
                [_const("k", 2.0), NodeDef(name="m", op="Mul", input=["x", "k:output:0"])], {"out": "m:z:0"})
    body2 = _fn("body2_fn", [("i", I32), ("acc", F32), ("n", I32)], [("i1", I32), ("acc1", F32), ("n1", I32)],
                [_const("one", 1, torch.int32), _const("two", 2, torch.int32), _const("zero", 0, torch.int32),
                 NodeDef(name="mod", op="FloorMod", input=["i", "two:output:0"]),
                 NodeDef(name="even", op="Equal", input=["mod:z:0", "zero:output:0"]),
                 NodeDef(name="pick", op="StatelessIf", input=["even:z:0", "acc"],
                         attr={"then_branch": _f("inc_fn"), "else_branch": _f("dbl_fn")}),
                 NodeDef(name="inc", op="AddV2", input=["i", "one:output:0"]),
                 NodeDef(name="n_id", op="Identity", input=["n"])],
                {"i1": "inc:z:0", "acc1": "pick:output:0", "n1": "n_id:output:0"})
    lib = FunctionDefLibrary(function=[COND, then2, else2, body2])
    g = Graph.from_graph_def(GraphDef(node=[
        _ph("n", I32), _ph("i0", I32), _const("acc0", 1.0),
        NodeDef(name="loop", op="StatelessWhile", input=["i0", "acc0", "n"],
                attr={"cond": _f("cond_fn"), "body": _f("body2_fn")}),
        NodeDef(name="acc", op="Identity", input=["loop:1"])], library=lib).encode())
    s = Session(g)
    for i0, n in ((0, 5), (1, 6), (2, 9)):
        acc = s.run("acc:0", {"n:0": torch.tensor(n, dtype=torch.int32), "i0:0": torch.tensor(i0, dtype=torch.int32)})
        want = 1.0
        for i in range(i0, n):
            want = want + 1 if i % 2 == 0 else want * 2
        assert float(acc) == want, (i0, n, float(acc), want)


def test_call_control_inputs_gate_the_inlined_body():
    """``StatefulPartitionedCall ^assign`` whose body reads the variable through an argument:
    the read waits for (and pruning keeps) the assign (inlining dropped the
    call's control inputs for every body node fed by an argument)."""
    g = _graph([NodeDef(name="v", op="VarHandleOp", attr={"dtype": AttrValue(type=F32), "shape": AttrValue(
        shape=TensorShapeProto.of([2])), "shared_name": AttrValue(s=b"v")}),
                _const("v_init", [3.0, 4.0]),
                NodeDef(name="assign", op="AssignVariableOp", input=["v", "v_init"], attr={"dtype": AttrValue(type=F32)}),
                _ph("x", F32),
                NodeDef(name="call", op="StatefulPartitionedCall", input=["v", "x", "^assign"],
                        attr={"f": _f("read_fn")})])
    s = Session(g)  # no separate init run: the call's control input must bring the assign
    assert torch.equal(s.run("call:0", {"x:0": torch.tensor([1.0, 1.0])}), torch.tensor([4.0, 5.0]))


def test_if_and_while_control_inputs_gate_their_arguments():
    nodes = [NodeDef(name="v", op="VarHandleOp", attr={"dtype": AttrValue(type=F32), "shape": AttrValue(
        shape=TensorShapeProto.of([2])), "shared_name": AttrValue(s=b"w")}),
             _const("v_init", [3.0, 4.0]),
             NodeDef(name="assign", op="AssignVariableOp", input=["v", "v_init"], attr={"dtype": AttrValue(type=F32)}),
             _ph("p", BOOL),
             NodeDef(name="rd", op="ReadVariableOp", input=["v"], attr={"dtype": AttrValue(type=F32)}),
             NodeDef(name="if", op="StatelessIf", input=["p", "rd", "^assign"],
                     attr={"then_branch": _f("then_fn"), "else_branch": _f("else_fn")})]
    from flink_tensorflow_amd.graph.functions import lower_functional_ops

    low = lower_functional_ops(_graph(nodes))
    assert "if/input_control" in low.nodes and low.nodes["if/input_control"].control_inputs == ["assign"]
    assert all(low.nodes[f"if/arg_{i}"].control_inputs == ["if/input_control"] for i in range(2))


def test_opdef_flags_round_trip_with_tf_field_numbers():
    """op_def.proto: is_aggregate = 16, is_stateful = 17 (is_stateful was
    written as tag 16 and came back as is_aggregate in TF)."""
    from flink_tensorflow_amd.proto.wire import scan

    sig = OpDef(name="f", is_stateful=True)
    raw = sig.encode()
    tags = {num for num, _, _ in scan(raw)}
    assert 17 in tags and 16 not in tags
    back = OpDef.decode(raw)
    assert back.is_stateful and not back.is_aggregate
    fd = FunctionDef(signature=OpDef(name="g", is_stateful=True, is_aggregate=True))
    again = FunctionDef.decode(fd.encode())
    assert again.signature.is_stateful and again.signature.is_aggregate
