"""Graph compiler: fused plan == interpreter (TF semantics), on host and on the GPU."""
import numpy as np
import pytest
import torch

from flink_tensorflow_amd.graph.compiler import CompiledFunction
from flink_tensorflow_amd.graph.graph import Graph
from flink_tensorflow_amd.graph.session import Session
from flink_tensorflow_amd.models.zoo.resnet import resnet50_graph_def


@pytest.fixture(scope="module")
def small_resnet():
    return Graph.from_graph_def(resnet50_graph_def(depth=26, image_hw=(72, 72), num_classes=64))


def _check_plan(graph, device, imgs):
    ref = Session(graph).run(["logits:0", "top_k:1"], {"images:0": imgs})
    plan = CompiledFunction(graph, {"images:0": (tuple(imgs.shape), "UINT8")}, ["logits:0", "top_k:1"], device,
                            strict=True)
    s = plan.summary()
    # 29 convs, the 4 projection shortcuts fused into their unit's expansion conv, the two
    # stage-1 block boundaries (unit 1 -> 2, stage 1 -> 2) fused into one step each; on the
    # GPU the 3 deep-K 1x1 reduce convs of stages 3/4 and the stage-3 entry reduce (K 512 -> 256)
    # run on the ping-pong GEMM (kernels/gemm_pp.hip)
    gpu = torch.device(device).type == "cuda"
    assert s["glue_ops"] == [] and s["fused_shortcuts"] == 4 and s["fused_tails"] == 2
    assert s["kinds"]["conv"] == (19 if gpu else 23)
    assert s["kinds"]["preprocess"] == 1
    # on the GPU the stem runs on the direct conv with pool1 fused into its epilogue
    assert s["fused_pools"] == (1 if torch.device(device).type == "cuda" else 0)
    logits, idx = plan({"images:0": imgs.to(device)})
    err = (logits.cpu() - ref[0]).abs().max().item() / ref[0].abs().max().item()
    assert err < 0.05, err
    # top-1 agrees unless the reference's top-2 are within bf16 noise
    p = torch.softmax(ref[0], -1)
    top2 = torch.topk(p, 2, -1).values
    ok = (idx[:, 0].cpu() == ref[1][:, 0]) | ((top2[:, 0] - top2[:, 1]) < 0.02)
    assert ok.all()
    return plan


def test_compiled_plan_host(small_resnet):
    imgs = torch.randint(0, 256, (2, 72, 72, 3), dtype=torch.uint8)
    _check_plan(small_resnet, "cpu", imgs)


@pytest.mark.gpu
def test_compiled_plan_gpu(small_resnet):
    imgs = torch.randint(0, 256, (3, 72, 72, 3), dtype=torch.uint8)
    plan = _check_plan(small_resnet, torch.device("cuda", 0), imgs)
    assert plan.summary()["hip_graph"]
    # replay is deterministic
    a = plan({"images:0": imgs.cuda()})[0]
    b = plan({"images:0": imgs.cuda()})[0]
    assert torch.equal(a, b)


def test_memory_reuse(small_resnet):
    plan = CompiledFunction(small_resnet, {"images:0": ((1, 72, 72, 3), "UINT8")}, ["probs:0"], "cpu")
    distinct = {s.outputs[0].buf.untyped_storage().data_ptr() for s in plan.steps if s.outputs[0].buf is not None}
    assert len(distinct) < len(plan.steps)  # buffers are recycled between layers


def test_s2d_stem_equivalence():
    """Stride-2 7x7 RGB stem == stride-1 4x4 conv over the space-to-depth input."""
    from flink_tensorflow_amd.graph.ops_nn import conv2d_tf, same_pads
    from flink_tensorflow_amd.ops import kernels as K

    img = torch.randint(0, 256, (2, 100, 90, 3), dtype=torch.uint8)
    w = torch.randn(7, 7, 3, 64)
    a = K.preprocess_images(img, (224, 224))
    ref = conv2d_tf(a[..., :3].float(), w, (2, 2), "SAME")
    pt, pb = same_pads(224, 7, 2)
    w2, pads = K.s2d_stem_weights(w, 224, 224, (pt, pb, pt, pb))
    b = K.preprocess_images(img, (224, 224), s2d=True)
    got = K.conv2d_nhwc(b, w2, pad=pads)
    assert pads == (1, 2, 1, 2)
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-2)
    # odd size (Inception's 3x3 / s2 VALID stem on 299 x 299): the last block row / column
    # is zero-filled past the image and meets only zero weights
    w3 = torch.randn(3, 3, 3, 32)
    a = K.preprocess_images(img, (75, 75))
    ref = conv2d_tf(a[..., :3].float(), w3, (2, 2), "VALID")
    w2, pads = K.s2d_stem_weights(w3, 75, 75, (0, 0, 0, 0))
    b = K.preprocess_images(img, (75, 75), s2d=True)
    assert b.shape == (2, 38, 38, 16) and (b[:, -1, :, 6:12] == 0).all() and (b[:, :, -1, 3:6] == 0).all()
    got = K.conv2d_nhwc(b, w2, pad=pads)
    assert pads == (0, 0, 0, 0) and got.shape == ref.shape == (2, 37, 37, 32)
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-2)


def test_plan_profile_and_debug_modes(monkeypatch):
    """Compiled-plan RunMetadata (one NodeExecStats per launch) and the eager debug modes:
    FTM_DEBUG_SYNC checks after each launch, FTM_DEBUG_POISON fills dead buffers with NaN
    bytes — results must be unchanged when the liveness plan is right."""
    import torch

    from flink_tensorflow_amd.graph.compiler import CompiledFunction
    from flink_tensorflow_amd.graph.graph import Graph
    from flink_tensorflow_amd.models.zoo.resnet import resnet50_graph_def

    g = Graph.from_graph_def(resnet50_graph_def(image_hw=(32, 32), out_hw=(32, 32), depth=26))
    feeds = {"images:0": ((2, 32, 32, 3), "UINT8")}
    img = torch.randint(0, 256, (2, 32, 32, 3), dtype=torch.uint8)
    base = CompiledFunction(g, feeds, ["logits:0"], "cpu", strict=True)
    ref = base({"images:0": img})[0]
    md = base.profile({"images:0": img})
    stats = md.step_stats.dev_stats[0].node_stats
    assert len(stats) == len(base.steps) and {s.timeline_label for s in stats} >= {"conv", "preprocess"}
    monkeypatch.setenv("FTM_DEBUG_POISON", "1")
    monkeypatch.setenv("FTM_DEBUG_SYNC", "1")
    dbg = CompiledFunction(g, feeds, ["logits:0"], "cpu", strict=True)
    assert dbg._poison_after  # some buffers die mid-plan
    out = dbg({"images:0": img})[0]
    assert torch.isfinite(out).all()
    torch.testing.assert_close(out, ref)


def _elementwise_graph():
    import numpy as np

    from flink_tensorflow_amd.graph.builder import GraphBuilder
    from flink_tensorflow_amd.graph.graph import Graph

    gb = GraphBuilder()
    x = gb.placeholder("x", "FLOAT", [2, 4, 4, 16])
    y = gb.mul(x, gb.constant("two", np.float32(2.0)), name="scale")
    y = gb.add(y, gb.constant("bias", np.linspace(-1, 1, 16).astype(np.float32)), name="shift")
    y = gb.relu(y, name="act")
    y = gb.lrn(y, 2, 1.0, 0.5, 0.75, name="lrn")
    y = gb.sub(y, x, name="diff")
    y = gb.op("Maximum", [y, gb.constant("floor", np.float32(-0.25))], name="clip")
    y = gb.div(gb.constant("one", np.float32(1.0)), gb.add(gb.op("Abs", [y], name="abs"),
                                                            gb.constant("eps", np.float32(1.0))), name="out")
    return Graph.from_graph_def(gb.build_graph_def())


def _check_elementwise(device):
    import torch

    from flink_tensorflow_amd.graph.compiler import CompiledFunction
    from flink_tensorflow_amd.graph.session import Session

    g = _elementwise_graph()
    x = torch.randn(2, 4, 4, 16)
    ref = Session(g).run(["clip:0"], {"x:0": x})[0]
    plan = CompiledFunction(g, {"x:0": ((2, 4, 4, 16), "FLOAT")}, ["clip:0"], device, strict=True)
    kinds = plan.summary()["kinds"]
    assert kinds.get("elementwise") == 5 and kinds.get("lrn") == 1, kinds
    got = plan({"x:0": x.to(device)})[0].cpu()
    torch.testing.assert_close(got, ref.float(), rtol=2e-2, atol=3e-2)


def test_standalone_elementwise_and_lrn_host():
    _check_elementwise("cpu")


@pytest.mark.gpu
def test_standalone_elementwise_and_lrn_gpu():
    import torch

    _check_elementwise(torch.device("cuda", 0))


@pytest.mark.gpu
def test_replay_from_staging_buffer_gpu(small_resnet):
    """``replay_from`` runs the preprocess head on the caller's buffer and replays the tail
    graph: same outputs as copy-into-input + full replay, and the input buffer is untouched."""
    dev = torch.device("cuda", 0)
    imgs = torch.randint(0, 256, (3, 72, 72, 3), dtype=torch.uint8, device=dev)
    other = torch.randint(0, 256, (3, 72, 72, 3), dtype=torch.uint8, device=dev)
    plan = CompiledFunction(small_resnet, {"images:0": ((3, 72, 72, 3), "UINT8")}, ["logits:0"], dev, strict=True)
    assert plan._head is not None and plan._graph_tail is not None
    ref = plan({"images:0": imgs})[0].clone()
    plan.input_buffer("images:0").copy_(other)
    plan.replay_from("images:0", imgs)
    got = plan.output_tensors()[0].float().clone()
    torch.cuda.synchronize()
    assert torch.equal(got, ref.float())
    assert torch.equal(plan.input_buffer("images:0"), other)
    # a non-contiguous source falls back to copy + full replay
    nc = imgs.permute(0, 2, 1, 3).contiguous().permute(0, 2, 1, 3)
    plan.replay_from("images:0", nc)
    torch.cuda.synchronize()
    assert torch.equal(plan.output_tensors()[0].float(), ref.float())


def test_head_bypass_refused_when_the_feed_has_other_readers():
    """``replay_from`` may skip the input copy only if the preprocess step is the raw feed's
    sole reader: a fetch of the feed itself, or of a Reshape alias of it, keeps the copy."""
    from flink_tensorflow_amd.graph.builder import GraphBuilder
    from flink_tensorflow_amd.models.zoo.resnet import resnet50_graph_def

    spec = {"images:0": ((2, 72, 72, 3), "UINT8")}
    gd = resnet50_graph_def(depth=26, image_hw=(72, 72), num_classes=8)
    plan = CompiledFunction(Graph.from_graph_def(gd), spec, ["logits:0"], "cpu", strict=True)
    assert plan._head_feed_step() is not None                      # sole reader: bypass allowed
    plan = CompiledFunction(Graph.from_graph_def(gd), spec, ["logits:0", "images:0"], "cpu")
    assert plan._head_feed_step() is None                          # the feed is fetched
    b = GraphBuilder()
    b.op("Reshape", ["images:0", b.constant("flat_shape", np.array([2, -1], np.int32))], name="flat_images")
    gd.node.extend(b.build_graph_def().node)
    plan = CompiledFunction(Graph.from_graph_def(gd), spec, ["logits:0", "flat_images:0"], "cpu")
    assert plan._head_feed_step() is None                          # a Reshape alias is fetched
