"""Graph compiler: fused plan == interpreter (TF semantics), on host and on the GPU."""
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
    assert s["glue_ops"] == [] and s["kinds"]["conv"] == 29 and s["kinds"]["preprocess"] == 1
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
