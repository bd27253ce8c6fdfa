"""Batch-slice chain (``EngineConfig.chain_batch``): the plan's leading run of large-activation
layers runs once per slice of images with slice-sized intermediates; outputs must equal the
unsliced plan's (graph/compiler.py ``_find_chain``)."""
import pytest
import torch

from flink_tensorflow_amd import config
from flink_tensorflow_amd.graph.compiler import CompiledFunction
from flink_tensorflow_amd.graph.graph import Graph
from flink_tensorflow_amd.models.zoo.resnet import resnet50_graph_def


@pytest.fixture(scope="module")
def small_resnet():
    # 72x72 images, resized to 224 in the graph: stage 1 at 56x56
    return Graph.from_graph_def(resnet50_graph_def(depth=26, image_hw=(72, 72), num_classes=64))


def _plans(graph, device, B, bs, **kw):
    feeds = {"images:0": ((B, 72, 72, 3), "UINT8")}
    fetch = ["logits:0", "top_k:1"]
    base = CompiledFunction(graph, feeds, fetch, device, strict=True, **kw)
    with config.override(chain_batch=bs, chain_min_hw=3136):
        ch = CompiledFunction(graph, feeds, fetch, device, strict=True, **kw)
    return base, ch


def test_chain_host_matches_unsliced(small_resnet):
    imgs = torch.randint(0, 256, (4, 72, 72, 3), dtype=torch.uint8)
    base, ch = _plans(small_resnet, "cpu", 4, 2)
    c = ch._chain
    assert c is not None and c[2] == 2 and c[3] == 2
    # every chain step is a stage-1 (18x18) or stem layer; the slice buffers are a fraction
    # of the batch's activations
    names = [s.name for s in ch.steps[c[0]:c[1]]]
    assert all(n.startswith(("conv1", "pool1", "block1/")) for n in names), names
    assert len(names) >= 5 and ch.chain_bytes > 0
    a = base({"images:0": imgs})
    b = ch({"images:0": imgs})
    torch.testing.assert_close(b[0], a[0], rtol=0, atol=1e-5)
    assert torch.equal(a[1], b[1])
    # per-step profile covers every slice of a chain step
    md = ch.profile({"images:0": imgs})
    assert len(md.step_stats.dev_stats[0].node_stats) == len(ch.steps)


def test_chain_edge_takes_the_stride2_readers(small_resnet):
    imgs = torch.randint(0, 256, (4, 72, 72, 3), dtype=torch.uint8)
    feeds = {"images:0": ((4, 72, 72, 3), "UINT8")}
    base = CompiledFunction(small_resnet, feeds, ["logits:0"], "cpu", strict=True)
    with config.override(chain_batch=2, chain_min_hw=3136, chain_edge=True):
        ch = CompiledFunction(small_resnet, feeds, ["logits:0"], "cpu", strict=True)
    names = [s.name for s in ch.steps[ch._chain[0]:ch._chain[1]]]
    # the stage-2 entry 3x3/s2 conv reads the 56x56 tail output: it joins the chain, and
    # that 56x56 tensor becomes a slice-sized internal value
    assert "block2/unit1/conv2/Conv2D" in names
    assert not any(n.startswith("block2/unit2") for n in names)
    torch.testing.assert_close(ch({"images:0": imgs})[0], base({"images:0": imgs})[0], rtol=0, atol=1e-5)


def test_chain_off_when_batch_not_divisible(small_resnet):
    with config.override(chain_batch=3, chain_min_hw=3136):
        plan = CompiledFunction(small_resnet, {"images:0": ((4, 72, 72, 3), "UINT8")}, ["logits:0"], "cpu",
                                strict=True)
    assert getattr(plan, "_chain", None) is None


@pytest.mark.gpu
def test_chain_gpu_matches_unsliced(small_resnet):
    dev = torch.device("cuda", 0)
    imgs = torch.randint(0, 256, (8, 72, 72, 3), dtype=torch.uint8)
    base, ch = _plans(small_resnet, dev, 8, 2)
    assert ch._chain is not None and ch.summary()["hip_graph"]
    a = base({"images:0": imgs.to(dev)})
    b = ch({"images:0": imgs.to(dev)})
    # the same kernels on the same images (a kernel may pick another tiling for fewer rows)
    assert (a[0] - b[0]).abs().max().item() <= 1e-2 * a[0].abs().max().item()
    assert (a[1][:, 0] == b[1][:, 0]).float().mean().item() >= 0.75
    # the head preprocess per H2D piece, then the tail graph (chain inside)
    src = imgs.to(dev)
    pieces = [(0, 3), (3, 8)]
    assert ch.replay_from_chunks("images:0", src, pieces, lambda i: None)
    torch.cuda.synchronize()
    assert torch.equal(ch.output_tensors()[0].float(), b[0])
