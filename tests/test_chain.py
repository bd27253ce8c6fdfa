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
    with config.override(chain_batch=0):
        base = CompiledFunction(graph, feeds, fetch, device, strict=True, **kw)
    with config.override(chain_batch=bs, chain_min_hw=3136, chain_edge=False):
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
    with config.override(chain_batch=0):
        base = CompiledFunction(small_resnet, feeds, ["logits:0"], "cpu", strict=True)
    with config.override(chain_batch=2, chain_min_hw=3136, chain_edge=True):
        ch = CompiledFunction(small_resnet, feeds, ["logits:0"], "cpu", strict=True)
    names = [s.name for s in ch.steps[ch._chain[0]:ch._chain[1]]]
    # the stage-2 entry 3x3/s2 conv reads the 56x56 tail output: it joins the chain, and
    # that 56x56 tensor becomes a slice-sized internal value
    assert "block2/unit1/conv2/Conv2D" in names
    assert not any(n.startswith("block2/unit2") for n in names)
    torch.testing.assert_close(ch({"images:0": imgs})[0], base({"images:0": imgs})[0], rtol=0, atol=1e-5)


def test_chain_auto_takes_the_inception_stem_not_resnet_stage1(small_resnet):
    """Default (auto): 32-image slices over the layers whose tensors reach 71x71 pixels per
    image, never across a persistent weight-resident kernel — Inception-v3's stem chains,
    ResNet-50 (56x56 stage 1 on persistent kernels) does not."""
    from flink_tensorflow_amd.models.zoo.inception_v3 import inception_v3_graph_def

    with config.override(chain_batch=-1, chain_min_hw=5041, chain_edge=True):
        rn = CompiledFunction(small_resnet, {"images:0": ((64, 72, 72, 3), "UINT8")}, ["logits:0"], "cpu",
                              strict=True)
        g = Graph.from_graph_def(inception_v3_graph_def(image_hw=(299, 299), top_k=5, seed=0))
        inc = CompiledFunction(g, {"images:0": ((64, 299, 299, 3), "UINT8")}, ["top_k:0"], "cpu", strict=True)
    # (the GPU plan fuses ResNet's stem conv and max pool into one launch, so nothing chains;
    # the host plan may chain those two steps, never stage 1)
    rc = getattr(rn, "_chain", None)
    assert rc is None or {s.name for s in rn.steps[rc[0]:rc[1]]} <= {"conv1/Conv2D", "pool1"}
    c = inc._chain
    assert c is not None and c[2] == 2 and c[3] == 32
    names = [s.name for s in inc.steps[c[0]:c[1]]]
    assert names[0].endswith("Conv2d_1a_3x3/Conv2D") and names[-1].endswith("MaxPool_5a_3x3"), names


def test_chain_short_last_slice(small_resnet):
    """A batch that is not a multiple of the slice (the dynamic batch buckets): 5 images in
    slices of 2 run 2 + 2 + 1, the last slice on the leading rows of the slice buffers."""
    imgs = torch.randint(0, 256, (5, 72, 72, 3), dtype=torch.uint8)
    base, ch = _plans(small_resnet, "cpu", 5, 2)
    c = ch._chain
    assert c is not None and c[2] == 3 and c[3] == 2
    torch.testing.assert_close(ch({"images:0": imgs})[0], base({"images:0": imgs})[0], rtol=0, atol=1e-5)
    with config.override(chain_batch=8, chain_min_hw=3136):  # one slice: nothing to chain
        plan = CompiledFunction(small_resnet, {"images:0": ((4, 72, 72, 3), "UINT8")}, ["logits:0"], "cpu",
                                strict=True)
    assert getattr(plan, "_chain", None) is None


@pytest.mark.gpu
def test_chain_gpu_matches_unsliced(small_resnet):
    dev = torch.device("cuda", 0)
    imgs = torch.randint(0, 256, (7, 72, 72, 3), dtype=torch.uint8)
    base, ch = _plans(small_resnet, dev, 7, 2)  # slices 2 + 2 + 2 + 1
    assert ch._chain is not None and ch.summary()["hip_graph"]
    a = base({"images:0": imgs.to(dev)})
    b = ch({"images:0": imgs.to(dev)})
    # the same kernels on the same images (a kernel may pick another tiling for fewer rows)
    assert (a[0] - b[0]).abs().max().item() <= 1e-2 * a[0].abs().max().item()
    assert (a[1][:, 0] == b[1][:, 0]).float().mean().item() >= 0.75
    # the head preprocess per H2D piece, then the tail graph (chain inside)
    src = imgs.to(dev)
    pieces = [(0, 3), (3, 7)]
    assert ch.replay_from_chunks("images:0", src, pieces, lambda i: None)
    torch.cuda.synchronize()
    assert torch.equal(ch.output_tensors()[0].float(), b[0])
