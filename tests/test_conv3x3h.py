"""Halo-staged 3x3 conv (kernels/conv3x3h.hip) against the fp32 reference conv."""
import pytest
import torch
import torch.nn.functional as F

from flink_tensorflow_amd.ops import kernels as K


def _brute_halo(N, H, W):
    Wp, Hp = W + 2, H + 2
    M = N * H * W
    P = [((m // (H * W)) * Hp + (m % (H * W)) // W) * Wp + (m % W) for m in range(M)]
    worst = 0
    for m0 in range(0, M, 128):
        worst = max(worst, P[min(m0 + 127, M - 1)] - P[m0])
    return worst + 2 * Wp + 3


def test_halo_len_matches_brute_force():
    for shape in [(2, 28, 28), (3, 14, 14), (6, 7, 7), (1, 9, 13), (2, 5, 40)]:
        assert K.conv3x3_halo_len(*shape) == _brute_halo(*shape)


def test_halo_eligibility_resnet_stages():
    # ResNet-50 stride-1 3x3 convs of stages 2-4 at the bench batch fit the 288-pixel halo
    for hw, c in [(28, 128), (14, 256), (7, 512)]:
        assert K.conv3x3_halo_eligible((256, hw, hw, c), (c, 3, 3, c), (1, 1), (1, 1, 1, 1), (1, 1), None, "relu")
    assert not K.conv3x3_halo_eligible((256, 56, 56, 64), (64, 3, 3, 64), (1, 1), (1, 1, 1, 1), (1, 1), None, "relu")
    assert not K.conv3x3_halo_eligible((8, 28, 28, 128), (128, 3, 3, 128), (2, 2), (1, 1, 1, 1), (1, 1), None, None)
    assert not K.conv3x3_halo_eligible((8, 28, 28, 96), (128, 3, 3, 96), (1, 1), (1, 1, 1, 1), (1, 1), None, None)


def test_halo_host_path_is_reference_conv():
    torch.manual_seed(0)
    x = torch.randn(2, 7, 7, 64)
    w = torch.randn(32, 3, 3, 64) / 24
    b = torch.randn(32)
    y = K.conv3x3_halo(x, w, b, "relu")
    ref = F.conv2d(x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), b, padding=1).relu().permute(0, 2, 3, 1)
    torch.testing.assert_close(y, ref, rtol=1e-4, atol=1e-4)


DEV = torch.device("cuda", 0)


def _case(N, H, W, C, Cout, act="relu", offset=0, extra=0):
    torch.manual_seed(N * 1000 + H * 10 + C + Cout)
    x = torch.randn(N, H, W, C).to(torch.bfloat16)
    w = (torch.randn(Cout, 3, 3, C) / (9 * C) ** 0.5).to(torch.bfloat16)
    b = torch.randn(Cout) * 0.1
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b, padding=1).permute(0, 2, 3, 1)
    if act == "relu":
        ref = ref.relu()
    out = torch.full((N, H, W, Cout + extra), 7.0, dtype=torch.bfloat16, device=DEV)
    K.conv3x3_halo(x.to(DEV), w.to(DEV), b.to(DEV), act, out=out, out_channel_offset=offset)
    torch.cuda.synchronize()
    got = out[..., offset:offset + Cout].float().cpu()
    torch.testing.assert_close(got, ref, rtol=2e-2, atol=2e-2)
    if extra:
        assert (out[..., :offset] == 7.0).all() and (out[..., offset + Cout:] == 7.0).all()


@pytest.mark.gpu
def test_conv3x3h_resnet_shapes_gpu():
    _case(4, 28, 28, 128, 128)      # stage 2: two 64-channel chunks, tiles across images
    _case(3, 14, 14, 256, 256)      # stage 3
    _case(5, 7, 7, 512, 512)        # stage 4: tiles span three images


@pytest.mark.gpu
def test_conv3x3h_tails_and_offsets_gpu():
    _case(1, 9, 13, 64, 200, act=None)                # M tail (117 pixels), Cout tail, no act
    _case(2, 5, 24, 192, 64, offset=64, extra=128)    # 5-row images, concat offset
    _case(3, 11, 3, 64, 136)                          # narrow rows, Cout 136 = 128 + 8


@pytest.mark.gpu
def test_conv3x3h_in_resnet_plan_gpu():
    """The compiled ResNet-50 routes its stride-1 stage 2-4 3x3 convs (10 layers) to the
    halo kernel and still matches the fp32 interpreter."""
    from flink_tensorflow_amd.graph.compiler import CompiledFunction
    from flink_tensorflow_amd.graph.graph import Graph
    from flink_tensorflow_amd.graph.session import Session
    from flink_tensorflow_amd.models.zoo.resnet import resnet50_graph_def

    from flink_tensorflow_amd.config import override

    g = Graph.from_graph_def(resnet50_graph_def(image_hw=(224, 224)))
    with override(conv3x3_halo=True):
        plan = CompiledFunction(g, {"images:0": ((2, 224, 224, 3), "UINT8")}, ["logits:0"], DEV, strict=True)
    assert plan.summary()["conv3x3h"] == 10, plan.summary()
    imgs = torch.randint(0, 255, (2, 224, 224, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(5))
    (got,) = plan({"images:0": imgs.to(DEV)})
    torch.cuda.synchronize()
    (ref,) = Session(g, device=torch.device("cpu")).run(["logits:0"], {"images:0": imgs})
    got, ref = got.float().cpu(), ref.float()
    err = (got - ref).abs().max().item() / max((ref.max(-1).values - ref.min(-1).values).max().item(), 1e-6)
    assert err < 0.03, err
