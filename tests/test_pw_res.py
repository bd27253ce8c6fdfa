"""Persistent identity-residual expansion conv (``ops.kernels.pw_res``, kernels/pw_res.hip)
against the fp32 PyTorch reference of the same op, and its routing in the compiled
ResNet-50 plan (the stage-2/3 bottleneck expands)."""
import pytest
import torch

from flink_tensorflow_amd.ops import kernels as K


def _case(M, K_, N, g):
    x = torch.randn(M, K_, generator=g).bfloat16()
    w = (torch.randn(N, K_, generator=g) / K_ ** 0.5).bfloat16()
    b = torch.randn(N, generator=g)
    r = torch.randn(M, N, generator=g).bfloat16()
    return x, w, b, r


def _ref(x, w, b, r):
    return torch.relu(x.float() @ w.float().t() + b + r.float())


def test_pw_res_host_reference():
    g = torch.Generator().manual_seed(0)
    x, w, b, r = _case(100, 128, 256, g)
    got = K.pw_res(x.float().reshape(4, 25, 128), w.float(), b, r.float().reshape(4, 25, 256))
    torch.testing.assert_close(got.reshape(100, 256), _ref(x, w, b, r), rtol=1e-5, atol=1e-4)
    with pytest.raises(ValueError):
        K.pw_res(torch.zeros(4, 64), torch.zeros(128, 64), torch.zeros(128), torch.zeros(4, 128))  # K = 64


@pytest.mark.gpu
@pytest.mark.parametrize("M,K_,N,tp", [(25088, 128, 512, 0), (12544 + 77, 256, 1024, 0), (300, 128, 128, 0),
                                       (1000, 256, 384, 128), (5000 + 3, 256, 512, 128), (12544, 256, 1024, 128)])
def test_pw_res_gpu(M, K_, N, tp):
    g = torch.Generator().manual_seed(M + N)
    x, w, b, r = _case(M, K_, N, g)
    dev = torch.device("cuda", 0)
    got = K.pw_res(x.to(dev), w.to(dev), b.to(dev), r.to(dev), tp=tp).float().cpu()
    ref = _ref(x, w, b, r)
    torch.testing.assert_close(got, ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())


@pytest.mark.gpu
def test_pw_res_gpu_channel_offset():
    """Writes at a channel offset of a wider output (concat-by-stride-write)."""
    g = torch.Generator().manual_seed(3)
    x, w, b, r = _case(640, 256, 256, g)
    dev = torch.device("cuda", 0)
    out = torch.zeros(640, 512, dtype=torch.bfloat16, device=dev)
    K.pw_res(x.to(dev), w.to(dev), b.to(dev), r.to(dev), out=out, out_channel_offset=128)
    ref = _ref(x, w, b, r)
    got = out.float().cpu()
    torch.testing.assert_close(got[:, 128:384], ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())
    assert (got[:, :128] == 0).all() and (got[:, 384:] == 0).all()


def test_resnet50_plan_routes_expands_to_pw_res():
    from flink_tensorflow_amd.graph.compiler import CompiledFunction
    from flink_tensorflow_amd.graph.graph import Graph
    from flink_tensorflow_amd.models.zoo.resnet import resnet50_graph_def

    g = Graph.from_graph_def(resnet50_graph_def(image_hw=(64, 64), num_classes=16))
    plan = CompiledFunction(g, {"images:0": ((2, 64, 64, 3), "UINT8")}, ["logits:0"], "cpu", strict=True)
    # stage 2: units 2-4, stage 3: units 2-6 (unit 1 of each stage fuses its projection)
    assert plan.summary()["pw_res"] == 8
