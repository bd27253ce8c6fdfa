"""Ping-pong 256x256 MFMA GEMM (``kernels/gemm_pp.hip``) vs a plain PyTorch fp32 reference.

Shapes cover the BERT-base projections at 32768 tokens (guide-style 8-phase kernel, the
hipBLASLt replacement), M / N tails, the split-K small-M heads (ResNet FC 2048->1000,
BERT pooler), the fused epilogues (bias, GELU, tanh, ReLU, residual) and the
concat-by-stride output offset.
"""
import pytest
import torch

from flink_tensorflow_amd.ops import kernels as K

DEV = torch.device("cuda", 0)


def _ref(x, w, b, r, act):
    y = x.float() @ w.float().t()
    if b is not None:
        y = y + b.float()
    if r is not None:
        y = y + r.float()
    return K._apply_act_ref(y, K.act_code(act))


def _close(got, ref, rtol=2e-2, atol_scale=1e-2):
    got = got.float()
    ref = ref.float().to(got.device)
    atol = atol_scale * max(ref.abs().max().item(), 1e-3)
    torch.testing.assert_close(got, ref, rtol=rtol, atol=atol)


def test_gemm_pp_host_reference_semantics():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(5, 64, generator=g)
    w = torch.randn(16, 64, generator=g)
    b = torch.randn(16, generator=g)
    out = torch.zeros(5, 40)
    K.gemm_pp(x, w, b, act="relu", out=out, out_col=8)
    torch.testing.assert_close(out[:, 8:24], torch.relu(x @ w.t() + b))
    assert out[:, :8].abs().sum() == 0 and out[:, 24:].abs().sum() == 0


def test_gemm_pp_split_heuristic():
    assert K.gemm_pp_splits(32768, 3072, 768) == 1
    assert K.gemm_pp_splits(2048, 2304, 768) == 1   # partial traffic would cost more than it saves
    assert K.gemm_pp_splits(50176, 256, 1024) == 1  # one wave of tiles already
    assert K.gemm_pp_splits(256, 1000, 2048) > 4    # FC head: 4 tiles -> split-K
    assert K.gemm_pp_splits(16, 768, 3072) > 4      # final-layer CLS rows
    assert K.gemm_pp_splits(256, 768, 128) == 1     # too shallow to split


CASES = [
    # M, N, K, act, residual, splits
    (32768, 2304, 768, None, False, 1),      # BERT QKV
    (32768, 768, 768, None, True, 1),        # BERT O-proj + residual
    (32768, 3072, 768, "gelu", False, 1),    # BERT FFN1 + GELU
    (32768, 768, 3072, None, True, 1),       # BERT FFN2 + residual
    (24611, 768, 768, None, True, 1),        # packed tokens: M tail
    (1000, 1000, 640, "relu", False, 1),     # M and N tails
    (300, 264, 64, None, False, 1),          # single K tile
    (448, 520, 192, "relu", True, 1),        # odd K-tile count, tails
    (256, 1000, 2048, None, False, None),    # ResNet FC head: auto split-K
    (256, 768, 768, "tanh", False, 4),       # BERT pooler, forced split
    (12544, 256, 1024, "relu", False, 1),    # ResNet stage-3 deep-K 1x1
    (3136, 512, 2048, "relu", True, 2),      # split + residual + act
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}x{c[1]}x{c[2]}-{c[3]}-r{int(c[4])}-s{c[5]}" for c in CASES])
def test_gemm_pp(case):
    M, N, Kd, act, has_res, splits = case
    g = torch.Generator(device=DEV).manual_seed(M * 7 + N + Kd)
    x = torch.randn(M, Kd, generator=g, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, Kd, generator=g, device=DEV) / Kd ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, generator=g, device=DEV)
    r = torch.randn(M, N, generator=g, device=DEV).to(torch.bfloat16) if has_res else None
    got = K.gemm_pp(x, w, b, r, act, splits=splits)
    torch.cuda.synchronize()
    _close(got, _ref(x, w, b, r, act))


@pytest.mark.gpu
def test_gemm_pp_layout_asymmetric():
    """x = I (256 rows), asymmetric w: out must equal w^T exactly (catches a transposed
    C write or a mis-swizzled fragment)."""
    M, N, Kd = 256, 256, 256
    x = torch.eye(M, Kd, device=DEV, dtype=torch.bfloat16)
    w = (torch.arange(N * Kd, device=DEV, dtype=torch.float32).reshape(N, Kd) % 251 - 125).to(torch.bfloat16)
    got = K.gemm_pp(x, w)
    torch.cuda.synchronize()
    assert torch.equal(got.float(), w.float().t())


@pytest.mark.gpu
def test_gemm_pp_out_col_and_no_bias():
    M, N, Kd = 512, 128, 128
    g = torch.Generator(device=DEV).manual_seed(3)
    x = torch.randn(M, Kd, generator=g, device=DEV).to(torch.bfloat16)
    w = torch.randn(N, Kd, generator=g, device=DEV).to(torch.bfloat16)
    out = torch.full((M, 3 * N), 7.0, device=DEV, dtype=torch.bfloat16)
    K.gemm_pp(x, w, out=out, out_col=N)
    torch.cuda.synchronize()
    _close(out[:, N:2 * N], _ref(x, w, None, None, None))
    assert (out[:, :N] == 7).all() and (out[:, 2 * N:] == 7).all()


@pytest.mark.gpu
def test_gemm_pp_graph_capture():
    M, N, Kd = 2048, 768, 768
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn(M, Kd, generator=g, device=DEV).to(torch.bfloat16)
    w = torch.randn(N, Kd, generator=g, device=DEV).to(torch.bfloat16)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    K.gemm_pp(x, w, out=out)  # warm-up outside capture
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        K.gemm_pp(x, w, out=out)
    x.copy_(torch.randn(M, Kd, generator=g, device=DEV).to(torch.bfloat16))
    graph.replay()
    torch.cuda.synchronize()
    _close(out, _ref(x, w, None, None, None))


@pytest.mark.gpu
@pytest.mark.parametrize("splits", [1, 3])
def test_gemm_pp_drelu_mask_epilogue(splits):
    """act='drelu': y = (mask > 0) ? x.w^T + b : 0 — the ReLU backward of a training step's
    dX GEMM, in the direct epilogue and in the split-K reduction."""
    g = torch.Generator(device=DEV).manual_seed(5)
    M, N, Kd = 1000, 512, 768
    x = torch.randn(M, Kd, generator=g, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, Kd, generator=g, device=DEV) / Kd ** 0.5).to(torch.bfloat16)
    h = torch.randn(M, N, generator=g, device=DEV).to(torch.bfloat16)
    got = K.gemm_pp(x, w, None, h, "drelu", splits=splits)
    ref = torch.where(h.float() > 0, x.float() @ w.float().t(), 0.0)
    torch.cuda.synchronize()
    assert bool((got[h <= 0] == 0).all())
    _close(got, ref)
    host = K.gemm_pp(x.cpu(), w.cpu(), None, h.cpu(), "drelu")
    _close(host, ref.cpu())
