"""Probe: torch.mm with out_dtype=float32 and out= on the GPU (bf16 operands)."""
import torch

a = torch.randn(64, 128, device="cuda").bfloat16()
b = torch.randn(128, 32, device="cuda").bfloat16()
o = torch.empty(64, 32, device="cuda")
try:
    torch.mm(a, b, out_dtype=torch.float32, out=o)
    print("mm out_dtype+out ok", torch.allclose(o, a.float() @ b.float(), atol=1e-1))
except Exception as e:  # noqa: BLE001
    print("mm out_dtype+out FAILED", type(e).__name__, str(e)[:200])
