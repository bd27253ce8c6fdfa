"""Debug print for conv2d_nhwc_fp8_multi vs its host reference: per segment, how many
elements differ and at which channels / pixels."""
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402

from flink_tensorflow_amd.ops import fp8 as Q  # noqa: E402

DEV = torch.device("cuda", 0)
torch.manual_seed(6)
N, H, W, C = 2, 13, 11, 96
x = torch.randn(N, H, W, C).relu()
sx = Q.scale_for(x.abs().max())
xq = Q.quantize(x, sx)
couts = (64, 48, 32, 16)
w = torch.randn(sum(couts), C) / C ** 0.5
wq, ws = Q.quantize_weight(w)
b = torch.randn(sum(couts)) * 0.1
lo = torch.tensor([0.0] * (64 + 48) + [float("-inf")] * 48)


def outs(dev):
    return [torch.zeros((N, H, W, 128), dtype=torch.uint8, device=dev),
            torch.zeros((N, H, W, 48), dtype=torch.uint8, device=dev),
            torch.zeros((N, H, W, 32), dtype=torch.bfloat16 if dev != "cpu" else torch.float32, device=dev),
            torch.zeros((N, H, W, 16), dtype=torch.uint8, device=dev)]


def segs(o):
    return [(o[0], 0, 64, 32, 0.02), (o[1], 64, 112, 0, 0.05), (o[2], 112, 144, 0, None), (o[3], 144, 160, 0, 0.01)]


ref = outs("cpu")
Q.conv2d_nhwc_fp8_multi(xq, sx, wq, (1, 1), ws, b, lo, segs(ref))
got = outs(DEV)
Q.conv2d_nhwc_fp8_multi(xq.to(DEV), sx, wq.to(DEV), (1, 1), ws.to(DEV), b.to(DEV), lo.to(DEV), segs(got))
torch.cuda.synchronize()
single = Q.conv2d_nhwc_fp8(xq.to(DEV), sx, wq.to(DEV), (1, 1), ws.to(DEV), b.to(DEV), act=None, cfg=8).float().cpu()
print("single-output lite (bf16) vs host conv:", (single - Q.conv2d_nhwc_fp8(xq, sx, wq, (1, 1), ws, b, act=None)).abs().max())
for i, (r, g) in enumerate(zip(ref, got)):
    g = g.cpu()
    if r.dtype == torch.uint8:
        rd, gd = Q.from_fp8_bytes(r), Q.from_fp8_bytes(g)
    else:
        rd, gd = r.float(), g.float()
    bad = (gd - rd).abs() > 0.13 * rd.abs() + 1e-3
    print(i, "bad", int(bad.sum()), "of", bad.numel())
    if bad.any():
        idx = bad.nonzero()[:6]
        for t in idx.tolist():
            print("   ", t, float(rd[tuple(t)]), float(gd[tuple(t)]))
        print("   channels with errors:", sorted(set(bad.nonzero()[:, 3].tolist()))[:40])
        print("   pixels with errors:", len(set(map(tuple, bad.nonzero()[:, :3].tolist()))))
