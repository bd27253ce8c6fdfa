"""Times the fused s2d preprocess (uint8 256x256x3 -> bilinear 224x224 -> normalize -> bf16
2x2 space-to-depth [B,112,112,16], the ResNet-50 stem input) at B=256: the row-staged LDS
kernel vs the one-thread-per-pixel kernel (FTM_PREPROCESS_PIXEL=1), interleaved rounds."""
import json
import os
import sys

import torch

sys.path.insert(0, __file__.rsplit("/bench/", 1)[0])
from flink_tensorflow_amd.ops import kernels as K  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    img = torch.randint(0, 256, (B, 256, 256, 3), dtype=torch.uint8, device=dev)
    out = torch.empty((B, 112, 112, 16), dtype=torch.bfloat16, device=dev)
    mean, std = (123.68, 116.78, 103.94), (58.4, 57.12, 57.38)
    times = {"rows": [], "pixel": []}
    res = {}
    for rnd in range(8):
        for form in ("rows", "pixel"):
            if form == "pixel":
                os.environ["FTM_PREPROCESS_PIXEL"] = "1"
            else:
                os.environ.pop("FTM_PREPROCESS_PIXEL", None)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                K.preprocess_images(img, (224, 224), mean, std, out=out, s2d=True)
            e1.record()
            e1.synchronize()
            res[form] = out.clone()
            if rnd:
                times[form].append(e0.elapsed_time(e1) / 10 * 1e3)
    nbytes = img.numel() + out.numel() * 2
    # Inception-v3 form: 299 x 299 -> 299 x 299 (897-byte, unaligned rows), s2d [B,150,150,16]
    img2 = torch.randint(0, 256, (B, 299, 299, 3), dtype=torch.uint8, device=dev)
    out2 = torch.empty((B, 150, 150, 16), dtype=torch.bfloat16, device=dev)
    t2 = {"rows": [], "pixel": []}
    for rnd in range(8):
        for form in ("rows", "pixel"):
            if form == "pixel":
                os.environ["FTM_PREPROCESS_PIXEL"] = "1"
            else:
                os.environ.pop("FTM_PREPROCESS_PIXEL", None)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                K.preprocess_images(img2, (299, 299), mean, std, out=out2, s2d=True)
            e1.record()
            e1.synchronize()
            res[form + "299"] = out2.clone()
            if rnd:
                t2[form].append(e0.elapsed_time(e1) / 10 * 1e3)
    os.environ.pop("FTM_PREPROCESS_PIXEL", None)
    for form, ts in t2.items():
        us = sorted(ts)[len(ts) // 2]
        print(json.dumps({"batch": B, "hw": 299, "form": form, "us": round(us, 1),
                          "max_abs_diff_vs_pixel": float((res[form + "299"].float() - res["pixel299"].float()).abs().max())}))
    for form, ts in times.items():
        us = sorted(ts)[len(ts) // 2]
        print(json.dumps({"batch": B, "form": form, "us": round(us, 1), "TB_s": round(nbytes / us / 1e6, 2),
                          "max_abs_diff_vs_pixel": float((res[form].float() - res["pixel"].float()).abs().max())}))


if __name__ == "__main__":
    main()
