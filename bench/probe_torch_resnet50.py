"""Library baseline probe: plain PyTorch-ROCm (MIOpen/hipBLASLt) ResNet-50 bf16 inference.

Used only to size the target our hand-written kernels must beat; not part of the product path.
"""
import time, json, sys
import torch
import torch.nn as nn
import torch.nn.functional as F


class Bottleneck(nn.Module):
    def __init__(self, cin, mid, cout, stride):
        super().__init__()
        self.c1 = nn.Conv2d(cin, mid, 1, bias=False); self.b1 = nn.BatchNorm2d(mid)
        self.c2 = nn.Conv2d(mid, mid, 3, stride, 1, bias=False); self.b2 = nn.BatchNorm2d(mid)
        self.c3 = nn.Conv2d(mid, cout, 1, bias=False); self.b3 = nn.BatchNorm2d(cout)
        self.down = None
        if stride != 1 or cin != cout:
            self.down = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        idt = x if self.down is None else self.down(x)
        y = F.relu(self.b1(self.c1(x)))
        y = F.relu(self.b2(self.c2(y)))
        y = self.b3(self.c3(y))
        return F.relu(y + idt)


class ResNet50(nn.Module):
    def __init__(self):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(), nn.MaxPool2d(3, 2, 1))
        layers = []
        cin = 64
        for mid, n, s in [(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]:
            for i in range(n):
                layers.append(Bottleneck(cin, mid, mid * 4, s if i == 0 else 1)); cin = mid * 4
        self.layers = nn.Sequential(*layers)
        self.fc = nn.Linear(2048, 1000)

    def forward(self, x):
        x = self.layers(self.stem(x))
        return self.fc(x.mean((2, 3)))


def main():
    dev = torch.device("cuda")
    print(torch.cuda.get_device_properties(0), flush=True)
    m = ResNet50().eval().to(dev).to(torch.bfloat16).to(memory_format=torch.channels_last)
    res = {}
    for B in [int(b) for b in (sys.argv[1:] or ["1", "64", "256"])]:
        x = torch.randn(B, 3, 224, 224, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        with torch.no_grad():
            for _ in range(3):
                m(x)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):
                    m(x)
            torch.cuda.current_stream().wait_stream(s)
            with torch.cuda.graph(g):
                y = m(x)
            for _ in range(3):
                g.replay()
            torch.cuda.synchronize()
            n = max(5, 2000 // B)
            t = time.perf_counter()
            for _ in range(n):
                g.replay()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) / n
        res[B] = {"ms": dt * 1e3, "img_s": B / dt}
        print(json.dumps({"B": B, "ms": round(dt * 1e3, 3), "img_per_s": round(B / dt, 1)}), flush=True)


if __name__ == "__main__":
    main()
