import sys, torch
sys.path.insert(0, '.')
from flink_tensorflow_amd import _ext
h = _ext.hip()
out = torch.zeros(64 * 4, dtype=torch.int16, device="cuda")
h.probe_tr_read(out.data_ptr(), 0, torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
o = out.cpu().view(64, 4).tolist()
for lane in range(0, 64):
    print(lane, [(v // 256, v % 256) for v in o[lane]])
