"""GPU count without touching the HIP runtime.

A launcher process (``bench.py --gpus N`` starting ``torch.distributed.run``) must not
initialise HIP before its ranks start: ``torch.cuda.device_count()`` goes through amdsmi on
ROCm and falls back to ``hipGetDeviceCount`` when that fails, which initialises the runtime
in the parent.  The KFD topology in sysfs lists every GPU agent (a node with a non-zero
``simd_count``; CPU nodes have none) and needs no library at all."""
from __future__ import annotations

import glob
import os

_VISIBLE = ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")


def sysfs_gpu_count(root: str = "/sys/class/kfd/kfd/topology/nodes") -> int:
    """GPUs the KFD driver exposes, narrowed by a ``*_VISIBLE_DEVICES`` list when one is
    set (the runtime applies the same masks)."""
    n = 0
    for props in glob.glob(os.path.join(root, "*", "properties")):
        try:
            with open(props) as f:
                for line in f:
                    k, _, v = line.partition(" ")
                    if k == "simd_count":
                        n += int(v) > 0
                        break
        except OSError:
            continue
    for var in _VISIBLE:
        v = os.environ.get(var)
        if v is not None:
            ids = [x for x in v.split(",") if x.strip() != ""]
            n = min(n, len(ids))
    return n
