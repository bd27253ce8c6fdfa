"""The data-parallel Wide&Deep step with the fixed-capacity owner exchange at RCCL world
size 1, for kernel traces (``rocprofv3 --kernel-trace --stats -- python3
tools/wd_bucketed_trace.py``): warm-up steps, the capture (2 warm-up + 1 calibrated step),
then ``--eager`` uncaptured steps and ``--replays`` graph replays.  Every step runs the
exchange's pull / push (radix unique, owner_buckets, RCCL all-to-alls, row gather /
scatter) and the fused step's kernels; the trace shows which kernels one DP step launches.
Prints one JSON line (step times, bucket capacities, overflow)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--eager", type=int, default=5)
    ap.add_argument("--replays", type=int, default=20)
    ap.add_argument("--tiny", action="store_true")
    a = ap.parse_args()
    import torch

    from flink_tensorflow_amd import _ext
    from flink_tensorflow_amd.models.zoo.wide_deep import (PackedBatchStager, WideDeepConfig, WideDeepTrainer,
                                                           pack_click_records, synthetic_click_records)
    from flink_tensorflow_amd.parallel import comm
    from flink_tensorflow_amd.parallel.sparse_exchange import BucketedOwnerExchange

    dev = torch.device("cuda", 0)
    c = comm.RcclCommunicator(0, 1, dev, unique_id=_ext.rccl().unique_id())
    comm.set_communicator(c)
    cfg = WideDeepConfig.tiny() if a.tiny else WideDeepConfig()
    B = 64 if a.tiny else a.batch
    t = WideDeepTrainer(cfg, device=dev, seed=0)
    t.open()
    ex = BucketedOwnerExchange(c)
    t._exchange = ex
    if t._fused is not None:
        t._fused.exchange = ex
    nx = min(8, cfg.num_fields - 1)
    rows = list(pack_click_records(synthetic_click_records(8 * B, cfg, seed=1, n_cross=nx), cfg, nx))
    stager = PackedBatchStager(cfg, B, dev, n_cross=nx)
    batches = [tuple(x.clone() for x in stager.stage(rows[i * B:(i + 1) * B])) for i in range(8)]
    for i in range(2):
        t.train_step(batch=batches[i])
    t.capture(batches[0])
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    g, t._graph = t._graph, None  # eager steps on the calibrated buckets
    for i in range(a.eager):
        t.train_step(batch=batches[i % 8])
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    t._graph = g
    for i in range(a.replays):
        t.train_step(batch=batches[i % 8])
    torch.cuda.synchronize(dev)
    t2 = time.perf_counter()
    ex.check()
    print(json.dumps({"batch": B, "eager_ms_per_step": round((t1 - t0) * 1e3 / max(1, a.eager), 3),
                      "replay_ms_per_step": round((t2 - t1) * 1e3 / max(1, a.replays), 3),
                      "captured": t._graph is not None, "bucket_capacities": {str(k): v for k, v in ex._caps.items()},
                      "overflow": int(ex.over.item())}), flush=True)
    del g  # the captured graph (RCCL kernels inside) goes before the communicator
    t.close()
    torch.cuda.synchronize(dev)
    comm.destroy()


if __name__ == "__main__":
    main()
