"""Wide&Deep data-parallel replica check under ``torch.distributed.run`` (any world size):
every rank trains the fused GPU step on its own synthetic records for a few steps with the
given communicator (``--fake``: the loopback test communicator, so several ranks can share
one GPU; default RCCL on ``cuda:LOCAL_RANK``), then prints one JSON line with checksums of
all dense parameters and both embedding tables.  Replicas must agree bit for bit: dense
gradients are all-reduced; row-sparse gradients go to the rows' owners (the owner exchange,
``parallel/sparse_exchange.py``: tables compared as merged owner shards) or are all-gathered
and merged deterministically (``FT_WD_SPARSE_EXCHANGE=allgather``)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fake", action="store_true")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--fused", type=int, default=1)
    a = ap.parse_args()
    import torch

    from flink_tensorflow_amd.models.zoo.wide_deep import WideDeepConfig, WideDeepTrainer, synthetic_click_records
    from flink_tensorflow_amd.parallel import comm

    rank, ws, local = comm.world()
    dev = torch.device("cuda", 0 if a.fake else comm.local_device(local))
    if a.fake:
        from flink_tensorflow_amd.parallel.fake import FakeCommunicator

        comm.set_communicator(FakeCommunicator(rank, ws, dev, comm.rendezvous_store(rank, ws)))
    else:
        comm.init_distributed(device=dev)
    cfg = WideDeepConfig.tiny(hidden=(128, 64), embed_dim=16)
    tr = WideDeepTrainer(cfg, device=dev, seed=7 + rank, fused=bool(a.fused))  # different init: rank 0's wins
    tr.open()
    recs = synthetic_click_records(256 * a.steps, cfg, seed=100 + rank)
    losses = [float(tr.train_step(recs[i * 256:(i + 1) * 256])) for i in range(a.steps)]
    torch.cuda.synchronize(dev)
    sd = dict(tr.model.state_dict())
    if tr._exchange is not None:  # owner-authoritative rows / Adagrad state: the merged shards
        for name in ("emb", "wide"):
            e = getattr(tr.model, name)
            sd[f"{name}.table"] = tr._exchange.merge_owner_shards(e.table.data)
            sd[f"{name}.accum"] = tr._exchange.merge_owner_shards(e.accum)
    sums = {k: [float(v.double().sum()), float(v.double().abs().sum())] for k, v in sorted(sd.items())}
    sys.stdout.write(json.dumps({"rank": rank, "fused": tr._fused is not None, "losses": losses, "sums": sums}) + "\n")  # one write per record
    sys.stdout.flush()
    tr.close()
    comm.destroy()


if __name__ == "__main__":
    main()
