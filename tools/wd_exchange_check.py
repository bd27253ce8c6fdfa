"""Row-sparse exchange check under ``torch.distributed.run`` (CPU, loopback communicator).

``--mode train``: every rank trains the Wide&Deep trainer (autograd path, tiny config) on
its own records twice — with the owner exchange (``parallel/sparse_exchange.py``) and with
the padded all-gather it replaces — and prints checksums of both tables, the merged
Adagrad state and the dense parameters for both runs: they must agree bit for bit, on
every rank.

``--mode overflow``: a bucketed exchange whose buckets are too small reports it
(``CapacityExceeded`` from ``check`` and from the delayed ``step_done`` check).

``--mode bytes``: the exchange alone at the benchmark's shapes (26 fields x 100k rows x 32,
wide 1,000,003 x 8, micro-batch 4096 per rank, Zipf ids of ``synthetic_click_records``):
prints the bytes this rank received in one step with each scheme.
"""
import argparse
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _digest(t) -> str:
    return hashlib.sha256(t.detach().cpu().contiguous().numpy().tobytes()).hexdigest()[:16]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["train", "bytes", "overflow"], default="train")
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    import torch

    from flink_tensorflow_amd import config as C
    from flink_tensorflow_amd.models.zoo.wide_deep import (WideDeepConfig, WideDeepTrainer, _sparse_sync,
                                                           synthetic_click_records)
    from flink_tensorflow_amd.parallel import comm
    from flink_tensorflow_amd.parallel.fake import FakeCommunicator

    rank, ws, _ = comm.world()
    comm.set_communicator(FakeCommunicator(rank, ws, "cpu", comm.rendezvous_store(rank, ws)))
    out = {"rank": rank, "world": ws}
    if a.mode == "train":
        cfg = WideDeepConfig.tiny(hidden=(32, 16), embed_dim=8, vocab_per_field=64, wide_buckets=257)
        recs = synthetic_click_records(128 * a.steps, cfg, seed=100 + rank)
        for mode in ("owner", "bucketed", "allgather"):
            C.set_current(C.EngineConfig(wd_sparse_exchange=mode))
            tr = WideDeepTrainer(cfg, device="cpu", seed=7 + rank, fused=False)
            tr.open()
            recv = []
            for i in range(a.steps):
                tr.train_step(recs[i * 128:(i + 1) * 128])
                if tr.exchange_stats is not None:
                    recv.append(tr.exchange_stats.received)
            m = tr.model
            acc, tab = {}, {}
            for name, e in (("emb", m.emb), ("wide", m.wide)):
                ex = tr._exchange
                acc[name] = ex.merge_owner_shards(e.accum) if ex is not None else e.accum
                tab[name] = ex.merge_owner_shards(e.table.data) if ex is not None else e.table
            out[mode] = {"emb": _digest(tab["emb"]), "wide": _digest(tab["wide"]),
                         "emb_accum": _digest(acc["emb"]), "wide_accum": _digest(acc["wide"]),
                         "dense": _digest(torch.cat([p.detach().reshape(-1) for p in m.dense_parameters()])),
                         "received": recv}
            tr.close()
    elif a.mode == "overflow":
        # every id owned by rank 0 and a small slack: rank 0's bucket cannot hold them
        from flink_tensorflow_amd.parallel.sparse_exchange import BucketedOwnerExchange, CapacityExceeded

        bx = BucketedOwnerExchange(comm.get(), slack=0.5, check_every=1)
        ids = torch.arange(0, 2000, 2, dtype=torch.int32)
        table = torch.zeros(4000, 8)
        accum = torch.full((4000, 8), 0.1)
        bx.pull(table, ids)
        bx.apply(table, accum, ids, torch.ones(ids.numel(), 8), 0.05)
        bx.step_done()  # schedules the sync-free copy of the counter
        raised = []
        for fn in (bx.check, bx.step_done):
            try:
                fn()
            except CapacityExceeded as e:
                raised.append(str(e)[:60])
        # a restarted job (attempt 2) opens its trainer with 4x the configured slack
        C.set_current(C.EngineConfig(wd_sparse_exchange="bucketed", wd_bucket_slack=1.5))
        tr = WideDeepTrainer(WideDeepConfig.tiny(), device="cpu", seed=7, fused=False)
        tr.restart_attempt = 2
        tr.open()
        out["overflow"] = {"capacity": bx.capacity(ids.numel(), 4000), "demand": int(bx.need.item()),
                           "raised": raised, "restart_slack": tr._exchange.slack}
        tr.close()
    else:
        cfg = WideDeepConfig()
        B = 4096
        recs = synthetic_click_records(B, cfg, seed=100 + rank)
        from flink_tensorflow_amd.ops.embedding import segment_sum
        from flink_tensorflow_amd.parallel.sparse_exchange import BucketedOwnerExchange, OwnerSparseExchange

        cats = torch.tensor([r[2] for r in recs], dtype=torch.int64)
        cross = torch.tensor([r[3] for r in recs], dtype=torch.int64)
        ids = (cats + torch.arange(cfg.num_fields) * cfg.vocab_per_field).reshape(-1)
        FV = cfg.num_fields * cfg.vocab_per_field
        ex = OwnerSparseExchange(comm.get())
        bx = BucketedOwnerExchange(comm.get())
        res = {}
        for name, V, D, keys in (("emb", FV, cfg.embed_dim, ids), ("wide", cfg.wide_buckets, 8, cross.reshape(-1))):
            g = torch.randn(keys.numel(), D)
            u, r = segment_sum(keys, g, V, static=True)
            table = torch.zeros(V, D)
            accum = torch.full((V, D), 0.1)
            ex.begin_step()
            ex.pull(table, u)
            ex.apply(table, accum, u, r, 0.05)
            st = ex.stats
            bx.begin_step()  # warm-up step: measures every site's demand
            bx.pull(table, u)
            bx.apply(table, accum, u, r, 0.05)
            bx.calibrate()  # buckets sized from it (what the trainer does before capturing)
            g2 = torch.randn(keys.numel(), D)
            u2, r2 = segment_sum(keys.flip(0), g2, V, static=True)  # another step, same ids
            bx.begin_step()
            bx.pull(table, u2)
            bx.apply(table, accum, u2, r2, 0.05)
            bx.check()
            # the padded all-gather receives (ws - 1) x (one id + one row) per lookup
            res[name] = {"owner_received": st.received, "rows_out": st.rows_out, "lookups": int(keys.numel()),
                         "bucketed_received": bx.stats.received, "bucket_capacity": bx.capacity(int(keys.numel()), V),
                         "bucket_demand": int(bx._site_need[(V, int(keys.numel()))].item()),
                         "allgather_received": (ws - 1) * int(keys.numel()) * (4 + 4 * D)}
            _sparse_sync  # noqa: B018 - the scheme priced above
        out["bytes"] = res
    sys.stdout.write(json.dumps(out) + "\n")
    sys.stdout.flush()
    comm.destroy()


if __name__ == "__main__":
    main()
