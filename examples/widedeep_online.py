#!/usr/bin/env python3
"""Wide&Deep online training as a streaming job (BASELINE config 4).

    python examples/widedeep_online.py [--records 400000] [--batch 4096] [--parallelism P]
                                       [--cpu] [--checkpoint-dir DIR] [--control-stream]

One DataStream job of P worker-process subtasks (one GPU each) running the lockstep
trainer (``runtime/lockstep.py``) — the reference's online-training operator, the
co-process function (``AbstractCoProcessFunction.scala:11-16``):

* each rank's clicks are generated in its own worker (``env.generate``, chained into the
  trainer) as blocks of packed 192-B rows; micro-batches of ``--batch`` records are
  training steps agreed across the ranks in rounds of up to ``--steps-per-round`` (the
  captured, padded fused GPU step: forward, backward on the MFMA training GEMM, sparse
  Adagrad on the radix-sorted rows, Adam; gradients all-reduced over RCCL when P > 1);
* ``--control-stream``: the reference's two-input shape — one coordinator click source
  rebalanced to the ranks, connected with a control stream whose ``eval`` ticks score a
  held-out batch (every record crosses the coordinator: the slower plumbing);
* the trainer is a ``CheckpointedModel``: with ``--checkpoint-dir`` the aligned barriers
  snapshot its weights, tables and optimizer state into bundle-V2 files.

Prints one JSON line: records/s trained, steps, first / last training loss, eval losses.
Data: synthetic Criteo-shaped clicks (13 dense, 26 categorical, 8 crossed features) with a
planted logistic signal, so the loss falls as the stream is consumed; random init.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flink_tensorflow_amd.models.zoo.wide_deep import (WideDeepConfig, WideDeepTrainer,  # noqa: E402
                                                       synthetic_click_records)
from flink_tensorflow_amd.runtime import StreamExecutionEnvironment  # noqa: E402
from flink_tensorflow_amd.runtime.lockstep import LockstepTrainer  # noqa: E402
from flink_tensorflow_amd.runtime.sources import CollectionSource  # noqa: E402


class EvalAtEnd(LockstepTrainer):
    """The lockstep trainer on one input (the click stream generated in each worker): the
    held-out log-loss is emitted once the stream has been trained on (the co-process form
    with a control stream of eval ticks is ``--control-stream``)."""

    def on_finished(self, out):
        self.on_eval(self.model.predict(self.eval_records), out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=400_000)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--max-delay-ms", type=float, default=20.0)
    ap.add_argument("--eval-every", type=float, default=0.5, help="seconds between eval ticks (--control-stream)")
    ap.add_argument("--checkpoint-dir", default=None)
    ap.add_argument("--cpu", action="store_true", help="tiny model on the host (plumbing check)")
    ap.add_argument("--parallelism", type=int, default=1,
                    help="P worker-process ranks (one per GPU) of ONE data-parallel trainer, kept in lockstep "
                         "(runtime/lockstep.py); each rank's clicks are generated in its own worker")
    ap.add_argument("--steps-per-round", type=int, default=8, help="agreed steps per lockstep round")
    ap.add_argument("--control-stream", action="store_true",
                    help="the reference's co-process shape: clicks from ONE coordinator source rebalanced to the "
                         "ranks, connected with a control stream of eval ticks (slower: every record crosses the "
                         "coordinator)")
    a = ap.parse_args()

    import torch

    from flink_tensorflow_amd.models.zoo.wide_deep import pack_click_records
    from flink_tensorflow_amd.runtime import RestartStrategy

    gpu = torch.cuda.is_available() and not a.cpu
    cfg = WideDeepConfig() if gpu else WideDeepConfig.tiny()
    batch = a.batch if gpu else min(a.batch, 256)
    n = a.records if gpu else min(a.records, 8 * batch)
    P = a.parallelism
    heldout = synthetic_click_records(batch, cfg, seed=1000)
    n_ticks = max(1, int(math.ceil(3.0 / max(1e-3, a.eval_every))))

    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(P)
    if a.checkpoint_dir:
        env.enable_checkpointing(1.0, a.checkpoint_dir)
    if P > 1:  # the subtasks form the job communicator (RCCL, one GPU each)
        env.enable_job_communicator(True)
        if os.environ.get("FT_WD_SPARSE_EXCHANGE", "owner") == "bucketed":  # overflow -> restart
            env.set_restart_strategy(RestartStrategy.fixed_delay(1, 0.0))
    trainer = WideDeepTrainer(cfg, device=(None if P > 1 else "cuda") if gpu else "cpu", seed=0)
    if a.control_stream:
        recs = synthetic_click_records(n, cfg, seed=7)
        clicks = env.add_source(CollectionSource(recs), "clicks", parallelism=1)
        ticks = env.add_source(CollectionSource(["eval"] * n_ticks, delay_s=a.eval_every), "control", parallelism=1)
        fn = LockstepTrainer(trainer, batch, a.max_delay_ms, heldout, steps_per_round=a.steps_per_round)
        sink = clicks.rebalance().connect(ticks).process(fn).name("widedeep-online").run_in_processes().collect_into()
    else:
        per = -(-n // P)

        def clicks(idx, par, start):  # runs in rank idx's worker: blocks of packed 192-B click rows
            rows = pack_click_records(synthetic_click_records(per, cfg, seed=7 + idx), cfg)
            for lo in range(start, per, batch):
                yield rows[lo:lo + batch]

        fn = EvalAtEnd(trainer, batch, a.max_delay_ms, heldout, steps_per_round=a.steps_per_round)
        sink = env.generate(clicks).run_in_processes().process(fn, "widedeep-online").run_in_processes() \
            .collect_into()
    t0 = time.perf_counter()
    res = env.execute("widedeep-online")
    wall = time.perf_counter() - t0
    out = sink.results()
    train = [o for o in out if o[0] == "train"]
    evals = [o for o in out if o[0] == "eval"]
    # ("train", step, rank, n, total, loss): one line per rank and step
    trained = sum(o[3] for o in train)
    train = sorted((o for o in train if o[2] == 0), key=lambda o: o[1])
    print(json.dumps({
        "job": "widedeep-online", "device": "gpu" if gpu else "cpu", "parallelism": P,
        "source": "coordinator + control stream" if a.control_stream else "generated in each worker",
        "records_trained": trained, "steps": len(train), "records_per_s_wall": round(trained / wall, 1),
        "wall_s": round(wall, 2), "first_loss": round(float(train[0][5]), 4) if train else None,
        "last_loss": round(float(train[-1][5]), 4) if train else None,
        "eval_losses": [round(e[3], 4) for e in evals], "checkpoints": len(res.checkpoints)}), flush=True)


if __name__ == "__main__":
    main()
