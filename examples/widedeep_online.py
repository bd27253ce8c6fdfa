#!/usr/bin/env python3
"""Wide&Deep online training as a streaming job (BASELINE config 4).

    python examples/widedeep_online.py [--records 400000] [--batch 4096] [--cpu]
                                       [--checkpoint-dir DIR] [--eval-every 0.5]

The job shape of the reference's streaming examples (``inception.scala:21-51``: a source,
one model operator, a sink), with the model operator the reference reserves for online
training — the co-process function (``AbstractCoProcessFunction.scala:11-16``):

    click source ──────────────┐
                               ├─ connect ─ ModelCoProcessFunction(WideDeepTrainer) ─ sink
    control source (eval ticks)┘

* input 1 (click records): buffered into micro-batches of ``--batch`` records (or whatever
  arrived within ``--max-delay-ms``, via a processing-time timer); each micro-batch is one
  training step — the hand-fused GPU step replayed as a hipGraph (forward, backward on the
  MFMA training GEMM, sparse Adagrad on the radix-sorted rows, Adam);
* input 2 (control): an ``eval`` tick scores a held-out micro-batch with the current model
  and emits its log-loss;
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
from flink_tensorflow_amd.runtime.model_functions import ModelCoProcessFunction  # noqa: E402
from flink_tensorflow_amd.runtime.sources import CollectionSource  # noqa: E402


class OnlineTrainer(ModelCoProcessFunction):
    """Clicks -> micro-batched training steps; control ticks -> held-out evaluation."""

    def __init__(self, model, batch: int, max_delay_ms: float, heldout):
        self._model = model
        self.batch = batch
        self.max_delay_s = max_delay_ms / 1e3
        self.heldout = heldout
        self.buf: list = []
        self.steps = 0
        self.t_first = None

    @property
    def model(self):
        return self._model

    def _train(self, out):
        if not self.buf:
            return
        recs, self.buf = self.buf, []
        if self.t_first is None:
            self.t_first = time.perf_counter()
        m = self.model
        if m.model.device.type == "cuda" and m._graph is None and len(recs) == self.batch:
            m.capture(m.collate(recs))  # whole step as one hipGraph for full micro-batches
        loss = m.train_step(recs)
        self.steps += 1
        # a device scalar (the captured step's loss buffer is reused): keep a copy, no sync
        out.collect(("train", self.steps, len(recs), loss.clone() if hasattr(loss, "clone") else loss))

    def process_element1(self, rec, ctx, out):
        if self.t_first is None and not self.buf:  # end of input trains the last partial batch
            ctx.timer_service().register_event_time_timer(float("inf"))
        if not self.buf:  # first record of a micro-batch: arm its deadline
            ctx.timer_service().register_processing_time_timer(time.time() + self.max_delay_s)
        self.buf.append(rec)
        if len(self.buf) >= self.batch:
            self._train(out)

    def on_timer(self, ts, ctx, out):
        self._train(out)

    def process_element2(self, tick, ctx, out):
        if tick == "eval":
            p = np.clip(np.asarray(self.model.predict(self.heldout), np.float64), 1e-7, 1 - 1e-7)
            y = np.asarray([r[0] for r in self.heldout], np.float64)
            out.collect(("eval", self.steps, len(y), float(-np.mean(y * np.log(p) + (1 - y) * np.log(1 - p)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=400_000)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--max-delay-ms", type=float, default=20.0)
    ap.add_argument("--eval-every", type=float, default=0.5, help="seconds between eval ticks")
    ap.add_argument("--checkpoint-dir", default=None)
    ap.add_argument("--cpu", action="store_true", help="tiny model on the host (plumbing check)")
    ap.add_argument("--parallelism", type=int, default=1,
                    help="P > 1: P worker-process ranks (one per GPU) of ONE data-parallel trainer, kept in "
                         "lockstep over the uneven rebalanced stream (runtime/lockstep.py)")
    a = ap.parse_args()

    import torch

    gpu = torch.cuda.is_available() and not a.cpu
    cfg = WideDeepConfig() if gpu else WideDeepConfig.tiny()
    batch = a.batch if gpu else min(a.batch, 256)
    n = a.records if gpu else min(a.records, 8 * batch)
    recs = synthetic_click_records(n + batch, cfg, seed=7)
    heldout, recs = recs[:batch], recs[batch:]
    n_ticks = max(1, int(math.ceil(3.0 / max(1e-3, a.eval_every))))

    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(a.parallelism)
    if a.checkpoint_dir:
        env.enable_checkpointing(1.0, a.checkpoint_dir)
    clicks = env.add_source(CollectionSource(recs), "clicks", parallelism=1)
    ticks = env.add_source(CollectionSource(["eval"] * n_ticks, delay_s=a.eval_every), "control", parallelism=1)
    if a.parallelism > 1:  # the subtasks form the job communicator (RCCL, one GPU each)
        env.enable_job_communicator(True)
        trainer = WideDeepTrainer(cfg, device=None if gpu else "cpu", seed=0)  # None: the subtask's GPU
        fn = LockstepTrainer(trainer, batch, a.max_delay_ms, heldout)
        sink = clicks.rebalance().connect(ticks).process(fn).name("widedeep-online").run_in_processes().collect_into()
    else:
        trainer = WideDeepTrainer(cfg, device="cuda" if gpu else "cpu", seed=0)
        fn = OnlineTrainer(trainer, batch, a.max_delay_ms, heldout)
        sink = clicks.connect(ticks).process(fn).name("widedeep-online").collect_into()
    t0 = time.perf_counter()
    res = env.execute("widedeep-online")
    wall = time.perf_counter() - t0
    out = sink.results()
    train = [o for o in out if o[0] == "train"]
    evals = [o for o in out if o[0] == "eval"]
    if a.parallelism > 1:  # ("train", step, rank, n, total, loss): one line per rank and step
        trained = sum(o[3] for o in train)
        train = sorted((o for o in train if o[2] == 0), key=lambda o: o[1])
        train = [(o[0], o[1], o[4], o[5]) for o in train]
    else:
        trained = sum(o[2] for o in train)
    print(json.dumps({
        "job": "widedeep-online", "device": "gpu" if gpu else "cpu", "records_trained": trained,
        "steps": len(train), "records_per_s_wall": round(trained / wall, 1), "wall_s": round(wall, 2),
        "first_loss": round(float(train[0][3]), 4) if train else None,
        "last_loss": round(float(train[-1][3]), 4) if train else None,
        "eval_losses": [round(e[3], 4) for e in evals], "checkpoints": len(res.checkpoints)}), flush=True)


if __name__ == "__main__":
    main()
