"""Collective online training over uneven streams.

``LockstepTrainer`` is a ``ModelCoProcessFunction`` — the reference's home for a model fed
by a data stream and a control stream (``AbstractCoProcessFunction.scala:11-16``) — whose
P parallel subtasks are the ranks of one data-parallel trainer (the job communicator,
``runtime/remote.py``).  Input 1 carries training records, input 2 control commands
(``"eval"``).  Every collective the trainer issues happens inside an agreed ROUND
(``parallel/step_agreement.py``), so the ranks never disagree about how many steps,
snapshots or row refreshes there are:

* a rank calls a round when it holds a full micro-batch, when its heartbeat timer fires
  (every ``max_delay_ms``: an idle rank — empty partition, skewed key, slow source — still
  takes part, so a peer with data waits at most that long), on an eval command, at a
  checkpoint barrier and at end of input;
* each round's step trains the pieces the ranks bring (``WideDeepTrainer.train_step(piece,
  counts=...)``: loss normalised by the round's global record count, zero gradients and no
  sparse rows from a rank with an empty piece);
* a barrier: the rank keeps taking part in rounds (bringing its buffered pre-barrier
  records) until every rank still running waits at the same barrier; then all snapshot
  after the same step — the trainer's snapshot is collective-free
  (``WideDeepTrainer.snapshot_state``: owner shards), the unconsumed records and counters
  go into operator state;
* an eval: in the round that carries the request every rank runs the row refresh for it
  (a collective under the owner exchange; ranks without a request refresh nothing), then
  the requesting rank scores its held-out records locally;
* end of input: the rank keeps taking part until every rank has ended and no records are
  left anywhere; then ``on_finished`` runs on all ranks at the same point (a safe place
  for a final collective, e.g. a replica digest).

Without a communicator (P = 1) the same code runs with a local table.
"""
from __future__ import annotations

import time

from .model_functions import ModelCoProcessFunction


class LockstepTrainer(ModelCoProcessFunction):
    def __init__(self, model, batch: int, max_delay_ms: float = 20.0, eval_records=None):
        super().__init__(model)
        self.batch = int(batch)
        self.max_delay_s = max_delay_ms / 1e3
        self.eval_records = eval_records
        self.buf: list = []
        self.steps = 0
        self.pending_evals = 0
        self.barriers = 0
        self._agree = None
        self._finished = False

    # ---- lifecycle
    def open(self, config=None):
        super().open(config)
        from ..parallel.step_agreement import StepAgreement

        self._agree = StepAgreement()

    @property
    def rank(self) -> int:
        return self._agree.rank if self._agree is not None else 0

    def on_start(self, ctx, out):
        self._arm(ctx)

    def _arm(self, ctx):
        ctx.timer_service().register_processing_time_timer(time.time() + self.max_delay_s)

    # ---- inputs
    def process_element1(self, rec, ctx, out):
        self.buf.append(rec)
        while len(self.buf) >= self.batch:
            self._round(out)

    def process_element2(self, cmd, ctx, out):
        if cmd == "eval" and self.eval_records:
            self.pending_evals += 1
            self._round(out)

    def on_timer(self, ts, ctx, out):  # heartbeat
        if self._finished:
            return
        self._round(out)
        self._arm(ctx)

    def on_barrier(self, ctx, out):
        if self._finished:
            return
        self.barriers += 1
        while True:
            plan = self._round(out, barrier=self.barriers)
            # every rank still running waits at this barrier (a rank whose input ended
            # takes no further checkpoints)
            live = [b for b, e in zip(plan.barrier, plan.ended) if not e]
            if live and all(b == self.barriers for b in live):
                return

    def on_end_of_input(self, ctx, out):
        if self._finished:
            return
        while not self._round(out, ended=True).finished:
            pass
        self._finished = True
        self.on_finished(out)

    # ---- the round
    def _round(self, out, ended: bool = False, barrier: int = -1):
        n = min(len(self.buf), self.batch)
        plan = self._agree.round(n, ended, barrier, self.pending_evals)
        if plan.step:
            piece, self.buf = self.buf[:n], self.buf[n:]
            loss = self.model.train_step(piece, counts=plan.counts)
            self.steps += 1
            self.on_step(plan, piece, loss, out)
        if any(plan.evals):
            mine = self.pending_evals > 0
            self.model.refresh_rows(self.eval_records if mine else None)
            if mine:
                self.pending_evals -= 1
                self.on_eval(self.model.predict(self.eval_records), out)
        return plan

    # ---- outputs (override to shape them)
    def on_step(self, plan, piece, loss, out):
        # a device scalar on a GPU (a captured step reuses its buffer): keep a copy, no sync
        out.collect(("train", self.steps, self.rank, len(piece), plan.total,
                     loss.clone() if hasattr(loss, "clone") else loss))

    def on_eval(self, probs, out):
        import numpy as np

        p = np.clip(np.asarray(probs, np.float64), 1e-7, 1 - 1e-7)
        y = np.asarray([r[0] for r in self.eval_records], np.float64)
        out.collect(("eval", self.steps, self.rank, float(-np.mean(y * np.log(p) + (1 - y) * np.log(1 - p)))))

    def on_finished(self, out):  # noqa: B027
        """Every rank reaches this together after the last agreed round."""

    # ---- checkpoints: the model's (collective-free) state + the unconsumed records
    def snapshot_state(self, ctx):
        super().snapshot_state(ctx)
        ctx.operator_state.blobs["lockstep"] = {"buf": list(self.buf), "steps": self.steps,
                                                "barriers": self.barriers, "evals": self.pending_evals}

    def initialize_state(self, ctx):
        super().initialize_state(ctx)
        st = ctx.operator_state.blobs.get("lockstep") if ctx.is_restored() else None
        if st:
            self.buf = list(st["buf"])
            self.steps, self.barriers, self.pending_evals = st["steps"], st["barriers"], st["evals"]
