"""Step agreement for collective training on uneven streams.

Every step of a data-parallel trainer is collective (the dense all-reduce, the sparse
row exchange), so every rank must run the same number of steps.  In a streaming job the
ranks' inputs are uneven: a rebalance leaves a remainder, a key skews, one rank's input
ends before another's, a checkpoint barrier or an eval request reaches one rank first.
Counting full micro-batches per rank hangs the job the first time those counts differ.

The protocol: time is cut into ROUNDS.  In each round every rank publishes one small
vector — how many records it brings, whether its input has ended, the checkpoint barrier
it is waiting at, whether it has an eval request — with one all-gather, and every rank
derives the same decision from the same table:

* some rank brings records → everyone runs ONE step; a rank with nothing enters it with
  zero gradients and no sparse rows, and the loss is normalised by the round's global
  record count, so the step is the gradient of the mean over the union of the pieces;
* every rank is waiting at the same barrier → everyone snapshots after this round (the
  snapshot is taken at the same step on every rank: a consistent distributed checkpoint
  with collective-free ``snapshot_state``);
* a rank has an eval request → everyone runs the (collective) row refresh for it;
* every rank's input has ended and nobody brings records → training is over (end of
  input is itself agreed, so no rank leaves while a peer still steps).

A rank calls ``round`` when it has a full micro-batch, when its heartbeat deadline passes
(``max_delay``: an idle rank still takes part, so a busy peer waits at most that long), at
a barrier and at end of input.  Rounds pair up by sequence number, so no rank can enter a
step its peers skip.  The single-rank case needs no communicator (the table is local).

The reference has no training; its home for an online-training operator is
the co-process function (``AbstractCoProcessFunction.scala:11-16``), which
``runtime/lockstep.py`` builds on this.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from . import comm as _comm

_FIELDS = 4  # records, ended, barrier (-1 none), eval requests


@dataclass(frozen=True)
class RoundPlan:
    """The decision of one round, identical on every rank."""

    counts: tuple[int, ...]     # records each rank brings to this round's step
    ended: tuple[bool, ...]     # rank's input is exhausted
    barrier: tuple[int, ...]    # barrier sequence number the rank waits at (-1: none)
    evals: tuple[int, ...]      # eval requests pending on the rank
    index: int = 0              # round number (same on every rank)

    @property
    def total(self) -> int:
        return sum(self.counts)

    @property
    def step(self) -> bool:
        return self.total > 0

    @property
    def finished(self) -> bool:
        return all(self.ended) and not self.step and not any(self.evals)

    @property
    def snapshot_barrier(self) -> int | None:
        """The barrier every rank waits at (snapshot after this round), else None."""
        b = set(self.barrier)
        return self.barrier[0] if len(b) == 1 and self.barrier[0] >= 0 else None


class StepAgreement:
    """One all-gather of a 4-int vector per round (``comm`` None or world 1: local)."""

    def __init__(self, communicator=None):
        c = communicator
        if c is None and _comm.is_dist():
            c = _comm.get()
        self.comm = c if c is not None and c.size > 1 else None
        self.rank = self.comm.rank if self.comm is not None else 0
        self.size = self.comm.size if self.comm is not None else 1
        self.rounds = 0

    def round(self, n: int, ended: bool = False, barrier: int = -1, evals: int = 0) -> RoundPlan:
        mine = [int(n), int(bool(ended)), int(barrier), int(evals)]
        idx = self.rounds
        self.rounds += 1
        if self.comm is None:
            return RoundPlan((mine[0],), (bool(mine[1]),), (mine[2],), (mine[3],), idx)
        dev = self.comm.device
        t = torch.tensor(mine, dtype=torch.int64, device=dev)
        out = torch.empty(self.size * _FIELDS, dtype=torch.int64, device=dev)
        self.comm.all_gather(out, t)
        tab = out.view(self.size, _FIELDS).cpu().tolist()  # host sync: the decision is taken on the host
        return RoundPlan(tuple(r[0] for r in tab), tuple(bool(r[1]) for r in tab), tuple(r[2] for r in tab),
                         tuple(r[3] for r in tab), idx)
