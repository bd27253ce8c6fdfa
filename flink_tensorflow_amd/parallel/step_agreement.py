"""Step agreement for collective training on uneven streams.

Every step of a data-parallel trainer is collective (the dense all-reduce, the sparse
row exchange), so every rank must run the same number of steps.  In a streaming job the
ranks' inputs are uneven: a rebalance leaves a remainder, a key skews, one rank's input
ends before another's, a checkpoint barrier or an eval request reaches one rank first.
Counting full micro-batches per rank hangs the job the first time those counts differ.

The protocol: time is cut into ROUNDS.  In each round every rank publishes one small
vector — how many full micro-batches it brings, the size of the partial piece it flushes
after them (0: none), whether its input has ended, the checkpoint barrier it is waiting
at, whether it has an eval request — and every rank derives the same decision from the
same table:

* the round runs ``k = max over ranks of (full + (partial > 0))`` steps; in step ``j`` a
  rank brings its ``j``-th piece, or nothing once it has none left — a rank with nothing
  enters the step with zero gradients and no sparse rows (on the GPU: a piece of padding
  rows, so every step has the captured step's shape), and the loss is normalised by the
  step's global record count, so each step is the gradient of the mean over the union of
  the pieces.  A busy rank therefore runs as many steps per round as it holds batches:
  an idle peer costs it one agreement per round, not one step per heartbeat;
* every rank is waiting at the same barrier → everyone snapshots after this round (the
  snapshot is taken at the same step on every rank: a consistent distributed checkpoint
  with collective-free ``snapshot_state``);
* a rank has an eval request → everyone runs the (collective) row refresh for it;
* every rank's input has ended and nobody brings records → training is over (end of
  input is itself agreed, so no rank leaves while a peer still steps).

The table travels over the HOST control channel when the communicator has one (the job's
rendezvous key/value store: ``HostChannel``), so agreeing never waits behind the training
collectives queued on the GPU — the host decides the next round while the previous
round's captured steps still run.  Without a store it is one all-gather on the
communicator.  Rounds pair up by sequence number, so no rank can enter a step its peers
skip.  The single-rank case needs no communicator (the table is local).

The reference has no training; its home for an online-training operator is
the co-process function (``AbstractCoProcessFunction.scala:11-16``), which
``runtime/lockstep.py`` builds on this.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass

import torch

from . import comm as _comm

_FIELDS = 6  # full batches, batch size, partial piece, ended, barrier (-1 none), eval requests


@dataclass(frozen=True)
class RoundPlan:
    """The decision of one round, identical on every rank."""

    pieces: tuple[tuple[int, ...], ...]  # per rank: the record counts of the pieces it brings
    ended: tuple[bool, ...]     # rank's input is exhausted
    barrier: tuple[int, ...]    # barrier sequence number the rank waits at (-1: none)
    evals: tuple[int, ...]      # eval requests pending on the rank
    index: int = 0              # round number (same on every rank)

    @property
    def k(self) -> int:
        """Steps this round runs."""
        return max((len(p) for p in self.pieces), default=0)

    def counts_at(self, j: int) -> tuple[int, ...]:
        """Records each rank brings to step ``j`` of the round."""
        return tuple(p[j] if j < len(p) else 0 for p in self.pieces)

    @property
    def counts(self) -> tuple[int, ...]:
        """Records per rank of the round's first step (all zero without a step)."""
        return self.counts_at(0)

    @property
    def total(self) -> int:
        """Records of the whole round."""
        return sum(sum(p) for p in self.pieces)

    @property
    def step(self) -> bool:
        return self.k > 0

    @property
    def finished(self) -> bool:
        return all(self.ended) and not self.step and not any(self.evals)

    @property
    def snapshot_barrier(self) -> int | None:
        """The barrier every rank waits at (snapshot after this round), else None."""
        b = set(self.barrier)
        return self.barrier[0] if len(b) == 1 and self.barrier[0] >= 0 else None


def _pieces(full: int, size: int, partial: int) -> tuple[int, ...]:
    return (size,) * full + ((partial,) if partial > 0 else ())


class HostChannel:
    """All-gather of small int vectors through the job's rendezvous key/value store: the
    control plane of ``StepAgreement``, off the GPU streams.  Round ``i`` lives under
    ``ctl/<i>/<rank>``; a rank entering round ``i`` deletes its key of round ``i - 2``
    (every peer has read it: they all published round ``i - 1``, which they could only do
    after reading ``i - 2``), so the store stays bounded."""

    def __init__(self, store, rank: int, size: int, prefix: str = "ctl"):
        self.store, self.rank, self.size, self.prefix = store, rank, size, prefix
        self.seq = 0

    def all_gather_ints(self, vec: list[int]) -> list[list[int]]:
        i = self.seq
        self.seq += 1
        n = len(vec)
        self.store.set(f"{self.prefix}/{i}/{self.rank}", struct.pack(f"<{n}q", *vec))
        if i >= 2:
            self.store.delete_key(f"{self.prefix}/{i - 2}/{self.rank}")
        keys = [f"{self.prefix}/{i}/{r}" for r in range(self.size)]
        vals = self.store.multi_get(keys)  # blocks until every rank has published
        return [list(struct.unpack(f"<{n}q", bytes(v))) for v in vals]


class StepAgreement:
    """One exchange of a 6-int vector per round (``comm`` None or world 1: local).

    ``control``: ``"host"`` (default when the communicator carries its rendezvous store:
    ``HostChannel``) or ``"device"`` (an all-gather on the communicator)."""

    def __init__(self, communicator=None, control: str | None = None):
        c = communicator
        if c is None and _comm.is_dist():
            c = _comm.get()
        self.comm = c if c is not None and c.size > 1 else None
        self.rank = self.comm.rank if self.comm is not None else 0
        self.size = self.comm.size if self.comm is not None else 1
        self.rounds = 0
        store = getattr(self.comm, "store", None) if self.comm is not None else None
        if control is None:
            control = "host" if store is not None else "device"
        if control == "host" and self.comm is not None and store is None:
            raise ValueError("StepAgreement: host control channel requested but the communicator has no store")
        self.control = control if self.comm is not None else "local"
        self._host = HostChannel(store, self.rank, self.size) if self.control == "host" else None

    def round(self, n: int = 0, ended: bool = False, barrier: int = -1, evals: int = 0, *,
              full: int = 0, batch: int = 0) -> RoundPlan:
        """This rank brings ``full`` pieces of ``batch`` records, then a partial piece of
        ``n`` records (``n`` may also be a whole batch: the one-piece form)."""
        mine = [int(full), int(batch), int(n), int(bool(ended)), int(barrier), int(evals)]
        idx = self.rounds
        self.rounds += 1
        if self.comm is None:
            tab = [mine]
        elif self._host is not None:
            tab = self._host.all_gather_ints(mine)
        else:
            dev = self.comm.device
            t = torch.tensor(mine, dtype=torch.int64, device=dev)
            out = torch.empty(self.size * _FIELDS, dtype=torch.int64, device=dev)
            self.comm.all_gather(out, t)
            tab = out.view(self.size, _FIELDS).cpu().tolist()  # host sync: the decision is taken on the host
        return RoundPlan(tuple(_pieces(r[0], r[1], r[2]) for r in tab), tuple(bool(r[3]) for r in tab),
                         tuple(r[4] for r in tab), tuple(r[5] for r in tab), idx)
