"""Test-only loopback communicator.

Runs the collective layer's logic — bucketing, rank routing, barrier alignment, metric
merging — in N CPU worker processes without GPUs, RCCL or gloo: every collective is a
round through the job's rendezvous key/value store (each rank publishes its bytes under a
sequence-numbered key, reads its peers', and reduces locally in rank order, so every rank
computes bit-identical results).  Semantics match ``RcclCommunicator`` (in place,
contiguous tensors, same reductions).  Never selected by product code; tests inject it
with ``comm.init_distributed(communicator=FakeCommunicator)``.
"""
from __future__ import annotations

import numpy as np
import torch

from .comm import Communicator


class FakeCommunicator(Communicator):
    capturable = False  # host round trips: never inside a hipGraph capture

    def __init__(self, rank: int, size: int, device="cpu", store=None):
        if store is None:
            raise ValueError("FakeCommunicator needs the rendezvous store")
        self.rank, self.size = rank, size
        self.device = torch.device(device)
        self._store = store
        self.store = store  # host control channel (parallel/step_agreement.py HostChannel)
        self._seq = 0

    _CHUNK = 4 << 20  # the TCP store rejects values above 8 MiB

    def _put(self, key: str, payload: bytes) -> None:
        n = max(1, -(-len(payload) // self._CHUNK))
        for i in range(n):
            self._store.set(f"{key}/{i}", payload[i * self._CHUNK:(i + 1) * self._CHUNK])
        self._store.set(key, str(n).encode())  # written last: the parts are complete

    def _take(self, key: str) -> bytes:
        n = int(self._store.get(key))
        return b"".join(self._store.get(f"{key}/{i}") for i in range(n))

    def _forget(self, key: str) -> None:
        n = int(self._store.get(key))
        for i in range(n):
            self._store.delete_key(f"{key}/{i}")
        self._store.delete_key(key)

    # one round: publish my payload, return everyone's (rank order)
    def _exchange(self, payload: bytes) -> list[bytes]:
        self._seq += 1
        key = f"fake/{self._seq}/"
        self._put(key + str(self.rank), payload)
        out = [payload if r == self.rank else self._take(key + str(r)) for r in range(self.size)]
        # the last reader of a round deletes it (bounded store growth over long tests)
        if self._store.add(key + "done", 1) == self.size:
            for r in range(self.size):
                self._forget(key + str(r))
            self._store.delete_key(key + "done")
        return out

    @staticmethod
    def _bytes(t: torch.Tensor) -> bytes:
        return t.detach().to("cpu").contiguous().reshape(-1).view(torch.uint8).numpy().tobytes()

    @staticmethod
    def _from(b: bytes, like: torch.Tensor) -> torch.Tensor:
        a = np.frombuffer(b, np.uint8).copy()
        return torch.from_numpy(a).view(like.dtype).reshape(like.shape)

    def broadcast(self, t, root=0):
        got = self._exchange(self._bytes(t) if self.rank == root else b"")
        if self.rank != root:
            t.copy_(self._from(got[root], t))

    def _reduce(self, parts: list[torch.Tensor], op: str) -> torch.Tensor:
        acc = parts[0].clone()
        for p in parts[1:]:
            if op in ("sum", "avg"):
                acc += p
            elif op == "prod":
                acc *= p
            elif op == "max":
                acc = torch.maximum(acc, p)
            elif op == "min":
                acc = torch.minimum(acc, p)
            else:
                raise ValueError(op)
        if op == "avg":
            acc = acc / len(parts) if acc.is_floating_point() else acc // len(parts)
        return acc

    def all_reduce(self, t, op="sum"):
        host = t.detach().to("cpu")
        parts = [self._from(b, host) for b in self._exchange(self._bytes(t))]
        t.copy_(self._reduce(parts, op).to(t.dtype))

    def all_gather(self, out, inp):
        if out.numel() != inp.numel() * self.size:
            raise ValueError("all_gather: out must hold size x inp elements")
        host = inp.detach().to("cpu")
        parts = [self._from(b, host).reshape(-1) for b in self._exchange(self._bytes(inp))]
        out.copy_(torch.cat(parts).view(out.shape))

    def reduce_scatter(self, out, inp, op="sum"):
        if inp.numel() != out.numel() * self.size:
            raise ValueError("reduce_scatter: inp must hold size x out elements")
        host = inp.detach().to("cpu")
        parts = [self._from(b, host).reshape(-1) for b in self._exchange(self._bytes(inp))]
        red = self._reduce(parts, op)
        n = out.numel()
        out.copy_(red[self.rank * n:(self.rank + 1) * n].view(out.shape))

    def all_to_all_v(self, out, out_splits, inp, in_splits):
        # one round: every rank publishes its whole send buffer; each takes its slice from
        # every peer (rank order), as RCCL's grouped send/recv delivers it
        offs = np.concatenate([[0], np.cumsum(list(in_splits))]).tolist()
        meta = np.asarray(offs, np.int64).tobytes()
        got = self._exchange(meta + self._bytes(inp))
        host = inp.detach().to("cpu")
        row = int(np.prod(inp.shape[1:])) if inp.dim() > 1 else 1
        nmeta = 8 * (self.size + 1)
        parts = []
        for r, b in enumerate(got):
            o = np.frombuffer(b[:nmeta], np.int64)
            raw = np.frombuffer(b[nmeta:], np.uint8).copy()
            flat = torch.from_numpy(raw).view(host.dtype) if raw.size else torch.empty(0, dtype=host.dtype)
            part = flat[o[self.rank] * row:o[self.rank + 1] * row]
            if part.numel() != out_splits[r] * row:
                raise ValueError(f"all_to_all_v: rank {r} sends {part.numel() // max(row, 1)} rows, expected "
                                 f"{out_splits[r]}")
            parts.append(part)
        out.copy_(torch.cat(parts).view(out.shape) if parts else out)

    def all_gather_object(self, obj):
        import pickle

        return [pickle.loads(b) for b in self._exchange(pickle.dumps(obj))]

    def barrier(self):
        self._exchange(b"")

    def destroy(self, abort: bool = False):
        # rank 0's process usually hosts the store: it must outlive every peer's last store
        # operation (the final round's deletions), or a peer's request hits a closed socket
        if abort:
            return
        if self.rank != 0:
            self._store.set(f"fake/closed/{self.rank}", b"1")
        else:
            self._store.wait([f"fake/closed/{r}" for r in range(1, self.size)])
