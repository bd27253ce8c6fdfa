"""HIP streams owned by the framework.

``torch.cuda.Stream()`` hands out streams round-robin from a fixed pool (32 per device and
priority), and ``torch.cuda.graph`` captures on a pool stream of its own.  In a process
with several GPU subtasks (threads), the 33rd pooled stream is the capture stream again:
a runner replaying on it while a sibling thread captures a hipGraph either puts its
launches into that graph or is rejected ("Cannot prepare for replay during capturing
stage").  Runner lanes, copy engines and captures therefore use streams created here with
``hipStreamCreateWithPriority`` (non-blocking), never shared with the pool or with another
live owner.
"""
from __future__ import annotations

import threading
import weakref

_lock = threading.Lock()
_capture_streams: dict = {}
_free: dict = {}  # (device index, priority) -> streams released by collected owners


def dedicated_stream(device=None, priority: int = 0, owner=None):
    """A non-blocking HIP stream on ``device``, used by nobody else while ``owner`` lives,
    wrapped as ``torch.cuda.ExternalStream``.

    Streams are never destroyed: torch's pinned-host allocator records events on every
    stream a pinned block was copied on when that block is freed, which can be after the
    owner is gone.  A collected owner's streams go back to a free list and are handed to
    the next owner instead (exclusive, unlike torch's round-robin pool)."""
    import torch

    dev = torch.device(device if device is not None else "cuda")
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    key = (dev.index, priority)
    with _lock:
        free = _free.get(key)
        ptr = free.pop() if free else None
    if ptr is None:
        from .. import _ext

        with torch.cuda.device(dev):
            ptr = _ext.hip().stream_create(priority)
    if owner is not None:
        weakref.finalize(owner, _release, key, ptr)
    return torch.cuda.ExternalStream(ptr, device=dev)


def _release(key, ptr):
    with _lock:
        _free.setdefault(key, []).append(ptr)


def capture_stream(device=None):
    """The per-device stream every hipGraph capture of this process runs on (captures are
    serialised by the capture lock, so one stream per device suffices)."""
    import torch

    dev = torch.device(device if device is not None else "cuda")
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    with _lock:
        s = _capture_streams.get(dev.index)
    if s is None:
        s = dedicated_stream(dev)  # takes ``_lock`` itself
        with _lock:
            s = _capture_streams.setdefault(dev.index, s)
    return s
