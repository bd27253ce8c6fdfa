"""Micro-batching GPU execution: pinned staging, side-stream H2D, hipGraph replay, D2H.

The reference runs one ``Session.run`` per record at batch 1 with four host copies per
image.  Here records are staged into GPU micro-batches:

::

    host:  gather B record payloads → pinned slot (C++ multithreaded memcpy, GIL released)
    copy stream:    pinned slot ──hipMemcpyAsync──▶ HBM staging slot      (event h2d[s])
    compute stream: wait h2d[s] → preprocess kernel on the staging slot (or D2D into the
                    plan's input) → hipGraph replay
                    → outputs ──hipMemcpyAsync──▶ pinned result slot       (event done[s])
    host:  (later) wait done[s] → emit results, per-record latency

``depth`` slots rotate, so the host assembles batch i+1 and the copy engine moves it while
the compute stream runs batch i.  Buckets: a batch of n records runs on the smallest
compiled bucket ≥ n (padding rows are zero and their outputs discarded).
"""
from __future__ import annotations

import bisect
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Sequence

import numpy as np
import torch

from ..utils.streams import dedicated_stream
from ..utils.tracing import capture_lock, trace_range

from .. import _ext


@dataclass
class BatchResult:
    outputs: list            # host tensors, first ``n`` rows valid
    n: int
    ingest_ts: np.ndarray    # per-record ingest timestamps (perf_counter seconds)
    done_ts: float
    tags: list = field(default_factory=list)

    @property
    def latencies(self) -> np.ndarray:
        return self.done_ts - self.ingest_ts


class _Slot:
    def __init__(self, bucket: int, rec_shape, rec_dtype, out_shapes, device, pin=True, timing=False):
        self.bucket = bucket
        self.pinned_in = torch.empty((bucket, *rec_shape), dtype=rec_dtype, pin_memory=pin)
        self.dev_in = torch.empty((bucket, *rec_shape), dtype=rec_dtype, device=device)
        self.pinned_out = [torch.empty(s, dtype=d, pin_memory=pin) for s, d in out_shapes]
        self.h2d = torch.cuda.Event()
        self.h2d_parts: list[torch.cuda.Event] = []  # one per staged piece (chunked head launch)
        self.done = torch.cuda.Event(enable_timing=timing)
        # timeline mode: GPU timestamps of the first H2D piece and of the plan's first kernel
        self.t_h2d = torch.cuda.Event(enable_timing=True) if timing else None
        self.t_start = torch.cuda.Event(enable_timing=True) if timing else None
        self.busy = False
        self.n = 0
        self.ts = None
        self.tags = None


class PipelinedGpuRunner:
    """Runs compiled plans over micro-batches with copy/compute overlap.

    ``plans``: ``{bucket_size: plan}`` where ``plan.input_buffer(feed)`` is the static
    device input and ``plan.replay()`` launches the captured graph; ``fetch_bufs(plan)``
    returns the device output tensors to bring back (small: top-k values/indices).  A plan
    with ``select(host_batch, n)`` chooses the concrete plan per batch from the staged
    host records (before the H2D copy).

    ``plans`` may also be a list of such dicts — one per **compute lane**: independent plan
    instances (own buffers) replayed on their own HIP streams, batches assigned round-robin,
    so consecutive micro-batches overlap on the GPU (the tail of one graph's kernels fills
    with the next graph's instead of idling CUs).  Results are always returned in
    submission order.
    """

    def __init__(self, plans, feed: str, fetch_bufs: Callable[[Any], Sequence[torch.Tensor]],
                 record_shape, record_dtype=torch.uint8, depth: int = 3, device=None, gather_threads: int = 8,
                 stage_chunk: int = 64, lane_offset_us: float = 0.0, freeze_gc: bool = True, timeline: bool = False,
                 interleave_head: bool = True, decode_threads: int | None = None, async_decode: bool = True):
        lanes = plans if isinstance(plans, (list, tuple)) else [plans]
        self.lanes = [dict(sorted(p.items())) for p in lanes]
        self.plans = self.lanes[0]
        self.buckets = list(self.plans)
        if any(list(p) != self.buckets for p in self.lanes):
            raise ValueError("every compute lane needs the same batch buckets")
        self.feed = feed
        self.fetch_bufs = fetch_bufs
        self.device = torch.device(device or "cuda")
        self.record_shape = tuple(record_shape)
        self.record_dtype = record_dtype
        self.record_bytes = int(np.prod(record_shape)) * torch.empty((), dtype=record_dtype).element_size()
        # framework-owned streams, not torch's pool (a pooled stream can be the one a sibling
        # subtask thread is capturing a hipGraph on: utils/streams.py)
        self.copy_stream = dedicated_stream(self.device, owner=self)
        # (lane 0 on a high-priority stream measured -1 to -5 %: profiles/r04_o)
        self.compute_streams = [dedicated_stream(self.device, owner=self) for _ in self.lanes]
        self.compute_stream = self.compute_streams[0]
        self.gather_threads = gather_threads
        # records that arrive as compressed JPEG bytes (``ImageInputFormat(defer_decode=True)``)
        # are decoded by the native pool straight into the pinned rows (csrc/jpeg.cpp)
        # (None: 32, at most the CPUs this process may run on — 32 measured best on the
        # MI355X box, 64 oversubscribed it: profiles/r06_jpeg)
        if decode_threads is None:
            import os

            decode_threads = max(1, min(32, len(os.sched_getaffinity(0))))
        self.decode_threads = decode_threads
        self.decode_fallbacks = 0
        self.async_decode = async_decode
        self._pending = None  # (DecodeJob, slot, bucket, payloads, ingest_ts, tags)
        self.stage_chunk = stage_chunk  # records per gather + H2D piece (0: whole batch at once)
        self.interleave_head = interleave_head  # launch each piece's head kernel inside the gather loop
        self._native = _ext.native()
        depth = max(depth, len(self.lanes) + 1)  # every lane busy + one batch being staged
        # batches in flight over ALL buckets (each bucket has its own ``depth`` slots): with
        # many buckets (dynamic batch sizes) the host could otherwise run dozens of batches
        # ahead of the GPU, adding queueing latency without adding throughput
        self.max_inflight = depth
        self.slots: dict[int, list[_Slot]] = {}
        for b, plan in self.plans.items():
            outs = [(tuple(t.shape), t.dtype) for t in fetch_bufs(plan)]
            self.slots[b] = [_Slot(b, self.record_shape, record_dtype, outs, self.device, timing=timeline)
                             for _ in range(depth)]
        # timeline: per harvested batch (lane, host submit s, GPU ms of first H2D / first kernel /
        # done relative to ``mark()``) — where a short timed window loses time to fill and drain
        self.timeline = [] if timeline else None
        self._mark = None
        self._next = {b: 0 for b in self.buckets}
        self._lane = 0
        self._inflight: list[_Slot] = []  # submission order
        # host seconds per phase (gather / select / launch / wait): where the driving
        # thread's time goes when the GPU is not saturated
        self.host_s = {"gather": 0.0, "select": 0.0, "launch": 0.0, "wait": 0.0}
        self.batches = 0
        # lane phase: when the pipeline starts from empty, the k-th lane to receive a batch
        # starts it k x lane_offset_us after the first (a stream-ordered delay kernel), so
        # the lanes begin in the staggered phase of the steady state (one lane's
        # memory-bound layers against another's compute-bound ones) instead of in step
        self.lane_offset_us = float(lane_offset_us) if len(self.lanes) > 1 else 0.0
        self._started: list[int] = []
        if freeze_gc:  # the plans are compiled: keep the GC's full passes off them
            from ..utils.gcfreeze import freeze_setup_objects

            freeze_setup_objects()

    def bucket_for(self, n: int) -> int:
        i = bisect.bisect_left(self.buckets, n)
        if i == len(self.buckets):
            raise ValueError(f"batch of {n} exceeds the largest bucket {self.buckets[-1]}")
        return self.buckets[i]

    # ------------------------------------------------------------------ submission
    def _is_jpeg(self, payloads) -> bool:
        return (isinstance(payloads[0], (bytes, bytearray, memoryview)) and len(self.record_shape) == 3
                and self.record_shape[2] == 3 and self.record_dtype == torch.uint8)

    def _reserve(self, n: int):
        """The bucket and ring slot of an n-record batch, with the slot's previous batch
        (and anything beyond the in-flight cap) harvested."""
        b = self.bucket_for(n)
        slots = self.slots[b]
        slot = slots[self._next[b]]
        self._next[b] = (self._next[b] + 1) % len(slots)
        t0 = time.perf_counter()
        finished = self._harvest_through(slot) if slot.busy else []
        while len(self._inflight) >= self.max_inflight:
            finished.append(self._harvest(self._inflight[0]))
        self.host_s["wait"] += time.perf_counter() - t0
        return b, slot, finished

    def submit(self, payloads: Sequence, ingest_ts: np.ndarray, tags: list | None = None) -> list[BatchResult]:
        """Stages ``payloads`` (buffer-protocol records of ``record_shape``) and launches the
        batch.  Returns results of earlier batches that completed (slot reuse).

        JPEG byte strings (``ImageInputFormat(defer_decode=True)``) are decoded by the
        native pool into the pinned slot; with ``async_decode`` that decode runs in the
        background and the batch is launched by the next ``submit`` / ``poll`` / ``drain``
        once it has landed, so the caller reads and batches the next records meanwhile."""
        payloads = list(payloads)
        finished = self._finish_pending(block=True)
        if self.async_decode and self._is_jpeg(payloads):
            b, slot, more = self._reserve(len(payloads))
            H, W, _ = self.record_shape
            base, cap = slot.pinned_in.data_ptr(), slot.pinned_in.numel() * slot.pinned_in.element_size()
            job = self._native.jpeg_decode_start(base, cap, payloads, self.record_bytes, H, W, self.decode_threads)
            self._pending = (job, slot, b, payloads, ingest_ts, tags)
            return finished + more
        b, slot, more = self._reserve(len(payloads))
        self._stage_launch(slot, b, payloads, ingest_ts, tags, decoded=False)
        return finished + more

    def _finish_pending(self, block: bool) -> list[BatchResult]:
        """Launches the batch whose JPEG decode runs in the background, once it has landed
        (waiting for it when ``block``); images the native decoder declined go through
        Pillow first."""
        if self._pending is None:
            return []
        job, slot, b, payloads, ingest_ts, tags = self._pending
        if not block and not job.done():
            return []
        self._pending = None
        t0 = time.perf_counter()
        st = job.wait()
        self.host_s["decode_wait"] = self.host_s.get("decode_wait", 0.0) + time.perf_counter() - t0
        bad = [k for k, code in enumerate(st) if code]
        if bad:
            from ..graph.ops_io import fit_image_bytes

            H, W, _ = self.record_shape
            for k in bad:
                slot.pinned_in[k].copy_(torch.from_numpy(np.ascontiguousarray(fit_image_bytes(bytes(payloads[k]), H, W))))
            self.decode_fallbacks += len(bad)
        self._stage_launch(slot, b, payloads, ingest_ts, tags, decoded=True)
        return []

    def _stage_launch(self, slot: _Slot, b: int, payloads: list, ingest_ts, tags, decoded: bool) -> None:
        n = len(payloads)
        t1 = time.perf_counter()
        # host gather into the pinned slot in pieces, each piece's H2D issued as soon as it is
        # staged (the DMA of piece i overlaps the gather of piece i+1: a batch reaches the GPU
        # one piece after its last record is gathered, not one whole-batch copy later); the
        # padding rows of a short batch are zeroed only when needed
        rb = self.record_bytes
        base, cap = slot.pinned_in.data_ptr(), slot.pinned_in.numel() * slot.pinned_in.element_size()
        step = self.stage_chunk if 0 < self.stage_chunk < n else n
        pieces = [(lo, min(n, lo + step)) for lo in range(0, n, step)]
        while len(slot.h2d_parts) < len(pieces):
            slot.h2d_parts.append(torch.cuda.Event())
        if slot.t_h2d is not None:
            slot.t_h2d.record(self.copy_stream)
            slot.t_submit = t1
        lane = self._lane
        plan = self.lanes[lane][b]
        stream = self.compute_streams[lane]
        # a plan whose head kernel runs per staged piece and that needs no host look at the
        # batch (``select``): each piece's head is launched right after its H2D, WHILE the
        # host gathers the next piece — the GPU starts one piece after the first records are
        # gathered instead of after the whole batch (the pipeline fill of a timed window)
        interleave = (self.interleave_head and len(pieces) > 1 and getattr(plan, "select", None) is None
                      and getattr(plan, "head_pieces_ok", None) is not None
                      and plan.head_pieces_ok(self.feed, slot.dev_in))
        if interleave:
            self._begin_lane(slot, lane, stream)
        jpeg = self._is_jpeg(payloads)
        with trace_range(f"gather[{n}/{b}]"):
            for i, (lo, hi) in enumerate(pieces):
                if decoded:
                    pass  # the rows are in the slot already (background decode)
                elif jpeg:
                    self._decode_into(slot, base, cap, lo, payloads[lo:hi])
                else:
                    self._native.gather_into(base + lo * rb, cap - lo * rb, payloads[lo:hi], rb, self.gather_threads)
                if n < b and hi == n:  # the padding rows of a short batch travel with the last piece
                    slot.pinned_in[n:].zero_()
                    hi = b
                    pieces[i] = (lo, b)
                with torch.cuda.stream(self.copy_stream):
                    slot.dev_in[lo:hi].copy_(slot.pinned_in[lo:hi], non_blocking=True)
                    slot.h2d_parts[i].record(self.copy_stream)
                if interleave:
                    with torch.cuda.stream(stream):
                        stream.wait_event(slot.h2d_parts[i])
                        plan.launch_head_piece(slot.dev_in, lo, hi)
        t2 = time.perf_counter()
        self._lane = (self._lane + 1) % len(self.lanes)
        select = getattr(plan, "select", None)
        if select is not None:  # e.g. the padding-free BERT encoder: pick a token-capacity plan
            plan = select(slot.pinned_in, n)
        t3 = time.perf_counter()
        if not interleave:
            self._begin_lane(slot, lane, stream)
        with torch.cuda.stream(self.copy_stream):
            slot.h2d.record(self.copy_stream)
        slot.lane = lane
        with torch.cuda.stream(stream):
            with trace_range(f"forward[{b}]@lane{lane}"):
                if interleave:
                    plan.replay_tail()
                else:
                    chunked = getattr(plan, "replay_from_chunks", None)
                    # head kernel per staged piece: the GPU starts on the first piece while
                    # the later ones are still in flight (shortens the pipeline fill)
                    if not (len(pieces) > 1 and chunked is not None and chunked(
                            self.feed, slot.dev_in, pieces, lambda i: stream.wait_event(slot.h2d_parts[i]))):
                        stream.wait_event(slot.h2d)
                        replay_from = getattr(plan, "replay_from", None)
                        if replay_from is not None:  # head kernel reads the staging slot: no D2D copy
                            replay_from(self.feed, slot.dev_in)
                        else:
                            plan.input_buffer(self.feed).copy_(slot.dev_in, non_blocking=True)
                            plan.replay()
            with trace_range("d2h"):
                for dst, src in zip(slot.pinned_out, self.fetch_bufs(plan)):
                    dst.copy_(src, non_blocking=True)
            slot.done.record(stream)
        slot.busy = True
        slot.n = n
        slot.ts = ingest_ts
        slot.tags = tags
        self._inflight.append(slot)
        t4 = time.perf_counter()
        hs = self.host_s
        hs["gather"] += t2 - t1
        hs["select"] += t3 - t2
        hs["launch"] += t4 - t3
        self.batches += 1

    def _decode_into(self, slot: _Slot, base: int, cap: int, lo: int, blobs: list) -> None:
        """JPEG byte strings -> RGB rows ``lo ..`` of the pinned slot: the native baseline
        decoder on the host pool, GIL released; what it does not take (progressive, another
        size, not a JPEG) goes through Pillow, resized to the record shape."""
        from ..graph.ops_io import decode_jpegs_into

        H, W, _ = self.record_shape
        rb = self.record_bytes
        self.decode_fallbacks += decode_jpegs_into(base + lo * rb, cap - lo * rb, blobs, rb, H, W,
                                                   self.decode_threads, rows=slot.pinned_in[lo:])

    def _begin_lane(self, slot: _Slot, lane: int, stream) -> None:
        """The lane's stream work that precedes a batch: the phase delay of a restarting
        pipeline and the batch's start stamp (timeline)."""
        if self.lane_offset_us > 0:
            if not self._inflight:  # the pipeline restarts from empty
                self._started.clear()
            if lane not in self._started:
                k = len(self._started)
                self._started.append(lane)
                if k:
                    _ext.hip().stream_delay(k * self.lane_offset_us, stream.cuda_stream)
        if slot.t_start is not None:  # after the lane's previous work, before this batch's h2d wait
            with torch.cuda.stream(stream):
                slot.t_start.record(stream)

    def _harvest(self, slot: _Slot) -> BatchResult:
        # event waits / queries are rejected while a sibling subtask thread captures a
        # hipGraph (its plans compile while this one already streams): query under the
        # capture lock, never block while holding it
        while True:
            with capture_lock():
                if slot.done.query():
                    break
            time.sleep(5e-5)
        slot.busy = False
        self._inflight.remove(slot)
        if self.timeline is not None and self._mark is not None:
            m = self._mark
            self.timeline.append({"lane": slot.lane, "n": slot.n, "submit_ms": round((slot.t_submit - m[1]) * 1e3, 3),
                                  "h2d_ms": round(m[0].elapsed_time(slot.t_h2d), 3),
                                  "start_ms": round(m[0].elapsed_time(slot.t_start), 3),
                                  "done_ms": round(m[0].elapsed_time(slot.done), 3)})
        return BatchResult([t.clone() for t in slot.pinned_out], slot.n, slot.ts, time.perf_counter(),
                           slot.tags or [])

    def _harvest_through(self, slot: _Slot) -> list[BatchResult]:
        """Harvests every in-flight batch up to and including ``slot`` (order preserved)."""
        out = []
        while self._inflight:
            head = self._inflight[0]
            out.append(self._harvest(head))
            if head is slot:
                break
        return out

    def mark(self):
        """Timeline origin: a GPU timestamp on the copy stream and the host clock, now."""
        if self.timeline is None:
            return
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(self.copy_stream)
        self._mark = (ev, time.perf_counter())
        self.timeline.clear()

    def poll(self) -> list[BatchResult]:
        """Launches a background-decoded batch that has landed, then harvests completed
        batches without blocking, oldest first, stopping at the first one still running."""
        out = self._finish_pending(block=False)
        while self._inflight:
            with capture_lock():
                ready = self._inflight[0].done.query()
            if not ready:
                break
            out.append(self._harvest(self._inflight[0]))
        return out

    def drain(self) -> list[BatchResult]:
        out = self._finish_pending(block=True)
        while self._inflight:
            out.append(self._harvest(self._inflight[0]))
        return out


class MicroBatcher:
    """Size/time-triggered batch formation (the operator-side half of micro-batching).

    ``add`` returns a full batch when ``max_batch`` records are pending; ``due`` tells the
    operator that the oldest pending record has waited ``max_delay_ms``; ``flush`` returns
    whatever is pending (on timers, barriers and end-of-input: a batch never straddles a
    checkpoint barrier)."""

    def __init__(self, max_batch: int, max_delay_ms: float):
        self.max_batch = max_batch
        self.max_delay = max_delay_ms / 1000.0
        self.items: list = []
        self.ts: list[float] = []

    def add(self, item, ts: float | None = None):
        self.items.append(item)
        self.ts.append(time.perf_counter() if ts is None else ts)
        if len(self.items) >= self.max_batch:
            return self.flush()
        return None

    def add_many(self, items: list, ts: float) -> list:
        """``add`` for a run of items arriving together: the full batches it completes."""
        out = []
        i = 0
        while i < len(items):
            k = min(len(items) - i, self.max_batch - len(self.items))
            self.items.extend(items[i:i + k])
            self.ts.extend([ts] * k)
            i += k
            if len(self.items) >= self.max_batch:
                out.append(self.flush())
        return out

    def due(self, now: float | None = None) -> bool:
        if not self.items:
            return False
        now = time.perf_counter() if now is None else now
        return now - self.ts[0] >= self.max_delay

    def flush(self):
        if not self.items:
            return None
        items, ts = self.items, np.asarray(self.ts)
        self.items, self.ts = [], []
        return items, ts

    def __len__(self):
        return len(self.items)
