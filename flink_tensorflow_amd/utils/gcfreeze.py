"""Keeps CPython's cyclic garbage collector off the long-lived setup objects.

A streaming job builds hundreds of thousands of Python objects once (imported modules,
parsed GraphDefs, compiled plans, weight wrappers): ~200k with ResNet-50 loaded.  A full
collection walks all of them — 20-70 ms with the GIL held — and in a pipelined GPU
runner that is a host stall long enough to let the compute lanes run dry (measured: a
3-4 ms gap in the submit loop of a 20-batch window, `profiles/r03_s3_window`).  After setup
``freeze_setup_objects()`` collects once and moves every surviving object into the
permanent generation (``gc.freeze``), so later collections scan only what the stream
itself allocates.

Frozen objects are still freed by reference counting; only reference cycles among them
are no longer reclaimed until ``gc.unfreeze()``.  A process that rebuilds its plans many
times can call ``unfreeze_setup_objects()`` when it tears a runner down."""
from __future__ import annotations

import gc
import threading

_lock = threading.Lock()


def freeze_setup_objects(collect: bool = True) -> int:
    """One collection (optional), then ``gc.freeze()``.  Returns the number of frozen
    objects.  Idempotent; cheap to call again after more setup."""
    from .tracing import capture_lock

    # under the capture lock: a collection finalises whatever became garbage anywhere in
    # the process (old plans' hipGraphs, arenas, pinned blocks) and must not do so while a
    # sibling subtask thread is inside a stream capture
    with capture_lock(), _lock:
        if collect:
            gc.collect()
        gc.freeze()
        return gc.get_freeze_count()


def unfreeze_setup_objects() -> None:
    """Returns the frozen objects to the oldest generation (their cycles become collectable
    again)."""
    with _lock:
        gc.unfreeze()
