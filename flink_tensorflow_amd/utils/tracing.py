"""Tracing hooks.

* ``trace_range(name)`` — a roctx range (``torch.cuda.nvtx`` is roctx on ROCm) around a
  pipeline stage (gather, H2D, plan replay, D2H, operator batches), so
  ``rocprofv3 --kernel-trace --marker-trace`` shows stages next to the kernels.  Enabled
  by ``FTM_TRACE=1``; otherwise a no-op context manager with no per-call cost beyond a
  flag check.
* ``debug_sync()`` / ``debug_poison()`` — the ordering-assertion and use-after-release
  debug modes of the compiled plans (``FTM_DEBUG_SYNC=1``: run eagerly and synchronize +
  check the HIP error state after every launch, naming the failing step;
  ``FTM_DEBUG_POISON=1``: fill every plan buffer with NaN bytes right after its last
  reader, so a liveness-planning bug reads poison instead of stale-but-plausible data).
"""
from __future__ import annotations

import contextlib
import os

_TRACE = os.environ.get("FTM_TRACE") == "1"


def tracing_enabled() -> bool:
    return _TRACE


def set_tracing(on: bool) -> None:
    global _TRACE
    _TRACE = bool(on)


@contextlib.contextmanager
def _range(name: str):
    import torch

    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()


def trace_range(name: str):
    if not _TRACE:
        return contextlib.nullcontext()
    try:
        import torch

        if not torch.cuda.is_available():
            return contextlib.nullcontext()
    except Exception:  # noqa: BLE001
        return contextlib.nullcontext()
    return _range(name)


def debug_sync() -> bool:
    return os.environ.get("FTM_DEBUG_SYNC") == "1"


def debug_poison() -> bool:
    return os.environ.get("FTM_DEBUG_POISON") == "1"


# ------------------------------------------------------------------ hipGraph capture
_CAPTURE_LOCK = None


def capture_lock():
    """The process-wide capture lock: hold it around a capture's warm-up and device
    synchronisation too (a device-wide synchronise while another thread captures is
    rejected by the runtime)."""
    import threading

    global _CAPTURE_LOCK
    if _CAPTURE_LOCK is None:
        _CAPTURE_LOCK = threading.RLock()
    return _CAPTURE_LOCK


def graph_capture(graph, stream=None, pool=None):
    """``torch.cuda.graph`` (hipGraph stream capture) safe next to other operator threads
    of the same process: captures are serialised, and ``thread_local`` error mode keeps a
    sibling subtask's allocations / launches on its own stream from invalidating (or being
    rejected by) this capture.  ``pool`` shares one private memory pool between graphs that
    never replay concurrently (e.g. the token-capacity plans of one encoder)."""
    import contextlib
    import threading

    import torch

    from .streams import capture_stream

    lock = capture_lock()

    @contextlib.contextmanager
    def _cm():
        import gc

        with lock:
            # a framework-owned capture stream: torch's default capture stream comes from the
            # stream pool and can coincide with a sibling subtask's replay stream (utils/streams.py)
            s = stream if stream is not None else capture_stream()
            # no automatic collection while capturing: a collection triggered by ANY thread
            # runs finalisers (graph / arena / pinned-block teardown) in the middle of the
            # capture (explicit collections take the capture lock: utils/gcfreeze.py)
            was_enabled = gc.isenabled()
            gc.disable()
            try:
                with torch.cuda.graph(graph, pool=pool, stream=s, capture_error_mode="thread_local"):
                    yield
            finally:
                if was_enabled:
                    gc.enable()

    return _cm()
