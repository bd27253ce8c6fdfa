"""Barrier alignment at end of input (``runtime/executor.py`` input loop).

Two channels: channel 0 sends barrier -> records -> EndOfInput; channel 1 (a source that
finished before the checkpoint trigger, so it never emits a barrier) sends only
EndOfInput, later.  The EndOfInput of channel 1 completes the alignment; channel 0's
blocked records and EndOfInput are replayed after it, and the task must still finish."""
import threading
import time
from types import SimpleNamespace

from flink_tensorflow_amd.runtime.executor import InputGate, _OpTask
from flink_tensorflow_amd.runtime.operators import END, Barrier, Record


class _Op:
    def __init__(self):
        self.seen, self.ended, self.snapshots = [], False, []

    def setup(self, ctx, out): pass
    def initialize(self, restore, restore_dir): pass
    def open(self): pass
    def close(self): pass
    def next_deadline(self): return None
    def on_idle(self, now): pass
    def process(self, rec, idx): self.seen.append(rec.value)
    def process_watermark(self, wm): pass
    def prepare_snapshot(self): pass
    def end_input(self): self.ended = True

    def snapshot_state(self, cid, d):
        self.snapshots.append((cid, list(self.seen)))
        return {}


class _Writer:
    def __init__(self):
        self.out = []

    def emit(self, e): self.out.append(e)
    def emit_side(self, tag, v): pass
    def flush(self): pass


def _task(op):
    job = SimpleNamespace(cancel=threading.Event(), attempt=0, config=None, rank=0, world_size=1, restore_dir=None,
                          coordinator=None, device_for=lambda node, st: None, chk_dir=lambda cid: None,
                          ack=lambda cid, key, state: None, wait_all_opened=lambda: None)
    node = SimpleNamespace(uid="op", name="op", parallelism=1, remote=False, make_operator=lambda: op)
    gate = InputGate(64)
    t = _OpTask(job, node, 0, _Writer(), None, gate, [(0, 0), (1, 0)])
    return t, gate


def test_end_of_input_completes_alignment_and_replays():
    op = _Op()
    t, gate = _task(op)
    q = gate.q
    q.put((0, Barrier(7, time.time())))
    q.put((0, Record("a", None)))
    q.put((0, Record("b", None)))
    q.put((0, END))
    th = threading.Thread(target=t.run, daemon=True)
    th.start()
    time.sleep(0.2)
    assert op.seen == [] and not op.ended  # channel 0 blocked behind its barrier
    q.put((1, END))
    th.join(timeout=5)
    assert not th.is_alive(), "task hung at end of input"
    assert op.snapshots == [(7, [])]  # snapshot taken before the blocked records
    assert op.seen == ["a", "b"] and op.ended
    assert any(isinstance(e, Barrier) and e.checkpoint_id == 7 for e in t.writer.out)
