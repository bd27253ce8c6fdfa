"""Framework-owned HIP streams (utils/streams.py): exclusive while the owner lives, back on a
free list (never destroyed) when it is collected, one capture stream per device.  The
HIP calls are faked here; tests/test_arena.py and test_remote.py run the real ones on a GPU."""
import contextlib
import gc
import threading

import pytest
import torch

from flink_tensorflow_amd.utils import streams


class _FakeLib:
    def __init__(self):
        self.created = 0

    def stream_create(self, priority=0):
        self.created += 1
        return 0x1000 + self.created

    def stream_destroy(self, ptr):  # pragma: no cover - must never be called
        raise AssertionError("streams are never destroyed")


@pytest.fixture()
def fake(monkeypatch):
    lib = _FakeLib()
    monkeypatch.setattr(streams, "_free", {})
    monkeypatch.setattr(streams, "_capture_streams", {})
    from flink_tensorflow_amd import _ext

    monkeypatch.setattr(_ext, "hip", lambda required=True: lib)
    monkeypatch.setattr(torch.cuda, "device", lambda d: contextlib.nullcontext())
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 0)
    monkeypatch.setattr(torch.cuda, "ExternalStream", lambda ptr, device=None: ("stream", ptr, str(device)))
    return lib


class _Owner:
    pass


def test_streams_are_exclusive_and_recycled(fake):
    a, b = _Owner(), _Owner()
    sa, sb = streams.dedicated_stream("cuda:0", owner=a), streams.dedicated_stream("cuda:0", owner=b)
    assert sa[1] != sb[1] and fake.created == 2
    del a
    gc.collect()
    sc = streams.dedicated_stream("cuda:0", owner=_Owner())  # reuses the collected owner's stream
    assert sc[1] == sa[1] and fake.created == 2
    sd = streams.dedicated_stream("cuda:0", priority=-1)      # other priority: a new stream
    assert sd[1] not in (sa[1], sb[1]) and fake.created == 3


def test_capture_stream_is_one_per_device_and_does_not_deadlock(fake):
    got = []
    ts = [threading.Thread(target=lambda: got.append(streams.capture_stream("cuda:0"))) for _ in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(10)
    assert not any(t.is_alive() for t in ts)
    assert len({s[1] for s in got}) == 1 and streams.capture_stream("cuda:0") == got[0]
    assert streams.capture_stream("cuda:1")[1] != got[0][1]
