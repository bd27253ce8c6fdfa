"""Tensor arena: native liveness offset planner, first-fit allocator, and compiled plans
sharing one subtask arena (activation slab + interned weights)."""
import numpy as np
import pytest
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from flink_tensorflow_amd import _ext
from flink_tensorflow_amd.batching.arena import ArenaExhausted, DeviceArena, plan_offsets
from flink_tensorflow_amd.graph.compiler import CompiledFunction
from flink_tensorflow_amd.graph.graph import Graph
from flink_tensorflow_amd.models.zoo.resnet import resnet50_graph_def


@settings(max_examples=200, deadline=None)
@given(st.lists(st.tuples(st.integers(0, 5000), st.integers(0, 30), st.integers(0, 10)), min_size=1, max_size=40))
def test_plan_offsets_never_overlaps_live_buffers(bufs):
    sizes = [b[0] for b in bufs]
    first = [b[1] for b in bufs]
    last = [b[1] + b[2] for b in bufs]
    offs, total = plan_offsets(sizes, first, last, 64)
    ext = [(o, o + max(-(-max(s, 1) // 64) * 64, 64)) for o, s in zip(offs, sizes)]
    for i in range(len(bufs)):
        assert offs[i] % 64 == 0 and ext[i][1] <= total
        for j in range(i):
            if last[i] < first[j] or last[j] < first[i]:
                continue  # never alive together
            assert ext[i][1] <= ext[j][0] or ext[j][1] <= ext[i][0], (i, j)
    # never worse than giving every buffer its own region
    assert total <= sum(e - s for s, e in ext)


def test_plan_offsets_reuses_dead_memory():
    # a chain: each buffer is read only by the next step -> two regions suffice
    n = 10
    offs, total = plan_offsets([1 << 20] * n, list(range(n)), [i + 1 for i in range(n)], 256)
    assert total == 2 << 20 and len(set(offs)) == 2


def test_offset_allocator_coalesces():
    a = _ext.native().OffsetAllocator(1 << 12, 256)
    blocks = [a.alloc(256) for _ in range(16)]
    assert blocks == [i * 256 for i in range(16)] and a.alloc(1) == -1
    for b in blocks[4:12]:
        a.free(b)
    assert a.largest_free == 8 * 256 and a.num_free_blocks == 1
    assert a.alloc(8 * 256) == 4 * 256
    with pytest.raises(ValueError):
        a.free(123)
    assert a.peak == 1 << 12


@pytest.fixture(scope="module")
def small_graph():
    return Graph.from_graph_def(resnet50_graph_def(depth=26, image_hw=(48, 48), num_classes=32))


def test_bucket_plans_share_one_arena(small_graph):
    arena = DeviceArena("cpu", budget_bytes=1 << 30)
    feeds = lambda b: {"images:0": ((b, 48, 48, 3), "UINT8")}  # noqa: E731
    p4 = CompiledFunction(small_graph, feeds(4), ["logits:0"], "cpu", strict=True, arena=arena)
    p2 = CompiledFunction(small_graph, feeds(2), ["logits:0"], "cpu", strict=True, arena=arena)
    st_ = arena.stats()
    # the smaller bucket reuses the bigger bucket's slab and its weights
    assert st_["slab_bytes"] == p4.activation_bytes >= p2.activation_bytes and st_["retired_slab_bytes"] == 0
    assert st_["interned_hits"] >= len(p2.params) - 2
    assert {t.data_ptr() for t in p2.params} <= {t.data_ptr() for t in p4.params}
    imgs = torch.randint(0, 256, (4, 48, 48, 3), dtype=torch.uint8)
    ref4 = CompiledFunction(small_graph, feeds(4), ["logits:0"], "cpu", strict=True)({"images:0": imgs})[0]
    ref2 = CompiledFunction(small_graph, feeds(2), ["logits:0"], "cpu", strict=True)({"images:0": imgs[:2]})[0]
    # interleaved replays on the shared slab give the private plans' results
    for _ in range(2):
        torch.testing.assert_close(p2({"images:0": imgs[:2]})[0], ref2)
        torch.testing.assert_close(p4({"images:0": imgs})[0], ref4)
    # the planned slab is far smaller than one buffer per produced value
    produced = sum(o.buf.numel() * o.buf.element_size() for s in p4.steps for o in s.outputs if o.buf is not None)
    assert p4.activation_bytes < 0.5 * produced


def test_arena_budget_is_enforced(small_graph):
    arena = DeviceArena("cpu", budget_bytes=1 << 20, chunk_bytes=1 << 16)
    with pytest.raises(ArenaExhausted):
        CompiledFunction(small_graph, {"images:0": ((8, 48, 48, 3), "UINT8")}, ["logits:0"], "cpu", arena=arena)


@pytest.mark.gpu
def test_arena_plans_gpu(small_graph):
    dev = torch.device("cuda", 0)
    arena = DeviceArena(dev, budget_bytes=8 << 30)
    feeds = lambda b: {"images:0": ((b, 48, 48, 3), "UINT8")}  # noqa: E731
    p4 = CompiledFunction(small_graph, feeds(4), ["logits:0"], dev, strict=True, arena=arena)
    p2 = CompiledFunction(small_graph, feeds(2), ["logits:0"], dev, strict=True, arena=arena)
    assert p4.summary()["hip_graph"] and arena.stats()["interned_hits"] > 0
    imgs = torch.randint(0, 256, (4, 48, 48, 3), dtype=torch.uint8)
    ref4 = CompiledFunction(small_graph, feeds(4), ["logits:0"], dev, strict=True)({"images:0": imgs.to(dev)})[0]
    ref2 = CompiledFunction(small_graph, feeds(2), ["logits:0"], dev, strict=True)({"images:0": imgs[:2].to(dev)})[0]
    for _ in range(2):
        torch.testing.assert_close(p2({"images:0": imgs[:2].to(dev)})[0], ref2)
        torch.testing.assert_close(p4({"images:0": imgs.to(dev)})[0], ref4)


@pytest.mark.gpu
def test_two_compute_lanes_keep_order_gpu(small_graph):
    """Two plan instances on two HIP streams (batches round-robin): results come back in
    submission order and equal the single-lane results."""
    import numpy as np

    from flink_tensorflow_amd.batching.engine import PipelinedGpuRunner

    dev = torch.device("cuda", 0)
    feeds = {"images:0": ((4, 48, 48, 3), "UINT8")}

    def lane():
        return {4: CompiledFunction(small_graph, feeds, ["top_k:0", "top_k:1"], dev, strict=True,
                                    arena=DeviceArena(dev, 4 << 30))}

    rng = np.random.default_rng(0)
    batches = [[rng.integers(0, 256, (48, 48, 3), dtype=np.uint8) for _ in range(4)] for _ in range(7)]

    def run(lanes):
        r = PipelinedGpuRunner(lanes, "images:0", lambda p: p.output_tensors(), (48, 48, 3), depth=3, device=dev)
        out = []
        for i, b in enumerate(batches):
            out += r.submit(b, np.full(4, float(i)), [i] * 4)
        out += r.drain()
        return out

    one, two = run(lane()), run([lane(), lane()])
    assert [r.tags[0] for r in two] == list(range(7))
    for a, b in zip(one, two):
        torch.testing.assert_close(a.outputs[0], b.outputs[0])
        assert torch.equal(a.outputs[1], b.outputs[1])


@pytest.mark.parametrize("stride,nbytes,threads", [(5003, 5003, 8), (196608, 196608, 8), (4099, 4000, 1),
                                                   (300000, 262145, 4), (64, 48, 8)])
def test_staging_gather_streaming_copy_exact(stride, nbytes, threads):
    """The staging gather's streaming (non-temporal) copy: odd sizes, unaligned destination
    rows, slices that cross the 256 KiB split, the single-thread and small-copy paths."""
    from flink_tensorflow_amd import _ext

    nat = _ext.native()
    rng = np.random.default_rng(7)
    recs = [rng.integers(0, 256, nbytes, dtype=np.uint8) for _ in range(37)]
    dst = np.zeros(1 + stride * len(recs) + 64, np.uint8)
    base = dst.ctypes.data + 1  # every row starts off 32-B alignment
    nat.gather_into(base, stride * len(recs), recs, stride, threads)
    for i, r in enumerate(recs):
        np.testing.assert_array_equal(dst[1 + i * stride:1 + i * stride + nbytes], r)
        assert not dst[1 + i * stride + nbytes:1 + (i + 1) * stride].any()  # nothing past the payload
    assert dst[0] == 0 and not dst[1 + stride * len(recs):].any()


def test_gc_freeze_moves_setup_objects_out_of_collection():
    import gc

    from flink_tensorflow_amd.utils.gcfreeze import freeze_setup_objects, unfreeze_setup_objects

    try:
        n = freeze_setup_objects(collect=False)
        assert n > 0 and gc.get_freeze_count() > 0
    finally:
        unfreeze_setup_objects()
    assert gc.get_freeze_count() == 0


@pytest.mark.gpu
def test_interleaved_head_pieces_match_whole_batch_gpu(small_graph):
    """Per-piece head kernels launched inside the host gather loop (``interleave_head``)
    give the same results as the head launched after the whole gather, full and short
    (padded) batches included, over two lanes."""
    import numpy as np

    from flink_tensorflow_amd.batching.engine import PipelinedGpuRunner

    dev = torch.device("cuda", 0)
    feeds = {"images:0": ((8, 48, 48, 3), "UINT8")}

    def lane():
        return {8: CompiledFunction(small_graph, feeds, ["top_k:0", "top_k:1"], dev, strict=True,
                                    arena=DeviceArena(dev, 4 << 30))}

    rng = np.random.default_rng(1)
    batches = [[rng.integers(0, 256, (48, 48, 3), dtype=np.uint8) for _ in range(8 if i % 3 else 6)]
               for i in range(7)]

    def run(interleave):
        lanes = [lane(), lane()]
        assert lanes[0][8].head_pieces_ok("images:0", torch.empty((8, 48, 48, 3), dtype=torch.uint8, device=dev))
        r = PipelinedGpuRunner(lanes, "images:0", lambda p: p.output_tensors(), (48, 48, 3), depth=3, device=dev,
                               stage_chunk=3, interleave_head=interleave)
        out = []
        for i, b in enumerate(batches):
            out += r.submit(b, np.full(len(b), float(i)), [i] * len(b))
        out += r.drain()
        return out

    a, b = run(True), run(False)
    assert [r.tags[0] for r in a] == list(range(7)) and [r.n for r in a] == [len(x) for x in batches]
    for x, y in zip(a, b):
        torch.testing.assert_close(x.outputs[0][: x.n], y.outputs[0][: y.n])
        assert torch.equal(x.outputs[1][: x.n], y.outputs[1][: y.n])



@pytest.mark.gpu
def test_stream_delay_and_lane_phase_gpu(small_graph):
    """``stream_delay`` holds a stream for the requested time (the lane-phase offset of a
    restarting pipeline); a runner with ``lane_offset_us`` gives the same results as one
    without, and delays only the second lane's first batch after each restart."""
    import numpy as np

    from flink_tensorflow_amd import _ext
    from flink_tensorflow_amd.batching.engine import PipelinedGpuRunner

    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        e0.record(s)
        _ext.hip().stream_delay(3000.0, s.cuda_stream)
        e1.record(s)
    e1.synchronize()
    assert 2.9 <= e0.elapsed_time(e1) < 20.0
    with pytest.raises(ValueError):
        _ext.hip().stream_delay(2e6, s.cuda_stream)

    feeds = {"images:0": ((8, 48, 48, 3), "UINT8")}

    def lane():
        return {8: CompiledFunction(small_graph, feeds, ["top_k:0", "top_k:1"], dev, strict=True,
                                    arena=DeviceArena(dev, 4 << 30))}

    rng = np.random.default_rng(2)
    batches = [[rng.integers(0, 256, (48, 48, 3), dtype=np.uint8) for _ in range(8)] for _ in range(6)]

    def run(offset):
        r = PipelinedGpuRunner([lane(), lane()], "images:0", lambda p: p.output_tensors(), (48, 48, 3), depth=3,
                               device=dev, lane_offset_us=offset, timeline=True)
        r.mark()
        out = []
        for i, b in enumerate(batches):
            out += r.submit(b, np.full(len(b), float(i)), [i] * len(b))
            if i == 2:  # drain: the pipeline restarts from empty at batch 3
                out += r.drain()
        out += r.drain()
        return out, r.timeline

    (a, _), (b, tl) = run(0.0), run(2000.0)
    for x, y in zip(a, b):
        assert torch.equal(x.outputs[1][: x.n], y.outputs[1][: y.n])
    # after each (re)start the second lane's first batch begins ~2 ms after the first batch
    # (its start stamp follows the delay kernel); the first lane is never delayed
    tl = sorted(tl, key=lambda t: t["submit_ms"])
    starts = [t["start_ms"] for t in tl]
    assert len(starts) == 6
    for i in (0, 3):
        assert starts[i + 1] - starts[i] >= 1.8, starts
