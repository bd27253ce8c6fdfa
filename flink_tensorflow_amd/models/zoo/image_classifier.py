"""Image-classification models served by the compiled CDNA4 plan.

``ImageClassifierModel`` is a ``GenericModel`` (frozen GraphDef + session, the
reference's ``InceptionModel`` shape: ``EX/inception/InceptionModel.scala:19-92``) that is
also a ``BatchedGpuModel``: on a GPU subtask ``open()`` compiles the graph for each batch
bucket (fused preprocess, implicit-GEMM convs, softmax+top-k) and wraps the plans in the
pipelined pinned-H2D / hipGraph runner; ``DataStream.map_with_model_batched`` then feeds
it micro-batches of raw uint8 images.  On a host subtask the same graph runs in the
interpreter (tests, CPU plumbing).

``label(images)`` is the synchronous ``LabelMethod`` equivalent: top-k (probability,
label) pairs per image (the reference sorts the full [M, N] matrix on the host).
"""
from __future__ import annotations

from typing import Callable, Sequence

import numpy as np
import torch

from ...graph.compiler import CompiledFunction
from ...proto.messages import GraphDef
from ...runtime.model_functions import BatchedGpuModel
from ...types.tensor_value import TensorValue
from ..core import DefaultGraphLoader, GenericModel, GraphDefGraphLoader, GraphLoader


class ImageClassifierModel(GenericModel, BatchedGpuModel):
    _TRANSIENT = ("_graph", "_session", "_plans", "_runner", "_arena", "_labels_cache")

    def __init__(self, graph_source: Callable[[], GraphDef] | str, image_hw: tuple[int, int],
                 buckets: Sequence[int] = (64, 256), top_k: int = 5, labels: Sequence[str] | None = None,
                 feed: str = "images:0", fetches: Sequence[str] = ("top_k:0", "top_k:1"), depth: int = 3,
                 device=None, use_graph: bool = True, precision: str = "bf16", calibration_images=None,
                 distributed_weights: bool = False, lanes: int = 2, lane_offset_us: float = 0.0):
        super().__init__(device)
        self.lanes = max(1, int(lanes))  # concurrent plan instances on their own HIP streams
        # lane phase at a pipeline restart (PipelinedGpuRunner): off by default — under light
        # load every batch that overlaps a running one would wait; throughput runs set it
        self.lane_offset_us = float(lane_offset_us)
        self.distributed_weights = distributed_weights  # DP: broadcast rank 0's compiled weights at open
        self.precision = precision
        self.calibration_images = calibration_images  # uint8 [n, H, W, 3] for fp8 scales (synthetic if None)
        self.graph_source = graph_source
        self.image_hw = tuple(image_hw)
        self.buckets = tuple(sorted(buckets))
        self.top_k = top_k
        self.labels = list(labels) if labels is not None else None
        self.feed = feed
        self.fetches = list(fetches)
        self.depth = depth
        self.use_graph = use_graph
        self._plans: dict | None = None
        self._runner = None
        self._arena = None

    @property
    def graph_loader(self) -> GraphLoader:
        if isinstance(self.graph_source, str):
            return DefaultGraphLoader(self.graph_source)
        return GraphDefGraphLoader(self.graph_source())

    # ------------------------------------------------------------------ lifecycle
    def open(self) -> None:
        super().open()
        dev = self._session.device
        if dev.type == "cuda":
            from ...batching.arena import DeviceArena
            from ...batching.engine import PipelinedGpuRunner
            from ...config import EngineConfig

            H, W = self.image_hw
            # per compute lane one arena: its bucket plans share that arena's activation slab
            # (largest compiled first) and interned weights; lanes replay concurrently
            budget = EngineConfig().arena_bytes(dev) // self.lanes
            self._arena = [DeviceArena(dev, budget, name=f"{type(self).__name__}/lane{i}") for i in range(self.lanes)]
            lanes = [{b: CompiledFunction(self._graph, {self.feed: ((b, H, W, 3), "UINT8")}, self.fetches, dev,
                                          use_graph=self.use_graph, strict=True, precision=self.precision,
                                          calibration=self._calibration(b), arena=arena)
                      for b in sorted(self.buckets, reverse=True)} for arena in self._arena]
            self._plans = lanes[0]
            if self.distributed_weights:
                from ...parallel import comm

                # in place, so the captured hipGraphs keep reading the same buffers
                comm.broadcast_tensors([t for ln in lanes for p in ln.values() for t in p.params], src=0)
            self._runner = PipelinedGpuRunner(lanes, self.feed, lambda p: p.output_tensors(), (H, W, 3),
                                              torch.uint8, depth=self.depth, device=dev,
                                              lane_offset_us=getattr(self, "lane_offset_us", 0.0),
                                              decode_threads=getattr(self, "decode_threads", None))

    def _calibration(self, b: int):
        if self.precision != "fp8" or self.calibration_images is None:
            return None
        imgs = torch.as_tensor(np.asarray(self.calibration_images, dtype=np.uint8))
        reps = -(-b // imgs.shape[0])
        return {self.feed: imgs.repeat(reps, 1, 1, 1)[:b]}

    def close(self) -> None:
        if self._runner is not None:
            self._runner.drain()
        self._runner = None
        self._plans = None
        self._arena = None
        super().close()

    def plan_summary(self) -> dict | None:
        return next(iter(self._plans.values())).summary() if self._plans else None

    def label_of(self, i: int) -> str:
        return self.labels[i] if self.labels and i < len(self.labels) else f"class_{i}"

    # ------------------------------------------------------------------ batched GPU API
    @staticmethod
    def _as_array(r) -> np.ndarray:
        if isinstance(r, tuple) and len(r) == 2 and isinstance(r[0], str):
            r = r[1]  # an ``ImageInputFormat`` record: (file name, decoded image or JPEG bytes)
        if isinstance(r, (bytes, bytearray)):
            return r  # compressed: decoded by the runner straight into the staging slot
        if isinstance(r, TensorValue):
            r = r.to_numpy()
        elif isinstance(r, torch.Tensor):
            r = r.cpu().numpy()
        a = np.asarray(r)
        if a.ndim == 4 and a.shape[0] == 1:
            a = a[0]
        return np.ascontiguousarray(a, dtype=np.uint8)

    def _label_table(self, n: int) -> list:
        """``label_of`` for every class index below ``n``, built once (the per-batch result
        conversion is 256 x top-k lookups on the worker's hot path)."""
        t = self.__dict__.get("_labels_cache")
        if t is None or len(t) < n:
            t = self.__dict__["_labels_cache"] = [self.label_of(i) for i in range(max(n, 1024))]
        return t

    def _results(self, br):
        vals, idxs = br.outputs[0][: br.n], br.outputs[1][: br.n]
        il = idxs.tolist()
        lab = self._label_table(max((max(r) for r in il), default=0) + 1)
        # tolist() already yields Python floats / ints
        res = [list(zip(vr, [lab[i] for i in ir])) for vr, ir in zip(vals.tolist(), il)]
        return res, br.tags, br.latencies

    def submit(self, records, ingest_ts, tags):
        if self._runner is None:  # host fallback: synchronous interpreter run
            out = self.label(records)
            import time

            return [(out, tags, time.perf_counter() - np.asarray(ingest_ts))]
        arrs = [self._as_array(r) for r in records]
        out = []
        # split into bucket-sized chunks
        cap = self.buckets[-1]
        for s in range(0, len(arrs), cap):
            chunk = arrs[s:s + cap]
            for br in self._runner.submit(chunk, np.asarray(ingest_ts[s:s + cap]), list(tags[s:s + cap])):
                out.append(self._results(br))
        return out

    def poll(self):
        return [self._results(b) for b in self._runner.poll()] if self._runner is not None else []

    def drain(self):
        return [self._results(b) for b in self._runner.drain()] if self._runner is not None else []

    # ------------------------------------------------------------------ synchronous API
    def label(self, images) -> list[list[tuple[float, str]]]:
        """Top-k ``(probability, label)`` per image (``InceptionModel.label`` +
        ``toTextLabels``)."""
        arrs = [self._as_array(r) for r in images]
        if any(isinstance(a, (bytes, bytearray)) for a in arrs):
            from ...graph.ops_io import decode_jpegs

            H, W = self.image_hw
            blobs = [a for a in arrs if isinstance(a, (bytes, bytearray))]
            dec = iter(decode_jpegs(blobs, H, W, getattr(self, "decode_threads", None) or 8))
            arrs = [next(dec) if isinstance(a, (bytes, bytearray)) else a for a in arrs]
        arrs = np.stack(arrs)
        sess = self.session()
        if self._plans is not None:
            n = len(arrs)
            b = next((bk for bk in self.buckets if bk >= n), None)
            if b is not None:
                buf = np.zeros((b, *arrs.shape[1:]), dtype=np.uint8)
                buf[:n] = arrs
                vals, idxs = self._plans[b]({self.feed: torch.from_numpy(buf).to(sess.device)})
                vals, idxs = vals[:n].cpu(), idxs[:n].cpu()
                return [[(float(v), self.label_of(int(i))) for v, i in zip(vr, ir)]
                        for vr, ir in zip(vals.tolist(), idxs.tolist())]
        vals, idxs = sess.run(self.fetches, {self.feed: torch.from_numpy(arrs)})
        return [[(float(v), self.label_of(int(i))) for v, i in zip(vr, ir)] for vr, ir in zip(vals.tolist(), idxs.tolist())]


class ResNet50Model(ImageClassifierModel):
    """ResNet-50 v1.5 (random-init frozen graph; BASELINE headline model)."""

    def __init__(self, image_hw=(256, 256), buckets=(64, 256), top_k=5, seed: int = 0, device=None, depth_layers=50,
                 **kw):
        self.seed = seed
        self.depth_layers = depth_layers
        super().__init__(self._make_graph, image_hw, buckets, top_k, device=device, **kw)

    def _make_graph(self) -> GraphDef:
        from .resnet import resnet50_graph_def

        return resnet50_graph_def(image_hw=self.image_hw, top_k=self.top_k, seed=self.seed, depth=self.depth_layers)


class InceptionV3Model(ImageClassifierModel):
    """Inception-v3 (random-init frozen graph) compiled for fp8 by default — BASELINE config
    5: e4m3 weights and activations on the CDNA4 fp8 MFMA, bucketed dynamic batching per
    operator (each micro-batch runs on the smallest captured bucket that holds it)."""

    def __init__(self, image_hw=(299, 299), buckets=(32, 64, 128, 256), top_k=5, seed: int = 0, device=None,
                 precision: str = "fp8", **kw):
        self.seed = seed
        super().__init__(self._make_graph, image_hw, buckets, top_k, device=device, precision=precision, **kw)

    def _make_graph(self) -> GraphDef:
        from .inception_v3 import inception_v3_graph_def

        return inception_v3_graph_def(image_hw=self.image_hw, top_k=self.top_k, seed=self.seed)
