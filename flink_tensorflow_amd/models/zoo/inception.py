"""The reference's Inception example models (SURVEY §2.7 X3–X7), MI355X-served.

* ``ImageNormalization`` — ``EX/inception/ImageNormalization.scala:14-91``: a GenericModel
  whose graph is built in code: ``Placeholder("input", STRING) → DecodeJpeg(3) →
  Cast(FLOAT) → ExpandDims(0) → ResizeBilinear(224,224) → Sub(117) → Div(1)``.
* ``InceptionModel`` — ``EX/inception/InceptionModel.scala:19-92``: a GenericModel over
  ``tensorflow_inception_graph.pb`` (input ``input`` [N,224,224,3] float normalized, output
  ``output`` [N,C] probabilities) and ``imagenet_comp_graph_label_strings.txt``.  The frozen
  graph is imported behind our own uint8 front end (``input_map``), so the GPU plan runs
  the fused resize/normalize kernel, the MFMA convs and a fused top-k.  When the model dir
  holds no ``.pb`` (there is no network access to fetch it), a GoogLeNet-shaped
  random-init graph with the same input/output names is synthesized.
* ``ImageInputFormat`` — ``EX/inception/ImageInputFormat.scala:24-85``: one record per
  ``*.jpg``/``*.jpeg`` file (``*.crdownload`` excluded; filters merged, B8); JPEG decode
  on the host (Pillow), normalization either on the host through ``ImageNormalization``
  (reference behaviour) or deferred to the fused GPU preprocess kernel.
* The package type aliases of ``EX/inception/package.scala:7-30`` (``ImageTensor``,
  ``ImageTensorValue``, ``ImageFile``, ``ImageFileTensor``, ``LabelTensor``): runtime-checked
  ``TypeTag``s (rank + element type) usable with ``tagged_as``.
"""
from __future__ import annotations

import os

import numpy as np

from ...graph.builder import GraphBuilder
from ...graph.graph import Graph
from ...proto.messages import GraphDef
from ...runtime.sources import WholeFileInputFormat
from ...types.tensor import StringTensor
from ...types.tensor_value import TensorValue
from ...utils import fs
from ..core import GenericModel, GraphDefGraphLoader, GraphLoader, ModelFunction
from ...types.names import TypedTensor, tagged_as
from ..signatures import LambdaMethod
from .image_classifier import ImageClassifierModel

# ---- EX/inception/package.scala:7-30
ImageTensor = TypedTensor(4, "FLOAT")          # TypedTensor[`4D`, Float]: [N, H, W, 3] normalized
ImageTensorValue = ImageTensor                 # TensorValue[`4D`, Float] (checked on to_tensor())
ImageFile = "ImageFile"                        # the ByteString tag of an encoded image file
ImageFileTensor = TypedTensor(0, "STRING")     # TypedTensor[`0D`, ByteString[ImageFile]]
LabelTensor = TypedTensor(2, "FLOAT")          # TypedTensor[`2D`, Float]: [N, classes] scores


def as_image_tensor(t):
    """``t.taggedAs[ImageTensor]`` (rank-4 float, checked)."""
    return tagged_as(t, ImageTensor)


def as_label_tensor(t):
    """``t.taggedAs[LabelTensor]`` (rank-2 float, checked)."""
    return tagged_as(t, LabelTensor)

IMAGE_H = IMAGE_W = 224
MEAN = 117.0
SCALE = 1.0


def image_normalization_graph_def(h=IMAGE_H, w=IMAGE_W, mean=MEAN, scale=SCALE) -> GraphDef:
    b = GraphBuilder()
    inp = b.placeholder("input", "STRING", [])
    x = b.decode_jpeg(inp, 3, name="DecodeJpeg")
    x = b.cast(x, "FLOAT", name="Cast")
    x = b.expand_dims(x, b.constant("make_batch", np.int32(0)), name="ExpandDims")
    x = b.resize_bilinear(x, b.constant("size", np.asarray([h, w], dtype=np.int32)), name="ResizeBilinear")
    x = b.sub(x, b.constant("mean", np.float32(mean)), name="Sub")
    b.div(x, b.constant("scale", np.float32(scale)), name="output")
    return b.build_graph_def()


class ImageNormalization(GenericModel):
    """``normalize(jpeg_bytes) -> float [1,224,224,3]`` (method ``inception/normalize``)."""

    METHOD = "inception/normalize"

    def __init__(self, device="cpu"):
        super().__init__(device)

    @property
    def graph_loader(self) -> GraphLoader:
        return GraphDefGraphLoader(image_normalization_graph_def())

    def normalize(self, jpeg: bytes):
        from ...proto.messages import SignatureDef, TensorInfo

        sd = SignatureDef(inputs={"inputs": TensorInfo(name="input:0")}, outputs={"outputs": TensorInfo(name="output:0")},
                          method_name=self.METHOD)
        m = LambdaMethod(self.METHOD, lambda v: {"inputs": StringTensor(v)}, lambda t: t["outputs"])
        return ModelFunction(self.session(), sd, m).apply(jpeg)


def googlenet_like_graph_def(num_classes: int = 1008, seed: int = 0, width: float = 0.5) -> GraphDef:
    """A random-init GoogLeNet-shaped graph with the inception5h I/O contract
    (``input`` float [N,224,224,3] → ``output`` softmax [N, num_classes])."""
    rng = np.random.default_rng(seed)
    b = GraphBuilder()

    def conv(x, cin, cout, k, s, name):
        w = (rng.standard_normal((k, k, cin, cout)) * np.sqrt(2.0 / (k * k * cin))).astype(np.float32)
        y = b.conv2d(x, b.constant(name + "_w", w), (s, s), "SAME", name=name)
        y = b.bias_add(y, b.constant(name + "_b", np.zeros(cout, np.float32)), name=name + "_pre_relu")
        return b.relu(y, name=name + "_relu")

    def c(n):
        return max(8, int(round(n * width / 8)) * 8)

    x = b.placeholder("input", "FLOAT", [None, 224, 224, 3])
    x = conv(x, 3, c(64), 7, 2, "conv2d0")
    x = b.max_pool(x, (3, 3), (2, 2), "SAME", name="maxpool0")
    x = b.lrn(x, 5, 1.0, 1e-4, 0.75, name="localresponsenorm0")  # as in inception5h
    x = conv(x, c(64), c(64), 1, 1, "conv2d1")
    x = conv(x, c(64), c(192), 3, 1, "conv2d2")
    x = b.lrn(x, 5, 1.0, 1e-4, 0.75, name="localresponsenorm1")
    x = b.max_pool(x, (3, 3), (2, 2), "SAME", name="maxpool1")
    cin = c(192)
    for i, (o1, r3, o3, r5, o5, pp) in enumerate([(64, 96, 128, 16, 32, 32), (128, 128, 192, 32, 96, 64)]):
        nm = f"mixed{i}"
        b1 = conv(x, cin, c(o1), 1, 1, nm + "_1x1")
        b2 = conv(conv(x, cin, c(r3), 1, 1, nm + "_3x3_bottleneck"), c(r3), c(o3), 3, 1, nm + "_3x3")
        b3 = conv(conv(x, cin, c(r5), 1, 1, nm + "_5x5_bottleneck"), c(r5), c(o5), 5, 1, nm + "_5x5")
        b4 = conv(b.max_pool(x, (3, 3), (1, 1), "SAME", name=nm + "_pool"), cin, c(pp), 1, 1, nm + "_pool_reduce")
        x = b.concat([b1, b2, b3, b4], 3, name=nm)
        cin = c(o1) + c(o3) + c(o5) + c(pp)
    x = b.max_pool(x, (3, 3), (2, 2), "SAME", name="maxpool4")
    x = b.mean(x, [1, 2], name="avgpool0")
    w = (rng.standard_normal((cin, num_classes)) * np.sqrt(1.0 / cin)).astype(np.float32)
    logits = b.bias_add(b.matmul(x, b.constant("softmax2_w", w), name="softmax2_pre_activation/matmul"),
                        b.constant("softmax2_b", np.zeros(num_classes, np.float32)), name="softmax2_pre_activation")
    b.softmax(logits, name="output")
    return b.build_graph_def()


def with_uint8_front_end(inner: GraphDef, image_hw, mean=MEAN, scale=SCALE, top_k=3,
                         inner_input="input:0", inner_output="output:0") -> GraphDef:
    """``images`` uint8 → Cast → ResizeBilinear(224) → Sub(mean) → Div(scale) →
    [inner graph] → ``top_k`` on its probabilities."""
    b = GraphBuilder()
    images = b.placeholder("images", "UINT8", [None, image_hw[0], image_hw[1], 3])
    x = b.cast(images, "FLOAT", name="Cast")
    x = b.resize_bilinear(x, b.constant("size", np.asarray([IMAGE_H, IMAGE_W], np.int32)), name="ResizeBilinear")
    x = b.sub(x, b.constant("mean", np.float32(mean)), name="Sub")
    b.div(x, b.constant("scale", np.float32(scale)), name="normalized")
    g = Graph.from_graph_def(b.build_graph_def())
    g.import_graph_def(inner, "net", input_map={inner_input: "normalized:0"})
    b2 = GraphBuilder()
    b2.top_k("net/" + inner_output, top_k, name="top_k")
    g.import_graph_def(b2.build_graph_def())
    return g.to_graph_def()


class InceptionModel(ImageClassifierModel):
    GRAPH_FILE = "tensorflow_inception_graph.pb"
    LABEL_FILE = "imagenet_comp_graph_label_strings.txt"

    def __init__(self, model_dir: str | None = None, image_hw=(IMAGE_H, IMAGE_W), top_k: int = 3,
                 buckets=(16, 64), device=None, **kw):
        self.model_dir = model_dir
        labels = None
        if model_dir and fs.exists(os.path.join(model_dir, self.LABEL_FILE)):
            labels = fs.read_all_lines(os.path.join(model_dir, self.LABEL_FILE))
        super().__init__(self._make_graph, image_hw, buckets, top_k, labels=labels, device=device, **kw)

    def _make_graph(self) -> GraphDef:
        pb = os.path.join(self.model_dir, self.GRAPH_FILE) if self.model_dir else None
        if pb and fs.exists(pb):
            inner = GraphDef.decode(fs.read_bytes(pb))
        else:
            inner = googlenet_like_graph_def()
        return with_uint8_front_end(inner, self.image_hw, top_k=self.top_k)


class ImageInputFormat(WholeFileInputFormat):
    """``(filename, image)`` records: decoded uint8 [H,W,3] (GPU-normalized downstream), or
    with ``normalize_on_host`` a float ``TensorValue`` [1,224,224,3] from
    ``ImageNormalization`` (the reference's behaviour)."""

    def __init__(self, include=None, exclude=None, normalize_on_host: bool = False, resize_to=None,
                 defer_decode: bool = False):
        super().__init__(include, exclude)
        self.configure(include=["*.jpg", "*.jpeg"], exclude=["*.crdownload"])
        self.normalize_on_host = normalize_on_host
        self.resize_to = resize_to
        # defer_decode: records carry the compressed bytes; a GPU image model decodes them
        # with the native pool straight into its staging slot (csrc/jpeg.cpp), so a ~20 KB
        # record crosses the job instead of a 196 KB decoded image and no per-image Python
        # decode runs in the reader
        self.defer_decode = defer_decode
        self.model = ImageNormalization() if normalize_on_host else None

    def open_input_format(self):
        if self.model is not None:
            self.model.open()

    def close_input_format(self):
        if self.model is not None:
            self.model.close()

    def read_record(self, path: str, data: bytes):
        if not data:
            return None
        if self.normalize_on_host:
            return os.path.basename(path), TensorValue.from_tensor(self.model.normalize(data))
        if self.defer_decode:
            return os.path.basename(path), data
        from ...graph.ops_io import decode_rgb

        img = decode_rgb(data)  # native baseline decoder, Pillow for the rest
        if self.resize_to is not None and img.shape[:2] != tuple(self.resize_to):
            from PIL import Image

            img = np.asarray(Image.fromarray(img).resize((self.resize_to[1], self.resize_to[0]), Image.BILINEAR))
        return os.path.basename(path), img
