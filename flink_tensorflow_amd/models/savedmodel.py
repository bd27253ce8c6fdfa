"""SavedModel support (SURVEY §2.2 M5–M8; native loader N4).

* ``SignatureConstants`` — identical strings to
  ``LIB/models/savedmodel/SignatureConstants.java:6-57``.
* ``SavedModelLoader`` / ``DefaultSavedModelLoader`` —
  ``LIB/models/savedmodel/{SavedModelLoader,DefaultSavedModelLoader}.scala``: ``metagraph``
  is readable at job-definition time and parses ONLY ``saved_model.pb`` (the reference
  loads the whole bundle including weights for it, B7); ``load()`` copies non-local model
  dirs to a local temp dir (deleted at exit), imports the graph, restores variables from
  the TensorBundle V2 checkpoint through the SaverDef restore op, resolves assets and runs
  the ``main_op``/``legacy_init_op``.
* ``TensorFlowModel`` — ``LIB/models/savedmodel/TensorFlowModel.scala:12-61``.  It is a
  ``CheckpointedModel`` (``LIB/streaming/models/CheckpointedModel.scala:24-46``, wired as
  SURVEY §3.5 / F9 designs it): on a checkpoint barrier the session's variables are
  written D2H as a TensorBundle V2 (the ``Saver`` format, ``LIB/io/Saver.scala:55-89``)
  under ``chk-N/models/savedmodel-<subtask>/``; on restore they are read back into the
  session, so variables a streaming job mutates (e.g. ``Assign`` driven by a co-process
  update stream) survive a restart.
"""
from __future__ import annotations

import abc
import os
from typing import Sequence

import torch

from ..graph.graph import Graph
from ..graph.session import Session
from ..proto.messages import AssetFileDef, MetaGraphDef, SavedModel, SignatureDef
from ..types.tensor import StringTensor
from ..utils import fs
from .core import CheckpointedModel, ModelFunction, RichModel, default_device

STATE_NAME = "savedmodel"  # checkpoint sub-directory of TensorFlowModel variables


class SignatureConstants:
    DEFAULT_SERVING_SIGNATURE_DEF_KEY = "serving_default"
    CLASSIFY_INPUTS = "inputs"
    CLASSIFY_METHOD_NAME = "tensorflow/serving/classify"
    CLASSIFY_OUTPUT_CLASSES = "classes"
    CLASSIFY_OUTPUT_SCORES = "scores"
    PREDICT_INPUTS = "inputs"
    PREDICT_METHOD_NAME = "tensorflow/serving/predict"
    PREDICT_OUTPUTS = "outputs"
    REGRESS_INPUTS = "inputs"
    REGRESS_METHOD_NAME = "tensorflow/serving/regress"
    REGRESS_OUTPUTS = "outputs"


SAVED_MODEL_FILENAME_PB = "saved_model.pb"
VARIABLES_DIRECTORY = "variables"
VARIABLES_FILENAME = "variables"
ASSETS_DIRECTORY = "assets"
MAIN_OP_KEY = "saved_model_main_op"
LEGACY_INIT_OP_KEY = "legacy_init_op"
ASSETS_KEY = "saved_model_assets"
TAG_SERVE = "serve"
TAG_TRAIN = "train"
TAG_GPU = "gpu"


def read_saved_model(path: str) -> SavedModel:
    return SavedModel.decode(fs.read_bytes(path.rstrip("/") + "/" + SAVED_MODEL_FILENAME_PB))


def select_meta_graph(sm: SavedModel, tags: Sequence[str]) -> MetaGraphDef:
    want = set(tags)
    for mg in sm.meta_graphs:
        if set(mg.meta_info_def.tags if mg.meta_info_def else []) == want:
            return mg
    avail = [list(mg.meta_info_def.tags) for mg in sm.meta_graphs]
    raise ValueError(f"no MetaGraphDef with tags {sorted(want)}; available: {avail}")


class SavedModelBundle:
    """A loaded SavedModel: graph + session (variables restored) + meta graph."""

    def __init__(self, graph: Graph, session: Session, meta_graph_def: MetaGraphDef, export_dir: str):
        self.graph = graph
        self.session = session
        self.meta_graph_def = meta_graph_def
        self.export_dir = export_dir

    def close(self):
        self.session.close()


def asset_file_defs(mg: MetaGraphDef) -> list[AssetFileDef]:
    if mg.asset_file_def:
        return list(mg.asset_file_def)
    cd = mg.collection_def.get(ASSETS_KEY)
    out = []
    if cd is not None and cd.any_list is not None:
        for a in cd.any_list.value:
            out.append(AssetFileDef.decode(a.value))
    return out


def _allocate_variables(sess: Session, var_prefix: str) -> bool:
    """Every variable of the bundle allocated (uninitialised) on the session's device from
    the index alone — no tensor data read.  False when a variable cannot be received by a
    broadcast (STRING), in which case the caller restores normally."""
    from ..io import bundle
    from ..types.dtypes import DataType

    with bundle.BundleReader(var_prefix) as r:
        specs = {k: r.dtype_and_shape(k) for k in r.keys()}
    if any(dt == DataType.STRING for dt, _ in specs.values()):
        return False
    dev = sess.device
    for k, (dt, shape) in specs.items():
        sess.variables[k] = torch.empty(shape, dtype=dt.torch, device=dev)
    return True


def load_bundle(local_dir: str, tags: Sequence[str], device=None, read_variables: bool = True) -> SavedModelBundle:
    """``read_variables=False``: variables are only allocated from the checkpoint index (a
    data-parallel rank that receives rank 0's values by broadcast)."""
    sm = read_saved_model(local_dir)
    mg = select_meta_graph(sm, tags)
    g = Graph.from_graph_def(mg.graph_def)
    sess = Session(g, device=device)
    var_prefix = os.path.join(local_dir, VARIABLES_DIRECTORY, VARIABLES_FILENAME)
    sd = mg.saver_def
    if sd is not None and sd.restore_op_name and os.path.exists(var_prefix + ".index"):
        if read_variables or not _allocate_variables(sess, var_prefix):
            sess.run(targets=[sd.restore_op_name.split(":")[0]],
                     feed_dict={sd.filename_tensor_name: StringTensor(var_prefix.encode())})
    asset_feeds = {}
    for a in asset_file_defs(mg):
        asset_feeds[a.tensor_info.name] = StringTensor(os.path.join(local_dir, ASSETS_DIRECTORY, a.filename).encode())
    for key in (MAIN_OP_KEY, LEGACY_INIT_OP_KEY):
        cd = mg.collection_def.get(key)
        if cd is not None and cd.node_list is not None and cd.node_list.value:
            sess.run(targets=[n.split(":")[0].lstrip("^") for n in cd.node_list.value], feed_dict=asset_feeds)
            break
    return SavedModelBundle(g, sess, mg, local_dir)


class SavedModelLoader(abc.ABC):
    @property
    @abc.abstractmethod
    def metagraph(self) -> MetaGraphDef:
        ...

    @abc.abstractmethod
    def load(self, device=None) -> SavedModelBundle:
        ...


class DefaultSavedModelLoader(SavedModelLoader):
    def __init__(self, export_path: str, tags: Sequence[str] = (TAG_SERVE,)):
        self.export_path = export_path
        self.tags = tuple(tags)
        self._metagraph: MetaGraphDef | None = None

    def __getstate__(self):
        return {"export_path": self.export_path, "tags": self.tags, "_metagraph": None}

    @property
    def metagraph(self) -> MetaGraphDef:
        if self._metagraph is None:  # parse saved_model.pb only (B7 fixed)
            self._metagraph = select_meta_graph(read_saved_model(self.export_path), self.tags)
        return self._metagraph

    def load(self, device=None, read_variables: bool = True) -> SavedModelBundle:
        local = fs.copy_to_local(self.export_path)
        return load_bundle(local, self.tags, device=device, read_variables=read_variables)


class TensorFlowModel(RichModel, CheckpointedModel):
    """A SavedModel-backed model.  Subclasses define ``loader``."""

    _TRANSIENT = ("_bundle", "_functions")

    def __init__(self, device=None, distributed_weights: bool = False):
        self.device = device
        # data parallel: rank 0 reads the variables, the other ranks receive them (RCCL
        # broadcast) instead of every rank reading the checkpoint
        self.distributed_weights = distributed_weights
        self._bundle: SavedModelBundle | None = None
        self._pending_restore: str | None = None

    @property
    @abc.abstractmethod
    def loader(self) -> SavedModelLoader:
        ...

    @property
    def metagraph(self) -> MetaGraphDef:
        return self.loader.metagraph

    def signature_def(self, name: str) -> SignatureDef | None:
        return self.metagraph.signature_def.get(name)

    def open(self) -> None:
        if self._bundle is not None:
            raise RuntimeError("model already open")  # checkState(bundle == null)
        dev = self.device if self.device is not None else default_device()
        from ..parallel import comm

        dist = self.distributed_weights and comm.is_dist()
        if dist and comm.rank_size()[0] != 0:
            try:
                self._bundle = self.loader.load(device=dev, read_variables=False)
            except TypeError:  # a custom loader without the option: it reads, rank 0's values win
                self._bundle = self.loader.load(device=dev)
        else:
            self._bundle = self.loader.load(device=dev)
        if dist:
            vs = self._bundle.session.variables
            comm.broadcast_tensors([vs[k] for k in sorted(vs) if isinstance(vs[k], torch.Tensor)], src=0)
            if hasattr(vs, "touch"):
                vs.touch()
        if self._pending_restore is not None:  # initialize_state ran before open()
            prefix, self._pending_restore = self._pending_restore, None
            self.restore_variables(prefix)

    def close(self) -> None:
        if self._bundle is not None:
            self._bundle.close()
        self._bundle = None
        self.__dict__.pop("_functions", None)

    @property
    def is_open(self) -> bool:
        return self._bundle is not None

    @property
    def bundle(self) -> SavedModelBundle:
        if self._bundle is None:
            raise RuntimeError(f"{type(self).__name__} is not open")
        return self._bundle

    def session(self) -> Session:
        return self.bundle.session

    def function(self, signature: str, method, **options) -> ModelFunction:
        """The ``ModelFunction`` of ``signature`` (cached per signature / method type /
        options, so its compiled plans live as long as the open model).  ``options`` go to
        ``ModelFunction`` (``compile``, ``batch_buckets``, ``precision``, ``strict``)."""
        key = (signature, type(method), tuple(sorted(options.items())))
        fns = self.__dict__.get("_functions")
        if fns is None:  # first use, or a descriptor unpickled in a subtask (transient field)
            fns = self.__dict__["_functions"] = {}
        fn = fns.get(key)
        if fn is None:
            sd = self.signature_def(signature)
            if sd is None:
                raise KeyError(f"no signature {signature!r}; available: {sorted(self.metagraph.signature_def)}")
            fn = ModelFunction(self.session, sd, method, **options)
            fns[key] = fn
        fn.method = method
        return fn

    @staticmethod
    def load(path: str, *tags: str) -> DefaultSavedModelLoader:
        return DefaultSavedModelLoader(path, tags or (TAG_SERVE,))

    # ---- CheckpointedModel: session variables <-> bundle V2 in the checkpoint
    def save_variables(self, prefix: str) -> str:
        from ..io.saver import VariableSaver

        return VariableSaver().save(self.session(), prefix)

    def restore_variables(self, prefix: str) -> None:
        from ..io.saver import VariableSaver

        VariableSaver().restore(self.session(), prefix)

    def snapshot_state(self, ctx) -> None:
        from ..runtime.model_functions import model_state_dir

        d = model_state_dir(ctx, STATE_NAME)
        if d is not None and self.is_open and self.session().variables:
            self.save_variables(os.path.join(d, "variables"))

    def initialize_state(self, ctx) -> None:
        if not ctx.is_restored() or ctx.checkpoint_dir is None:
            return
        prefix = os.path.join(ctx.checkpoint_dir, "models", f"{STATE_NAME}-{ctx.subtask_index}", "variables")
        if not os.path.exists(prefix + ".index"):
            return
        if self.is_open:
            self.restore_variables(prefix)
        else:
            self._pending_restore = prefix


class SavedModel_(TensorFlowModel):
    """Concrete TensorFlowModel over a path (for users who don't subclass)."""

    def __init__(self, path: str, tags: Sequence[str] = (TAG_SERVE,), device: str | torch.device | None = None,
                 distributed_weights: bool = False):
        super().__init__(device, distributed_weights)
        self._loader = DefaultSavedModelLoader(path, tags)

    @property
    def loader(self) -> SavedModelLoader:
        return self._loader


SavedModelModel = SavedModel_
