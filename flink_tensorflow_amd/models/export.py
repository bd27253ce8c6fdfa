"""SavedModel export: writes ``saved_model.pb`` + ``variables/`` (TensorBundle V2) + assets.

The reference only *loads* SavedModels (built by TF elsewhere).  To exercise the same
load path on models created here (the MNIST-MLP plumbing config, online-training
snapshots) we emit real TF 1.x SavedModels: the graph gets ``VariableV2``/``Assign``
initialisers and a sharded V2 saver subgraph (``save/Const``, ``SaveV2``,
``MergeV2Checkpoints``, ``RestoreV2``, ``save/restore_all``) with a matching ``SaverDef``,
so ``DefaultSaver`` and ``TensorFlowModel.open`` work on them exactly as on TF exports.
"""
from __future__ import annotations

import os
import shutil
from typing import Mapping

import numpy as np
import torch

from ..graph.builder import GraphBuilder
from ..io import bundle
from ..proto.messages import (CollectionDef, MetaGraphDef, MetaInfoDef, NodeList, OpDefRaw, OpList, SavedModel,
                              SaverDef, SignatureDef, TensorInfo, TensorShapeProto)
from ..types.dtypes import DataType


def add_saver(b: GraphBuilder, var_names: list[str], var_dtypes: list[DataType]) -> SaverDef:
    """Appends TF's sharded V2 saver subgraph for ``var_names``."""
    with b.name_scope("save"):
        fname = b.constant("Const", b"model")
        tmp_suffix = b.constant("StringJoin/inputs_1", b"_temp_ftm/part")
        join = b.op("StringJoin", [fname, tmp_suffix], name="StringJoin", separator=b"", N=2)
        shard = b.constant("ShardedFilename/shard", np.int32(0))
        nsh = b.constant("num_shards", np.int32(1))
        sfn = b.op("ShardedFilename", [join, shard, nsh], name="ShardedFilename")
        names = b.constant("SaveV2/tensor_names", np.asarray([n.encode() for n in var_names], dtype=object))
        slices = b.constant("SaveV2/shape_and_slices", np.asarray([b""] * len(var_names), dtype=object))
        save = b.op("SaveV2", [sfn, names, slices] + [f"{n}:0" for n in var_names], name="SaveV2",
                    dtypes=list(var_dtypes))
        dep = b.op("Identity", [sfn], name="control_dependency", control=[save], T=DataType.STRING)
        prefixes = b.op("Pack", [sfn], name="MergeV2Checkpoints/checkpoint_prefixes", control=[dep], N=1,
                        T=DataType.STRING, axis=0)
        merge = b.op("MergeV2Checkpoints", [prefixes, fname], name="MergeV2Checkpoints", delete_old_dirs=True)
        ident = b.op("Identity", [fname], name="Identity", control=[dep, merge], T=DataType.STRING)
        assigns = []
        for i, (n, dt) in enumerate(zip(var_names, var_dtypes)):
            rn = b.constant(f"RestoreV2_{i}/tensor_names", np.asarray([n.encode()], dtype=object))
            rs = b.constant(f"RestoreV2_{i}/shape_and_slices", np.asarray([b""], dtype=object))
            r = b.op("RestoreV2", [fname, rn, rs], name=f"RestoreV2_{i}", dtypes=[dt])
            assigns.append(b.op("Assign", [f"{n}:0", r], name=f"Assign_{i}", validate_shape=True, use_locking=True))
        shard_op = b.no_op("restore_shard", control=assigns)
        b.no_op("restore_all", control=[shard_op])
    return SaverDef(filename_tensor_name=fname, save_tensor_name=ident, restore_op_name="save/restore_all",
                    max_to_keep=5, sharded=True, keep_checkpoint_every_n_hours=10000.0, version=SaverDef.V2)


def tensor_info(name: str, dtype, shape) -> TensorInfo:
    return TensorInfo(name=name, dtype=int(DataType.of(dtype)), tensor_shape=TensorShapeProto.of(shape))


def export_saved_model(export_dir: str, builder: GraphBuilder, variables: Mapping[str, object],
                       signatures: Mapping[str, SignatureDef], tags=("serve",), assets: Mapping[str, bytes] | None = None,
                       overwrite: bool = True) -> str:
    """``variables``: ``{variable node name: initial value}`` — must already exist in the
    graph as ``VariableV2`` nodes (use ``GraphBuilder.variable_with_init``)."""
    if os.path.exists(export_dir):
        if not overwrite:
            raise FileExistsError(export_dir)
        shutil.rmtree(export_dir)
    os.makedirs(os.path.join(export_dir, "variables"))
    names = sorted(variables)
    import torch

    dts = [DataType.from_torch(torch.as_tensor(np.asarray(variables[n])).dtype) for n in names]
    saver_def = add_saver(builder, names, dts)
    init_op = builder.no_op("init", control=[builder.variables[n] for n in names if n in builder.variables])
    gd = builder.build_graph_def()
    ops = sorted({n.op for n in gd.node})
    mg = MetaGraphDef(
        meta_info_def=MetaInfoDef(tags=list(tags), tensorflow_version="ftm-amd", meta_graph_version="",
                                  stripped_op_list=OpList(op=[OpDefRaw(name=o) for o in ops])),
        graph_def=gd, saver_def=saver_def, signature_def=dict(signatures),
        collection_def={"variables": CollectionDef(node_list=NodeList(value=names)),
                        "trainable_variables": CollectionDef(node_list=NodeList(value=names)),
                        "init_op": CollectionDef(node_list=NodeList(value=[init_op.split(":")[0]]))})
    sm = SavedModel(saved_model_schema_version=1, meta_graphs=[mg])
    with open(os.path.join(export_dir, "saved_model.pb"), "wb") as f:
        f.write(sm.encode())
    bundle.save_tensors(os.path.join(export_dir, "variables", "variables"),
                        {n: torch.as_tensor(np.asarray(variables[n])) for n in names})
    if assets:
        os.makedirs(os.path.join(export_dir, "assets"))
        for k, v in assets.items():
            with open(os.path.join(export_dir, "assets", k), "wb") as f:
                f.write(v)
    return export_dir


def graph_def_to_saved_model(export_dir: str, graph_def, signatures: Mapping[str, SignatureDef],
                             tags=("serve",), min_elems: int = 2, overwrite: bool = True) -> str:
    """Exports a frozen GraphDef as a TF 1.x SavedModel whose weights are **variables**:
    every floating-point ``Const`` with at least ``min_elems`` elements becomes a
    ``VariableV2`` of the same name (consumers keep reading ``name:0``), initialised by a
    ``name/Assign`` from ``name/initial_value`` and restored from ``variables/`` by the
    saver subgraph — the layout TF's ``freeze_graph`` undoes."""
    from ..graph.tensor_proto import tensor_from_proto

    b = GraphBuilder()
    variables: dict[str, object] = {}
    for nd in graph_def.node:
        if nd.op == "Const":
            t = tensor_from_proto(nd.attr["value"].tensor)
            if isinstance(t, torch.Tensor) and t.is_floating_point() and t.numel() >= min_elems:
                variables[nd.name] = t.numpy()
                continue
        b.nodes.append(nd)
        b._names.add(nd.name)
    for name, val in variables.items():
        init = b.constant(f"{name}/initial_value", val)
        v = b.op("VariableV2", name=name, dtype=DataType.from_torch(torch.as_tensor(val).dtype),
                 shape=TensorShapeProto.of(val.shape), container=b"", shared_name=b"")
        assert v == f"{name}:0", v
        asg = b.op("Assign", [f"{name}:0", init], name=f"{name}/Assign", validate_shape=True, use_locking=True)
        b.variables[name] = asg.split(":")[0]
    return export_saved_model(export_dir, b, variables, signatures, tags=tags, overwrite=overwrite)
