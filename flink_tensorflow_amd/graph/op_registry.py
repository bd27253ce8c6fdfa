"""Op kernel registry for the graph executor.

Each TF op type maps to ``fn(ctx, node, *inputs) -> tuple(outputs)``.  Kernels implement
TF 1.x semantics on ``torch.Tensor`` / ``StringTensor`` values (host or HBM).  This is
the replacement for libtensorflow's CPU op kernels that the reference runs
(op inventory §2.11).  GPU-hot ops reach the hand-written HIP kernels
through the compiled-plan path (``graph/compiler.py``); the interpreter here is the
TF-semantics reference path.
"""
from __future__ import annotations

from typing import Callable

_REGISTRY: dict[str, Callable] = {}
# ops whose first input is a variable reference that must NOT be dereferenced
REF_INPUT_OPS = {"Assign", "AssignAdd", "AssignSub", "ScatterUpdate", "ScatterAdd", "ScatterSub", "IsVariableInitialized",
                 "AssignVariableOp", "AssignAddVariableOp", "AssignSubVariableOp", "ReadVariableOp", "ResourceGather"}
STATEFUL_OPS = {"VariableV2", "Variable", "VarHandleOp", "Assign", "AssignAdd", "AssignSub", "SaveV2", "RestoreV2",
                "MergeV2Checkpoints", "Save", "Restore", "AssignVariableOp", "AssignAddVariableOp",
                "AssignSubVariableOp", "ScatterUpdate", "ScatterAdd", "ScatterSub", "RandomUniform",
                "RandomStandardNormal", "TruncatedNormal", "Print", "PrintV2"}


def register(*names: str):
    def deco(fn):
        for n in names:
            _REGISTRY[n] = fn
        return fn

    return deco


def lookup(op: str) -> Callable:
    try:
        return _REGISTRY[op]
    except KeyError:
        raise NotImplementedError(f"op {op!r} is not supported by the executor") from None


def supported_ops() -> set[str]:
    return set(_REGISTRY)


class OpContext:
    """Per-run execution context handed to kernels."""

    def __init__(self, session, device, run_options=None):
        self.session = session
        self.device = device
        self.run_options = run_options or {}

    @property
    def variables(self):
        return self.session.variables
