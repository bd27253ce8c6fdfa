"""``Saver`` / ``DefaultSaver`` — ``LIB/io/Saver.scala:14-89``.

Drives the graph's saver subgraph described by a ``SaverDef``:

* ``save(session, path)`` feeds ``filename_tensor_name`` with the path (STRING scalar),
  fetches ``save_tensor_name`` and returns its string value (the written prefix);
* ``restore(session, path)`` feeds the same tensor and targets ``restore_op_name``.

The SaveV2/RestoreV2/MergeV2Checkpoints kernels write/read TensorBundle V2 through the
native bundle I/O, so checkpoints interoperate with TF.  ``VariableSaver`` is the
graph-free variant used by the streaming checkpoint backend: it writes the session's
variable store (or any ``{name: tensor}`` dict) straight to a bundle.
"""
from __future__ import annotations

import abc

from ..proto.messages import SaverDef
from ..types.tensor import StringTensor
from . import bundle


class Saver(abc.ABC):
    @abc.abstractmethod
    def save(self, session, path: str) -> str:
        ...

    @abc.abstractmethod
    def restore(self, session, path: str) -> None:
        ...

    @staticmethod
    def create(saver_def: SaverDef) -> "DefaultSaver":
        return DefaultSaver(saver_def)


class DefaultSaver(Saver):
    def __init__(self, saver_def: SaverDef):
        if saver_def is None:
            raise ValueError("graph has no SaverDef")
        self.saver_def = saver_def

    def save(self, session, path: str) -> str:
        out = session.run(self.saver_def.save_tensor_name,
                          {self.saver_def.filename_tensor_name: StringTensor(path.encode())})
        return out.item().decode() if isinstance(out, StringTensor) else str(out)

    def restore(self, session, path: str) -> None:
        session.run(targets=[self.saver_def.restore_op_name.split(":")[0]],
                    feed_dict={self.saver_def.filename_tensor_name: StringTensor(path.encode())})


class VariableSaver(Saver):
    """Saves/restores a session's variable store without a saver subgraph."""

    def save(self, session, path: str) -> str:
        bundle.save_tensors(path, {k: v for k, v in session.variables.items() if v is not None})
        return path

    def restore(self, session, path: str) -> None:
        with bundle.BundleReader(path) as r:
            for k in r.keys():
                val = r.read(k, device=getattr(session, "device", None))
                cur = session.variables.get(k)
                if cur is not None and hasattr(cur, "copy_") and tuple(cur.shape) == tuple(val.shape):
                    cur.copy_(val)
                    if hasattr(session.variables, "touch"):
                        session.variables.touch()
                else:
                    session.variables[k] = val
