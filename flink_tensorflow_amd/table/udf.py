"""User-defined scalar functions of the Table API, including model-backed ones.

``ScalarFunction`` mirrors Flink's: ``eval(*args)`` plus an ``open``/``close`` lifecycle
run on each parallel subtask.  ``ModelScalarFunction`` is the Table-API face of the
reference's ``mapWithModel`` (``LIB/streaming/package.scala:15-43``): the wrapped model is
opened on the subtask's device in ``open`` (``ModelAwareFunction`` semantics,
``LIB/common/functions/util/ModelAwareFunction.scala:10-19``) and ``fn(model, *args)`` is
evaluated per row, so ``SELECT classify(features) FROM events`` runs the TF graph inside a
streaming SQL query.
"""
from __future__ import annotations

from typing import Callable

from .expressions import Call, lit_if


class ScalarFunction:
    def __init__(self, fn: Callable | None = None, name: str | None = None):
        self.fn = fn
        self.name = name or getattr(fn, "__name__", type(self).__name__)

    def open(self, ctx) -> None:  # noqa: B027 - optional hook
        pass

    def close(self) -> None:  # noqa: B027 - optional hook
        pass

    def eval(self, *args):
        if self.fn is None:
            raise NotImplementedError(f"{type(self).__name__}.eval")
        return self.fn(*args)

    def eval_bound(self, env, *args):
        return self.eval(*args)

    def __call__(self, *args) -> Call:
        return Call(self.name, [lit_if(a) for a in args], None, udf=self)


def udf(fn: Callable | None = None, name: str | None = None):
    """``udf(f)`` or ``@udf`` / ``@udf(name=...)``: a ``ScalarFunction`` from a callable."""
    if fn is None:
        return lambda f: ScalarFunction(f, name)
    return ScalarFunction(fn, name)


class ModelScalarFunction(ScalarFunction):
    """``fn(model, *args)`` per row with ``model`` opened on the subtask's GPU."""

    def __init__(self, model, fn: Callable, name: str = "model_udf"):
        super().__init__(None, name)
        if model is None or fn is None:
            raise ValueError("model and function must not be None")
        self.model = model
        self.model_fn = fn

    def open(self, ctx) -> None:
        from ..runtime.model_functions import open_model

        open_model(self.model, getattr(ctx, "device", None))

    def close(self) -> None:
        from ..runtime.model_functions import close_model

        close_model(self.model)

    def eval(self, *args):
        return self.model_fn(self.model, *args)
