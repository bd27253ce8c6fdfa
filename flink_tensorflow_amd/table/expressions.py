"""Expression DSL of the Table API: ``col("x") * 2 + lit(1)``, comparisons, boolean logic,
aggregates (``col("x").sum``), window properties (``col("w").start``) and scalar function
calls (user functions and models).

Expressions are trees evaluated against a ``Row``; aggregates are evaluated by the
group-aggregate operators through ``Accumulator`` objects that support retraction (needed
for aggregates over updating tables).
"""
from __future__ import annotations

import math
from typing import Any, Callable, Sequence


class Row(tuple):
    """An immutable row with named fields: ``row.user``, ``row["user"]``, ``row[0]``."""

    __slots__ = ()
    _fields: tuple = ()

    def __new__(cls, values: Sequence = (), fields: Sequence[str] = ()):
        r = super().__new__(cls, tuple(values))
        return r

    @classmethod
    def of(cls, fields: Sequence[str], values: Sequence) -> "Row":
        if len(fields) != len(values):
            raise ValueError(f"row has {len(values)} values for {len(fields)} fields")
        sub = _row_class(tuple(fields))
        return tuple.__new__(sub, tuple(values))

    def __getattr__(self, name):
        try:
            return tuple.__getitem__(self, type(self)._fields.index(name))
        except ValueError:
            raise AttributeError(name) from None

    def __getitem__(self, k):
        if isinstance(k, str):
            return tuple.__getitem__(self, type(self)._fields.index(k))
        return tuple.__getitem__(self, k)

    def as_dict(self) -> dict:
        return dict(zip(type(self)._fields, self))

    def __repr__(self):
        return "Row(" + ", ".join(f"{f}={v!r}" for f, v in zip(type(self)._fields, self)) + ")"

    def __reduce__(self):
        return (Row.of, (type(self)._fields, tuple(self)))


_ROW_CLASSES: dict[tuple, type] = {}


def _row_class(fields: tuple) -> type:
    c = _ROW_CLASSES.get(fields)
    if c is None:
        c = type("Row", (Row,), {"__slots__": (), "_fields": fields})
        _ROW_CLASSES[fields] = c
    return c


# ------------------------------------------------------------------ expressions
class Expr:
    __hash__ = object.__hash__

    # arithmetic
    def __add__(self, o): return BinOp("+", self, lit_if(o))
    def __radd__(self, o): return BinOp("+", lit_if(o), self)
    def __sub__(self, o): return BinOp("-", self, lit_if(o))
    def __rsub__(self, o): return BinOp("-", lit_if(o), self)
    def __mul__(self, o): return BinOp("*", self, lit_if(o))
    def __rmul__(self, o): return BinOp("*", lit_if(o), self)
    def __truediv__(self, o): return BinOp("/", self, lit_if(o))
    def __rtruediv__(self, o): return BinOp("/", lit_if(o), self)
    def __mod__(self, o): return BinOp("%", self, lit_if(o))
    def __neg__(self): return Call("neg", [self], lambda a: -a)

    # comparison (SQL three-valued: None compares as None)
    def __eq__(self, o): return BinOp("=", self, lit_if(o))  # type: ignore[override]
    def __ne__(self, o): return BinOp("<>", self, lit_if(o))  # type: ignore[override]
    def __lt__(self, o): return BinOp("<", self, lit_if(o))
    def __le__(self, o): return BinOp("<=", self, lit_if(o))
    def __gt__(self, o): return BinOp(">", self, lit_if(o))
    def __ge__(self, o): return BinOp(">=", self, lit_if(o))

    # boolean
    def __and__(self, o): return BinOp("AND", self, lit_if(o))
    def __or__(self, o): return BinOp("OR", self, lit_if(o))
    def __invert__(self): return Call("NOT", [self], lambda a: None if a is None else not a)

    def is_null(self): return Call("IS NULL", [self], lambda a: a is None, null_safe=True)
    def is_not_null(self): return Call("IS NOT NULL", [self], lambda a: a is not None, null_safe=True)

    def alias(self, name: str) -> "Alias":
        return Alias(self, name)

    def cast(self, typ: type) -> "Expr":
        return Call(f"CAST({typ.__name__})", [self], typ)

    # aggregates
    @property
    def sum(self): return Agg("sum", self)
    @property
    def count(self): return Agg("count", self)
    @property
    def avg(self): return Agg("avg", self)
    @property
    def min(self): return Agg("min", self)
    @property
    def max(self): return Agg("max", self)

    # evaluation
    def eval(self, row, env=None):
        raise NotImplementedError

    def name(self) -> str:
        return str(self)

    def columns(self) -> set[str]:
        return set().union(*[c.columns() for c in self.children()]) if self.children() else set()

    def children(self) -> list["Expr"]:
        return []

    def aggregates(self) -> list["Agg"]:
        return [a for c in self.children() for a in c.aggregates()]

    def udfs(self) -> list:
        return [u for c in self.children() for u in c.udfs()]


def lit_if(v) -> Expr:
    return v if isinstance(v, Expr) else Lit(v)


class Col(Expr):
    def __init__(self, name: str):
        self.col = name

    def eval(self, row, env=None):
        return row[self.col]

    def name(self):
        return self.col

    def columns(self):
        return {self.col}

    @property
    def start(self):
        return WindowProp(self.col, "start")

    @property
    def end(self):
        return WindowProp(self.col, "end")

    def __repr__(self):
        return self.col


class Lit(Expr):
    def __init__(self, v):
        self.v = v

    def eval(self, row, env=None):
        return self.v

    def __repr__(self):
        return repr(self.v)


def _arith(op: str, a, b):
    if a is None or b is None:
        return None
    if op == "+":
        return a + b
    if op == "-":
        return a - b
    if op == "*":
        return a * b
    if op == "/":
        return a / b
    if op == "%":
        return a % b
    raise ValueError(op)


_CMP = {"=": lambda a, b: a == b, "<>": lambda a, b: a != b, "<": lambda a, b: a < b, "<=": lambda a, b: a <= b,
        ">": lambda a, b: a > b, ">=": lambda a, b: a >= b}


class BinOp(Expr):
    def __init__(self, op: str, left: Expr, right: Expr):
        self.op, self.left, self.right = op, left, right

    def children(self):
        return [self.left, self.right]

    def eval(self, row, env=None):
        if self.op == "AND":
            a = self.left.eval(row, env)
            if a is False:
                return False
            b = self.right.eval(row, env)
            if b is False:
                return False
            return None if a is None or b is None else True
        if self.op == "OR":
            a = self.left.eval(row, env)
            if a is True:
                return True
            b = self.right.eval(row, env)
            if b is True:
                return True
            return None if a is None or b is None else False
        a, b = self.left.eval(row, env), self.right.eval(row, env)
        if self.op in _CMP:
            return None if a is None or b is None else _CMP[self.op](a, b)
        return _arith(self.op, a, b)

    def __repr__(self):
        return f"({self.left!r} {self.op} {self.right!r})"


class Call(Expr):
    """A scalar function applied to argument expressions."""

    def __init__(self, fname: str, args: list[Expr], fn: Callable, null_safe: bool = False, udf=None):
        self.fname, self.args, self.fn, self.null_safe, self.udf = fname, args, fn, null_safe, udf

    def children(self):
        return self.args

    def eval(self, row, env=None):
        vals = [a.eval(row, env) for a in self.args]
        if not self.null_safe and any(v is None for v in vals):
            return None
        if self.udf is not None:
            return self.udf.eval_bound(env, *vals)
        return self.fn(*vals)

    def udfs(self):
        own = [self.udf] if self.udf is not None else []
        return own + super().udfs()

    def __repr__(self):
        return f"{self.fname}({', '.join(map(repr, self.args))})"


class Alias(Expr):
    def __init__(self, expr: Expr, name: str):
        self.expr, self.alias_name = expr, name

    def children(self):
        return [self.expr]

    def eval(self, row, env=None):
        return self.expr.eval(row, env)

    def name(self):
        return self.alias_name

    def __repr__(self):
        return f"{self.expr!r} AS {self.alias_name}"


class WindowProp(Expr):
    """``w.start`` / ``w.end`` of a group window (resolved by the window aggregate)."""

    def __init__(self, window: str, prop: str):
        self.window, self.prop = window, prop

    def eval(self, row, env=None):
        w = env.get("__window__") if env else None
        if w is None:
            raise ValueError(f"{self!r} is only defined in a window aggregation")
        return getattr(w, self.prop)

    def name(self):
        return f"{self.window}_{self.prop}"

    def __repr__(self):
        return f"{self.window}.{self.prop}"


class Agg(Expr):
    """An aggregate call; ``expr`` None means COUNT(*)."""

    def __init__(self, kind: str, expr: Expr | None, distinct: bool = False):
        self.kind, self.expr, self.distinct = kind, expr, distinct

    def children(self):
        return [self.expr] if self.expr is not None else []

    def aggregates(self):
        return [self]

    def eval(self, row, env=None):
        # inside an aggregate projection the accumulated value is looked up by identity
        return env["__aggs__"][id(self)]

    def name(self):
        inner = self.expr.name() if self.expr is not None else "star"
        return f"{self.kind}_{inner}"

    def accumulator(self) -> "Accumulator":
        return Accumulator(self.kind, self.distinct)

    def __repr__(self):
        return f"{self.kind.upper()}({'*' if self.expr is None else repr(self.expr)})"


class Accumulator:
    """Retractable accumulator: sum / count / avg keep running totals; min / max keep a
    value multiset so retracting the current extreme is exact."""

    def __init__(self, kind: str, distinct: bool = False):
        if kind not in ("sum", "count", "avg", "min", "max"):
            raise ValueError(f"unknown aggregate {kind!r}")
        self.kind, self.distinct = kind, distinct
        self.n = 0
        self.total = 0
        self.counts: dict = {}

    def add(self, v, sign: int = 1):
        if v is None and self.kind != "count":
            return
        if self.distinct or self.kind in ("min", "max"):
            c = self.counts.get(v, 0) + sign
            if c:
                self.counts[v] = c
            else:
                self.counts.pop(v, None)
            if self.distinct:
                return
        if v is None:  # COUNT(col) skips NULLs, COUNT(*) passes a non-None marker
            return
        self.n += sign
        if self.kind in ("sum", "avg"):
            self.total += sign * v

    def result(self):
        if self.distinct:
            vals = list(self.counts)
            if self.kind == "count":
                return len(vals)
            if not vals:
                return None
            return {"sum": sum, "avg": lambda x: sum(x) / len(x), "min": min, "max": max}[self.kind](vals)
        if self.kind == "count":
            return self.n
        if self.n == 0:
            return None
        if self.kind == "sum":
            return self.total
        if self.kind == "avg":
            return self.total / self.n
        return (min if self.kind == "min" else max)(self.counts)

    @property
    def empty(self) -> bool:
        return self.n == 0 and not self.counts


# ------------------------------------------------------------------ constructors
def col(name: str) -> Col:
    return Col(name)


def lit(v) -> Lit:
    return Lit(v)


def count_star() -> Agg:
    return Agg("count", None)


def call(fn: "ScalarFunction | Callable", *args) -> Call:
    """Applies a scalar function (``ScalarFunction``, ``ModelScalarFunction`` or a plain
    callable) to argument expressions."""
    from .udf import ScalarFunction, udf

    f = fn if isinstance(fn, ScalarFunction) else udf(fn)
    return f(*args)


BUILTINS: dict[str, Callable] = {
    "ABS": abs,
    "UPPER": lambda s: s.upper(),
    "LOWER": lambda s: s.lower(),
    "CHAR_LENGTH": len,
    "ROUND": lambda x, n=0: round(x, int(n)),
    "SQRT": math.sqrt,
    "EXP": math.exp,
    "LN": math.log,
    "FLOOR": math.floor,
    "CEIL": math.ceil,
    "POWER": lambda a, b: a ** b,
    "MOD": lambda a, b: a % b,
}


def builtin(name: str, *args: Expr) -> Call:
    if name.upper() == "COALESCE":
        return Call("COALESCE", list(args), lambda *v: next((x for x in v if x is not None), None), null_safe=True)
    fn = BUILTINS.get(name.upper())
    if fn is None:
        raise KeyError(f"unknown function {name}")
    return Call(name.upper(), list(args), fn)


def output_name(e: Expr, i: int) -> str:
    if isinstance(e, (Col, Alias, WindowProp, Agg)):
        return e.name()
    return f"EXPR${i}"


def row_env(fields: Sequence[str], values: Sequence) -> dict[str, Any]:
    return dict(zip(fields, values))
