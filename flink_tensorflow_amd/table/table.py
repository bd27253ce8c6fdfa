"""Table API over the streaming runtime (the Flink ``Table``/``StreamTableEnvironment``
surface named by BASELINE.json's north star; the reference itself stops at DataStream).

A ``Table`` is a logical view of a ``DataStream`` of ``Row``s with a schema, plus its
changelog kind:

* **append** tables carry plain rows (sources, projections, filters, window aggregates,
  joins of append tables);
* **retract** tables carry ``(is_add, Row)`` change messages (non-windowed group
  aggregates: each update retracts the group's previous row and adds the new one).

Relational operators compile to DataStream operators of the runtime, so tables inherit
parallelism, keyed state, event-time windows, checkpoints and restarts:

=========================  ====================================================
``select`` / ``where``     map / filter (expressions evaluated per row)
``group_by().select()``    ``key_by`` + keyed process with retractable accumulators
``window().group_by()``    ``key_by`` + tumbling/sliding event- or processing-time window
``join``                   ``connect`` + keyed co-process (inner equi-join, list state)
``union_all``              union
model scalar functions     a rich map that opens the model on the subtask's device
=========================  ====================================================
"""
from __future__ import annotations

from collections import Counter
from dataclasses import dataclass
from typing import Any, Iterable, Sequence

from ..runtime import functions as F
from ..runtime.operators import SlidingEventTimeWindows, TumblingEventTimeWindows, TumblingProcessingTimeWindows
from ..runtime.state import ListStateDescriptor, ValueStateDescriptor
from .expressions import Agg, Alias, BinOp, Col, Expr, Row, WindowProp, col, output_name


class TableError(ValueError):
    pass


# ------------------------------------------------------------------ group windows
@dataclass
class GroupWindow:
    kind: str                 # "tumble" | "slide"
    size: float
    slide: float | None = None
    time_col: str | None = None
    alias_name: str | None = None

    def on(self, time_col) -> "GroupWindow":
        self.time_col = time_col.name() if isinstance(time_col, Expr) else str(time_col)
        return self

    def alias(self, name: str) -> "GroupWindow":
        self.alias_name = name
        return self


class _TumbleBuilder:
    def over(self, size_s: float) -> GroupWindow:
        return GroupWindow("tumble", float(size_s))


class _SlideBuilder:
    class _Over:
        def __init__(self, size):
            self.size = size

        def every(self, slide_s: float) -> GroupWindow:
            return GroupWindow("slide", self.size, float(slide_s))

    def over(self, size_s: float) -> "_SlideBuilder._Over":
        return _SlideBuilder._Over(float(size_s))


Tumble = _TumbleBuilder()
Slide = _SlideBuilder()


# ------------------------------------------------------------------ row functions
def _to_row_fn(fields: tuple):
    def to_row(v):
        if isinstance(v, Row):
            if type(v)._fields == fields:
                return v
            return Row.of(fields, [v[f] for f in fields])
        if isinstance(v, dict):
            return Row.of(fields, [v.get(f) for f in fields])
        if isinstance(v, (tuple, list)):
            return Row.of(fields, v)
        return Row.of(fields, (v,))

    return to_row


class _ExprFunction(F.RichFunction):
    """Shared lifecycle: opens every scalar/model function used by its expressions on the
    subtask (after the operator cloned the whole expression tree for this subtask)."""

    def _exprs(self) -> list[Expr]:
        return []

    def open(self, config=None):
        ctx = getattr(self, "_runtime_context", None)
        for e in self._exprs():
            for u in e.udfs():
                u.open(ctx)

    def close(self):
        for e in self._exprs():
            for u in e.udfs():
                u.close()


class _Project(_ExprFunction, F.MapFunction):
    def __init__(self, exprs: list[Expr], out_fields: tuple, retract: bool):
        super().__init__()
        self.exprs, self.out_fields, self.retract = exprs, out_fields, retract

    def _exprs(self):
        return self.exprs

    def map(self, value):
        if self.retract:
            flag, row = value
            return flag, Row.of(self.out_fields, [e.eval(row) for e in self.exprs])
        return Row.of(self.out_fields, [e.eval(value) for e in self.exprs])


class _Where(_ExprFunction, F.FilterFunction):
    def __init__(self, pred: Expr, retract: bool):
        super().__init__()
        self.pred, self.retract = pred, retract

    def _exprs(self):
        return [self.pred]

    def filter(self, value):
        return self.pred.eval(value[1] if self.retract else value) is True


def _project_agg(exprs, out_fields, row, accs_by_id, window=None):
    env = {"__aggs__": {k: a.result() for k, a in accs_by_id.items()}, "__window__": window}
    return Row.of(out_fields, [e.eval(row, env) for e in exprs])


class _GroupAgg(_ExprFunction, F.ProcessFunction):
    """Non-windowed GROUP BY: retractable accumulators per key; emits a retraction of the
    group's previous result row and the new row on every change."""

    def __init__(self, exprs, out_fields, aggs, having, retract_in: bool):
        super().__init__()
        self.exprs, self.out_fields, self.aggs, self.having, self.retract_in = exprs, out_fields, aggs, having, retract_in

    def _exprs(self):
        return list(self.exprs) + ([self.having] if self.having is not None else [])

    def open(self, config=None):
        super().open(config)
        ctx = self.get_runtime_context()
        self.acc = ctx.get_state(ValueStateDescriptor("accs"))
        self.last = ctx.get_state(ValueStateDescriptor("last"))

    def process_element(self, value, ctx, out):
        flag, row = value if self.retract_in else (True, value)
        st = self.acc.value()
        if st is None:
            st = {"n": 0, "accs": [a.accumulator() for a in self.aggs]}
        sign = 1 if flag else -1
        st["n"] += sign
        for a, acc in zip(self.aggs, st["accs"]):
            acc.add(a.expr.eval(row) if a.expr is not None else 1, sign)
        new = None
        if st["n"] > 0:
            new = _project_agg(self.exprs, self.out_fields, row, {id(a): acc for a, acc in zip(self.aggs, st["accs"])})
            if self.having is not None:
                hv = _project_agg([self.having], ("h",), row, {id(a): acc for a, acc in zip(self.aggs, st["accs"])})
                if hv[0] is not True:
                    new = None
        old = self.last.value()
        if st["n"] > 0:
            self.acc.update(st)
        else:
            self.acc.clear()
        if old == new:
            return
        if old is not None:
            out.collect((False, old))
        if new is not None:
            out.collect((True, new))
        self.last.update(new)


class _WindowAgg(_ExprFunction):
    def __init__(self, exprs, out_fields, aggs, having):
        super().__init__()
        self.exprs, self.out_fields, self.aggs, self.having = exprs, out_fields, aggs, having

    def _exprs(self):
        return list(self.exprs) + ([self.having] if self.having is not None else [])

    def _emit(self, window, inputs, out):
        rows = list(inputs)
        if not rows:
            return
        accs = [a.accumulator() for a in self.aggs]
        for r in rows:
            for a, acc in zip(self.aggs, accs):
                acc.add(a.expr.eval(r) if a.expr is not None else 1)
        by_id = {id(a): acc for a, acc in zip(self.aggs, accs)}
        if self.having is not None:
            if _project_agg([self.having], ("h",), rows[0], by_id, window)[0] is not True:
                return
        out.collect(_project_agg(self.exprs, self.out_fields, rows[0], by_id, window))


class _KeyedWindowAgg(_WindowAgg, F.WindowFunction):
    def apply(self, key, window, inputs, out):
        self._emit(window, inputs, out)


class _AllWindowAgg(_WindowAgg, F.AllWindowFunction):
    def apply(self, window, inputs, out):
        self._emit(window, inputs, out)


class _Join(_ExprFunction, F.CoProcessFunction):
    """Inner equi-join of two append tables: each side's rows are kept in keyed list
    state and every arrival is joined with the other side's rows for its key."""

    def __init__(self, out_fields, residual: Expr | None):
        super().__init__()
        self.out_fields, self.residual = out_fields, residual

    def _exprs(self):
        return [self.residual] if self.residual is not None else []

    def open(self, config=None):
        super().open(config)
        ctx = self.get_runtime_context()
        self.left = ctx.get_list_state(ListStateDescriptor("left"))
        self.right = ctx.get_list_state(ListStateDescriptor("right"))

    def _emit(self, l, r, out):
        row = Row.of(self.out_fields, tuple(l) + tuple(r))
        if self.residual is None or self.residual.eval(row) is True:
            out.collect(row)

    def process_element1(self, value, ctx, out):
        self.left.add(value)
        for r in self.right.get():
            self._emit(value, r, out)

    def process_element2(self, value, ctx, out):
        self.right.add(value)
        for l in self.left.get():
            self._emit(l, value, out)


def _key_fn(key_exprs: list[Expr], retract: bool):
    def key(v):
        row = v[1] if retract else v
        return tuple(e.eval(row) for e in key_exprs)

    return key


# ------------------------------------------------------------------ table
class Table:
    def __init__(self, t_env: "StreamTableEnvironment", stream, fields: Sequence[str], kind: str = "append",
                 time_attrs: dict | None = None, plan: str = ""):
        self.t_env = t_env
        self.stream = stream
        self.fields = tuple(fields)
        self.kind = kind
        self.time_attrs = dict(time_attrs or {})
        self.plan = plan

    # ---- schema
    def get_schema(self) -> list[str]:
        return list(self.fields)

    def print_schema(self):
        print("(\n" + ",\n".join(f"  `{f}`" + (f" *{self.time_attrs[f].upper()}*" if f in self.time_attrs else "")
                                 for f in self.fields) + "\n)")

    def explain(self) -> str:
        return self.plan

    @property
    def is_append_only(self) -> bool:
        return self.kind == "append"

    def _check_cols(self, exprs: Iterable[Expr], allow=()):
        for e in exprs:
            for c in e.columns():
                if c not in self.fields and c not in allow:
                    raise TableError(f"column {c!r} not in {list(self.fields)}")

    def _derive(self, stream, fields, kind=None, time_attrs=None, op=""):
        return Table(self.t_env, stream, fields, kind or self.kind,
                     self.time_attrs if time_attrs is None else time_attrs, f"{op}\n  {self.plan}".rstrip())

    # ---- relational operators
    def select(self, *exprs) -> "Table":
        exprs = _expand(self, exprs)
        if any(e.aggregates() for e in exprs):
            return GroupedTable(self, []).select(*exprs)
        self._check_cols(exprs)
        out = _out_fields(exprs)
        ta = {output_name(e, i): self.time_attrs[e.col] for i, e in enumerate(exprs)
              if isinstance(e, Col) and e.col in self.time_attrs}
        s = self.stream.map(_Project(exprs, out, self.kind == "retract"), name="select")
        return self._derive(s, out, time_attrs=ta, op=f"Project({', '.join(map(repr, exprs))})")

    def add_columns(self, *exprs) -> "Table":
        return self.select(*[col(f) for f in self.fields], *exprs)

    def drop_columns(self, *names) -> "Table":
        drop = {n.name() if isinstance(n, Expr) else n for n in names}
        return self.select(*[col(f) for f in self.fields if f not in drop])

    def rename_columns(self, **mapping) -> "Table":
        return self.select(*[col(f).alias(mapping.get(f, f)) for f in self.fields])

    def where(self, pred: Expr) -> "Table":
        self._check_cols([pred])
        s = self.stream.filter(_Where(pred, self.kind == "retract"), name="where")
        return self._derive(s, self.fields, op=f"Filter({pred!r})")

    filter = where

    def group_by(self, *keys) -> "GroupedTable":
        return GroupedTable(self, [_as_expr(k) for k in keys])

    def window(self, w: GroupWindow) -> "WindowedTable":
        if w.time_col is None or w.alias_name is None:
            raise TableError("a group window needs .on(time attribute) and .alias(name)")
        if w.time_col not in self.time_attrs:
            raise TableError(f"{w.time_col!r} is not a time attribute (declare rowtime= or proctime=)")
        return WindowedTable(self, w)

    def union_all(self, other: "Table") -> "Table":
        if other.fields != self.fields or other.kind != self.kind:
            raise TableError("union_all needs identical schemas and changelog kinds")
        return self._derive(self.stream.union(other.stream), self.fields, op="UnionAll")

    def join(self, right: "Table", on: Expr) -> "Table":
        if self.kind != "append" or right.kind != "append":
            raise TableError("join supports append-only tables")
        clash = set(self.fields) & set(right.fields)
        if clash:
            raise TableError(f"join inputs share column names {sorted(clash)}; rename first")
        lk, rk, residual = _split_equi(on, set(self.fields), set(right.fields))
        if not lk:
            raise TableError("join needs at least one equality between the two tables")
        out = self.fields + right.fields
        s = self.stream.connect(right.stream).key_by(_key_fn(lk, False), _key_fn(rk, False)) \
            .process(_Join(out, residual), name="join")
        return Table(self.t_env, s, out, "append", {}, f"Join({on!r})\n  {self.plan}\n  {right.plan}")

    def map_with_model(self, model, fn, out_field: str = "prediction") -> "Table":
        """Adds ``fn(model, row)`` as a column (``mapWithModel`` on a table)."""
        from .udf import ModelScalarFunction

        f = ModelScalarFunction(model, lambda m, *vals: fn(m, Row.of(self.fields, vals)), name="map_with_model")
        return self.add_columns(f(*[col(c) for c in self.fields]).alias(out_field))

    def map_with_model_batched(self, model, fn, out_field: str = "prediction", max_batch: int = 64,
                               max_delay_ms: float = 5.0) -> "Table":
        """Adds ``fn(model, rows) -> [value per row]`` as a column, evaluated on
        micro-batches of up to ``max_batch`` rows (or whatever arrived within
        ``max_delay_ms``) by the batched model operator — one GPU launch per batch instead
        of one per row (e.g. ``fn = lambda m, rows: m.predict([r.text for r in rows])``)."""
        if self.kind != "append":
            raise TableError("map_with_model_batched needs an append-only table")
        out = self.fields + (out_field,)

        def batch(m, rows, fn=fn, out=out):
            vals = list(fn(m, rows))
            if len(vals) != len(rows):
                raise TableError(f"model function returned {len(vals)} values for {len(rows)} rows")
            return [Row.of(out, tuple(r) + (v,)) for r, v in zip(rows, vals)]

        s = self.stream.map_with_model_batched(model, batch, max_batch=max_batch, max_delay_ms=max_delay_ms,
                                               name="table-batched-model")
        return self._derive(s, out, op=f"BatchedModelMap({out_field})")

    # ---- conversions
    def to_data_stream(self):
        return self.t_env.to_data_stream(self)

    def to_retract_stream(self):
        return self.t_env.to_retract_stream(self)

    def execute(self) -> "TableResult":
        sink = self.stream.collect_into()
        self.t_env.env.execute("table")
        return TableResult(self, sink.results())

    def to_pandas(self):
        import pandas as pd

        rows = self.execute().collect()
        return pd.DataFrame([list(r) for r in rows], columns=list(self.fields))


class GroupedTable:
    def __init__(self, table: Table, keys: list[Expr], window: GroupWindow | None = None):
        self.table, self.keys, self.window = table, keys, window

    def select(self, *exprs, having: Expr | None = None) -> Table:
        t = self.table
        exprs = _expand(t, exprs)
        allow = {self.window.alias_name} if self.window else set()
        t._check_cols(exprs + ([having] if having is not None else []), allow)
        t._check_cols(self.keys)
        aggs = []
        for e in exprs + ([having] if having is not None else []):
            for a in e.aggregates():
                if not any(a is b for b in aggs):  # identity: Expr.__eq__ builds a predicate
                    aggs.append(a)
        key_cols = set().union(*[k.columns() for k in self.keys]) if self.keys else set()
        for e in exprs:  # non-aggregated columns must be grouping columns
            bare = _bare_columns(e)
            if not bare <= key_cols:
                raise TableError(f"{e!r} uses {sorted(bare - key_cols)} which is neither grouped nor aggregated")
        out = _out_fields(exprs)
        desc = f"{'Window' if self.window else 'Group'}Aggregate(keys={self.keys!r}, select={exprs!r})"
        if self.window is None:
            retract_in = t.kind == "retract"
            keyed = t.stream.key_by(_key_fn(self.keys, retract_in))
            s = keyed.process(_GroupAgg(exprs, out, aggs, having, retract_in), name="group-agg")
            return Table(t.t_env, s, out, "retract", {}, f"{desc}\n  {t.plan}")
        if t.kind != "append":
            raise TableError("group windows need an append-only input")
        w = self.window
        event = t.time_attrs[w.time_col] == "rowtime"
        if w.kind == "tumble":
            asg = TumblingEventTimeWindows(w.size) if event else TumblingProcessingTimeWindows(w.size)
        else:
            if not event:
                raise TableError("sliding windows need an event-time (rowtime) attribute")
            asg = SlidingEventTimeWindows(w.size, w.slide)
        if self.keys:
            s = t.stream.key_by(_key_fn(self.keys, False)).window(asg).apply(
                _KeyedWindowAgg(exprs, out, aggs, having), name="window-agg")
        else:
            s = t.stream.window_all(asg).apply(_AllWindowAgg(exprs, out, aggs, having), name="window-agg")
        return Table(t.t_env, s, out, "append", {}, f"{desc} over {w}\n  {t.plan}")


class WindowedTable:
    def __init__(self, table: Table, window: GroupWindow):
        self.table, self.window = table, window

    def group_by(self, *keys) -> GroupedTable:
        ks = [_as_expr(k) for k in keys]
        if not any(isinstance(k, Col) and k.col == self.window.alias_name for k in ks):
            raise TableError(f"a windowed group_by must include the window alias {self.window.alias_name!r}")
        ks = [k for k in ks if not (isinstance(k, Col) and k.col == self.window.alias_name)]
        return GroupedTable(self.table, ks, self.window)


class TableResult:
    def __init__(self, table: Table, messages: list):
        self.table = table
        self.messages = messages

    def changelog(self) -> list:
        return list(self.messages) if self.table.kind == "retract" else [(True, r) for r in self.messages]

    def collect(self) -> list:
        """Rows of the result; an updating table is materialised (its changelog applied)."""
        if self.table.kind == "append":
            return list(self.messages)
        bag = Counter()
        for flag, row in self.messages:
            bag[row] += 1 if flag else -1
        out = []
        for row, n in bag.items():
            if n < 0:
                raise TableError(f"changelog retracts {row!r} more often than it was added")
            out.extend([row] * n)
        return out

    def print(self):
        for r in self.collect():
            print(r)


# ------------------------------------------------------------------ helpers
def _as_expr(e) -> Expr:
    return e if isinstance(e, Expr) else col(str(e))


def _expand(t: Table, exprs) -> list[Expr]:
    out = []
    for e in exprs:
        if isinstance(e, str) and e == "*":
            out.extend(col(f) for f in t.fields)
        else:
            out.append(_as_expr(e))
    return out


def _out_fields(exprs) -> tuple:
    names = [output_name(e, i) for i, e in enumerate(exprs)]
    if len(set(names)) != len(names):
        raise TableError(f"duplicate output columns {names}; use .alias()")
    return tuple(names)


def _bare_columns(e: Expr) -> set[str]:
    """Columns referenced outside aggregate calls and window properties."""
    if isinstance(e, (Agg, WindowProp)):
        return set()
    if isinstance(e, Col):
        return {e.col}
    return set().union(*[_bare_columns(c) for c in e.children()]) if e.children() else set()


def _split_equi(on: Expr, left: set, right: set):
    conj = []

    def flatten(e):
        if isinstance(e, BinOp) and e.op == "AND":
            flatten(e.left)
            flatten(e.right)
        else:
            conj.append(e)

    flatten(on)
    lk, rk, rest = [], [], []
    for c in conj:
        if isinstance(c, BinOp) and c.op == "=":
            lc, rc = c.left.columns(), c.right.columns()
            if lc and rc and lc <= left and rc <= right:
                lk.append(c.left)
                rk.append(c.right)
                continue
            if lc and rc and lc <= right and rc <= left:
                lk.append(c.right)
                rk.append(c.left)
                continue
        rest.append(c)
    residual = None
    for c in rest:
        residual = c if residual is None else BinOp("AND", residual, c)
    return lk, rk, residual


class StreamTableEnvironment:
    """``StreamTableEnvironment.create(env)``: tables from/to DataStreams, a catalog of
    temporary views and functions, and ``sql_query``."""

    def __init__(self, env):
        self.env = env
        self.views: dict[str, Table] = {}
        self.functions: dict[str, Any] = {}

    @staticmethod
    def create(env) -> "StreamTableEnvironment":
        return StreamTableEnvironment(env)

    def from_data_stream(self, stream, *fields, rowtime: str | None = None, proctime: str | None = None,
                         max_out_of_orderness_s: float = 0.0) -> Table:
        """Rows from tuples / dicts / Rows / scalars.  ``rowtime`` names the event-time
        column (timestamps + bounded-out-of-orderness watermarks are assigned from it);
        ``proctime`` appends a processing-time attribute column."""
        if len(fields) == 1 and isinstance(fields[0], (list, tuple)):
            fields = tuple(fields[0])
        fields = tuple(f.name() if isinstance(f, Expr) else f for f in fields)
        if not fields:
            raise TableError("from_data_stream needs the field names")
        s = stream.map(_to_row_fn(fields), name="to-row")
        ta = {}
        if rowtime is not None:
            if rowtime not in fields:
                raise TableError(f"rowtime {rowtime!r} is not a field")
            idx = fields.index(rowtime)
            s = s.assign_timestamps_and_watermarks(lambda r, i=idx: r[i], max_out_of_orderness_s)
            ta[rowtime] = "rowtime"
        if proctime is not None:
            import time as _t

            out = fields + (proctime,)
            s = s.map(lambda r, out=out: Row.of(out, tuple(r) + (_t.time(),)), name="proctime")
            fields = out
            ta[proctime] = "proctime"
        return Table(self, s, fields, "append", ta, f"DataStreamScan({', '.join(fields)})")

    def from_elements(self, rows: Sequence, fields: Sequence[str], **kw) -> Table:
        return self.from_data_stream(self.env.from_collection(list(rows)), tuple(fields), **kw)

    def create_temporary_view(self, name: str, table: Table) -> None:
        self.views[name] = table

    def from_path(self, name: str) -> Table:
        if name not in self.views:
            raise TableError(f"no table {name!r} (registered: {sorted(self.views)})")
        return self.views[name]

    def create_temporary_function(self, name: str, fn) -> None:
        from .udf import ScalarFunction, udf

        self.functions[name.upper()] = fn if isinstance(fn, ScalarFunction) else udf(fn, name)

    def sql_query(self, query: str) -> Table:
        from .sql import plan_query

        return plan_query(self, query)

    def to_data_stream(self, table: Table):
        if table.kind != "append":
            raise TableError("an updating (retract) table cannot become an append DataStream; "
                             "use to_retract_stream")
        return table.stream

    def to_append_stream(self, table: Table):
        return self.to_data_stream(table)

    def to_retract_stream(self, table: Table):
        if table.kind == "retract":
            return table.stream
        return table.stream.map(lambda r: (True, r), name="as-retract")

    def to_changelog_stream(self, table: Table):
        return self.to_retract_stream(table)


__all__ = ["GroupWindow", "GroupedTable", "Slide", "StreamTableEnvironment", "Table", "TableError", "TableResult",
           "Tumble", "WindowedTable", "Alias"]
