"""A streaming SQL subset planned onto the Table API.

::

    SELECT [DISTINCT] item [, item]* FROM view
      [WHERE cond]
      [GROUP BY [TUMBLE(t, INTERVAL 'n' unit) | HOP(t, INTERVAL slide, INTERVAL size),] expr [, expr]*]
      [HAVING cond]

    item := * | expr [[AS] name]
    expr := literals (numbers, 'strings', TRUE/FALSE/NULL), columns, + - * / %, comparisons
            (= <> != < <= > >=), AND / OR / NOT, IS [NOT] NULL, BETWEEN a AND b,
            aggregates (COUNT(*), COUNT/SUM/AVG/MIN/MAX([DISTINCT] e)), window bounds
            (TUMBLE_START/TUMBLE_END/HOP_START/HOP_END(t, ...)), built-ins (ABS, UPPER, LOWER,
            ROUND, SQRT, EXP, LN, FLOOR, CEIL, POWER, MOD, CHAR_LENGTH, COALESCE) and functions
            registered with ``create_temporary_function`` — including model-backed
            ``ModelScalarFunction``s.

Group windows follow Flink's group-window SQL: ``TUMBLE``/``HOP`` in GROUP BY over a
rowtime or proctime attribute; ``*_START``/``*_END`` in the select list.
``SELECT DISTINCT`` is a GROUP BY over all selected expressions.
"""
from __future__ import annotations

import re

from .expressions import Agg, BinOp, Call, Col, Expr, Lit, WindowProp, builtin, col
from .table import GroupWindow, Table, TableError

_TOKEN = re.compile(r"""\s*(?:
    (?P<num>\d+\.\d*|\.\d+|\d+)
  | (?P<str>'(?:[^']|'')*')
  | (?P<qid>`[^`]+`|"[^"]+")
  | (?P<id>[A-Za-z_][A-Za-z0-9_]*)
  | (?P<op><>|!=|<=|>=|=|<|>|\+|-|\*|/|%|\(|\)|,|\.)
)""", re.VERBOSE)

_KEYWORDS = {"SELECT", "DISTINCT", "FROM", "WHERE", "GROUP", "BY", "HAVING", "AS", "AND", "OR", "NOT", "IS", "NULL",
             "TRUE", "FALSE", "INTERVAL", "BETWEEN"}
_UNITS = {"SECOND": 1.0, "SECONDS": 1.0, "MINUTE": 60.0, "MINUTES": 60.0, "HOUR": 3600.0, "HOURS": 3600.0,
          "MILLISECOND": 1e-3, "MILLISECONDS": 1e-3, "DAY": 86400.0, "DAYS": 86400.0}
_AGGS = {"COUNT", "SUM", "AVG", "MIN", "MAX"}


def tokenize(sql: str) -> list[tuple[str, str]]:
    pos, out = 0, []
    sql = sql.strip().rstrip(";")
    while pos < len(sql):
        m = _TOKEN.match(sql, pos)
        if not m or m.end() == pos:
            raise TableError(f"SQL syntax error near {sql[pos:pos + 20]!r}")
        pos = m.end()
        kind = m.lastgroup
        text = m.group(kind)
        if kind == "id" and text.upper() in _KEYWORDS:
            out.append(("kw", text.upper()))
        elif kind == "qid":
            out.append(("id", text[1:-1]))
        elif kind == "str":
            out.append(("str", text[1:-1].replace("''", "'")))
        else:
            out.append((kind, text))
    out.append(("eof", ""))
    return out


class _Parser:
    def __init__(self, t_env, sql: str):
        self.t_env = t_env
        self.toks = tokenize(sql)
        self.i = 0
        self.window: GroupWindow | None = None

    # ---- token helpers
    def peek(self, k=0):
        return self.toks[self.i + k]

    def next(self):
        t = self.toks[self.i]
        self.i += 1
        return t

    def accept(self, kind, text=None) -> bool:
        t = self.peek()
        if t[0] == kind and (text is None or t[1].upper() == text):
            self.i += 1
            return True
        return False

    def expect(self, kind, text=None):
        if not self.accept(kind, text):
            raise TableError(f"SQL: expected {text or kind}, found {self.peek()[1]!r}")

    # ---- query
    def query(self) -> Table:
        self.expect("kw", "SELECT")
        distinct = self.accept("kw", "DISTINCT")
        items = self.select_list()
        self.expect("kw", "FROM")
        name = self.next()
        if name[0] != "id":
            raise TableError("SQL: FROM expects a view name")
        table = self.t_env.from_path(name[1])
        where = having = None
        group: list[Expr] | None = None
        if self.accept("kw", "WHERE"):
            where = self.expr()
        if self.accept("kw", "GROUP"):
            self.expect("kw", "BY")
            group = [self.group_item()]
            while self.accept("op", ","):
                group.append(self.group_item())
            group = [g for g in group if g is not None]
        if self.accept("kw", "HAVING"):
            having = self.expr()
        if self.peek()[0] != "eof":
            raise TableError(f"SQL: unexpected {self.peek()[1]!r}")
        if where is not None:
            table = table.where(where)
        if len(items) == 1 and isinstance(items[0], str):  # SELECT * (not ==: Expr.__eq__ is a predicate)
            items = [col(f) for f in table.fields]
        if distinct:
            if group is not None:
                raise TableError("SQL: DISTINCT with GROUP BY is not supported")
            group = [e.expr if hasattr(e, "alias_name") else e for e in items]
        if self.window is not None:
            wt = table.window(self.window).group_by(col(self.window.alias_name), *(group or []))
            return wt.select(*items, having=having)
        if group is not None or any(e.aggregates() for e in items):
            return table.group_by(*(group or [])).select(*items, having=having)
        if having is not None:
            raise TableError("SQL: HAVING needs GROUP BY or aggregates")
        return table.select(*items)

    def select_list(self):
        if self.accept("op", "*"):
            return ["*"]
        items = [self.select_item()]
        while self.accept("op", ","):
            items.append(self.select_item())
        return items

    def select_item(self) -> Expr:
        e = self.expr()
        if self.accept("kw", "AS"):
            t = self.next()
            return e.alias(t[1])
        if self.peek()[0] == "id":
            return e.alias(self.next()[1])
        return e

    def group_item(self):
        t = self.peek()
        if t[0] == "id" and t[1].upper() in ("TUMBLE", "HOP") and self.peek(1) == ("op", "("):
            self.next()
            self.expect("op", "(")
            tcol = self.expr()
            self.expect("op", ",")
            a = self.interval()
            if t[1].upper() == "TUMBLE":
                w = GroupWindow("tumble", a)
            else:  # HOP(t, slide, size)
                self.expect("op", ",")
                w = GroupWindow("slide", self.interval(), a)
            self.expect("op", ")")
            if self.window is not None and (self.window.kind, self.window.size, self.window.slide) != \
                    (w.kind, w.size, w.slide):
                raise TableError("SQL: one group window per query")
            w.on(tcol).alias("$w")
            self.window = w
            return None
        return self.expr()

    def interval(self) -> float:
        self.expect("kw", "INTERVAL")
        t = self.next()
        if t[0] not in ("str", "num"):
            raise TableError("SQL: INTERVAL expects a quoted amount")
        unit = self.next()[1].upper()
        if unit not in _UNITS:
            raise TableError(f"SQL: unknown interval unit {unit}")
        return float(t[1]) * _UNITS[unit]

    # ---- expressions (precedence climbing)
    def expr(self) -> Expr:
        return self.or_()

    def or_(self):
        e = self.and_()
        while self.accept("kw", "OR"):
            e = BinOp("OR", e, self.and_())
        return e

    def and_(self):
        e = self.not_()
        while self.accept("kw", "AND"):
            e = BinOp("AND", e, self.not_())
        return e

    def not_(self):
        if self.accept("kw", "NOT"):
            return ~self.not_()
        return self.cmp()

    def cmp(self):
        e = self.add()
        t = self.peek()
        if t[0] == "op" and t[1] in ("=", "<>", "!=", "<", "<=", ">", ">="):
            self.next()
            op = "<>" if t[1] == "!=" else t[1]
            return BinOp(op, e, self.add())
        if self.accept("kw", "IS"):
            neg = self.accept("kw", "NOT")
            self.expect("kw", "NULL")
            return e.is_not_null() if neg else e.is_null()
        if self.accept("kw", "BETWEEN"):
            lo = self.add()
            self.expect("kw", "AND")
            hi = self.add()
            return BinOp("AND", BinOp(">=", e, lo), BinOp("<=", e, hi))
        return e

    def add(self):
        e = self.mul()
        while self.peek()[0] == "op" and self.peek()[1] in ("+", "-"):
            op = self.next()[1]
            e = BinOp(op, e, self.mul())
        return e

    def mul(self):
        e = self.unary()
        while self.peek()[0] == "op" and self.peek()[1] in ("*", "/", "%"):
            op = self.next()[1]
            e = BinOp(op, e, self.unary())
        return e

    def unary(self):
        if self.accept("op", "-"):
            return -self.unary()
        if self.accept("op", "+"):
            return self.unary()
        return self.primary()

    def primary(self) -> Expr:
        t = self.next()
        if t[0] == "num":
            return Lit(float(t[1]) if "." in t[1] else int(t[1]))
        if t[0] == "str":
            return Lit(t[1])
        if t == ("kw", "TRUE"):
            return Lit(True)
        if t == ("kw", "FALSE"):
            return Lit(False)
        if t == ("kw", "NULL"):
            return Lit(None)
        if t == ("op", "("):
            e = self.expr()
            self.expect("op", ")")
            return e
        if t[0] == "id":
            if self.accept("op", "("):
                return self.call(t[1])
            return Col(t[1])
        raise TableError(f"SQL: unexpected {t[1]!r}")

    def call(self, name: str) -> Expr:
        up = name.upper()
        if up in _AGGS:
            if up == "COUNT" and self.accept("op", "*"):
                self.expect("op", ")")
                return Agg("count", None)
            distinct = self.accept("kw", "DISTINCT")
            arg = self.expr()
            self.expect("op", ")")
            return Agg(up.lower(), arg, distinct)
        if up in ("TUMBLE_START", "TUMBLE_END", "HOP_START", "HOP_END"):
            depth = 1  # skip the (time, interval...) arguments: the query has one group window
            while depth:
                t = self.next()
                if t == ("op", "("):
                    depth += 1
                elif t == ("op", ")"):
                    depth -= 1
                elif t[0] == "eof":
                    raise TableError("SQL: unterminated call")
            return WindowProp("$w", "start" if up.endswith("START") else "end")
        args = []
        if not self.accept("op", ")"):
            args.append(self.expr())
            while self.accept("op", ","):
                args.append(self.expr())
            self.expect("op", ")")
        fn = self.t_env.functions.get(up)
        if fn is not None:
            return fn(*args)
        try:
            return builtin(up, *args)
        except KeyError:
            raise TableError(f"SQL: unknown function {name}") from None


def plan_query(t_env, sql: str) -> Table:
    return _Parser(t_env, sql).query()


__all__ = ["plan_query", "tokenize", "Call"]
