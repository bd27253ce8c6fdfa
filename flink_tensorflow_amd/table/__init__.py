"""Table API and streaming SQL on the DataStream runtime (see ``table.py``)."""
from .expressions import Accumulator, Agg, Expr, Row, call, col, count_star, lit
from .sql import plan_query, tokenize
from .table import (GroupedTable, GroupWindow, Slide, StreamTableEnvironment, Table, TableError, TableResult, Tumble,
                    WindowedTable)
from .udf import ModelScalarFunction, ScalarFunction, udf

__all__ = ["Accumulator", "Agg", "Expr", "GroupWindow", "GroupedTable", "ModelScalarFunction", "Row",
           "ScalarFunction", "Slide", "StreamTableEnvironment", "Table", "TableError", "TableResult", "Tumble",
           "WindowedTable", "call", "col", "count_star", "lit", "plan_query", "tokenize", "udf"]
