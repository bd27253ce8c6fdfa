"""Table API + streaming SQL: projections, filters, updating group aggregates with
retractions, event-time group windows, joins, UDFs and a model-backed SQL function
(the SavedModel fixture of the reference's RegressITCase behind ``SELECT``)."""
import pytest

from flink_tensorflow_amd.models import RegressionMethod, TensorFlowModel
from flink_tensorflow_amd.runtime import StreamExecutionEnvironment
from flink_tensorflow_amd.table import (ModelScalarFunction, Row, Slide, StreamTableEnvironment, TableError, Tumble,
                                        col, lit, tokenize, udf)
from flink_tensorflow_amd.types import example, feature

ORDERS = [("alice", 10, 0.5), ("bob", 5, 1.2), ("alice", 7, 1.9), ("carol", 3, 2.1), ("bob", 20, 2.5),
          ("alice", 1, 3.7), ("carol", 8, 3.9)]


def _env(p=2):
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(p)
    return env, StreamTableEnvironment.create(env)


def _orders(t_env, env, rowtime=True):
    return t_env.from_data_stream(env.from_collection(ORDERS), "user", "amount", "ts",
                                  rowtime="ts" if rowtime else None)


def test_rows():
    r = Row.of(("a", "b"), (1, "x"))
    assert r.a == 1 and r["b"] == "x" and r[0] == 1 and r.as_dict() == {"a": 1, "b": "x"}
    import pickle

    assert pickle.loads(pickle.dumps(r)) == r and pickle.loads(pickle.dumps(r)).b == "x"


def test_select_where_expressions():
    env, t_env = _env()
    t = _orders(t_env, env)
    res = t.where((col("amount") > 4) & (col("user") != "carol")) \
        .select(col("user"), (col("amount") * 2 + 1).alias("score"), lit("x").alias("tag")).execute().collect()
    assert sorted(res) == [("alice", 15, "x"), ("alice", 21, "x"), ("bob", 11, "x"), ("bob", 41, "x")]
    assert res[0].score in (15, 21, 11, 41)


def test_group_by_retracts_and_materialises():
    env, t_env = _env(3)
    t = _orders(t_env, env)
    out = t.group_by(col("user")).select(col("user"), col("amount").sum.alias("total"),
                                         col("amount").count.alias("n"), col("amount").max.alias("mx"))
    assert not out.is_append_only
    res = out.execute()
    assert sorted(res.collect()) == [("alice", 18, 3, 10), ("bob", 25, 2, 20), ("carol", 11, 2, 8)]
    log = res.changelog()
    assert any(flag is False for flag, _ in log)  # updates retract the previous result row
    with pytest.raises(TableError):
        t_env.to_data_stream(out)


def test_aggregate_over_updating_table():
    """A second aggregation consumes the first one's retractions: count of users per
    order count."""
    env, t_env = _env()
    per_user = _orders(t_env, env).group_by(col("user")).select(col("user"), col("amount").count.alias("n"))
    hist = per_user.group_by(col("n")).select(col("n"), col("user").count.alias("users"))
    assert sorted(hist.execute().collect()) == [(2, 2), (3, 1)]


def test_tumbling_and_sliding_event_time_windows():
    env, t_env = _env()
    t = _orders(t_env, env)
    w = t.window(Tumble.over(2.0).on(col("ts")).alias("w")).group_by(col("w"), col("user")) \
        .select(col("user"), col("w").start.alias("ws"), col("w").end.alias("we"), col("amount").sum.alias("s"))
    assert sorted(w.execute().collect()) == [("alice", 0.0, 2.0, 17), ("alice", 2.0, 4.0, 1), ("bob", 0.0, 2.0, 5),
                                             ("bob", 2.0, 4.0, 20), ("carol", 2.0, 4.0, 11)]
    env, t_env = _env()
    t = _orders(t_env, env)
    s = t.window(Slide.over(2.0).every(1.0).on(col("ts")).alias("w")).group_by(col("w")) \
        .select(col("w").start.alias("ws"), col("amount").count.alias("n"))
    assert sorted(s.execute().collect()) == [(-1.0, 1), (0.0, 3), (1.0, 4), (2.0, 4), (3.0, 2)]


def test_join_and_union():
    env, t_env = _env()
    orders = _orders(t_env, env, rowtime=False)
    users = t_env.from_elements([("alice", "DE"), ("bob", "FR")], ["name", "country"])
    j = orders.join(users, col("user") == col("name")).select(col("user"), col("country"), col("amount"))
    assert sorted(j.execute().collect()) == [("alice", "DE", 1), ("alice", "DE", 7), ("alice", "DE", 10),
                                             ("bob", "FR", 5), ("bob", "FR", 20)]
    env, t_env = _env()
    a = t_env.from_elements([(1,), (2,)], ["x"])
    b = t_env.from_elements([(3,)], ["x"])
    assert sorted(a.union_all(b).execute().collect()) == [(1,), (2,), (3,)]


def test_sql_queries():
    env, t_env = _env()
    t_env.create_temporary_view("orders", _orders(t_env, env))
    t_env.create_temporary_function("bonus", lambda a: a * 10)
    q = t_env.sql_query("SELECT user, SUM(amount) AS total, COUNT(*) AS n FROM orders "
                        "WHERE amount BETWEEN 2 AND 15 GROUP BY user HAVING COUNT(*) >= 1")
    assert sorted(q.execute().collect()) == [("alice", 17, 2), ("bob", 5, 1), ("carol", 11, 2)]
    env, t_env = _env()
    t_env.create_temporary_view("orders", _orders(t_env, env))
    t_env.create_temporary_function("bonus", udf(lambda a: a * 10, "bonus"))
    q = t_env.sql_query("SELECT UPPER(user) AS u, bonus(amount) b FROM orders WHERE NOT user = 'bob' AND ts < 2")
    assert sorted(q.execute().collect()) == [("ALICE", 70), ("ALICE", 100)]
    env, t_env = _env()
    t_env.create_temporary_view("orders", _orders(t_env, env))
    q = t_env.sql_query("SELECT user, TUMBLE_START(ts, INTERVAL '2' SECOND) AS ws, MAX(amount) AS m "
                        "FROM orders GROUP BY TUMBLE(ts, INTERVAL '2' SECOND), user")
    assert q.is_append_only
    assert sorted(q.execute().collect()) == [("alice", 0.0, 10), ("alice", 2.0, 1), ("bob", 0.0, 5),
                                             ("bob", 2.0, 20), ("carol", 2.0, 8)]
    env, t_env = _env()
    t_env.create_temporary_view("orders", _orders(t_env, env))
    q = t_env.sql_query("SELECT DISTINCT user FROM orders")
    assert sorted(q.execute().collect()) == [("alice",), ("bob",), ("carol",)]
    with pytest.raises(TableError):
        t_env.sql_query("SELECT user, amount FROM orders GROUP BY user")  # amount neither grouped nor aggregated
    assert tokenize("SELECT 'it''s'")[1] == ("str", "it's")


class HalfPlusTwo(TensorFlowModel):
    def __init__(self, path):
        super().__init__(device="cpu")
        self._loader = TensorFlowModel.load(path, "serve")

    @property
    def loader(self):
        return self._loader


def test_model_function_in_sql(half_plus_two):
    """The reference's regress_x_to_y SavedModel signature as a SQL scalar function."""
    env, t_env = _env(2)
    t_env.create_temporary_view("xs", t_env.from_elements([(float(v),) for v in range(4)], ["x"]))

    def regress(model, x):
        fn = model.function("regress_x_to_y", RegressionMethod())
        return float(fn.apply([example(("x", feature(x)))]).reshape(-1)[0])

    t_env.create_temporary_function("half_plus_two", ModelScalarFunction(HalfPlusTwo(half_plus_two), regress))
    q = t_env.sql_query("SELECT x, half_plus_two(x) AS y FROM xs WHERE x >= 1")
    assert sorted(q.execute().collect()) == [(1.0, 2.5), (2.0, 3.0), (3.0, 3.5)]
    # the Table-level mapWithModel
    env, t_env = _env(1)
    t = t_env.from_elements([(float(v),) for v in range(2)], ["x"])
    out = t.map_with_model(HalfPlusTwo(half_plus_two), lambda m, row: regress(m, row.x), "y").execute().collect()
    assert sorted(out) == [(0.0, 2.0), (1.0, 2.5)]


def test_batched_model_column(half_plus_two):
    """Micro-batched model inference on a table: one SavedModel call per batch of rows."""
    env, t_env = _env(1)
    t = t_env.from_elements([(float(v), f"r{v}") for v in range(40)], ["x", "tag"])

    def regress_batch(model, rows):
        fn = model.function("regress_x_to_y", RegressionMethod())
        ys = fn.apply([example(("x", feature(r.x))) for r in rows]).reshape(-1).tolist()
        return ys

    out = t.map_with_model_batched(HalfPlusTwo(half_plus_two), regress_batch, "y", max_batch=16).where(
        col("y") > 20).execute().collect()
    assert sorted((r.x, r.y) for r in out) == [(float(v), 0.5 * v + 2) for v in range(37, 40)]
    assert all(r.tag == f"r{int(r.x)}" for r in out)
