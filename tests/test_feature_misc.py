"""RandomSplitter / SQLTransformer (LIBT/feature/{RandomSplitterTest,SQLTransformerTest}.java)."""
import math

import pytest

from flink_ml_amd import Table, Vectors
from flink_ml_amd.models import RandomSplitter, SQLTransformer
from flink_ml_amd.utils.java import JavaRandom, java_random_doubles
from tests.spmd import run_spmd

SQL_ROWS = [(0, 1.0, 3.0), (1, 2.0, 3.0), (2, 2.0, 2.0), (3, 4.0, 2.0)]


def _t():
    return Table.from_rows(SQL_ROWS, ["id", "v1", "v2"])


def test_random_splitter(tmp_path):
    s = RandomSplitter()
    assert s.get_weights() == (1.0, 1.0)
    s.set_weights(0.3, 0.4).set_seed(5)
    assert s.get_weights() == (0.3, 0.4) and s.get_seed() == 5
    with pytest.raises(ValueError):
        RandomSplitter().set_weights(1.0)
    with pytest.raises(ValueError):
        RandomSplitter().set_weights(1.0, -1.0)
    data = Table.from_rows([(i,) for i in range(1000)], ["x"])
    sp = RandomSplitter().set_weights(2.0, 1.0, 2.0)
    p = str(tmp_path / "rs")
    sp.save(p)
    outs = RandomSplitter.load(p).transform(data)
    assert len(outs) == 3 and sum(o.num_rows for o in outs) == 1000
    for o, e in zip(outs, (400, 200, 400)):
        assert abs(o.num_rows / e - 1.0) < 0.1
    again = sp.transform(data)
    assert [o.num_rows for o in outs] == [o.num_rows for o in again]
    assert sorted(x for o in outs for x in o.get_list("x")) == list(range(1000))


def test_native_java_random_doubles():
    r = JavaRandom(12345)
    assert [r.next_double() for _ in range(5)] == java_random_doubles(12345, 5).tolist()


@pytest.mark.parametrize("stmt,expected", [
    ("SELECT *, (v1 + v2) AS v3, (v1 * v2) AS v4 FROM __THIS__",
     {(0, 1.0, 3.0, 4.0, 3.0), (1, 2.0, 3.0, 5.0, 6.0), (2, 2.0, 2.0, 4.0, 4.0), (3, 4.0, 2.0, 6.0, 8.0)}),
    ("SELECT *, SQRT(v1) AS v3 FROM __THIS__",
     {(0, 1.0, 3.0, 1.0), (1, 2.0, 3.0, math.sqrt(2.0)), (2, 2.0, 2.0, math.sqrt(2.0)), (3, 4.0, 2.0, 2.0)}),
    ("SELECT v2, SUM(v1) AS v3 FROM __THIS__ GROUP BY v2", {(3.0, 3.0), (2.0, 6.0)}),
    ("SELECT SUM(v1) AS v3 FROM __THIS__", {(9.0,)}),
])
def test_sql_transformer(stmt, expected, tmp_path):
    s = SQLTransformer().set_statement(stmt)
    p = str(tmp_path / "sql")
    s.save(p)
    assert set(SQLTransformer.load(p).transform(_t())[0].rows()) == expected


def test_sql_transformer_validation_and_vectors():
    s = SQLTransformer().set_statement("SELECT * FROM __THIS__")
    assert s.get_statement() == "SELECT * FROM __THIS__"
    with pytest.raises(ValueError, match="statement is given an invalid value SELECT \\* FROM __THAT__"):
        SQLTransformer().set_statement("SELECT * FROM __THAT__")
    tv = Table.from_rows([(0, Vectors.dense(1, 2)), (1, Vectors.dense(3, 4))], ["id", "vec"])
    out = SQLTransformer().set_statement("SELECT vec, id * 2 AS d FROM __THIS__ WHERE id > 0").transform(tv)[0]
    assert out.column_names == ["vec", "d"]
    assert out.rows()[0][0] == Vectors.dense(3, 4) and out.rows()[0][1] == 2


def _spmd_sql(rank, world):
    t = _t().partition(rank, world)
    g = SQLTransformer().set_statement("SELECT v2, SUM(v1) AS v3 FROM __THIS__ GROUP BY v2").transform(t)[0].rows()
    r = SQLTransformer().set_statement("SELECT id, v1 + v2 AS s FROM __THIS__").transform(t)[0].rows()
    return g, r


def test_sql_transformer_distributed():
    res = run_spmd(_spmd_sql, 2)
    assert set(x for g, _ in res for x in g) == {(3.0, 3.0), (2.0, 6.0)}
    assert sorted(x for _, r in res for x in r) == [(0, 4.0), (1, 5.0), (2, 4.0), (3, 6.0)]


# ---- device-columnar SQL evaluator vs the SQLite path (same statements, same table)

def _rand_table(n=500, seed=0):
    import numpy as np
    import torch

    rng = np.random.default_rng(seed)
    return Table({"id": torch.arange(n, dtype=torch.int64),
                  "v1": torch.from_numpy(rng.random(n)),
                  "v2": torch.from_numpy(rng.integers(0, 5, n).astype(np.float64)),
                  "vec": torch.from_numpy(rng.random((n, 3)))}, num_rows=n)


def _rows_close(a, b):
    assert len(a) == len(b)
    for ra, rb in zip(sorted(a, key=repr), sorted(b, key=repr)):
        assert len(ra) == len(rb)
        for x, y in zip(ra, rb):
            if isinstance(x, float) or isinstance(y, float):
                assert math.isclose(float(x), float(y), rel_tol=1e-12, abs_tol=1e-12), (ra, rb)
            else:
                assert x == y, (ra, rb)


@pytest.mark.parametrize("stmt", [
    "SELECT id, v1, ABS(v1 - 0.5) AS a FROM __THIS__",
    "SELECT id, v1 * 2 + v2 / 3 AS a, -v1 AS b FROM __THIS__ WHERE v1 > 0.3 AND NOT v2 < 1",
    "SELECT id % 3 AS m, id / 3 AS d, (id + 1) * 2 - 7 AS e FROM __THIS__",
    "SELECT v2, COUNT(*) AS c, SUM(v1) AS s, MIN(v1) AS lo, MAX(v1) AS hi, AVG(v1) AS av FROM __THIS__ GROUP BY v2",
    "SELECT CASE WHEN v1 > 0.5 THEN 1.0 WHEN v1 > 0.25 THEN 0.5 ELSE 0.0 END AS flag FROM __THIS__",
    "SELECT id FROM __THIS__ WHERE v1 BETWEEN 0.2 AND 0.4 OR id IN (1, 2, 3)",
    "SELECT POWER(v1, 2) AS p, MOD(id, 4) AS m, CEIL(v1 * 10) AS c, FLOOR(v1 * 10) AS f FROM __THIS__",
    "SELECT id % 4 AS k, SUM(v1) AS s, COUNT(v1) AS n FROM __THIS__ GROUP BY id % 4",
    "SELECT SUM(v1) AS s, MAX(id) AS m FROM __THIS__ WHERE v2 >= 2",
    "SELECT SQRT(v1) AS r, EXP(v1) AS e, LN(v1 + 1) AS l FROM __THIS__",
])
def test_sql_device_matches_sqlite(stmt):
    from flink_ml_amd.models.feature import sql_device
    from flink_ml_amd.models.feature.misc import run_sql

    t = _rand_table()
    dev = sql_device.evaluate(stmt, t)
    ref = run_sql(stmt, t.select(*[c for c in t.column_names if c != "vec"]))
    assert dev.num_rows == ref.num_rows
    _rows_close(dev.rows(), ref.rows())


def test_sql_device_passthrough_and_fallback():
    from flink_ml_amd.models.feature import sql_device
    from flink_ml_amd.models.feature.misc import run_sql

    t = _rand_table(50)
    out = sql_device.evaluate("SELECT *, v1 + v2 AS s FROM __THIS__ WHERE id < 10", t)
    assert out.column_names == ["id", "v1", "v2", "vec", "s"] and out.num_rows == 10
    assert out.column("vec").shape == (10, 3)  # vector column carried by reference (gathered by WHERE)
    assert sql_device.evaluate("SELECT v1 * 2 FROM __THIS__", t).column_names == ["EXPR$0"]
    for stmt in ("SELECT id FROM __THIS__ ORDER BY v1 NULLS FIRST", "SELECT 'a' AS s FROM __THIS__",
                 "SELECT id / (id - id) AS z FROM __THIS__", "SELECT COUNT(DISTINCT v2) FROM __THIS__"):
        with pytest.raises(sql_device.Unsupported):
            sql_device.evaluate(stmt, t)
    # the transformer falls back to the host engine for those
    got = SQLTransformer().set_statement("SELECT id FROM __THIS__ ORDER BY v1 NULLS FIRST LIMIT 3").transform(t)[0]
    assert got.num_rows == 3
    # ORDER BY / LIMIT / DISTINCT run on the device (round 5) and match the host engine
    stmt = "SELECT id FROM __THIS__ ORDER BY v1 LIMIT 3"
    assert sql_device.evaluate(stmt, t).rows() == run_sql(stmt, t).rows()


def _spmd_sql_fallback(rank, world):
    t = _t().partition(rank, world)
    # integer division by zero only on the rank holding id == 1: every rank must fall back together
    g = SQLTransformer().set_statement("SELECT v2, SUM(id / (id - 1)) AS s FROM __THIS__ GROUP BY v2").transform(t)[0]
    a = SQLTransformer().set_statement("SELECT v2, COUNT(*) AS c, MAX(v1) AS m FROM __THIS__ GROUP BY v2") \
        .transform(t)[0].rows()
    return g.num_rows, a


def test_sql_device_distributed_agreement():
    res = run_spmd(_spmd_sql_fallback, 2)
    assert sum(n for n, _ in res) == 2
    assert set(x for _, a in res for x in a) == {(3.0, 2, 2.0), (2.0, 2, 4.0)}


def _spmd_sql_where_edge(rank, world):
    t = _t().partition(rank, world)
    # WHERE division by zero on one rank only: the aggregate's ranks still take one path together
    a = SQLTransformer().set_statement(
        "SELECT v2, COUNT(*) AS c FROM __THIS__ WHERE id / (id - 1) >= 0 GROUP BY v2").transform(t)[0].rows()
    # WHERE filters every row on every rank, no GROUP BY: Flink returns one row of NULLs
    e = SQLTransformer().set_statement("SELECT SUM(v1) AS s, MAX(id) AS m FROM __THIS__ WHERE id < 0") \
        .transform(t)[0].rows()
    return a, e


def test_sql_distributed_where_agreement_and_empty_input():
    """WHERE errors join the aggregate's rank agreement; an input every rank
    filters to nothing gives NULLs (host fallback), not sentinel values."""
    res = run_spmd(_spmd_sql_where_edge, 2)
    for _, e in res:
        for row in e:
            assert all(v is None or (isinstance(v, float) and math.isnan(v)) for v in row), e
    assert sum(len(e) for _, e in res) == 1
    assert sum(c for a, _ in res for (_, c) in a) >= 1
