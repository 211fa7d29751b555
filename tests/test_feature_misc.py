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
