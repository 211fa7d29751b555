"""Flink SQL semantics the SQLTransformer pins beyond the reference's own statements
(``SQLTransformerTest.java`` covers projections, SQRT and SUM only; the reference hands the
statement to Flink's planner, ``SQLTransformer.java:86-107``). Flink itself is not importable
here, so the expected values below are Flink's documented / Java-arithmetic results written out
by hand — parity is asserted against those rules, not against a running Flink — and both engines
of this framework (the device-columnar evaluator and the SQLite host fallback) must agree with them:

* integer ``/`` truncates toward zero, ``%`` / ``MOD`` keep the dividend's sign (Java);
* ``CAST(double AS INT|BIGINT)`` truncates toward zero; ``ROUND`` is half away from zero
  (BigDecimal HALF_UP on the double's value); ``CEIL`` / ``FLOOR`` / ``SIGN`` of a DOUBLE are DOUBLE;
* ``AVG`` of an integer column is an integer: BIGINT sum / BIGINT count truncated toward zero
  (Flink's IntegralAvgAggFunction); ``SUM`` keeps its argument's type (an INT sum wraps like
  Java's ``int``, device engine);
* NULLs (host engine): aggregates skip them, ``COUNT(*)`` does not, an all-NULL ``SUM`` is NULL,
  a comparison with NULL is UNKNOWN so ``WHERE`` drops the row whichever way it is negated, and
  ``ORDER BY`` puts NULLs first ascending / last descending (Flink's planner: NULL sorts lowest).
"""
import math

import pytest
import torch

from flink_ml_amd import Table
from flink_ml_amd.models import SQLTransformer
from flink_ml_amd.models.feature import sql_device
from flink_ml_amd.models.feature.misc import run_sql


def _ints():
    return Table({"k": torch.tensor([0, 0, 1, 1, 2, 2, 2], dtype=torch.int64),
                  "i": torch.tensor([1, 2, -1, -2, 3, 4, 4], dtype=torch.int32),
                  "x": torch.tensor([-2.7, 2.7, 2.5, -2.5, 7.0, -7.0, 0.5], dtype=torch.float64)}, num_rows=7)


def _both(stmt, t):
    """(device rows, host rows) of one statement."""
    return sql_device.evaluate(stmt, t).rows(), run_sql(stmt, t).rows()


def test_integral_avg_truncates_toward_zero_and_keeps_int_type():
    t = _ints()
    stmt = "SELECT k, AVG(i) AS a, SUM(i) AS s, COUNT(i) AS n FROM __THIS__ GROUP BY k"
    dev, host = _both(stmt, t)
    expected = {(0, 1, 3, 2), (1, -1, -3, 2), (2, 3, 11, 3)}  # 1.5 -> 1, -1.5 -> -1, 11/3 -> 3
    assert set(dev) == expected and set(host) == expected
    out = sql_device.evaluate(stmt, t)
    assert out.column("a").dtype == torch.int32 and out.column("s").dtype == torch.int32
    # a floating column's AVG stays floating
    dev, host = _both("SELECT AVG(x) AS a FROM __THIS__", t)
    assert math.isclose(dev[0][0], 0.5 / 7, rel_tol=1e-12) and math.isclose(host[0][0], 0.5 / 7, rel_tol=1e-12)


def test_int_sum_wraps_like_java_int_on_the_device():
    t = Table({"i": torch.tensor([2 ** 31 - 1, 1], dtype=torch.int32),
               "b": torch.tensor([2 ** 31 - 1, 1], dtype=torch.int64)}, num_rows=2)
    out = sql_device.evaluate("SELECT SUM(i) AS s, SUM(b) AS t FROM __THIS__", t).rows()
    assert out == [(-2 ** 31, 2 ** 31)]  # INT wraps, BIGINT does not


@pytest.mark.parametrize("expr,expected", [
    ("-7 / 2", -3), ("7 / 2", 3), ("-7 % 3", -1), ("7 % -3", 1), ("MOD(-7, 3)", -1), ("7 / 2.0", 3.5),
    ("CAST(-2.7 AS INT)", -2), ("CAST(2.7 AS BIGINT)", 2), ("CAST(-0.5 AS INT)", 0),
    ("ROUND(2.5)", 3.0), ("ROUND(-2.5)", -3.0), ("ROUND(0.125, 2)", 0.13), ("ROUND(-0.125, 2)", -0.13),
    ("CEIL(2.1)", 3.0), ("FLOOR(-2.1)", -3.0), ("SIGN(-3.5)", -1.0),
])
def test_scalar_rules_on_both_engines(expr, expected):
    t = Table({"id": torch.arange(3, dtype=torch.int64)}, num_rows=3)
    stmt = "SELECT %s AS v FROM __THIS__" % expr
    dev, host = _both(stmt, t)
    for rows in (dev, host):
        assert len(rows) == 3
        v = rows[0][0]
        assert type(v) is type(expected) and v == expected, (expr, rows[0], expected)


def test_column_rules_on_both_engines():
    t = _ints()
    stmt = "SELECT CAST(x AS INT) AS c, ROUND(x) AS r, i / 2 AS q, i % 2 AS m, CEIL(x) AS up FROM __THIS__"
    dev, host = _both(stmt, t)
    expected = [(-2, -3.0, 0, 1, -2.0), (2, 3.0, 1, 0, 3.0), (2, 3.0, 0, -1, 3.0), (-2, -3.0, -1, 0, -2.0),
                (7, 7.0, 1, 1, 7.0), (-7, -7.0, 2, 0, -7.0), (0, 1.0, 2, 0, 1.0)]
    assert dev == expected and host == expected


def test_round_of_int_and_sign_of_nan_on_both_engines():
    """ROUND(INT) stays an INT on the SQLite engine too (its built-in returns REAL), and
    SIGN(NaN) is NaN (Math.signum), not 0."""
    t = _ints()
    dev, host = _both("SELECT ROUND(i) AS r, SIGN(i) AS s FROM __THIS__", t)
    expected = [(1, 1), (2, 1), (-1, -1), (-2, -1), (3, 1), (4, 1), (4, 1)]
    assert host == expected and all(isinstance(r[0], int) for r in host)
    assert dev == expected
    tn = Table({"x": torch.tensor([float("nan"), -3.0, 0.0], dtype=torch.float64)}, num_rows=3)
    from flink_ml_amd.models.feature.misc import _sign, run_sql

    got = sql_device.evaluate("SELECT SIGN(x) AS s FROM __THIS__", tn).get_list("s")
    assert got[0] != got[0] and got[1:] == [-1.0, 0.0]
    # SQLite stores a NaN as NULL (it has no NaN), so the host engine sees SIGN(NULL); the function
    # itself propagates NaN
    assert _sign(float("nan")) != _sign(float("nan")) and _sign(-2.0) == -1.0 and _sign(3) == 1
    r2 = run_sql("SELECT ROUND(x, 1) AS r FROM __THIS__", Table({"x": torch.tensor([2.25, -2.25, 1.05],
                                                                                    dtype=torch.float64)},
                                                                  num_rows=3)).get_list("r")
    assert r2 == [2.3, -2.3, 1.1]


def _nulls():
    return Table.from_rows([(0, 1.0, 3), (0, None, 4), (1, None, None), (1, None, 5), (2, 4.0, None)],
                           ["k", "x", "j"])


def test_null_aggregates_and_count_star():
    rows = SQLTransformer().set_statement(
        "SELECT k, COUNT(*) AS c, COUNT(x) AS cx, SUM(x) AS sx, AVG(j) AS aj FROM __THIS__ GROUP BY k"
    ).transform(_nulls())[0].rows()
    got = {r[0]: r[1:] for r in rows}
    assert got[0] == (2, 1, 1.0, 3)      # AVG(INT) 3.5 -> 3
    assert got[1][:2] == (2, 0) and got[1][2] is None and got[1][3] == 5
    assert got[2][:3] == (1, 1, 4.0) and got[2][3] is None


def test_null_comparisons_drop_the_row_either_way():
    t = _nulls()
    a = SQLTransformer().set_statement("SELECT k FROM __THIS__ WHERE x > 2").transform(t)[0].get_list("k")
    b = SQLTransformer().set_statement("SELECT k FROM __THIS__ WHERE NOT (x > 2)").transform(t)[0].get_list("k")
    assert a == [2] and b == [0]  # the three NULL-x rows are in neither


def test_null_ordering_lowest():
    t = _nulls()
    asc = SQLTransformer().set_statement("SELECT j FROM __THIS__ ORDER BY j").transform(t)[0].get_list("j")
    desc = SQLTransformer().set_statement("SELECT j FROM __THIS__ ORDER BY j DESC").transform(t)[0].get_list("j")
    assert asc[:2] == [None, None] and asc[2:] == [3, 4, 5]
    assert desc[:3] == [5, 4, 3] and desc[3:] == [None, None]


def _mixed():
    return Table({"k": torch.tensor([2, 0, 1, 0, 2, 1], dtype=torch.int64),
                  "x": torch.tensor([1.5, 9.0, -2.0, 4.0, 0.5, 3.0], dtype=torch.float64),
                  "i": torch.tensor([3, 1, 2, 1, 3, 5], dtype=torch.int32)}, num_rows=6)


@pytest.mark.parametrize("stmt,expected", [
    ("SELECT x FROM __THIS__ ORDER BY x", [(-2.0,), (0.5,), (1.5,), (3.0,), (4.0,), (9.0,)]),
    ("SELECT x FROM __THIS__ ORDER BY x DESC LIMIT 2", [(9.0,), (4.0,)]),
    ("SELECT k, x FROM __THIS__ ORDER BY k DESC, x", [(2, 0.5), (2, 1.5), (1, -2.0), (1, 3.0), (0, 4.0), (0, 9.0)]),
    ("SELECT k, x FROM __THIS__ ORDER BY 2 LIMIT 2 OFFSET 1", [(2, 0.5), (2, 1.5)]),
    ("SELECT x AS v FROM __THIS__ ORDER BY i, v DESC", [(9.0,), (4.0,), (-2.0,), (1.5,), (0.5,), (3.0,)]),
    ("SELECT k, SUM(i) AS s FROM __THIS__ GROUP BY k HAVING SUM(i) > 4 ORDER BY s DESC", [(1, 7), (2, 6)]),
    ("SELECT k, COUNT(*) AS c FROM __THIS__ GROUP BY k HAVING k <> 1 ORDER BY k", [(0, 2), (2, 2)]),
    ("SELECT DISTINCT k FROM __THIS__ ORDER BY k DESC", [(2,), (1,), (0,)]),
    ("SELECT DISTINCT k, i FROM __THIS__ ORDER BY k, i", [(0, 1), (1, 2), (1, 5), (2, 3)]),
])
def test_order_limit_distinct_having_on_both_engines(stmt, expected):
    """ORDER BY (names, positions, aliases, input columns not in the output; stable, multi-key),
    LIMIT / OFFSET, DISTINCT and HAVING evaluate on the device (no host fallback) and agree with
    the SQLite engine and the hand-written Flink results."""
    t = _mixed()
    dev, host = _both(stmt, t)
    assert dev == expected and host == expected


def test_order_by_nan_is_the_largest_double_on_the_device():
    """Double.compare: NaN after +inf ascending, first descending (SQLite has no NaN: NULL)."""
    t = Table({"x": torch.tensor([1.0, float("nan"), -math.inf, math.inf], dtype=torch.float64)}, num_rows=4)
    asc = sql_device.evaluate("SELECT x FROM __THIS__ ORDER BY x", t).get_list("x")
    desc = sql_device.evaluate("SELECT x FROM __THIS__ ORDER BY x DESC", t).get_list("x")
    assert asc[:3] == [-math.inf, 1.0, math.inf] and asc[3] != asc[3]
    assert desc[0] != desc[0] and desc[1:] == [math.inf, 1.0, -math.inf]


@pytest.mark.parametrize("expr,expected", [
    ("LOG(8.0)", math.log(8.0)), ("LOG(2, 8)", 3.0), ("LOG2(8.0)", 3.0), ("ATAN2(1.0, 1.0)", math.pi / 4),
    ("COT(1.0)", 1 / math.tan(1.0)), ("SINH(1.0)", math.sinh(1.0)), ("COSH(1.0)", math.cosh(1.0)),
    ("TANH(0.5)", math.tanh(0.5)), ("TRUNCATE(-2.77, 1)", -2.7), ("TRUNCATE(2.77)", 2.0), ("TRUNCATE(7)", 7),
    ("TRUNCATE(123.456, -1)", 120.0), ("PI()", math.pi), ("E()", math.e), ("IF(1 < 2, 2.5, 3.5)", 2.5),
    ("DEGREES(PI())", 180.0), ("LEAST(3, 1, 2)", 1), ("GREATEST(1.5, 2.5)", 2.5),
])
def test_more_scalar_functions_on_both_engines(expr, expected):
    t = Table({"id": torch.arange(2, dtype=torch.int64)}, num_rows=2)
    dev, host = _both("SELECT %s AS v FROM __THIS__" % expr, t)
    for rows in (dev, host):
        v = rows[0][0]
        assert type(v) is type(expected) and math.isclose(v, expected, rel_tol=1e-12, abs_tol=1e-15), (expr, v)


def test_math_outside_the_domain_is_nan_on_the_device():
    """Java's Math: SQRT(-1), LN(-1), ASIN(2) are NaN (not an error) — literals and columns."""
    t = Table({"x": torch.tensor([-1.0, 2.0], dtype=torch.float64)}, num_rows=2)
    r = sql_device.evaluate("SELECT SQRT(-1.0) AS a, LN(x) AS b, ASIN(x) AS c FROM __THIS__", t).rows()
    assert all(v != v for v in (r[0][0], r[0][1], r[1][2]))
    assert math.isclose(r[1][1], math.log(2.0))
    from flink_ml_amd.models.feature.sql_device import java_math

    assert java_math(math.sqrt, -1.0) != java_math(math.sqrt, -1.0) and java_math(math.exp, 1e6) == math.inf


def test_order_by_over_ranks_falls_back():
    t = _mixed()
    with pytest.raises(sql_device.Unsupported):
        sql_device.evaluate("SELECT x FROM __THIS__ ORDER BY x", t, world=2, rank=0)


@pytest.mark.parametrize("expr,expected", [
    ("TRUNCATE(0.29, 2)", 0.29), ("ROUND(2.675, 2)", 2.68), ("ROUND(-2.675, 2)", -2.68), ("ROUND(1.005, 2)", 1.01),
    ("TRUNCATE(-0.29, 2)", -0.29), ("ROUND(1e20, 10)", 1e20), ("TRUNCATE(1e20, 10)", 1e20),
    ("TRUNCATE(-17, -1)", -10),
])
def test_decimal_rounding_of_doubles_on_both_engines(expr, expected):
    """Flink rounds a double's shortest decimal form (BigDecimal.valueOf): 0.29·100 and
    2.675·100 are 28.999… and 267.4999… in binary, yet TRUNCATE(0.29, 2) = 0.29 and
    ROUND(2.675, 2) = 2.68; ROUND(1e20, 10) is 1e20 (no 28-digit decimal context overflow)."""
    t = Table({"id": torch.arange(2, dtype=torch.int64)}, num_rows=2)
    dev, host = _both("SELECT %s AS v FROM __THIS__" % expr, t)
    for rows in (dev, host):
        v = rows[0][0]
        assert type(v) is type(expected) and v == expected, (expr, v)


def test_decimal_rounding_of_double_columns_matches_the_host_engine():
    """The device engine's exact elementwise ROUND / TRUNCATE (decimal boundary test by correctly
    rounded division + Dekker product error) against the host's Decimal(repr(x)) on values built to
    sit on decimal boundaries, for d = 0..6; out-of-range magnitudes fall back to the host engine."""
    import random

    from flink_ml_amd.models.feature.misc import _round, _truncate

    rnd = random.Random(7)
    vals = [0.29, 2.675, -2.675, 1.005, 0.125, -0.0, 1.15, 2.5, -2.5, 1e-9, 123456.785]
    for _ in range(4000):
        q = rnd.randint(-10 ** 7, 10 ** 7)
        vals.append(q / 10 ** rnd.randint(0, 7) + rnd.choice([0.0, 5e-4, 5e-3, 0.5, 5e-7]))
        vals.append(rnd.uniform(-1e4, 1e4))
    x = torch.tensor(vals, dtype=torch.float64)
    for d in range(7):
        for half_up, f in ((True, _round), (False, _truncate)):
            got = sql_device.decimal_round(x, d, half_up).tolist()
            want = [f(v, d) for v in vals]
            assert got == want, next((v, g, w) for v, g, w in zip(vals, got, want) if g != w)
    t = Table({"x": torch.tensor([0.29, 2.675, -1.005], dtype=torch.float64)}, num_rows=3)
    dev, host = _both("SELECT TRUNCATE(x, 2) AS t, ROUND(x, 2) AS r FROM __THIS__", t)
    assert dev == host == [(0.29, 0.29), (2.67, 2.68), (-1.0, -1.01)]
    with pytest.raises(sql_device.Unsupported):
        sql_device.decimal_round(torch.tensor([1e15]), 3, True)
