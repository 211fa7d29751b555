"""RandomSplitter and SQLTransformer (reference ``LIB/feature/{randomsplitter,sqltransformer}``).

* RandomSplitter: each rank draws ``java.util.Random(Tuple2.of(seed, rank).hashCode())``
  doubles (native host loop, bit-identical to ``SplitterOperator``) and routes row i to split
  ``#{cumulative fractions < r_i}`` — one searchsorted and one gather per output.
* SQLTransformer: statements in the device subset (projections, arithmetic, built-in math
  functions, WHERE, GROUP BY with SUM/COUNT/AVG/MIN/MAX — ``sql_device.py``) are evaluated
  column-at-a-time on the input's device. Anything else runs on SQLite (stdlib) with the input's
  scalar columns; vector/object columns pass through as opaque references. Row-wise statements
  run per rank; statements that aggregate, sort, join or de-duplicate are evaluated over the
  gathered table and the result is re-partitioned round-robin.
"""
from __future__ import annotations

import math
import re
import sqlite3
from typing import List

import numpy as np
import torch

from ...api.stage import AlgoOperator
from ...common.param import HasSeed
from ...io import read_write as rw
from ...param.param import FloatArrayParam, ParamValidator, StringParam
from ...parallel import comm
from ...table import Table, compact_column
from ...utils.java import _i32, java_long_hash, java_random_doubles
from .common import get_world_distributed


def _weights_ok(w) -> bool:
    return w is not None and len(w) > 1 and all(x > 0.0 for x in w)


@rw.register_stage
class RandomSplitter(AlgoOperator, HasSeed):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.randomsplitter.RandomSplitter"
    WEIGHTS = FloatArrayParam("weights", "The weights of data splitting.", (1.0, 1.0),
                              ParamValidator(_weights_ok, "weightsValidator"))

    def transform(self, *inputs) -> List[Table]:
        from ...parallel.context import get_context

        t = inputs[0]
        w = np.asarray(self.get(self.WEIGHTS), dtype=np.float64)
        # the reference accumulates currentSum / weightSum element by element
        acc, fr = 0.0, []
        for x in w:
            acc += x
            fr.append(acc / w.sum())
        fractions = np.asarray(fr)
        rank = get_context().rank
        # Tuple2.of(Long seed, Integer subtask).hashCode()
        r = java_random_doubles(_i32(31 * java_long_hash(int(self.get_seed())) + rank), t.num_rows)
        split = np.searchsorted(fractions, r, side="left")
        return [t.take(torch.from_numpy(np.nonzero(split == i)[0])) for i in range(len(w))]


_GLOBAL_SQL = re.compile(r"\b(GROUP\s+BY|ORDER\s+BY|DISTINCT|JOIN|LIMIT|OFFSET|UNION|INTERSECT|EXCEPT|HAVING|OVER|"
                         r"COUNT|SUM|AVG|MIN|MAX|STDDEV\w*|VAR\w*|COLLECT|LISTAGG)\b", re.IGNORECASE)
_REF = "\x00fmlx-ref:"


def _statement_ok(s) -> bool:
    return s is not None and "__THIS__" in s


class _FlinkAvg:
    """AVG with Flink's result type: over integral values the average of an INT / BIGINT column is
    integral (Flink's IntegralAvgAggFunction: BIGINT sum / BIGINT count, Java division — truncated
    toward zero); over anything floating it is the floating mean. NULLs are skipped; no rows → NULL."""

    def __init__(self):
        self.s, self.n, self.ints = 0, 0, True

    def step(self, v):
        if v is None:
            return
        if not isinstance(v, int):
            self.ints = False
        self.s += v
        self.n += 1

    def finalize(self):
        if self.n == 0:
            return None
        if self.ints:
            q = abs(self.s) // self.n
            return q if self.s >= 0 else -q
        return self.s / self.n


def _keep_type(fn):
    """CEIL / FLOOR / SIGN of a DOUBLE stay DOUBLE (Python's return ints); of an integer, integer."""
    return lambda x: None if x is None else (float(fn(x)) if isinstance(x, float) else int(fn(x)))


def _java_mod(a, b):
    """MOD / % with Java semantics: the dividend's sign; integral for integers (Flink's MOD(INT, INT)
    is INT)."""
    if a is None or b is None:
        return None
    if isinstance(a, int) and isinstance(b, int):
        if b == 0:
            return None
        r = abs(a) % abs(b)
        return r if a >= 0 else -r
    return math.fmod(a, b)


def _sign(x):
    """SIGN with Java's Math.signum / Integer.signum: NaN stays NaN, the input's type is kept."""
    if x is None:
        return None
    if isinstance(x, float):
        return x if x != x else float((x > 0) - (x < 0))
    return (x > 0) - (x < 0)


def _decimal(x: float, d: int, rounding) -> float:
    """A double rounded at d decimals the way Flink does it: its shortest decimal representation
    (``BigDecimal.valueOf``) is rounded, under a context wide enough for any double's digits (the
    default 28 digits raised InvalidOperation for ROUND(1e20, 10))."""
    from decimal import Decimal, localcontext

    v = Decimal(repr(x))
    with localcontext() as ctx:
        ctx.prec = max(28, v.adjusted() + max(d, 0) + 4)
        if d >= 0:
            return float(v.quantize(Decimal(1).scaleb(-d), rounding=rounding))
        return float(v.scaleb(d).quantize(Decimal(1), rounding=rounding).scaleb(-d))


def _round(x, d=0):
    """ROUND(x[, d]) as Flink: HALF_UP (ties away from zero) at d decimals (d < 0: tens, hundreds…),
    keeping the input's type — ROUND(INT) is an INT (SQLite's built-in returns REAL). Doubles round
    their shortest decimal representation (BigDecimal.valueOf), so ROUND(2.675, 2) = 2.68."""
    from decimal import ROUND_HALF_UP, Decimal

    if x is None or d is None:
        return None
    d = int(d)
    if isinstance(x, float):
        if x != x or x in (float("inf"), float("-inf")):
            return x
        return _decimal(x, d, ROUND_HALF_UP)
    if d >= 0:
        return x
    return int(Decimal(x).scaleb(d).quantize(Decimal(1), rounding=ROUND_HALF_UP).scaleb(-d))


def _truncate(x, d=0):
    """TRUNCATE(x[, d]): toward zero at d decimals, the input's type kept (Flink). Doubles truncate
    their shortest decimal representation: TRUNCATE(0.29, 2) = 0.29 (0.29·100 is 28.999… in binary)."""
    from decimal import ROUND_DOWN

    if x is None or d is None:
        return None
    d = int(d)
    if isinstance(x, int):
        return x if d >= 0 else (1 if x >= 0 else -1) * (abs(x) // 10 ** -d) * 10 ** -d
    if x != x or x in (float("inf"), float("-inf")):
        return x
    return _decimal(x, d, ROUND_DOWN)


def _least(*a):
    return None if any(v is None for v in a) else min(a)


def _greatest(*a):
    return None if any(v is None for v in a) else max(a)


def _register_functions(con: sqlite3.Connection) -> None:
    from .sql_device import java_math

    def f1(fn):  # NULL in, NULL out; outside the domain NaN like Java's Math (Python raises)
        return lambda x: None if x is None else java_math(fn, x)

    for name, fn in (("SQRT", math.sqrt), ("LN", math.log), ("LOG10", math.log10), ("EXP", math.exp),
                     ("ABS", abs), ("SIN", math.sin), ("COS", math.cos), ("TAN", math.tan), ("ASIN", math.asin),
                     ("ACOS", math.acos), ("ATAN", math.atan), ("DEGREES", math.degrees),
                     ("RADIANS", math.radians), ("LOG2", math.log2), ("SINH", math.sinh), ("COSH", math.cosh),
                     ("TANH", math.tanh), ("COT", lambda a: 1.0 / math.tan(a)), ("LOG", math.log)):
        con.create_function(name, 1, f1(fn), deterministic=True)
    con.create_function("LOG", 2, lambda b, x: None if b is None or x is None else
                        java_math(lambda u, v: math.log(v) / math.log(u), b, x), deterministic=True)
    con.create_function("ATAN2", 2, lambda a, b: None if a is None or b is None else math.atan2(a, b),
                        deterministic=True)
    con.create_function("TRUNCATE", 1, _truncate, deterministic=True)
    con.create_function("TRUNCATE", 2, _truncate, deterministic=True)
    con.create_function("PI", 0, lambda: math.pi, deterministic=True)
    con.create_function("E", 0, lambda: math.e, deterministic=True)
    con.create_function("IF", 3, lambda c, a, b: a if c else b, deterministic=True)
    con.create_function("LEAST", -1, _least, deterministic=True)
    con.create_function("GREATEST", -1, _greatest, deterministic=True)
    for name, fn in (("CEIL", math.ceil), ("CEILING", math.ceil), ("FLOOR", math.floor)):
        con.create_function(name, 1, _keep_type(fn), deterministic=True)
    con.create_function("SIGN", 1, _sign, deterministic=True)
    con.create_function("ROUND", 1, _round, deterministic=True)
    con.create_function("ROUND", 2, _round, deterministic=True)
    con.create_function("POWER", 2, lambda a, b: None if a is None or b is None else math.pow(a, b),
                        deterministic=True)
    con.create_function("MOD", 2, _java_mod, deterministic=True)
    con.create_aggregate("AVG", 1, _FlinkAvg)


def _sql_value(v):
    if v is None or isinstance(v, (int, float, str, bytes)):
        return v
    if isinstance(v, (np.integer,)):
        return int(v)
    if isinstance(v, (np.floating,)):
        return float(v)
    if isinstance(v, (bool, np.bool_)):
        return int(v)
    return None  # replaced by a reference token below


def run_sql(statement: str, t: Table) -> Table:
    names = t.column_names
    cols = [t.get_list(n) for n in names]
    objects = []
    rows = []
    for i in range(t.num_rows):
        row = []
        for j, c in enumerate(cols):
            v = c[i]
            sv = _sql_value(v)
            if sv is None and v is not None:
                sv = "%s%d" % (_REF, len(objects))
                objects.append(v)
            row.append(sv)
        rows.append(row)
    con = sqlite3.connect(":memory:")
    try:
        _register_functions(con)
        qn = ", ".join('"%s"' % n for n in names)
        con.execute('CREATE TABLE __fmlx_this (%s)' % qn)
        if rows:
            con.executemany('INSERT INTO __fmlx_this VALUES (%s)' % ", ".join("?" * len(names)), rows)
        cur = con.execute(statement.replace("__THIS__", "__fmlx_this"))
        out_names = [d[0] for d in cur.description]
        data = cur.fetchall()
    finally:
        con.close()

    def unref(v):
        if isinstance(v, str) and v.startswith(_REF):
            return objects[int(v[len(_REF):])]
        return v

    out_cols = {}
    for j, n in enumerate(out_names):
        vals = [unref(r[j]) for r in data]
        if vals and all(isinstance(v, float) or isinstance(v, int) for v in vals) and any(
                isinstance(v, float) for v in vals):
            vals = [float(v) for v in vals]
        out_cols[n] = compact_column(vals)
    return Table(out_cols, num_rows=len(data))


@rw.register_stage
class SQLTransformer(AlgoOperator):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.sqltransformer.SQLTransformer"
    STATEMENT = StringParam("statement", "SQL statement.", None, ParamValidator(_statement_ok, "statement"))

    def transform(self, *inputs) -> List[Table]:
        from . import sql_device

        t = inputs[0]
        stmt = self.get(self.STATEMENT)
        world, rank = 1, 0
        if get_world_distributed():
            from ...parallel.context import get_context

            world, rank = get_context().world_size, get_context().rank
        # the statement subset a feature pipeline uses runs column-at-a-time on the device
        # (sql_device.py); the rest falls back to SQLite over host rows
        out = sql_device.try_evaluate(stmt, t, world, rank)
        if out is not None:
            return [out]
        if get_world_distributed() and _GLOBAL_SQL.search(stmt):
            from ...parallel.context import get_context

            ctx = get_context()
            full = Table.concat(comm.all_gather_object(t.to("cpu")))
            return [run_sql(stmt, full).partition(ctx.rank, ctx.world_size)]
        return [run_sql(stmt, t.to("cpu"))]
