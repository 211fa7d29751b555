"""Device-columnar evaluator for SQLTransformer statements (reference
``flink-ml-lib/.../feature/sqltransformer/SQLTransformer.java:86-107``, which hands the statement to
Flink's table planner).

The subset a feature pipeline uses is evaluated column-at-a-time on the columns' own device — the
input never leaves HBM, ``SELECT *`` columns (vectors, sparse, strings included) pass through by
reference, and a ``WHERE`` is one mask + one gather per column:

    SELECT [ALL | DISTINCT] item, ... FROM __THIS__ [WHERE cond] [GROUP BY expr, ... [HAVING cond]]
           [ORDER BY expr [ASC | DESC], ...] [LIMIT n [OFFSET m]]
    item  := * | expr [[AS] alias]
    expr  := arithmetic (+ - * / %, unary -), comparisons (= <> != < <= > >=), AND / OR / NOT,
             BETWEEN, IN (...), IS [NOT] NULL, CASE WHEN ... THEN ... [ELSE ...] END,
             CAST(x AS DOUBLE|FLOAT|INT|INTEGER|BIGINT|BOOLEAN), numeric literals, TRUE / FALSE,
             ABS SQRT LN LOG LOG2 LOG10 EXP CEIL CEILING FLOOR SIN COS TAN COT ASIN ACOS ATAN ATAN2
             SINH COSH TANH SIGN DEGREES RADIANS POWER MOD ROUND TRUNCATE LEAST GREATEST PI E IF
             COALESCE,
             aggregates SUM COUNT(*|x) AVG MIN MAX (with or without GROUP BY)

Types follow Flink: integer op integer stays integer ('/' truncates toward zero, '%' keeps the
dividend's sign), anything with a floating operand is floating, comparisons are BOOLEAN, unnamed
expressions are called ``EXPR$<i>``, SUM keeps its argument's type and AVG of an integer column is
an integer (sum / count truncated toward zero, Flink's IntegralAvgAggFunction), CAST to INT /
BIGINT truncates toward zero, ROUND is half away from zero, TRUNCATE toward zero, LOG(x) is the
natural log and LOG(b, x) = LN(x) / LN(b), math outside a function's domain is NaN (Java's Math).
GROUP BY and DISTINCT output is ordered by key (ascending). ORDER BY is a stable lexicographic sort
over output columns (names, 1-based positions or expressions of them) with NaN the largest
DOUBLE (Double.compare). Distributed: row-wise statements run per rank; aggregates are computed per
rank, the small partial tables are all-gathered and merged on every rank, and the result is dealt
round-robin; ORDER BY / LIMIT need the global order and fall back when world > 1.

Anything outside the subset (strings, joins, windows, NULL results, integer division by zero, ...)
raises ``Unsupported`` and the caller falls back to the host SQL engine.
"""
from __future__ import annotations

import math
import re
from typing import List, NamedTuple, Optional

import numpy as np
import torch

from ...table import Table


class Unsupported(Exception):
    pass


_TOKEN = re.compile(r"""\s*(?:
    (?P<num>(?:\d+\.\d*|\.\d+|\d+)(?:[eE][+-]?\d+)?)
  | (?P<id>[A-Za-z_][A-Za-z0-9_$]*)
  | "(?P<qid>[^"]+)"
  | `(?P<bid>[^`]+)`
  | (?P<str>'(?:[^']|'')*')
  | (?P<op><=|>=|<>|!=|\|\||[-+*/%(),=<>])
)""", re.VERBOSE)

_KEYWORDS = {"SELECT", "ALL", "FROM", "WHERE", "GROUP", "BY", "AS", "AND", "OR", "NOT", "BETWEEN", "IN", "IS",
             "NULL", "CASE", "WHEN", "THEN", "ELSE", "END", "CAST", "TRUE", "FALSE", "DISTINCT", "ORDER", "HAVING",
             "LIMIT", "JOIN", "UNION", "OVER", "TABLE"}
_AGGS = {"SUM", "COUNT", "AVG", "MIN", "MAX"}


def _tokenize(s: str):
    out, pos = [], 0
    s = s.rstrip().rstrip(";")
    while pos < len(s):
        if s[pos:].strip() == "":
            break
        m = _TOKEN.match(s, pos)
        if not m or m.end() == pos:
            raise Unsupported("cannot tokenize at %r" % s[pos:pos + 20])
        pos = m.end()
        if m.group("num") is not None:
            out.append(("num", m.group("num")))
        elif m.group("id") is not None:
            w = m.group("id")
            out.append(("kw", w.upper()) if w.upper() in _KEYWORDS else ("id", w))
        elif m.group("qid") is not None or m.group("bid") is not None:
            out.append(("id", m.group("qid") or m.group("bid")))
        elif m.group("str") is not None:
            out.append(("str", m.group("str")[1:-1].replace("''", "'")))
        else:
            out.append(("op", m.group("op")))
    out.append(("eof", None))
    return out


# ---- AST: tuples ("col", name) ("lit", value) ("un", op, a) ("bin", op, a, b) ("fn", NAME, [args])
#      ("agg", NAME, arg|None) ("case", [(cond, val)], else) ("cast", a, type) ("isnull", a, negate)
#      ("in", a, [vals], negate) ("star",)

class Query(NamedTuple):
    items: list
    where: object
    group: Optional[list]
    having: object
    order: list  # [(expr, descending)]
    limit: Optional[int]
    offset: int
    distinct: bool


class _Parser:
    def __init__(self, toks):
        self.t = toks
        self.i = 0

    def peek(self, k=0):
        return self.t[self.i + k]

    def take(self):
        tok = self.t[self.i]
        self.i += 1
        return tok

    def accept(self, kind, val=None):
        tok = self.peek()
        if tok[0] == kind and (val is None or tok[1] == val):
            self.i += 1
            return tok
        return None

    def expect(self, kind, val=None):
        tok = self.accept(kind, val)
        if tok is None:
            raise Unsupported("expected %s %s, got %r" % (kind, val, self.peek()))
        return tok

    def query(self):
        self.expect("kw", "SELECT")
        self.accept("kw", "ALL")
        distinct = bool(self.accept("kw", "DISTINCT"))
        items = [self.item()]
        while self.accept("op", ","):
            items.append(self.item())
        self.expect("kw", "FROM")
        src = self.expect("id")[1]
        if src != "__THIS__":
            raise Unsupported("FROM %s" % src)
        where = group = having = None
        order, limit, offset = [], None, 0
        if self.accept("kw", "WHERE"):
            where = self.expr()
        if self.accept("kw", "GROUP"):
            self.expect("kw", "BY")
            group = [self.expr()]
            while self.accept("op", ","):
                group.append(self.expr())
        if self.accept("kw", "HAVING"):
            having = self.expr()
        if self.accept("kw", "ORDER"):
            self.expect("kw", "BY")
            while True:
                e = self.expr()
                desc = False
                if self.peek()[0] == "id" and self.peek()[1].upper() in ("ASC", "DESC"):
                    desc = self.take()[1].upper() == "DESC"
                if self.peek()[0] == "id" and self.peek()[1].upper() == "NULLS":
                    raise Unsupported("NULLS FIRST / LAST")
                order.append((e, desc))
                if not self.accept("op", ","):
                    break
        if self.accept("kw", "LIMIT"):
            tok = self.expect("num")
            if not re.fullmatch(r"\d+", tok[1]):
                raise Unsupported("LIMIT %s" % tok[1])
            limit = int(tok[1])
            if self.peek()[0] == "id" and self.peek()[1].upper() == "OFFSET":
                self.take()
                tok = self.expect("num")
                if not re.fullmatch(r"\d+", tok[1]):
                    raise Unsupported("OFFSET %s" % tok[1])
                offset = int(tok[1])
        self.expect("eof")
        return Query(items, where, group, having, order, limit, offset, distinct)

    def item(self):
        if self.accept("op", "*"):
            return ("star",), None
        e = self.expr()
        alias = None
        if self.accept("kw", "AS"):
            alias = self.expect("id")[1]
        elif self.peek()[0] == "id":
            alias = self.take()[1]
        return e, alias

    def expr(self):
        a = self.and_()
        while self.accept("kw", "OR"):
            a = ("bin", "OR", a, self.and_())
        return a

    def and_(self):
        a = self.not_()
        while self.accept("kw", "AND"):
            a = ("bin", "AND", a, self.not_())
        return a

    def not_(self):
        if self.accept("kw", "NOT"):
            return ("un", "NOT", self.not_())
        return self.cmp()

    def cmp(self):
        a = self.add()
        tok = self.peek()
        if tok[0] == "op" and tok[1] in ("=", "<>", "!=", "<", "<=", ">", ">="):
            self.take()
            return ("bin", "<>" if tok[1] == "!=" else tok[1], a, self.add())
        neg = False
        if tok == ("kw", "NOT") and self.peek(1)[1] in ("BETWEEN", "IN"):
            self.take()
            neg = True
        if self.accept("kw", "BETWEEN"):
            lo = self.add()
            self.expect("kw", "AND")
            hi = self.add()
            e = ("bin", "AND", ("bin", ">=", a, lo), ("bin", "<=", a, hi))
            return ("un", "NOT", e) if neg else e
        if self.accept("kw", "IN"):
            self.expect("op", "(")
            vals = [self.add()]
            while self.accept("op", ","):
                vals.append(self.add())
            self.expect("op", ")")
            return ("in", a, vals, neg)
        if self.accept("kw", "IS"):
            negate = bool(self.accept("kw", "NOT"))
            self.expect("kw", "NULL")
            return ("isnull", a, negate)
        return a

    def add(self):
        a = self.mul()
        while self.peek()[0] == "op" and self.peek()[1] in ("+", "-"):
            a = ("bin", self.take()[1], a, self.mul())
        if self.peek() == ("op", "||"):
            raise Unsupported("string concatenation")
        return a

    def mul(self):
        a = self.unary()
        while self.peek()[0] == "op" and self.peek()[1] in ("*", "/", "%"):
            a = ("bin", self.take()[1], a, self.unary())
        return a

    def unary(self):
        if self.accept("op", "-"):
            return ("un", "-", self.unary())
        if self.accept("op", "+"):
            return self.unary()
        return self.primary()

    def primary(self):
        tok = self.take()
        kind, v = tok
        if kind == "num":
            if re.fullmatch(r"\d+", v):
                return ("lit", int(v))
            return ("lit", float(v))
        if kind == "str":
            raise Unsupported("string literal")
        if kind == "op" and v == "(":
            e = self.expr()
            self.expect("op", ")")
            return e
        if kind == "kw":
            if v in ("TRUE", "FALSE"):
                return ("lit", v == "TRUE")
            if v == "CAST":
                self.expect("op", "(")
                e = self.expr()
                self.expect("kw", "AS")
                ty = self.expect("id")[1].upper()
                self.expect("op", ")")
                return ("cast", e, ty)
            if v == "CASE":
                whens = []
                while self.accept("kw", "WHEN"):
                    c = self.expr()
                    self.expect("kw", "THEN")
                    whens.append((c, self.expr()))
                other = self.expr() if self.accept("kw", "ELSE") else ("lit", None)
                self.expect("kw", "END")
                if not whens:
                    raise Unsupported("CASE without WHEN")
                return ("case", whens, other)
            raise Unsupported("keyword %s" % v)
        if kind == "id":
            if self.accept("op", "("):
                name = v.upper()
                if name in _AGGS:
                    if self.peek() == ("kw", "DISTINCT"):
                        raise Unsupported("aggregate DISTINCT")
                    if name == "COUNT" and self.accept("op", "*"):
                        arg = None
                    else:
                        arg = self.expr()
                    self.expect("op", ")")
                    if self.peek() == ("kw", "OVER"):
                        raise Unsupported("window function")
                    return ("agg", name, arg)
                args = []
                if not self.accept("op", ")"):
                    args.append(self.expr())
                    while self.accept("op", ","):
                        args.append(self.expr())
                    self.expect("op", ")")
                return ("fn", name, args)
            return ("col", v)
        raise Unsupported("unexpected token %r" % (tok,))


def parse(statement: str):
    return _Parser(_tokenize(statement)).query()


# ---- evaluation

def java_math(fn, *a):
    """A scalar math function with Java's Math semantics: outside the domain NaN (Python raises),
    overflow ±inf."""
    try:
        return fn(*a)
    except ValueError:
        return math.nan
    except OverflowError:
        return math.inf
    except ZeroDivisionError:
        return math.inf


# |x|·10^d below this: a decimal boundary (ROUND: a half-point; TRUNCATE: a multiple of 10^-d)
# that lies in x's rounding interval is x's shortest decimal representation itself — the interval
# (≤ 2^-52·|x| wide, ≤ 1/16 in units of 10^-d) holds no other decimal of d + 1 digits — see
# decimal_round
_DEC_EXACT = float(2 ** 48)


def _two_product_err(a: torch.Tensor, s: float, p: torch.Tensor) -> torch.Tensor:
    """a·s − p exactly, for p = fl(a·s) (Dekker's product with Veltkamp splits: every step is an
    exact fp64 operation; separate elementwise kernels, so nothing is contracted into an fma)."""
    def split(v):
        c = v * 134217729.0  # 2^27 + 1
        hi = c - (c - v)
        return hi, v - hi

    ah, al = split(a)
    bh, bl = split(torch.full_like(a, s))
    return ((ah * bh - p) + ah * bl + al * bh) + al * bl


def decimal_round(a: torch.Tensor, d: int, half_up: bool) -> torch.Tensor:
    """ROUND (half away from zero) / TRUNCATE (toward zero) of doubles at d decimals with Flink's
    semantics: the SHORTEST decimal representation is rounded (``BigDecimal.valueOf``), not the
    binary value — ROUND(2.675, 2) = 2.68 and TRUNCATE(0.29, 2) = 0.29, although 2.675·100 and
    0.29·100 are 267.49999999999997 and 28.999999999999996 in binary.

    Exact elementwise, without decimal strings: with s = 10^d (exact for d <= 22) and y = |x|·s,
    * a boundary c (TRUNCATE: k/s, ROUND: (2k+1)/(2s), k next to floor(y)) is x's shortest decimal
      iff the correctly rounded quotient c equals |x| — then the result is decided by c;
    * otherwise no boundary lies in x's rounding interval, so x and its decimal round alike, and
      the binary value y + e (e the product's exact error, ``_two_product_err``) decides: its side of
      a boundary is the sign of (y − boundary) + e, an exact difference plus one rounding.
    Elements with |x|·s ≥ 2^48 (and d outside 0..22) are left to the host engine (Unsupported)."""
    if d < 0 or d > 22:
        raise Unsupported("ROUND / TRUNCATE of a DOUBLE at d < 0 or d > 22")
    x = a.to(torch.float64)
    s = float(10 ** d)
    ax = torch.abs(x)
    y = ax * s
    fin = torch.isfinite(x)
    big = fin & (y >= _DEC_EXACT)
    if bool(big.any()):
        raise Unsupported("ROUND / TRUNCATE beyond the exactly decided range")
    e = _two_product_err(ax, s, y)
    k = torch.floor(y)
    if half_up:
        # the half-point next to y (k − 1/2 is ≥ 1/2 − ulp away); the decimal tie rounds away from zero
        tie = (2 * k + 1) / (2 * s) == ax
        side = ((y - k) - 0.5) + e >= 0  # binary value at or above k + 1/2
        r = torch.where(tie | side, k + 1, k)
    else:
        on_k = k / s == ax
        on_k1 = (k + 1) / s == ax
        below = (y == k) & (e < 0)  # y rounded up onto k: the binary value is just below it
        r = torch.where(on_k1, k + 1, torch.where(on_k, k, torch.where(below, k - 1, k)))
    out = torch.where(fin, torch.copysign(r / s, x), x)
    return out.to(a.dtype)


def _is_int(x) -> bool:
    if isinstance(x, torch.Tensor):
        return not x.dtype.is_floating_point and x.dtype != torch.bool
    return isinstance(x, int) and not isinstance(x, bool)


def _is_float(x) -> bool:
    return x.dtype.is_floating_point if isinstance(x, torch.Tensor) else isinstance(x, float)


def _num(x):
    if isinstance(x, torch.Tensor):
        if x.dtype == torch.bool:
            raise Unsupported("arithmetic on BOOLEAN")
        return x
    if x is None or isinstance(x, bool):
        raise Unsupported("arithmetic on NULL / BOOLEAN literal")
    return x


_FN1 = {
    "ABS": torch.abs, "SQRT": torch.sqrt, "LN": torch.log, "LOG10": torch.log10, "EXP": torch.exp,
    "SIN": torch.sin, "COS": torch.cos, "TAN": torch.tan, "ASIN": torch.asin, "ACOS": torch.acos,
    "ATAN": torch.atan, "DEGREES": torch.rad2deg, "RADIANS": torch.deg2rad, "LOG2": torch.log2,
    "SINH": torch.sinh, "COSH": torch.cosh, "TANH": torch.tanh, "COT": lambda a: 1.0 / torch.tan(a),
}
# host tensors go through numpy: its sqrt is correctly rounded like Java's Math.sqrt (torch's
# vectorised CPU sqrt is not: sqrt(2.0) comes out one ulp low)
_FN1_NP = {
    "ABS": np.abs, "SQRT": np.sqrt, "LN": np.log, "LOG10": np.log10, "EXP": np.exp, "SIN": np.sin, "COS": np.cos,
    "TAN": np.tan, "ASIN": np.arcsin, "ACOS": np.arccos, "ATAN": np.arctan, "DEGREES": np.degrees,
    "RADIANS": np.radians, "LOG2": np.log2, "SINH": np.sinh, "COSH": np.cosh, "TANH": np.tanh,
    "COT": lambda a: 1.0 / np.tan(a),
}
_FN1_PY = {
    "ABS": abs, "SQRT": math.sqrt, "LN": math.log, "LOG10": math.log10, "EXP": math.exp, "SIN": math.sin,
    "COS": math.cos, "TAN": math.tan, "ASIN": math.asin, "ACOS": math.acos, "ATAN": math.atan,
    "DEGREES": math.degrees, "RADIANS": math.radians, "LOG2": math.log2, "SINH": math.sinh, "COSH": math.cosh,
    "TANH": math.tanh, "COT": lambda a: 1.0 / math.tan(a),
}


class _Eval:
    def __init__(self, t: Table, n: int, device):
        self.t = t
        self.n = n
        self.device = device

    def col(self, name):
        names = self.t.column_names
        if name not in names:
            low = [c for c in names if c.lower() == name.lower()]
            if len(low) != 1:
                raise Unsupported("unknown column %s" % name)
            name = low[0]
        c = self.t.column(name)
        if not isinstance(c, torch.Tensor) or c.dim() != 1:
            raise Unsupported("column %s is not a scalar device column" % name)
        return c

    def full(self, x):
        if isinstance(x, torch.Tensor):
            return x
        if x is None:
            raise Unsupported("NULL result column")
        dt = torch.bool if isinstance(x, bool) else (torch.int64 if isinstance(x, int) else torch.float64)
        return torch.full((self.n,), x, dtype=dt, device=self.device)

    def __call__(self, e):
        kind = e[0]
        if kind == "col":
            return self.col(e[1])
        if kind == "lit":
            return e[1]
        if kind == "un":
            a = self(e[2])
            if e[1] == "-":
                return -_num(a)
            return ~self.boolean(a) if isinstance(a, torch.Tensor) else (not a)
        if kind == "bin":
            return self.binary(e[1], self(e[2]), self(e[3]))
        if kind == "fn":
            return self.fn(e[1], [self(a) for a in e[2]])
        if kind == "cast":
            return self.cast(self(e[1]), e[2])
        if kind == "case":
            out = self(e[2])
            for cond, val in reversed(e[1]):
                v = self(val)
                if out is None or v is None:
                    raise Unsupported("CASE with NULL branch")
                c = self.boolean(self(cond))
                v, o = self.promote(v, out)
                out = torch.where(c, self.full(v), self.full(o))
            return out
        if kind == "isnull":
            a = self(e[1])
            isn = torch.zeros(self.n, dtype=torch.bool, device=self.device) if isinstance(a, torch.Tensor) else (a is None)
            return ~isn if e[2] else isn
        if kind == "in":
            a = self(e[1])
            hit = None
            for v in e[2]:
                h = self.binary("=", a, self(v))
                hit = h if hit is None else (hit | h)
            return ~hit if e[3] else hit
        if kind == "agg":
            raise Unsupported("aggregate outside an aggregate query")
        raise Unsupported(kind)

    def boolean(self, x):
        if isinstance(x, torch.Tensor) and x.dtype == torch.bool:
            return x
        if isinstance(x, bool):
            return self.full(x)
        raise Unsupported("non-boolean condition")

    @staticmethod
    def promote(a, b):
        if isinstance(a, torch.Tensor) and isinstance(b, torch.Tensor) and a.dtype != b.dtype:
            dt = torch.promote_types(a.dtype, b.dtype)
            return a.to(dt), b.to(dt)
        return a, b

    def binary(self, op, a, b):
        if op in ("AND", "OR"):
            a, b = self.boolean(a), self.boolean(b)
            return a & b if op == "AND" else a | b
        if op in ("=", "<>", "<", "<=", ">", ">="):
            if a is None or b is None:
                raise Unsupported("comparison with NULL")
            if op not in ("=", "<>"):
                a, b = _num(a), _num(b)
            a = self.full(a)
            return {"=": torch.eq, "<>": torch.ne, "<": torch.lt, "<=": torch.le, ">": torch.gt, ">=": torch.ge}[op](a, b)
        a, b = _num(a), _num(b)
        both_int = _is_int(a) and _is_int(b)
        if op == "+":
            return a + b
        if op == "-":
            return a - b
        if op == "*":
            return a * b
        if op in ("/", "%"):
            if both_int:
                if isinstance(b, torch.Tensor):
                    if bool((b == 0).any()):
                        raise Unsupported("integer division by zero")
                elif b == 0:
                    raise Unsupported("integer division by zero")
                if op == "/":
                    if not isinstance(a, torch.Tensor) and not isinstance(b, torch.Tensor):
                        return int(a / b)
                    return torch.div(self.full(a) if not isinstance(a, torch.Tensor) else a, b, rounding_mode="trunc")
                return torch.fmod(self.full(a) if not isinstance(a, torch.Tensor) else a, b)
            if op == "/":
                if not _is_float(a) and not _is_float(b):
                    a = a.to(torch.float64) if isinstance(a, torch.Tensor) else float(a)
                return a / b if isinstance(a, torch.Tensor) or isinstance(b, torch.Tensor) else \
                    (a / b if b != 0 else (math.nan if a == 0 else math.copysign(math.inf, a)))
            return torch.fmod(self.full(a) if not isinstance(a, torch.Tensor) else a, b)
        raise Unsupported(op)

    def fn(self, name, args):
        if name in _FN1 and len(args) == 1:
            a = _num(args[0])
            if not isinstance(a, torch.Tensor):
                return java_math(_FN1_PY[name], a)
            if name != "ABS" and not a.dtype.is_floating_point:
                a = a.to(torch.float64)
            if a.device.type == "cpu":
                with np.errstate(all="ignore"):
                    return torch.from_numpy(np.asarray(_FN1_NP[name](a.contiguous().numpy())))
            return _FN1[name](a)
        if name in ("CEIL", "CEILING", "FLOOR") and len(args) == 1:
            a = _num(args[0])
            f = torch.ceil if name != "FLOOR" else torch.floor
            if isinstance(a, torch.Tensor):
                return f(a) if a.dtype.is_floating_point else a
            return float((math.ceil if name != "FLOOR" else math.floor)(a)) if isinstance(a, float) else a
        if name == "SIGN" and len(args) == 1:
            a = _num(args[0])
            if isinstance(a, torch.Tensor):  # Math.signum: NaN stays NaN (torch.sign gives 0)
                return torch.where(torch.isnan(a), a, torch.sign(a)) if a.dtype.is_floating_point else torch.sign(a)
            return a if a != a else type(a)((a > 0) - (a < 0))
        if name == "POWER" and len(args) == 2:
            a, b = _num(args[0]), _num(args[1])
            if not isinstance(a, torch.Tensor):
                a = self.full(float(a))
            return torch.pow(a.to(torch.float64) if not a.dtype.is_floating_point else a, b)
        if name == "MOD" and len(args) == 2:
            return self.binary("%", args[0], args[1])
        if name in ("ROUND", "TRUNCATE") and len(args) in (1, 2):
            a = _num(args[0])
            d = int(args[1]) if len(args) == 2 else 0
            if _is_int(a) and d >= 0:
                return a  # ROUND / TRUNCATE of an INT at d >= 0 is the INT itself
            if not isinstance(a, torch.Tensor):
                from .misc import _round, _truncate

                return (_round if name == "ROUND" else _truncate)(a, d)
            if _is_int(a):  # tens, hundreds…: integer arithmetic, ties away from zero
                p = 10 ** -d
                m = torch.abs(a) + (p // 2 if name == "ROUND" else 0)
                return torch.sign(a) * (m // p) * p
            if not _is_float(a):
                raise Unsupported(name + " of a non-numeric value")
            return decimal_round(a, d, name == "ROUND")
        if name == "LOG" and len(args) in (1, 2):  # Flink: LOG(x) = LN(x), LOG(b, x) = LN(x) / LN(b)
            if len(args) == 1:
                return self.fn("LN", args)
            return self.binary("/", self.fn("LN", [args[1]]), self.fn("LN", [args[0]]))
        if name == "ATAN2" and len(args) == 2:
            a, b = _num(args[0]), _num(args[1])
            if not isinstance(a, torch.Tensor) and not isinstance(b, torch.Tensor):
                return math.atan2(a, b)
            a, b = self.full(a), self.full(b)
            return torch.atan2(a.to(torch.float64) if not a.dtype.is_floating_point else a,
                               b.to(torch.float64) if not b.dtype.is_floating_point else b)
        if name in ("PI", "E") and not args:
            return math.pi if name == "PI" else math.e
        if name == "IF" and len(args) == 3:
            c = self.boolean(args[0])
            a, b = self.promote(self.full(_num(args[1])), self.full(_num(args[2])))
            return torch.where(self.full(c), a, b)
        if name == "COALESCE" and args:
            vals = [v for v in args if v is not None]
            if not vals:
                raise Unsupported("COALESCE of NULLs")
            out = self.full(_num(vals[0]))  # device values are never NULL: the first non-NULL argument
            for v in vals[1:]:
                out, _ = self.promote(out, self.full(_num(v)))
            return out
        if name in ("LEAST", "GREATEST") and len(args) >= 2:
            out = self.full(_num(args[0]))
            for x in args[1:]:
                out, x = self.promote(out, self.full(_num(x)))
                out = torch.minimum(out, x) if name == "LEAST" else torch.maximum(out, x)
            return out
        raise Unsupported("function %s/%d" % (name, len(args)))

    def cast(self, a, ty):
        a = self.full(a)
        if ty in ("DOUBLE",):
            return a.to(torch.float64)
        if ty in ("FLOAT", "REAL"):
            return a.to(torch.float32)
        if ty in ("INT", "INTEGER"):
            return (torch.trunc(a) if a.dtype.is_floating_point else a).to(torch.int32)
        if ty == "BIGINT":
            return (torch.trunc(a) if a.dtype.is_floating_point else a).to(torch.int64)
        if ty == "BOOLEAN":
            return a != 0 if a.dtype != torch.bool else a
        raise Unsupported("CAST AS %s" % ty)


def _has_agg(e) -> bool:
    if isinstance(e, list):
        return any(_has_agg(x) for x in e)
    if not isinstance(e, tuple) or not e:
        return False
    if e[0] == "agg":
        return True
    return any(_has_agg(x) for x in e[1:] if isinstance(x, (tuple, list)))


def _out_name(e, alias, idx, used):
    if alias:
        name = alias
    elif e[0] == "col":
        name = e[1]
    else:
        name = "EXPR$%d" % idx
    if name in used:
        raise Unsupported("duplicate output column %s" % name)
    used.add(name)
    return name


def _device_of(t: Table):
    for n in t.column_names:
        c = t.column(n)
        if isinstance(c, torch.Tensor):
            return c.device
    return torch.device("cpu")


def evaluate(statement: str, t: Table, world: int = 1, rank: int = 0) -> Table:
    """Runs ``statement`` against ``t`` on the columns' device; raises ``Unsupported`` outside the
    subset. ``world > 1``: aggregates are merged across ranks and dealt round-robin."""
    q = parse(statement)
    items, where, group = q.items, q.where, q.group
    if (q.order or q.limit is not None) and world > 1:
        raise Unsupported("ORDER BY / LIMIT over ranks (needs the global order)")
    if q.distinct:
        # SELECT DISTINCT e1, e2, ... = GROUP BY e1, e2, ... (ordered by key like every GROUP BY)
        if group is not None or q.having is not None or any(_has_agg(e) or e[0] == "star" for e, _ in items):
            raise Unsupported("DISTINCT with aggregates, GROUP BY or *")
        group = [e for e, _ in items]
    dev = _device_of(t)
    aggregate = group is not None or any(_has_agg(e) for e, _ in items)
    if q.having is not None and not aggregate:
        raise Unsupported("HAVING without aggregation")
    werr = None
    if where is not None:
        try:
            ev = _Eval(t, t.num_rows, dev)
            mask = ev.boolean(ev(where))
            if _has_agg(where):
                raise Unsupported("aggregate in WHERE")
            t = t.take(torch.nonzero(mask, as_tuple=True)[0])
        except Unsupported as e:
            # a data-dependent failure (integer division by zero) may hit one rank only: an
            # aggregate's ranks must still agree on the path, so it joins the agreement
            if not (aggregate and world > 1):
                raise
            werr = e
    if not aggregate:
        ev = _Eval(t, t.num_rows, dev)
        out, used = {}, set()
        for i, (e, alias) in enumerate(items):
            if e[0] == "star":
                for c in t.column_names:
                    if c in used:
                        raise Unsupported("duplicate output column %s" % c)
                    used.add(c)
                    out[c] = t.column(c)
                continue
            name = _out_name(e, alias, i, used)
            out[name] = ev.full(ev(e))
        res = Table(out, num_rows=t.num_rows)
        return _order_limit(res, q, t) if q.order or q.limit is not None else res
    res = _aggregate(items, group or [], t, dev, world, rank, werr, having=q.having)
    return _order_limit(res, q, None) if q.order or q.limit is not None else res


def _order_limit(res: Table, q: "Query", src: Optional[Table]) -> Table:
    """ORDER BY (stable, lexicographic; NaN the largest DOUBLE as Double.compare) then LIMIT /
    OFFSET over the result rows. Keys: output columns by name or 1-based position, or expressions
    of output columns — and, for row-wise statements (``src``: the filtered input, row-aligned with
    the result), of input columns the output does not shadow."""
    n = res.num_rows
    dev = _device_of(res) if res.column_names else torch.device("cpu")
    perm = torch.arange(n, device=dev)
    if q.order:
        names = res.column_names
        ctx = {c: res.column(c) for c in names}
        if src is not None:
            for c in src.column_names:
                ctx.setdefault(c, src.column(c))
        ev = _Eval(Table(ctx, num_rows=n), n, dev)
        keys = []
        for e, desc in q.order:
            if e[0] == "lit" and isinstance(e[1], int) and not isinstance(e[1], bool):
                if not 1 <= e[1] <= len(names):
                    raise Unsupported("ORDER BY position %d" % e[1])
                k = res.column(names[e[1] - 1])
            else:
                k = ev.full(ev(e))
            if not isinstance(k, torch.Tensor) or k.dim() != 1:
                raise Unsupported("ORDER BY a non-scalar column")
            keys.append((k.to(torch.int8) if k.dtype == torch.bool else k, desc))
        for k, desc in reversed(keys):
            perm = perm[torch.sort(k[perm], stable=True, descending=desc).indices]
    if q.limit is not None or q.offset:
        perm = perm[q.offset:q.offset + q.limit if q.limit is not None else None]
    return res.take(perm)


# ---- aggregation: per-group partial states (sum, count, min, max) so ranks can merge them

def _local_states(items, group, t: Table, dev, world, having=None):
    if any(e[0] == "star" for e, _ in items):
        raise Unsupported("SELECT * with aggregates")
    ev = _Eval(t, t.num_rows, dev)
    keys = [ev.full(ev(g)) for g in group]
    for k in keys:
        if k.dtype == torch.bool:
            raise Unsupported("BOOLEAN group key")
    aggs = []  # (name, arg tensor | None)

    def collect(e):
        for gi, g in enumerate(group):
            if e == g:
                return ("keyref", gi)
        if e[0] == "agg":
            arg = None if e[2] is None else ev.full(ev(e[2]))
            if e[1] in ("SUM", "AVG", "MIN", "MAX") and arg is not None and arg.dtype == torch.bool:
                raise Unsupported("%s over BOOLEAN" % e[1])
            aggs.append((e[1], arg))
            return ("aggref", len(aggs) - 1)
        if e[0] in ("bin",):
            return (e[0], e[1], collect(e[2]), collect(e[3]))
        if e[0] == "un":
            return ("un", e[1], collect(e[2]))
        if e[0] == "fn":
            return ("fn", e[1], [collect(a) for a in e[2]])
        if e[0] == "cast":
            return ("cast", collect(e[1]), e[2])
        if e[0] == "lit":
            return e
        raise Unsupported("non-grouped expression in an aggregate query")

    outs = [(collect(e), alias) for e, alias in items]
    having_c = collect(having) if having is not None else None
    n = t.num_rows
    if keys:
        K = torch.stack([k.to(torch.float64) if k.dtype.is_floating_point else k.to(torch.int64) for k in keys], 1) \
            if len({k.dtype.is_floating_point for k in keys}) == 1 else None
        if K is None:
            raise Unsupported("mixed integer / floating group keys")
        uk, inv = torch.unique(K, dim=0, return_inverse=True)
        ng = uk.shape[0]
    else:
        uk = torch.zeros((1, 0), dtype=torch.int64, device=dev)
        inv = torch.zeros(n, dtype=torch.int64, device=dev)
        ng = 1
    # partial states per aggregate
    states = []
    cnt_all = torch.zeros(ng, dtype=torch.int64, device=dev).index_add_(0, inv, torch.ones(n, dtype=torch.int64,
                                                                                           device=dev))
    for name, arg in aggs:
        if arg is None:
            states.append({"count": cnt_all})
            continue
        acc = torch.float64 if arg.dtype.is_floating_point else torch.int64
        st = {"count": cnt_all}
        if name in ("SUM", "AVG"):
            st["sum"] = torch.zeros(ng, dtype=acc, device=dev).index_add_(0, inv, arg.to(acc))
        if name == "MIN":
            st["min"] = torch.full((ng,), math.inf if acc == torch.float64 else 2 ** 62, dtype=acc,
                                   device=dev).scatter_reduce_(0, inv, arg.to(acc), "amin")
        if name == "MAX":
            st["max"] = torch.full((ng,), -math.inf if acc == torch.float64 else -2 ** 62, dtype=acc,
                                   device=dev).scatter_reduce_(0, inv, arg.to(acc), "amax")
        st["dtype"] = arg.dtype
        states.append(st)
    if not keys and world == 1 and n == 0:
        raise Unsupported("aggregate over an empty input (NULL result)")
    return aggs, states, outs, keys, uk, ng, having_c


def _aggregate(items, group, t: Table, dev, world, rank, werr=None, having=None) -> Table:
    err, local = werr, None
    if err is None:
        try:
            local = _local_states(items, group, t, dev, world, having)
        except Unsupported as e:
            err = e
    if world > 1:
        # every rank must take the same path: the merge below and the host fallback are collective
        from ...parallel import comm

        if not all(comm.all_gather_object(err is None)):
            raise Unsupported("some rank cannot evaluate the statement on the device: %s" % err)
    elif err is not None:
        raise err
    aggs, states, outs, keys, uk, ng, having_c = local
    if world > 1:
        uk, states, _ = _merge_ranks(uk, states, dev, bool(keys))
        ng = uk.shape[0]
        if not keys and states and int(states[0]["count"].sum().item()) == 0:
            # no rows on any rank (e.g. WHERE filtered everything): Flink returns NULLs, which
            # only the host fallback produces; the merged count is the same on every rank, so
            # every rank takes the fallback together
            raise Unsupported("aggregate over an empty input (NULL result)")
    res = {}
    used = set()
    key_cols = [uk[:, i].to(keys[i].dtype) for i in range(len(keys))]

    def value(e):
        if e[0] == "aggref":
            name, _ = aggs[e[1]]
            st = states[e[1]]
            if name == "COUNT":
                return st["count"]
            if name == "SUM":
                # Flink: SUM keeps its argument's type (an INT sum wraps like Java's int)
                return st["sum"].to(st["dtype"]) if st["dtype"] in (torch.float32, torch.int32, torch.int16,
                                                                      torch.int8) else st["sum"]
            if name == "AVG":
                if not st["dtype"].is_floating_point:
                    # Flink's IntegralAvgAggFunction: BIGINT sum / BIGINT count truncated toward
                    # zero, in the argument's type
                    return torch.div(st["sum"], st["count"], rounding_mode="trunc").to(st["dtype"])
                return st["sum"] / st["count"].to(torch.float64)
            if name == "MIN":
                return st["min"].to(st["dtype"])
            return st["max"].to(st["dtype"])
        if e[0] == "keyref":
            return key_cols[e[1]]
        if e[0] == "lit":
            return e[1]
        sub = _Eval(Table({}, num_rows=ng), ng, dev)
        if e[0] == "bin":
            return sub.binary(e[1], value(e[2]), value(e[3]))
        if e[0] == "un":
            a = value(e[2])
            return -a if e[1] == "-" else ~sub.boolean(a)
        if e[0] == "fn":
            return sub.fn(e[1], [value(a) for a in e[2]])
        if e[0] == "cast":
            return sub.cast(value(e[1]), e[2])
        raise Unsupported(e[0])

    for i, (e, alias) in enumerate(outs):
        name = alias or (group[e[1]][1] if e[0] == "keyref" and group[e[1]][0] == "col" else "EXPR$%d" % i)
        if name in used:
            raise Unsupported("duplicate output column %s" % name)
        used.add(name)
        v = value(e)
        res[name] = v if isinstance(v, torch.Tensor) else torch.full((ng,), v, device=dev)
    out = Table(res, num_rows=ng)
    if having_c is not None:  # the groups whose HAVING condition holds (evaluated on the merged states)
        keep = _Eval(Table({}, num_rows=ng), ng, dev).boolean(value(having_c))
        out = out.take(torch.nonzero(keep if isinstance(keep, torch.Tensor) else
                                     torch.full((ng,), bool(keep), device=dev), as_tuple=True)[0])
        ng = out.num_rows
    if world > 1:
        out = out.take(torch.arange(rank, ng, world, device=dev))
    return out


def _merge_ranks(uk, states, dev, keyed):
    """All-gathers every rank's partial group states (small) and merges them by key."""
    from ...parallel import comm

    payload = {"uk": uk.cpu(), "states": [{k: (v.cpu() if isinstance(v, torch.Tensor) else v) for k, v in st.items()}
                                          for st in states]}
    parts = comm.all_gather_object(payload)
    UK = torch.cat([p["uk"] for p in parts]).to(dev)
    if keyed:
        uk2, inv = torch.unique(UK, dim=0, return_inverse=True)
    else:
        uk2 = UK[:1]
        inv = torch.zeros(UK.shape[0], dtype=torch.int64, device=dev)
    ng = uk2.shape[0]
    merged = []
    for j, st in enumerate(states):
        m = {"dtype": st.get("dtype")}
        for key in ("count", "sum", "min", "max"):
            if key not in st:
                continue
            cat = torch.cat([p["states"][j][key] for p in parts]).to(dev)
            if key in ("count", "sum"):
                m[key] = torch.zeros(ng, dtype=cat.dtype, device=dev).index_add_(0, inv, cat)
            else:
                fill = (math.inf if key == "min" else -math.inf) if cat.dtype.is_floating_point else \
                    (2 ** 62 if key == "min" else -2 ** 62)
                m[key] = torch.full((ng,), fill, dtype=cat.dtype, device=dev).scatter_reduce_(
                    0, inv, cat, "amin" if key == "min" else "amax")
        merged.append(m)
    cnt = merged[0]["count"] if merged else None
    return uk2, merged, cnt


def try_evaluate(statement: str, t: Table, world: int = 1, rank: int = 0) -> Optional[Table]:
    try:
        return evaluate(statement, t, world, rank)
    except Unsupported:
        return None


__all__: List[str] = ["Unsupported", "parse", "evaluate", "try_evaluate"]
