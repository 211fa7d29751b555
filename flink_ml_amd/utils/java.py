"""Bit-exact re-implementations of the JVM behaviours the reference depends on
(SURVEY §7.4 "RNG compatibility"):

* ``java_string_hash`` — ``String.hashCode`` (default seeds: ``HasSeed.java:27-35``).
* ``JavaRandom`` — ``java.util.Random`` 48-bit LCG incl. ``nextInt(bound)``, ``nextDouble``,
  ``nextGaussian`` (KMeans init sampling ``DataStreamUtils.java:647-696``, data generators,
  MinHash coefficients).
* ``tuple2_hash`` — ``Tuple2.of(a, b).hashCode()`` (``RowGenerator`` per-task seed).
* ``java_long_hash``, ``java_double_hash``.
"""
from __future__ import annotations

import math
import struct


def _i32(x: int) -> int:
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= (1 << 31) else x


def _i64(x: int) -> int:
    x &= 0xFFFFFFFFFFFFFFFF
    return x - (1 << 64) if x >= (1 << 63) else x


def java_string_hash(s: str) -> int:
    h = 0
    units = s.encode("utf-16-be")
    for k in range(0, len(units), 2):
        h = (31 * h + ((units[k] << 8) | units[k + 1])) & 0xFFFFFFFF
    return _i32(h)


_HASH_SIG = False


def java_string_hashes(strings) -> "np.ndarray":
    """``String.hashCode()`` of many strings at once (native loop over their UTF-16 units)."""
    import ctypes

    import numpy as np

    from ..ops import native

    global _HASH_SIG
    if not _HASH_SIG:
        native.register_host_sigs({"fmlx_java_string_hashes": [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                                               ctypes.c_void_p]})
        _HASH_SIG = True
    strings = list(strings)
    n = len(strings)
    out = np.zeros(n, dtype=np.int32)
    if n == 0:
        return out
    raw = "".join(strings).encode("utf-16-le", "surrogatepass")
    units = np.frombuffer(raw, dtype=np.uint16) if raw else np.zeros(1, dtype=np.uint16)
    lens = np.fromiter(map(len, strings), dtype=np.int64, count=n)
    if int(lens.sum()) != len(raw) // 2:  # astral characters take two UTF-16 units
        lens = np.fromiter((len(w.encode("utf-16-le", "surrogatepass")) // 2 for w in strings), dtype=np.int64,
                           count=n)
    offs = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lens, out=offs[1:])
    native.host().fmlx_java_string_hashes(units.ctypes.data, offs.ctypes.data, n, out.ctypes.data)
    return out


def java_long_hash(v: int) -> int:
    v &= 0xFFFFFFFFFFFFFFFF
    return _i32(v ^ (v >> 32))


def java_int_hash(v: int) -> int:
    return _i32(v)


def java_double_hash(d: float) -> int:
    if d != d:
        bits = 0x7FF8000000000000
    else:
        bits = struct.unpack(">q", struct.pack(">d", d))[0]
    return java_long_hash(bits)


def java_hash(obj) -> int:
    if obj is None:
        return 0
    if isinstance(obj, bool):
        return 1231 if obj else 1237
    if isinstance(obj, int):
        if -(1 << 31) <= obj < (1 << 31):
            return _i32(obj)
        return java_long_hash(obj)
    if isinstance(obj, float):
        return java_double_hash(obj)
    if isinstance(obj, str):
        return java_string_hash(obj)
    raise TypeError("no Java hash for %r" % type(obj))


def _table_size_for(n: int) -> int:
    cap = 1
    while cap < n:
        cap <<= 1
    return max(cap, 1)


def java_hashmap_order(keys, hash_fn=java_hash, initial_capacity: int = 16):
    """Iteration order of a ``java.util.HashMap`` / ``HashSet`` filled with ``keys`` in that order
    (no treeified bins): by bucket of the final table, then insertion order (Java's resize split
    keeps the relative order inside a bucket). ``initial_capacity`` mirrors ``new HashMap<>(n)``."""
    keys = list(keys)
    cap = _table_size_for(initial_capacity)
    size = 0
    for _ in keys:
        size += 1
        if size > cap * 0.75:
            cap *= 2

    if hash_fn is java_string_hash and len(keys) > 256 and all(isinstance(k, str) for k in keys):
        # many string keys: hashes in one native pass, buckets and the stable order in numpy
        import numpy as np

        h = java_string_hashes(keys).view(np.uint32).astype(np.uint64)
        b = (h ^ (h >> np.uint64(16))) & np.uint64(cap - 1)
        return [keys[i] for i in np.argsort(b, kind="stable").tolist()]

    def bucket(k):
        h = hash_fn(k) & 0xFFFFFFFF
        return (h ^ (h >> 16)) & (cap - 1)

    return [k for _, _, k in sorted(((bucket(k), i, k) for i, k in enumerate(keys)), key=lambda x: (x[0], x[1]))]


def java_double_to_string(d: float) -> str:
    """``Double.toString``: plain notation for 1e-3 <= |d| < 1e7, else ``d.dddE±n``; shortest
    round-trip digits (same digit selection as Python's ``repr``)."""
    if d != d:
        return "NaN"
    if d in (float("inf"), float("-inf")):
        return "Infinity" if d > 0 else "-Infinity"
    if d == 0:
        return "-0.0" if math.copysign(1.0, d) < 0 else "0.0"
    a = abs(d)
    if 1e-3 <= a < 1e7:
        r = repr(d)
        if "e" in r or "E" in r:
            r = "%.17f" % d
            r = r.rstrip("0")
        if "." not in r:
            r += ".0"
        if r.endswith("."):
            r += "0"
        return r
    mant, exp = ("%r" % a).lower().split("e") if "e" in repr(a) else (repr(a), "0")
    if "e" not in repr(a):
        # repr printed a plain number (e.g. 12345678.0): normalise to scientific
        digits = repr(a).replace(".", "").lstrip("0").rstrip("0") or "0"
        ip = repr(a).split(".")[0]
        e = len(ip.lstrip("0")) - 1 if ip.strip("0") else -(len(repr(a).split(".")[1]) - len(
            repr(a).split(".")[1].lstrip("0")) + 1)
        mant = digits[0] + "." + (digits[1:] or "0")
        exp = str(e)
    else:
        if "." not in mant:
            mant += ".0"
        e = int(exp)
        exp = str(e)
    return ("-" if d < 0 else "") + mant + "E" + exp


def java_number_to_string(v) -> str:
    """``String.valueOf(Number)`` for the boxed types the reference accepts."""
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, int):
        return str(v)
    return java_double_to_string(float(v))


def tuple2_hash(a, b) -> int:
    """``org.apache.flink.api.java.tuple.Tuple2.hashCode``: 31*hash(f0) + hash(f1)."""
    return _i32(31 * java_hash(a) + java_hash(b))


class JavaRandom:
    """``java.util.Random`` (48-bit LCG)."""

    _MULT = 0x5DEECE66D
    _ADD = 0xB
    _MASK = (1 << 48) - 1

    def __init__(self, seed: int):
        self.set_seed(seed)
        self._next_gaussian = None

    def set_seed(self, seed: int) -> None:
        self._seed = (seed ^ self._MULT) & self._MASK
        self._next_gaussian = None

    def next(self, bits: int) -> int:
        self._seed = (self._seed * self._MULT + self._ADD) & self._MASK
        return _i32(self._seed >> (48 - bits))

    def next_int(self, bound: int = None) -> int:
        if bound is None:
            return self.next(32)
        if bound <= 0:
            raise ValueError("bound must be positive")
        r = self.next(31)
        m = bound - 1
        if (bound & m) == 0:
            return _i32((bound * r) >> 31)
        u = r
        while True:
            r = u % bound
            if u - r + m < (1 << 31):
                return r
            u = self.next(31)

    def next_long(self) -> int:
        return _i64((self.next(32) << 32) + self.next(32))

    def next_boolean(self) -> bool:
        return self.next(1) != 0

    def next_double(self) -> float:
        return ((self.next(26) << 27) + self.next(27)) * (1.0 / (1 << 53))

    def next_float(self) -> float:
        return self.next(24) / float(1 << 24)

    def next_gaussian(self) -> float:
        if self._next_gaussian is not None:
            g = self._next_gaussian
            self._next_gaussian = None
            return g
        while True:
            v1 = 2 * self.next_double() - 1
            v2 = 2 * self.next_double() - 1
            s = v1 * v1 + v2 * v2
            if 0 < s < 1:
                break
        mul = math.sqrt(-2 * math.log(s) / s)
        self._next_gaussian = v2 * mul
        return v1 * mul

    nextInt = next_int
    nextLong = next_long
    nextDouble = next_double
    nextGaussian = next_gaussian


def java_random_doubles(seed: int, n: int):
    """``n`` successive ``new Random(seed).nextDouble()`` values (native host loop)."""
    import ctypes

    import numpy as np

    from ..ops import native

    out = np.empty(n, dtype=np.float64)
    if n:
        lib = native.host()
        fn = lib.fmlx_java_next_doubles
        fn.argtypes, fn.restype = [ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p], None
        fn(int(seed), int(n), out.ctypes.data)
    return out
