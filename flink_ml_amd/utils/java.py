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
