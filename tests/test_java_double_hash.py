"""FeatureHasher's `col=Double.toString(v)` murmur3 hashing: the device kernel
(``ops/csrc/javastr.hip``) against the host runtime (``csrc/host/javastr.cpp``, std::to_chars
shortest digits), and the kernel's multiplier tables against exact shortest-digit results."""
import math
import random
import struct

import numpy as np
import pytest
import torch

from flink_ml_amd.ops import hashing


def _values(n_random=20000, seed=7):
    rnd = random.Random(seed)
    vals = [rnd.random() for _ in range(n_random)]
    vals += [struct.unpack("<d", struct.pack("<Q", rnd.getrandbits(64)))[0] for _ in range(n_random)]
    vals += [float(i) for i in range(-50, 3000)] + [10.0 ** k for k in range(-300, 300)]
    vals += [5e-324, -5e-324, 2.2250738585072014e-308, 1.7976931348623157e308, 0.1, 0.2, 0.3, 1 / 3, 2 ** -44,
             9007199254740993.0, 1e23, 123456789012345678.0, 1e-3, 9.999999999999998e-4, 1e7, 9999999.999999998,
             0.0, -0.0, math.inf, -math.inf, math.nan, 0.5, 100.0, 1234567.0, 12345678.0]
    return np.array(vals, dtype=np.float64)


def _shortest(v, inv, pw):
    """Python transliteration of the kernel's digit generation (same tables)."""
    M = (1 << 64) - 1

    def mulshift(m, mul, j):
        lo, hi = mul
        h0 = (m * lo) >> 64
        l1, h1 = (m * hi) & M, (m * hi) >> 64
        s = h0 + l1
        h1 += s >> 64
        s &= M
        d = j - 64
        return ((h1 << (64 - d)) | (s >> d)) & M

    def p5f(x):
        c = 0
        while x % 5 == 0:
            x //= 5
            c += 1
        return c

    bits = struct.unpack("<Q", struct.pack("<d", v))[0]
    ie, im = (bits >> 52) & 0x7FF, bits & ((1 << 52) - 1)
    m2, e2 = (1 << 52) | im, ie - 1075
    if ie and -52 <= e2 <= 0 and not m2 & ((1 << -e2) - 1):
        x, e = m2 >> -e2, 0
        while x % 10 == 0:
            x //= 10
            e += 1
        return x, e
    e2, m2 = (-1076, im) if ie == 0 else (ie - 1077, (1 << 52) | im)
    ab, mv, mms = m2 % 2 == 0, 4 * m2, 1 if (im or ie <= 1) else 0
    vmtz = vrtz = False
    if e2 >= 0:
        q = ((e2 * 78913) >> 18) - (e2 > 3)
        e10, mul = q, inv[q]
        i = -e2 + q + 125 + ((q * 1217359) >> 19)
        vr, vp, vm = (mulshift(x, mul, i) for x in (4 * m2, 4 * m2 + 2, 4 * m2 - 1 - mms))
        if q <= 21:
            if mv % 5 == 0:
                vrtz = p5f(mv) >= q
            elif ab:
                vmtz = p5f(mv - 1 - mms) >= q
            else:
                vp -= p5f(mv + 2) >= q
    else:
        q = ((-e2 * 732923) >> 20) - (-e2 > 1)
        e10, i = q + e2, -e2 - q
        j = q - (((i * 1217359) >> 19) + 1 - 125)
        vr, vp, vm = (mulshift(x, pw[i], j) for x in (4 * m2, 4 * m2 + 2, 4 * m2 - 1 - mms))
        if q <= 1:
            vrtz = True
            if ab:
                vmtz = mms == 1
            else:
                vp -= 1
        elif q < 63:
            vrtz = mv & ((1 << q) - 1) == 0
    removed = last = 0
    if vmtz or vrtz:
        while vp // 10 > vm // 10:
            vmtz &= vm % 10 == 0
            vrtz &= last == 0
            last = vr % 10
            vr, vp, vm, removed = vr // 10, vp // 10, vm // 10, removed + 1
        if vmtz:
            while vm % 10 == 0:
                vrtz &= last == 0
                last = vr % 10
                vr, vp, vm, removed = vr // 10, vp // 10, vm // 10, removed + 1
        if vrtz and last == 5 and vr % 2 == 0:
            last = 4
        return vr + ((vr == vm and (not ab or not vmtz)) or last >= 5), e10 + removed
    ru = False
    if vp // 100 > vm // 100:
        ru = vr % 100 >= 50
        vr, vp, vm, removed = vr // 100, vp // 100, vm // 100, removed + 2
    while vp // 10 > vm // 10:
        ru = vr % 10 >= 5
        vr, vp, vm, removed = vr // 10, vp // 10, vm // 10, removed + 1
    return vr + (vr == vm or ru), e10 + removed


def test_tables_give_shortest_round_trip_digits():
    inv_t, pw_t = hashing.ryu_tables("cpu")
    inv = [(int(a) & (2 ** 64 - 1), int(b)) for a, b in inv_t.view(-1, 2).tolist()]
    pw = [(int(a) & (2 ** 64 - 1), int(b)) for a, b in pw_t.view(-1, 2).tolist()]
    for v in _values(3000):
        if v == 0 or not math.isfinite(v):
            continue
        digits, e = _shortest(abs(float(v)), inv, pw)
        assert float("%de%d" % (digits, e)) == abs(float(v))          # round trips
        r = repr(abs(float(v))).replace(".", "").split("e")[0].strip("0")
        assert str(digits).rstrip("0") == r or len(str(digits)) <= len(r)  # and is no longer than repr


@pytest.mark.gpu
def test_device_hash_matches_host():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    vals = _values()
    for prefix in ("f0=", "", "a much longer column name="):
        host = hashing.hash_prefixed_doubles(prefix, vals)
        dev = hashing.hash_prefixed_doubles_device(prefix, torch.from_numpy(vals).cuda()).cpu().numpy()
        bad = np.nonzero(host != dev)[0]
        assert bad.size == 0, [(vals[i], host[i], dev[i]) for i in bad[:5]]


@pytest.mark.gpu
def test_feature_hasher_device_categorical_matches_host():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from flink_ml_amd import Table
    from flink_ml_amd.models import FeatureHasher

    rng = np.random.default_rng(3)
    x = rng.random(5000)
    y = rng.integers(0, 7, 5000).astype(np.float64)
    fh = FeatureHasher().set_input_cols("a", "b").set_categorical_cols("a", "b").set_output_col("o") \
        .set_num_features(1000)
    gpu = fh.transform(Table({"a": torch.from_numpy(x).cuda(), "b": torch.from_numpy(y).cuda()}))[0].column("o")
    cpu = fh.transform(Table({"a": torch.from_numpy(x), "b": torch.from_numpy(y)}))[0].column("o")
    assert torch.equal(gpu.indices.cpu(), cpu.indices.cpu()) and torch.equal(gpu.indptr.cpu(), cpu.indptr.cpu())
