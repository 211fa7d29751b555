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


def _treemap_rows(cols, cats, nf):
    """The reference's per-row TreeMap (FeatureHasher.java:118-141, updateMap :184-194) in Python:
    numeric columns first, then categorical, the first value of an index stored as is."""

    def idx(h):
        h = int(h)
        a = h if h == -(1 << 31) else abs(h)
        return a % nf

    names = list(cols)
    num = [c for c in names if c not in cats]
    n = len(cols[names[0]])
    hnum = {c: idx(hashing.hash_strings([c])[0]) for c in num}
    hcat = {c: hashing.hash_prefixed_doubles(c + "=", np.asarray(cols[c], dtype=np.float64)) for c in cats}
    rows = []
    for r in range(n):
        m = {}
        for c in num:
            k = hnum[c]
            m[k] = m[k] + float(cols[c][r]) if k in m else float(cols[c][r])
        for c in cats:
            k = idx(hcat[c][r])
            m[k] = m[k] + 1.0 if k in m else 1.0
        rows.append(sorted(m.items()))
    return rows


@pytest.mark.gpu
def test_feature_hasher_device_rows_match_treemap():
    """The per-row device assembly (csrc/hash.hip fh_rows_kernel) against the reference TreeMap
    semantics, exactly — a small numFeatures forces collisions between numeric and categorical
    features, -0.0 must survive as a first value — and against the general sort-unique path."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from flink_ml_amd import Table
    from flink_ml_amd.models import FeatureHasher
    from flink_ml_amd.models.feature import text

    rng = np.random.default_rng(11)
    n = 3000
    cols = {"f0": rng.normal(size=n), "f1": rng.integers(0, 5, n).astype(np.float64), "f2": rng.normal(size=n),
            "f3": rng.integers(0, 9, n).astype(np.float64), "f4": rng.normal(size=n)}
    cols["f0"][:50] = -0.0
    cats = ["f1", "f3"]
    for nf in (3, 7, 1000):
        fh = FeatureHasher().set_input_cols(*cols).set_categorical_cols(*cats).set_output_col("o").set_num_features(nf)
        tab = Table({c: torch.from_numpy(v).cuda() for c, v in cols.items()})
        got = fh.transform(tab)[0].column("o")
        ip, ix, vv = got.indptr.cpu().numpy(), got.indices.cpu().numpy(), got.values.cpu().numpy()
        want = _treemap_rows(cols, cats, nf)
        for r in range(n):
            row = list(zip(ix[ip[r]:ip[r + 1]].tolist(), vv[ip[r]:ip[r + 1]].tolist()))
            assert [k for k, _ in row] == [k for k, _ in want[r]], (nf, r)
            assert all(struct.pack("<d", a) == struct.pack("<d", b) for (_, a), (_, b) in zip(row, want[r])), (nf, r)
        saved = text.FH_ROWS_MAX_COLS
        text.FH_ROWS_MAX_COLS = 0  # the general path on the same device tensors
        try:
            gen = fh.transform(tab)[0].column("o")
        finally:
            text.FH_ROWS_MAX_COLS = saved
        assert torch.equal(gen.indptr.cpu(), got.indptr.cpu()) and torch.equal(gen.indices.cpu(), got.indices.cpu())
        torch.testing.assert_close(gen.values.cpu(), got.values.cpu(), rtol=1e-12, atol=1e-12)
