"""GPU numerics of the feature kernels (colstats.hip, hash.hip) against fp64 torch references, and
device-resident fit/transform of the scalers/encoders matching the CPU results."""
import numpy as np
import pytest
import torch

from flink_ml_amd import Table, Vectors

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.bfloat16])
@pytest.mark.parametrize("shape", [(1, 3), (1000, 37), (70000, 300)])
def test_colstats_kernel(dtype, shape):
    from flink_ml_amd.ops import features as fo

    g = torch.Generator().manual_seed(3)
    X = (torch.randn(shape, generator=g, dtype=torch.float64) * 3 + 1).to(dtype).cuda()
    st = fo.column_stats(X)
    Xd = X.double()
    tol = dict(rtol=1e-9, atol=1e-6)
    torch.testing.assert_close(st["sum"], Xd.sum(0), **tol)
    torch.testing.assert_close(st["sumsq"], (Xd * Xd).sum(0), **tol)
    torch.testing.assert_close(st["min"], Xd.min(0).values, rtol=0, atol=0)
    torch.testing.assert_close(st["max"], Xd.max(0).values, rtol=0, atol=0)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_affine_kernel(dtype):
    from flink_ml_amd.ops import features as fo

    X = torch.randn(5000, 129, dtype=torch.float64).to(dtype).cuda()
    sub = torch.randn(129, dtype=torch.float64).cuda()
    mul = torch.rand(129, dtype=torch.float64).cuda()
    add = torch.randn(129, dtype=torch.float64).cuda()
    out = fo.affine_cols(X, sub, mul, add)
    ref = (X.double() - sub) * mul + add
    torch.testing.assert_close(out.double(), ref, rtol=1e-6, atol=1e-5)
    out2 = fo.affine_cols(X, None, mul, None)
    torch.testing.assert_close(out2.double(), X.double() * mul, rtol=1e-6, atol=1e-5)


def test_murmur3_device_matches_host():
    from flink_ml_amd.ops import hashing

    words = ["HashingTFTest", "Hashing", "Term", "Frequency", "Test", "", "ünïcødé", "a" * 37] * 50
    for mode, mod in ((0, 262144), (1, 1000)):
        dev = hashing.hash_strings_device(words, mod, mode, torch.device("cuda")).cpu().numpy()
        h = hashing.hash_strings(words)
        host = hashing.non_negative_mod(h, mod) if mode == 0 else np.fmod(np.abs(h.astype(np.int64)), mod)
        np.testing.assert_array_equal(dev, host)


def test_scalers_on_device_match_cpu():
    from flink_ml_amd.models import KBinsDiscretizer, MinMaxScaler, StandardScaler

    rng = np.random.default_rng(0)
    X = rng.normal(size=(4096, 16))
    tc = Table({"input": torch.from_numpy(X)}, num_rows=4096)
    tg = Table({"input": torch.from_numpy(X).cuda()}, num_rows=4096)
    for est in (StandardScaler().set_with_mean(True), MinMaxScaler()):
        oc = est.fit(tc).transform(tc)[0].column("output")
        og = est.fit(tg).transform(tg)[0].column("output")
        assert og.is_cuda
        torch.testing.assert_close(og.double().cpu(), oc.double().cpu(), rtol=1e-5, atol=1e-5)
    kb = KBinsDiscretizer().set_strategy("uniform").set_num_bins(7)
    bc = kb.fit(tc).transform(tc)[0].column("output")
    bg = kb.fit(tg).transform(tg)[0].column("output")
    assert torch.equal(bg.cpu(), bc.cpu())


def test_hashing_tf_device():
    from flink_ml_amd.models import HashingTF

    t = Table.from_rows([(["HashingTFTest", "Hashing", "Term", "Frequency", "Test"],)] * 3000, ["input"])
    out = HashingTF().transform(t)[0].get_list("output")
    assert out[0] == Vectors.sparse(262144, [67564, 89917, 113827, 131486, 228971], [1.0] * 5)


@pytest.mark.parametrize("binary", [False, True])
def test_hashing_tf_rows_kernel_matches_general_path(binary):
    """The per-document device count (csrc/hash.hip tf_rows_kernel) against the general
    sort-unique path: repeated terms, empty documents, colliding buckets (small numFeatures),
    and a document longer than TF_ROWS_MAX_LEN (the whole column falls back)."""
    from flink_ml_amd.models import HashingTF
    from flink_ml_amd.models.feature import text

    rng = np.random.default_rng(5)
    vocab = ["w%d" % i for i in range(40)] + ["ünï", ""]
    docs = [[vocab[j] for j in rng.integers(0, len(vocab), rng.integers(0, 20))] for _ in range(3000)]
    for extra in ([], [["w1"] * 40]):
        t = Table.from_rows([(d,) for d in docs + extra], ["input"])
        for nf in (7, 262144):
            tf = HashingTF().set_num_features(nf).set_binary(binary)
            got = tf.transform(t)[0].column("output")
            saved = text.TF_ROWS_MAX_LEN
            text.TF_ROWS_MAX_LEN = 0
            try:
                ref = tf.transform(t)[0].column("output")
            finally:
                text.TF_ROWS_MAX_LEN = saved
            assert torch.equal(got.indptr.cpu(), ref.indptr.cpu())
            assert torch.equal(got.indices.cpu().long(), ref.indices.cpu().long())
            assert torch.equal(got.values.cpu(), ref.values.cpu())


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.bfloat16])
@pytest.mark.parametrize("shape,G", [((100000, 100), 10), ((3000, 300), 1), ((777, 5), 32)])
def test_group_colstats_kernel(dtype, shape, G):
    from flink_ml_amd.ops import features as fo

    g = torch.Generator().manual_seed(1)
    X = torch.randn(shape, generator=g, dtype=torch.float64).to(dtype)
    gi = torch.randint(0, G, (shape[0],), generator=g)
    w = torch.randn(shape[0], generator=g, dtype=torch.float64)
    S, s, q = fo.group_colstats(X.cuda(), gi.cuda(), G, w.cuda())
    Xd = X.double()
    ref = torch.zeros(G, shape[1], dtype=torch.float64).index_add_(0, gi, Xd * w[:, None])
    torch.testing.assert_close(S.cpu(), ref, rtol=1e-9, atol=1e-8)
    torch.testing.assert_close(s.cpu(), Xd.sum(0), rtol=1e-9, atol=1e-8)
    torch.testing.assert_close(q.cpu(), (Xd * Xd).sum(0), rtol=1e-9, atol=1e-8)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_radix_select_gpu(dtype):
    from flink_ml_amd.ops.quantile import kth_smallest

    X = (torch.randn(200000, 6, dtype=torch.float64) * 100).to(dtype)
    X[::7, 2] = float("nan")
    k = torch.tensor([1, 1000, 100000, 150000, 199999, 200000])
    k[2] = 100
    got = kth_smallest(X.cuda(), k.cuda()).cpu()
    for j in range(6):
        col = X[:, j][~torch.isnan(X[:, j])]
        kj = min(int(k[j]), col.numel())
        assert got[j] == torch.sort(col).values[kj - 1]


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("d", [3, 37])
def test_radix_hist_kernel_multi_quantile(dtype, d):
    from flink_ml_amd.ops.quantile import column_quantiles, kth_smallest_device

    g = torch.Generator().manual_seed(d)
    X = (torch.randn(100003, d, generator=g, dtype=torch.float64) * 50).to(dtype)
    X[::5, 0] = float("nan")
    X[:, -1] = torch.round(X[:, -1] / 20)  # many duplicates
    X[:1000, 1] = -0.0
    n_valid = (~torch.isnan(X)).sum(0)
    ks = torch.stack([torch.ones(d, dtype=torch.int64), n_valid // 3, n_valid // 2 + 1, n_valid])
    got = kth_smallest_device(X.cuda(), ks.cuda()).cpu()
    for j in range(d):
        col = torch.sort(X[:, j][~torch.isnan(X[:, j])]).values
        for q in range(4):
            assert got[q, j] == col[int(ks[q, j]) - 1], (q, j)
    # through the public entry point (device path) vs the host radix select
    ps = [0.25, 0.5, 0.75]
    dev = column_quantiles(X.cuda(), ps, 0.001).cpu()
    host = column_quantiles(X, ps, 0.001)
    assert torch.equal(dev, host)
    Xn = X.clone()
    Xn[:, 0] = float("nan")  # (the counts come from the select's first histogram on the device)
    with pytest.raises(RuntimeError, match="without any records"):
        column_quantiles(Xn.cuda(), ps, 0.001)


@pytest.mark.parametrize("handle", ["keep", "skip", "error"])
def test_bucketizer_kernel_matches_cpu(handle):
    """csrc/colstats.hip bucketize_kernel against the CPU searchsorted path: exact hits on every
    split (the last one maps to the last bucket), NaN and out-of-range values, infinite splits,
    and a split array too long for the LDS copy."""
    from flink_ml_amd.models import Bucketizer

    rng = np.random.default_rng(2)
    long_sp = np.sort(rng.normal(size=5000)).tolist()
    sp = [[-0.5, 0.0, 0.5, 1.0], [float("-inf"), -1.0, 1.0, float("inf")], long_sp]
    cols = {}
    for i, s in enumerate(sp):
        v = rng.normal(size=20000)
        fin = [x for x in s if np.isfinite(x)]
        v[:len(fin)] = fin
        if handle == "error":  # every value inside the splits' range
            v = np.clip(v, s[0], s[-1])
        else:
            v[-7:] = [np.nan, -5.0, 5.0, -0.0, np.inf, -np.inf, 0.25]
        cols["c%d" % i] = v
    bz = Bucketizer().set_input_cols(*cols).set_output_cols(*["o%d" % i for i in range(3)]) \
        .set_splits_array(sp).set_handle_invalid(handle)
    ref = bz.transform(Table({k: torch.from_numpy(v) for k, v in cols.items()}, num_rows=20000))[0]
    got = bz.transform(Table({k: torch.from_numpy(v).cuda() for k, v in cols.items()}, num_rows=20000))[0]
    assert got.num_rows == ref.num_rows
    for i in range(3):
        assert got.column("o%d" % i).is_cuda
        assert torch.equal(got.column("o%d" % i).cpu(), ref.column("o%d" % i).cpu())
    if handle == "error":
        bad = Table({"c0": torch.tensor([0.1, float("nan")], dtype=torch.float64).cuda()}, num_rows=2)
        with pytest.raises(RuntimeError, match="invalid value"):
            Bucketizer().set_input_cols("c0").set_output_cols("o").set_splits_array([sp[0]]).transform(bad)


@pytest.mark.parametrize("missing", [float("nan"), -1.0])
def test_imputer_mean_kernel_matches_cpu(missing):
    """csrc/colstats.hip masked_sum_kernel (Imputer mean without a filtered copy) against the CPU
    path: NaNs and missingValue entries skipped, an all-missing column raises on both."""
    from flink_ml_amd.models import Imputer

    rng = np.random.default_rng(8)
    cols = {}
    for i in range(3):
        v = rng.normal(size=300_001) * (i + 1)
        v[rng.integers(0, v.size, 5000)] = np.nan
        v[rng.integers(0, v.size, 5000)] = -1.0
        cols["f%d" % i] = v
    imp = Imputer().set_input_cols(*cols).set_output_cols("a", "b", "c").set_missing_value(missing)
    ref = imp.fit(Table({k: torch.from_numpy(v) for k, v in cols.items()}, num_rows=300_001)).get_model_data()[0]
    got = imp.fit(Table({k: torch.from_numpy(v).cuda() for k, v in cols.items()}, num_rows=300_001)) \
        .get_model_data()[0]
    r, g = ref.get_list(ref.column_names[0])[0], got.get_list(got.column_names[0])[0]
    assert set(r) == set(g)
    for k in r:
        assert abs(r[k] - g[k]) <= 1e-12 * max(1.0, abs(r[k])), (k, r[k], g[k])


def test_count_vectorizer_tfdf_kernel():
    """csrc/hash.hip cv_tfdf_kernel against numpy per-term tf / df / first position, and the fitted
    vocabulary against the torch path (skewed term frequencies, empty and repeated-term
    documents, unused dictionary entries), with and without minDF / maxDF."""
    from flink_ml_amd.models import CountVectorizer
    from flink_ml_amd.models.feature import text
    from flink_ml_amd.table import StringArrayColumn

    rng = np.random.default_rng(6)
    V, nd = 300, 20000
    vocab = ["t%03d" % i for i in range(V)]
    lens = rng.integers(0, 40, nd)
    codes = np.minimum(rng.zipf(1.3, int(lens.sum())) - 1, V - 10).astype(np.int32)  # last 9 unused
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    col = StringArrayColumn(torch.from_numpy(off).cuda(), torch.from_numpy(codes).cuda(), vocab)
    from flink_ml_amd.utils.strtable import StrTable

    tab, sums, firsts = text._cv_counts_device(col, StrTable.from_strings(vocab), V, len(codes))
    tf = np.bincount(codes, minlength=V)
    df = np.zeros(V, dtype=np.int64)
    for d in range(nd):
        df[np.unique(codes[off[d]:off[d + 1]])] += 1
    first = np.full(V, len(codes))
    for p in range(len(codes) - 1, -1, -1):
        first[codes[p]] = p
    present = np.nonzero(tf)[0]
    present = present[np.argsort(first[present], kind="stable")]
    assert tab.take_strings(np.arange(len(tab))) == [vocab[i] for i in present]
    np.testing.assert_array_equal(sums[:, 0], tf[present])
    np.testing.assert_array_equal(sums[:, 1], df[present])
    np.testing.assert_array_equal(firsts, first[present])
    t = Table({"input": col}, num_rows=nd)
    for kw in ({}, {"min_df": 3.0, "max_df": 0.5}):
        cv = CountVectorizer().set_vocabulary_size(50)
        if kw:
            cv = cv.set_min_df(kw["min_df"]).set_max_df(kw["max_df"])
        got = cv.fit(t).get_model_data()[0].get_list("vocabulary")[0]
        saved = text.CV_TFDF_MAX_V
        text.CV_TFDF_MAX_V = 0
        try:
            ref = cv.fit(t).get_model_data()[0].get_list("vocabulary")[0]
        finally:
            text.CV_TFDF_MAX_V = saved
        assert list(got) == list(ref)


@pytest.mark.parametrize("n", [1, 2, 3])
def test_ngram_presence_kernels_match_sort_path(n):
    """csrc/hash.hip ngram_mark_kernel / ngram_emit_kernel against the sort-unique path on the same
    device column: rows shorter than n (no grams), empty rows, repeated grams."""
    from flink_ml_amd.models import NGram
    from flink_ml_amd.models.feature import text
    from flink_ml_amd.table import StringArrayColumn

    rng = np.random.default_rng(n)
    vocab = ["a", "bb", "c c", "ü", "e"]
    lens = rng.integers(0, 6, 5000)
    codes = rng.integers(0, len(vocab), int(lens.sum())).astype(np.int32)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    col = StringArrayColumn(torch.from_numpy(off).cuda(), torch.from_numpy(codes).cuda(), vocab)
    t = Table({"input": col}, num_rows=len(lens))
    ng = NGram().set_n(n)
    got = ng.transform(t)[0].column("output")
    saved = text.NGRAM_DENSE_MAX
    text.NGRAM_DENSE_MAX = 0
    try:
        ref = ng.transform(t)[0].column("output")
    finally:
        text.NGRAM_DENSE_MAX = saved
    assert list(got.vocab) == list(ref.vocab)
    assert torch.equal(got.offsets.cpu(), ref.offsets.cpu())
    assert torch.equal(got.codes.cpu().long(), ref.codes.cpu().long())
    assert [list(r) for r in got][:50] == [list(r) for r in ref][:50]


def test_bounded_distinct_counts_kernel():
    """csrc/catstats.hip small_distinct_kernel: exact counts up to cap (merged over many row
    chunks), cap + 1 beyond it (early exit), NaN one value and −0 == +0; VectorIndexer on the GPU
    picks the same categorical columns and maps as on the CPU."""
    from flink_ml_amd.models import VectorIndexer
    from flink_ml_amd.ops import catstats

    rng = np.random.default_rng(12)
    n, cap = 300_000, 20
    cols = [rng.integers(0, 5, n), rng.integers(0, cap, n), rng.integers(0, cap + 1, n), rng.normal(size=n),
            rng.integers(0, 3, n).astype(np.float64)]
    X = np.stack([np.asarray(c, dtype=np.float64) for c in cols], 1)
    X[::7, 4] = np.nan
    X[::5, 0] = -0.0  # -0 == +0 (0 is among the values)
    got = catstats.bounded_distinct_counts(torch.from_numpy(X).cuda(), cap)
    assert got.tolist() == [5, 20, 21, 21, 4]
    Xc = X[:, :3]
    t_cpu = Table({"input": torch.from_numpy(Xc)}, num_rows=n)
    t_gpu = Table({"input": torch.from_numpy(Xc).cuda()}, num_rows=n)
    vi = VectorIndexer().set_max_categories(cap)
    m_cpu = vi.fit(t_cpu).get_model_data()[0]
    m_gpu = vi.fit(t_gpu).get_model_data()[0]
    name = m_cpu.column_names[0]
    assert m_cpu.get_list(name) == m_gpu.get_list(name)


@pytest.mark.parametrize("order", ["arbitrary", "frequencyDesc", "alphabetAsc"])
def test_string_indexer_code_counts_kernel(order):
    """StringIndexer on a device dictionary column (counts and first positions from the one-pass
    code-count kernel over pseudo-documents) against the same strings as a host list column;
    unused dictionary entries, a column longer than one segment."""
    from flink_ml_amd.models import StringIndexer
    from flink_ml_amd.ops import catstats
    from flink_ml_amd.table import StringColumn

    rng = np.random.default_rng(4)
    vocab = ["s%02d" % i for i in range(60)]
    codes = np.minimum(rng.zipf(1.5, 50_000) - 1, 49).astype(np.int32)  # entries 50..59 unused
    cnt, first = catstats.code_counts_first(torch.from_numpy(codes).cuda(), len(vocab))
    np.testing.assert_array_equal(cnt, np.bincount(codes, minlength=len(vocab)))
    ref_first = np.full(len(vocab), len(codes))
    for p in range(len(codes) - 1, -1, -1):
        ref_first[codes[p]] = p
    np.testing.assert_array_equal(first, ref_first)
    si = StringIndexer().set_input_cols("s").set_output_cols("o").set_string_order_type(order)
    dev = si.fit(Table({"s": StringColumn(torch.from_numpy(codes).cuda(), vocab)}, num_rows=len(codes)))
    host = si.fit(Table({"s": [vocab[c] for c in codes]}, num_rows=len(codes)))
    a, b = dev.get_model_data()[0], host.get_model_data()[0]
    assert a.get_list(a.column_names[0]) == b.get_list(b.column_names[0])


@pytest.mark.parametrize("handle", ["skip", "error", "keep"])
def test_vector_assembler_device_nan_check(handle):
    """VectorAssembler on device columns: the NaN check through the masked-sum kernel (no NaN:
    nothing filtered) and the torch mask path when a NaN is present, as on the CPU."""
    from flink_ml_amd.models import VectorAssembler

    rng = np.random.default_rng(9)
    a, b = rng.normal(size=1000), rng.normal(size=(1000, 3))
    va = VectorAssembler().set_input_cols("a", "b").set_output_col("o").set_input_sizes(1, 3) \
        .set_handle_invalid(handle)
    for with_nan in (False, True):
        a2 = a.copy()
        if with_nan:
            a2[17] = np.nan
        tg = Table({"a": torch.from_numpy(a2).cuda(), "b": torch.from_numpy(b).cuda()}, num_rows=1000)
        tc = Table({"a": torch.from_numpy(a2), "b": torch.from_numpy(b)}, num_rows=1000)
        if with_nan and handle == "error":
            with pytest.raises(RuntimeError, match="NaN"):
                va.transform(tg)
            continue
        g, c = va.transform(tg)[0], va.transform(tc)[0]
        assert g.num_rows == c.num_rows == (999 if with_nan and handle == "skip" else 1000)
        torch.testing.assert_close(g.column("o").cpu(), c.column("o").cpu(), rtol=0, atol=0, equal_nan=True)
