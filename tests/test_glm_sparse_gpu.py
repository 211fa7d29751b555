"""Sparse SGD rounds through the per-batch transpose (glm.hip glm_csr_fwd_kernel +
glm_csc_bwd_kernel) vs the fp64 host trainer on the densified data, and vs the atomic scatter
kernel it replaces. Rows have 0..40 non-zeros (empty rows and empty columns included) and n is not
a multiple of the batch, so the truncated last batch and the wrap-around are exercised."""
import numpy as np
import pytest
import torch

from tests.spmd import run_spmd

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _csr(n, d, seed, max_nnz=40, dtype=torch.float64):
    g = torch.Generator(device="cpu").manual_seed(seed)
    counts = torch.randint(0, max_nnz + 1, (n,), generator=g)
    indptr = torch.zeros(n + 1, dtype=torch.int64)
    indptr[1:] = torch.cumsum(counts, 0)
    nnz = int(indptr[-1])
    idx = torch.empty(nnz, dtype=torch.int32)
    for r in range(n):  # distinct sorted columns per row
        c = int(counts[r])
        if c:
            idx[indptr[r]:indptr[r + 1]] = torch.sort(torch.randperm(d - 5, generator=g)[:c]).values.to(torch.int32)
    vals = (torch.rand(nnz, generator=g, dtype=torch.float64) * 2 - 1).to(dtype)
    dense = torch.zeros((n, d), dtype=torch.float64)
    rows = torch.repeat_interleave(torch.arange(n), counts)
    dense[rows, idx.long()] = vals.to(torch.float64)
    y = (dense @ torch.linspace(-1, 1, d, dtype=torch.float64) > 0).double()
    w = torch.rand(n, generator=g, dtype=torch.float64) + 0.5
    return indptr, idx, vals, dense, y, w


def _sparse_col(indptr, idx, vals, d, device):
    from flink_ml_amd.table import SparseColumn

    return SparseColumn(indptr.to(device), idx.to(device), vals.to(device), d)


def _use_path(monkeypatch, path):
    """'bucket': the single-visit round (glm_sparse.hip glm_bkt_*, the default for fits visiting
    each batch < TILE_MIN_VISITS times); 'csc': the transposed rounds."""
    from flink_ml_amd.ops import glm as gk

    monkeypatch.setattr(gk, "BUCKETS", path == "bucket")


def _check_path(tr, path):
    assert (tr.bkt is not None) == (path == "bucket") and (tr.csc is not None) == (path == "csc")


@pytest.mark.parametrize("path", ["bucket", "csc"])
@pytest.mark.parametrize("graph", [False, True])
def test_sparse_sgd_transpose_path_matches_host(graph, path, monkeypatch):
    _need_gpu()
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer, TorchGlmTrainer

    _use_path(monkeypatch, path)

    n, d = 2300, 700
    indptr, idx, vals, dense, y, w = _csr(n, d, 3)
    for loss in ("logistic", "hinge", "leastsquare"):
        for reg, en in ((0.0, 0.0), (0.1, 0.5)):
            sgd = SGD(max_iter=9, learning_rate=0.1, global_batch_size=500, tol=1e-9, reg=reg, elastic_net=en)
            ref = TorchGlmTrainer(sgd, np.zeros(d), dense, y, w, loss).fit()
            tr = DeviceGlmTrainer(sgd, np.zeros(d), _sparse_col(indptr, idx, vals, d, "cuda"), y.cuda(), w.cuda(),
                                  loss, use_graph=graph)
            _check_path(tr, path)
            got = tr.fit()
            assert tr.rounds_executed() == 9
            assert np.allclose(got, ref, atol=1e-10, rtol=1e-10), (loss, reg, en, np.abs(got - ref).max())


@pytest.mark.parametrize("path", ["bucket", "csc"])
@pytest.mark.parametrize("max_nnz", [40, 300])
def test_sparse_weighted_and_unweighted_rounds_match_host(max_nnz, path, monkeypatch):
    """Short rows and rows spanning several load steps of a lane group, weighted and unweighted
    (the backward takes Σweight from the row count when unweighted), with tol termination decided
    on the device from the loss the last arriving block sums."""
    _need_gpu()
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer, TorchGlmTrainer

    _use_path(monkeypatch, path)

    n, d = 1900, 900
    indptr, idx, vals, dense, y, w = _csr(n, d, 11 + max_nnz, max_nnz=max_nnz)
    for wt in (None, w):
        sgd = SGD(max_iter=8, learning_rate=0.1, global_batch_size=333, tol=1e-9, reg=0.05, elastic_net=0.5)
        ref = TorchGlmTrainer(sgd, np.zeros(d), dense, y, wt, "logistic").fit()
        tr = DeviceGlmTrainer(sgd, np.zeros(d), _sparse_col(indptr, idx, vals, d, "cuda"), y.cuda(),
                              None if wt is None else wt.cuda(), "logistic")
        _check_path(tr, path)
        got = tr.fit()
        assert tr.rounds_executed() == 8
        assert np.allclose(got, ref, atol=1e-10, rtol=1e-10), np.abs(got - ref).max()
    sgd2 = SGD(max_iter=200, learning_rate=1.0, global_batch_size=n, tol=0.3)
    r2 = TorchGlmTrainer(sgd2, np.zeros(d), dense, y, None, "logistic")
    c2 = r2.fit()
    t2 = DeviceGlmTrainer(sgd2, np.zeros(d), _sparse_col(indptr, idx, vals, d, "cuda"), y.cuda(), None, "logistic")
    g2 = t2.fit()
    assert t2.rounds_executed() == r2.rounds
    assert np.abs(g2 - c2).max() < 1e-8 * max(1.0, np.abs(c2).max())


def test_sparse_sgd_fp32_transpose_vs_atomic_and_termination(monkeypatch):
    _need_gpu()
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer, TorchGlmTrainer

    n, d = 5000, 3000
    indptr, idx, vals, dense, y, w = _csr(n, d, 8, dtype=torch.float32)
    sgd = SGD(max_iter=15, learning_rate=0.5, global_batch_size=1024, tol=1e-9)
    ref = TorchGlmTrainer(sgd, np.zeros(d), dense, y, None, "hinge").fit()
    X = _sparse_col(indptr, idx, vals, d, "cuda")
    bk = DeviceGlmTrainer(sgd, np.zeros(d), X, y.cuda(), None, "hinge")
    assert bk.bkt is not None and bk.csc is None
    got_b = bk.fit()
    from flink_ml_amd.ops import glm as gk

    monkeypatch.setattr(gk, "BUCKETS", False)
    a = DeviceGlmTrainer(sgd, np.zeros(d), X, y.cuda(), None, "hinge")
    assert a.csc is not None and a.csc.G in (4, 8, 16, 32, 64)
    got = a.fit()
    monkeypatch.setattr(gk, "TRANSPOSE", False)
    b = DeviceGlmTrainer(sgd, np.zeros(d), X, y.cuda(), None, "hinge")
    assert b.csc is None and b.bkt is None
    old = b.fit()
    scale = np.abs(ref).max()
    assert np.abs(got_b - ref).max() < 1e-5 * scale
    assert np.abs(got - ref).max() < 1e-5 * scale
    assert np.abs(old - ref).max() < 1e-5 * scale
    # tol-based termination is decided on the device from the round's loss sum
    monkeypatch.setattr(gk, "TRANSPOSE", True)
    monkeypatch.setattr(gk, "BUCKETS", True)
    sgd2 = SGD(max_iter=200, learning_rate=1.0, global_batch_size=5000, tol=0.3)
    r2 = TorchGlmTrainer(sgd2, np.zeros(d), dense, y, None, "logistic")
    c2 = r2.fit()
    t2 = DeviceGlmTrainer(sgd2, np.zeros(d), X, y.cuda(), None, "logistic")
    g2 = t2.fit()
    assert t2.rounds_executed() == r2.rounds
    assert np.abs(g2 - c2).max() < 1e-5 * max(1.0, np.abs(c2).max())


def _sparse_worker(rank, world, path):
    import numpy as np
    import torch

    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer, TorchGlmTrainer
    from flink_ml_amd.ops import glm as gk

    gk.BUCKETS = path == "bucket"
    gk.TILE_MIN_VISITS = 0 if path == "tiled" else 10 ** 6

    n, d = 1500 + 400 * rank, 300
    indptr, idx, vals, dense, y, w = _csr(n, d, 40 + rank)
    sgd = SGD(max_iter=7, learning_rate=0.1, global_batch_size=900, tol=1e-9, reg=0.05, elastic_net=0.3)
    ref = TorchGlmTrainer(sgd, np.zeros(d), dense, y, w, "hinge").fit()
    tr = DeviceGlmTrainer(sgd, np.zeros(d), _sparse_col(indptr, idx, vals, d, "cuda:0"), y.cuda(), w.cuda(), "hinge")
    if path == "bucket":
        assert tr.bkt is not None and tr.csc is None
    else:
        assert tr.csc is not None and (tr.csc.ET > 0) == (path == "tiled")
    got = tr.fit()
    return float(np.abs(got - ref).max()), got.tobytes()


@pytest.mark.parametrize("path", ["bucket", "untiled", "tiled"])
def test_sparse_sgd_two_ranks_one_gpu(path):
    """The feedback path (backward writes the gradient row for the all-reduce): bucket round,
    untiled and tiled transposed rounds."""
    _need_gpu()
    env = {"FMLX_DEVICE": "cuda:0", "FMLX_XGMI": "0"}
    res = run_spmd(_sparse_worker, 2, path, env=env, timeout=300)
    assert res[0][0] < 1e-10 and res[1][0] < 1e-10
    assert res[0][1] == res[1][1]  # replicas identical


@pytest.mark.parametrize("run_max,vdtype,d,B,skew,bucket", [
    (1, torch.float32, 3_001, 1_000, False, True), (3, torch.float64, 3_001, 1_000, False, True),
    (4, torch.float32, 3_001, 1_000, False, "unpacked"),   # the unpacked bucket pass
    (16, torch.float32, 3_001, 1_000, False, True),
    (16, torch.float32, 3_001, 1_000, False, False),      # two LSD passes + the column-pointer kernel
    (4, torch.float32, 700, 1_000, False, True),          # 10 column bits: one LSD pass
    (6, torch.float32, 1_000_000, 1_000, False, True),    # 20 column bits (the SVC shape's width)
    (5, torch.float32, 3_001, 4_000, True, True),         # buckets of > 8192 entries: chunked
])
def test_batch_csc_device_transpose_matches_host(run_max, vdtype, d, B, skew, bucket, monkeypatch):
    """Per-batch column-major copies built on the device (csc_build.hip keys → radix.hip: a stable
    pass on the high column bits + one block per (batch, 1024-column) bucket writing rows, values
    and column pointers; or LSD passes + the column-pointer kernel; runs of consecutive batches in
    one sort) equal the host construction exactly — also after the storage, first sized for the
    leading batches of a short fit, grows to the whole partition (pointers move: ``version``)."""
    _need_gpu()
    from flink_ml_amd.ops import glm as gk

    monkeypatch.setattr(gk, "CSC_TILE", 0)  # the plain column-major layout (tiles: test below)
    monkeypatch.setattr(gk, "CSC_RUN_MAX", run_max)
    monkeypatch.setattr(gk, "CSC_BUCKET", bool(bucket))
    monkeypatch.setattr(gk, "CSC_PACK", bucket != "unpacked")
    g = torch.Generator().manual_seed(0)
    n = 20_037
    lens = torch.randint(0, 12, (n,), generator=g)
    lens[3 * B:4 * B] = 0  # an empty batch
    indptr = torch.zeros(n + 1, dtype=torch.int64)
    indptr[1:] = torch.cumsum(lens, 0)
    rows = []
    for k in lens.tolist():
        if skew and torch.rand(1, generator=g).item() < 0.8:  # most rows inside the first 1024 columns
            rows.append(torch.sort(torch.randperm(1024, generator=g)[:k]).values)
        else:
            rows.append(torch.sort(torch.randint(0, d, (4 * k + 4,), generator=g).unique()[:k]).values)
    idx = torch.cat(rows).to(torch.int32)
    lens = torch.tensor([len(r) for r in rows])
    indptr[1:] = torch.cumsum(lens, 0)
    vals = torch.rand(int(indptr[-1]), generator=g, dtype=torch.float64).to(vdtype)
    dev = gk.BatchCsc.alloc(indptr.cuda(), idx.cuda(), vals.cuda(), n, d, B, max_rounds=5)
    dev.ensure([0, 1, 2, 3, 4])
    assert dev.cap == 5 and dev.version == 0 and dev.erow.numel() == int(indptr[5 * B])
    dev.ensure([0, 1, 2, 7, 8, 12, 19, 20, dev.P - 1])
    assert dev.cap == dev.P and dev.version == 1
    dev.ensure(range(dev.P))
    host = gk.BatchCsc.alloc(indptr, idx, vals, n, d, B)
    host.ensure(range(host.P))
    assert torch.equal(dev.colptr.cpu(), host.colptr)
    assert torch.equal(dev.erow.cpu(), host.erow)
    assert torch.equal(dev.evals.cpu(), host.evals)


def _untile(csc, b):
    """The plain column-major (erow, evals) of batch b rebuilt from its tiled layout, checking the
    tile invariants on the way."""
    d, rb, EL, ET = csc.d, csc.rb, csc.EL, csc.ET
    j0, j1 = csc.bounds[b], csc.bounds[b + 1]
    cp = csc.colptr[b].cpu().numpy()
    nt = int(csc.ntiles[b])
    tl = csc.tiles[b, :nt + 1, 0].cpu().numpy()
    assert np.array_equal(csc.tiles[b, :nt + 1, 1].cpu().numpy(), cp[tl])  # each tile's first entry
    er = csc.erow[j0:j1].cpu().numpy().astype(np.int64) & 0xFFFFFFFF
    ev = csc.evals[j0:j1].cpu().numpy()
    assert tl[0] == 0 and tl[nt] == d and np.all(np.diff(tl) > 0)
    rows = np.empty(j1 - j0, dtype=np.int64)
    vals = np.empty_like(ev)
    heavy = 0
    for t in range(nt):
        k0, k1 = cp[tl[t]], cp[tl[t + 1]]
        r = er[k0:k1] & ((1 << rb) - 1)
        assert np.all(np.diff(r) >= 0), "rows sorted inside a tile"
        if tl[t + 1] - tl[t] == 1 and k1 - k0 > EL:
            heavy += 1
            rows[k0:k1], vals[k0:k1] = r, ev[k0:k1]
            continue
        assert k1 - k0 <= ET
        pos = er[k0:k1] >> rb
        assert sorted(pos.tolist()) == list(range(k1 - k0))
        rows[k0 + pos], vals[k0 + pos] = r, ev[k0:k1]
    return rows, vals, heavy


@pytest.mark.parametrize("vdtype,tile,d,B", [
    (torch.float32, 64, 3_001, 1_000), (torch.float64, 64, 3_001, 1_000),
    (torch.float32, 1024, 1_000_000, 1_000), (torch.float32, -1, 3_001, 4_000),
])
def test_batch_csc_row_sorted_tiles(vdtype, tile, d, B, monkeypatch):
    """The tiled layout of the tiled backward (csc_build.hip csc_tiles / csc_tile_keys / sort /
    csc_tile_store): tiles cover the columns, light tiles hold ≤ ET entries row-sorted with a
    permutation of their column-ordered slots, one column of > EL entries is its own (heavy) tile,
    and undoing the permutation gives the plain layout exactly."""
    _need_gpu()
    from flink_ml_amd.ops import glm as gk

    g = torch.Generator().manual_seed(1)
    n = 9_013
    lens = torch.randint(0, 12, (n,), generator=g)
    rows = []
    for k in lens.tolist():
        r = torch.randint(1, d, (4 * k + 4,), generator=g).unique()[:k]
        if torch.rand(1, generator=g).item() < 0.7:
            r = torch.cat([torch.zeros(1, dtype=r.dtype), r])  # column 0 in most rows: heavy
        rows.append(torch.sort(r).values)
    idx = torch.cat(rows).to(torch.int32)
    indptr = torch.zeros(n + 1, dtype=torch.int64)
    indptr[1:] = torch.cumsum(torch.tensor([len(r) for r in rows]), 0)
    vals = torch.rand(int(indptr[-1]), generator=g, dtype=torch.float64).to(vdtype)
    monkeypatch.setattr(gk, "CSC_TILE", 0)
    plain = gk.BatchCsc.build(indptr.cuda(), idx.cuda(), vals.cuda(), n, d, B)
    monkeypatch.setattr(gk, "CSC_TILE", tile)
    monkeypatch.setattr(gk, "TILE_MIN_VISITS", 0)
    csc = gk.BatchCsc.alloc(indptr.cuda(), idx.cuda(), vals.cuda(), n, d, B, max_rounds=3)
    assert csc.ET == (tile if tile > 0 else (16384 if vdtype == torch.float64 else 32768))
    csc.ensure([0, 1, 2])
    csc.ensure(range(csc.P))  # storage growth copies the built tiles
    heavy = 0
    for b in range(csc.P):
        j0, j1 = csc.bounds[b], csc.bounds[b + 1]
        r, v, h = _untile(csc, b)
        heavy += h
        assert np.array_equal(r, plain.erow[j0:j1].cpu().numpy()), b
        assert np.array_equal(v, plain.evals[j0:j1].cpu().numpy()), b
    assert torch.equal(csc.colptr.cpu(), plain.colptr.cpu())
    if tile == 64:
        assert heavy >= csc.P - 1  # column 0 in every full batch (the last holds 13 rows)


@pytest.mark.parametrize("vdtype,d,B,S,rbb", [
    (torch.float32, 3_001, 1_000, 8, 11), (torch.float64, 3_001, 5_000, 8, 11),  # 3 row blocks (last partial)
    (torch.float32, 1_000_000, 4_500, 8, 11), (torch.float32, 5, 2_100, 8, 11),  # wide; fewer columns than S
    (torch.float32, 3_001, 5_000, 1, 11), (torch.float32, 3_001, 5_000, 5, 10),
])
def test_batch_csr_forward_cells(vdtype, d, B, S, rbb, monkeypatch):
    """The forward's cell layout (csc_build.hip cell_keys / sorts / cell_bounds / cell_rekey /
    cell_store): every batch's entries as row-block × column-split cells, each cell's entries
    column-sorted (rows ascending within a column), packed (column − s·CS) | row-major rank << cb,
    with per-(cell, row) offsets — the same (row, column, value) set as the CSR batch, also after
    storage growth; ``cmax`` is the largest cell."""
    _need_gpu()
    from flink_ml_amd.ops import glm as gk

    monkeypatch.setattr(gk, "TILE_MIN_VISITS", 0)
    monkeypatch.setattr(gk, "CELLS", True)
    monkeypatch.setattr(gk, "CELL_SPLITS", S)
    monkeypatch.setattr(gk, "CELL_RBB", rbb)
    g = torch.Generator().manual_seed(5)
    n = 12_345
    lens = torch.randint(0, 12, (n,), generator=g)
    lens[B:2 * B] = 0  # an empty batch
    # rows with unsorted column lists too (CSR order inside a row is kept, not assumed sorted)
    rows = [torch.randint(0, d, (4 * k + 4,), generator=g).unique()[:k] for k in lens.tolist()]
    rows = [r[torch.randperm(len(r), generator=g)] if i % 3 == 0 else r for i, r in enumerate(rows)]
    idx = torch.cat(rows).to(torch.int32)
    indptr = torch.zeros(n + 1, dtype=torch.int64)
    indptr[1:] = torch.cumsum(torch.tensor([len(r) for r in rows]), 0)
    vals = torch.rand(int(indptr[-1]), generator=g, dtype=torch.float64).to(vdtype)
    csc = gk.BatchCsc.alloc(indptr.cuda(), idx.cuda(), vals.cuda(), n, d, B, max_rounds=2)
    if gk.DETERMINISTIC:
        assert csc.cells == 0
        return
    S_ = min(S, d)
    RB = 1 << rbb
    assert csc.cells == -(-min(B, n) // RB) * S_ and csc.S == S_ and csc.rbb == rbb
    csc.ensure([0, 1])
    csc.ensure(range(csc.P))
    ent = csc.cent.cpu().numpy().astype(np.int64) & 0xFFFFFFFF
    cv = csc.cval.cpu().numpy()
    roff = csc.roff.cpu().numpy().astype(np.int64)
    ip = indptr.numpy()
    big = 0
    for b in range(csc.P):
        r0, r1 = b * B, min(n, (b + 1) * B)
        j0, j1 = int(ip[r0]), int(ip[r1])
        nrb = -(-(r1 - r0) // RB)
        o = roff[b]
        assert o[0] == 0 and np.all(np.diff(o) >= 0) and np.all(o[nrb * S_ * RB:] == j1 - j0)
        got = []
        for c in range(nrb * S_):
            rb, sp = divmod(c, S_)
            k0, k1 = o[c * RB], o[(c + 1) * RB]
            big = max(big, k1 - k0)
            x = ent[j0 + k0:j0 + k1]
            col = sp * csc.CS + (x & ((1 << csc.cb) - 1))
            pos = x >> csc.cb
            assert sorted(pos.tolist()) == list(range(k1 - k0)), "row-major ranks: a permutation"
            assert np.all(np.diff(col * (1 << 32) + pos) > 0), "column-sorted, rows ascending inside a column"
            rowof = np.repeat(np.arange(RB), np.diff(o[c * RB:(c + 1) * RB + 1]))  # row of each rank
            row = rb * RB + rowof[pos]
            assert np.all(col < min(d, (sp + 1) * csc.CS)) and np.all(row < r1 - r0)
            got += list(zip(row.tolist(), col.tolist(), cv[j0 + k0:j0 + k1].tolist()))
        rr = np.repeat(np.arange(r1 - r0), np.diff(ip[r0:r1 + 1]))
        want = list(zip(rr.tolist(), idx[j0:j1].tolist(), vals[j0:j1].numpy().tolist()))
        assert sorted(got) == sorted(want), b
    assert csc.cmax == big


@pytest.mark.parametrize("tile", [0, 64, 2048])
@pytest.mark.parametrize("vdtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("cells", [False, True, 5])
def test_sparse_sgd_tiled_backward_matches_host(tile, vdtype, cells, monkeypatch):
    """Whole fits through the tiled backward (light and heavy tiles; the feedback path is the
    two-rank test above) and the cell forward or the row-group forward, against the fp64 host
    trainer, weighted and not."""
    _need_gpu()
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer, TorchGlmTrainer

    n, d = 5100, 800  # 2000-row batches in 1024-row blocks: partial last blocks, a 1100-row batch
    indptr, idx, vals, dense, y, w = _csr(n, d, 21, max_nnz=60, dtype=vdtype)
    from flink_ml_amd.ops import glm as gk

    monkeypatch.setattr(gk, "CSC_TILE", tile)
    monkeypatch.setattr(gk, "TILE_MIN_VISITS", 0)
    monkeypatch.setattr(gk, "CELLS", bool(cells))
    if cells is not True and cells:
        monkeypatch.setattr(gk, "CELL_SPLITS", cells)  # 2 row blocks × 5: a grid of 10 (uneven per XCD)
    from flink_ml_amd.ops import native

    # cells in the default XCD-aware block order, and (odd grid) in launch order
    for wt, xcd in ((None, 1), (w, 1)) + (((w, 0),) if cells is not True and cells else ()):
        sgd = SGD(max_iter=9, learning_rate=0.2, global_batch_size=2000, tol=1e-9, reg=0.05, elastic_net=0.4)
        ref = TorchGlmTrainer(sgd, np.zeros(d), dense, y, wt, "hinge").fit()
        tr = DeviceGlmTrainer(sgd, np.zeros(d), _sparse_col(indptr, idx, vals, d, "cuda"), y.cuda(),
                              None if wt is None else wt.cuda(), "hinge")
        assert tr.csc is not None and tr.csc.ET == tile
        assert (tr.csc.cells > 0) == (cells and not gk.DETERMINISTIC)
        native.kernels().fmlx_glm_set_cell_xcd(xcd)
        try:
            got = tr.fit()
        finally:
            native.kernels().fmlx_glm_set_cell_xcd(1)
        tol = 1e-10 if vdtype == torch.float64 else 1e-5
        assert np.abs(got - ref).max() <= tol * max(1.0, np.abs(ref).max()), (tile, xcd, np.abs(got - ref).max())


def _tol_stop_worker(rank, world, check_every):
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer

    n, d = 6000, 400
    indptr, idx, vals, dense, y, w = _csr(n, d, 40 + rank, max_nnz=30, dtype=torch.float32)
    # tol far above any hinge loss: the iteration stops after its first round, so every launched
    # round after it is predicated off on the device — but each still issues its host all-reduce,
    # which only matches its peer's if both ranks break after the same number of launched rounds
    sgd = SGD(max_iter=60, learning_rate=0.2, global_batch_size=2000, tol=1e9)
    tr = DeviceGlmTrainer(sgd, np.zeros(d), _sparse_col(indptr, idx, vals, d, "cuda"), y.cuda(), None, "hinge",
                          check_every=check_every)
    coef = tr.fit()
    return coef, tr.rounds_executed(), tr._launched


@pytest.mark.parametrize("check_every", [1, 3])
def test_two_rank_sparse_fit_stops_on_tol_in_lockstep(check_every):
    """the polled termination check must make every rank break after the same
    launched round; a rank seeing the stop one interval earlier left its peer's all-reduces
    unmatched. Two gloo ranks on one GPU, host all-reduce per round (TAIL_FEEDBACK)."""
    _need_gpu()
    env = {"FMLX_DEVICE": "cuda:0", "FMLX_XGMI": "0"}
    res = run_spmd(_tol_stop_worker, 2, check_every, env=env, timeout=300)
    (c0, r0, l0), (c1, r1, l1) = res
    assert r0 == r1 == 1
    assert l0 == l1 < 60
    assert np.array_equal(c0, c1)



@pytest.mark.parametrize("vdtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("chunk", [32768, 1024])
def test_bucket_round_skew_pieces_and_chunks_match_host(vdtype, chunk, monkeypatch):
    """The single-visit bucket round on awkward inputs: most entries in the first column slice
    (a bucket summed in several chunks through the accumulator: chunk = 1024), rows of up to 300
    entries (a forward block's entries staged in several LDS pieces), empty rows, a truncated
    last batch, weighted and not, with elastic net — against the fp64 host trainer."""
    _need_gpu()
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer, TorchGlmTrainer
    from flink_ml_amd.ops import glm as gk

    monkeypatch.setattr(gk.BucketRound, "CHUNK", chunk)
    n, d = 5100, 3000
    g = torch.Generator().manual_seed(5)
    counts = torch.randint(0, 301, (n,), generator=g)
    counts[100:140] = 0
    indptr = torch.zeros(n + 1, dtype=torch.int64)
    indptr[1:] = torch.cumsum(counts, 0)
    rows = []
    for c in counts.tolist():
        hot = torch.randperm(64, generator=g)[: c // 2]  # half of every row in columns 0..63
        cold = 64 + torch.randperm(d - 64, generator=g)[: c - len(hot)]
        rows.append(torch.sort(torch.cat([hot, cold])).values)
    idx = torch.cat(rows).to(torch.int32)
    vals = (torch.rand(len(idx), generator=g, dtype=torch.float64) * 2 - 1).to(vdtype)
    dense = torch.zeros((n, d), dtype=torch.float64)
    dense[torch.repeat_interleave(torch.arange(n), counts), idx.long()] = vals.double()
    y = (dense @ torch.linspace(-1, 1, d, dtype=torch.float64) > 0).double()
    w = torch.rand(n, generator=g, dtype=torch.float64) + 0.5
    for wt in (None, w):
        sgd = SGD(max_iter=7, learning_rate=0.3, global_batch_size=2000, tol=1e-12, reg=0.02, elastic_net=0.3)
        ref = TorchGlmTrainer(sgd, np.zeros(d), dense, y, wt, "hinge").fit()
        tr = DeviceGlmTrainer(sgd, np.zeros(d), _sparse_col(indptr, idx, vals, d, "cuda"), y.cuda(),
                              None if wt is None else wt.cuda(), "hinge")
        assert tr.bkt is not None and tr.bkt.nb > 1
        got = tr.fit()
        assert tr.rounds_executed() == 7
        tol = 1e-10 if vdtype == torch.float64 else 2e-5
        assert np.abs(got - ref).max() <= tol * max(1.0, np.abs(ref).max()), np.abs(got - ref).max()
