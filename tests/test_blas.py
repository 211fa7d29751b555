"""Device BLAS (ops/blas.py, csrc/blas.hip) against fp64 torch references of the reference's
BLAS.java semantics (flink-ml-core/.../linalg/BLAS.java:30-204): dense rows in bf16 / fp32 /
fp64 and CSR rows, on CPU (torch path) and on the GPU (HIP kernels)."""
import math

import numpy as np
import pytest
import torch

from flink_ml_amd.ops import blas
from flink_ml_amd.table import SparseColumn

DEVS = ["cpu"] + (["cuda"] if torch.cuda.is_available() else [])


def _dense(n, d, seed, dtype=torch.float64):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(n, d, generator=g, dtype=torch.float64)).to(dtype)


def _csr(n, d, nnz, seed):
    g = np.random.default_rng(seed)
    indptr = [0]
    idx, val = [], []
    for _ in range(n):
        k = int(g.integers(0, nnz + 1))
        cols = np.sort(g.choice(d, size=k, replace=False))
        idx.extend(cols.tolist())
        val.extend(g.normal(size=k).tolist())
        indptr.append(len(idx))
    return SparseColumn(torch.tensor(indptr), torch.tensor(idx, dtype=torch.int32), torch.tensor(val, dtype=torch.float64), d)


def _tol(dtype):
    return {torch.float64: 1e-12, torch.float32: 1e-5, torch.bfloat16: 1e-5}[dtype]


def _to(x, dev):
    if isinstance(x, SparseColumn):
        return SparseColumn(x.indptr.to(dev), x.indices.to(dev), x.values.to(dev), x.size)
    return x.to(dev)


def _mark(dev):
    return [pytest.mark.gpu] if dev == "cuda" else []


CASES = [pytest.param(dev, dt, d, marks=_mark(dev)) for dev in ["cpu", "cuda"]
         for dt in (torch.float64, torch.float32, torch.bfloat16) for d in (3, 17, 100, 1000)]


def _need(dev):
    if dev == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("dev,dtype,d", CASES)
def test_dense_reductions_and_gemv(dev, dtype, d):
    _need(dev)
    X, Y = _dense(513, d, d, dtype), _dense(513, d, d + 1, dtype)
    v = torch.randn(d, dtype=torch.float64)
    Xr, Yr = X.double(), Y.double()
    tol = _tol(dtype) * max(1, d)
    for p in (1.0, 2.0, 3.5, math.inf):
        got = blas.row_norm(_to(X, dev), p).double().cpu()
        assert torch.allclose(got, torch.linalg.vector_norm(Xr, ord=p, dim=1), rtol=tol, atol=tol), p
    assert torch.allclose(blas.row_dot(_to(X, dev), _to(Y, dev)).double().cpu(), (Xr * Yr).sum(1), rtol=tol, atol=tol)
    # gemv: the vector is rounded to the rows' dtype on the device (like the rows themselves)
    vr = v.to(dtype).double() if dev == "cuda" else v
    assert torch.allclose(blas.gemv(_to(X, dev), v).double().cpu(), Xr @ vr, rtol=tol, atol=tol)
    m = torch.randn(513, dtype=torch.float64)
    assert torch.allclose(blas.gemv_t(_to(X, dev), m).cpu(), Xr.t() @ m, rtol=tol, atol=tol)


@pytest.mark.parametrize("dev,dtype,d", CASES)
def test_dense_elementwise(dev, dtype, d):
    _need(dev)
    X = _dense(300, d, 7, dtype)
    v = torch.randn(d, dtype=torch.float64)
    tol = max(_tol(dtype), 1e-6 if dtype == torch.float32 else 0)
    Xr = X.double()
    for p in (1.0, 2.0, 3.0, math.inf):
        got = blas.normalize(_to(X, dev), p).double().cpu()
        ref = Xr / torch.linalg.vector_norm(Xr, ord=p, dim=1)[:, None]
        assert torch.allclose(got, ref, rtol=tol * 10, atol=tol * 10), p
    assert torch.allclose(blas.hdot(v, _to(X, dev)).double().cpu(), Xr * v[None, :], rtol=tol, atol=tol)
    if dtype != torch.bfloat16:
        Y = _dense(300, d, 8, dtype)
        a = torch.randn(300, dtype=torch.float64)
        Yd = _to(Y.clone(), dev)
        blas.axpby(a.to(dtype) if dtype == torch.float32 else a, _to(X, dev), 0.5, Yd)
        ar = a.to(dtype).double() if dtype == torch.float32 else a
        assert torch.allclose(Yd.double().cpu(), ar[:, None] * Xr + 0.5 * Y.double(), rtol=tol, atol=tol)
        Z = _to(Y.clone(), dev)
        blas.scal(2.0, Z)
        assert torch.allclose(Z.double().cpu(), 2.0 * Y.double(), rtol=tol, atol=tol)
    cols = [d - 1, 0, d // 2]
    assert torch.equal(blas.gather_cols(_to(X, dev), cols).cpu(), X[:, cols])


@pytest.mark.parametrize("dev", [pytest.param(d, marks=_mark(d)) for d in ["cpu", "cuda"]])
def test_csr_ops(dev):
    _need(dev)
    X, Y = _csr(400, 1000, 30, 1), _csr(400, 1000, 30, 2)
    Xd, Yd = X.to_dense(torch.float64), Y.to_dense(torch.float64)
    v = torch.randn(1000, dtype=torch.float64)
    Xg, Yg = _to(X, dev), _to(Y, dev)
    for p in (1.0, 2.0, 2.5, math.inf):
        assert torch.allclose(blas.row_norm(Xg, p).cpu().double(), torch.linalg.vector_norm(Xd, ord=p, dim=1),
                              rtol=1e-12, atol=1e-12), p
    assert torch.allclose(blas.gemv(Xg, v).cpu().double(), Xd @ v, rtol=1e-12, atol=1e-12)
    assert torch.allclose(blas.row_dot(Xg, Yg).cpu().double(), (Xd * Yd).sum(1), rtol=1e-12, atol=1e-12)
    h = blas.hdot(v, Xg)
    assert torch.allclose(_to(h, "cpu").to_dense(torch.float64), Xd * v[None, :], rtol=1e-12, atol=1e-12)
    nrm = blas.normalize(Xg, 2.0)
    ref = Xd / torch.linalg.vector_norm(Xd, dim=1)[:, None]
    got = _to(nrm, "cpu").to_dense(torch.float64)
    ok = torch.isfinite(ref).all(1)  # empty rows divide 0 by 0 (NaN-free: no stored values)
    assert torch.allclose(got[ok], ref[ok], rtol=1e-12, atol=1e-12)
    Yacc = torch.zeros(400, 1000, dtype=torch.float64, device=dev)
    blas.csr_axpy_dense(2.0, Xg, Yacc, k=500)
    ref = 2.0 * Xd
    ref[:, 500:] = 0
    assert torch.allclose(Yacc.cpu(), ref, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("dev", [pytest.param(d, marks=_mark(d)) for d in ["cpu", "cuda"]])
def test_interaction(dev):
    _need(dev)
    a, b, c = _dense(50, 3, 1), _dense(50, 4, 2), _dense(50, 1, 3)
    got = blas.interaction([_to(a, dev), _to(b, dev), _to(c, dev)]).cpu()
    ref = (a[:, :, None, None] * b[:, None, :, None] * c[:, None, None, :]).reshape(50, -1)
    assert torch.allclose(got, ref, rtol=1e-14, atol=1e-14)


def test_invalid_p_rejected():
    with pytest.raises(ValueError):
        blas.row_norm(torch.ones(2, 2), 0.5)


@pytest.mark.parametrize("dev", [pytest.param(d, marks=_mark(d)) for d in ["cpu", "cuda"]])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_gather_prod_polynomial_terms(dev, dtype):
    _need(dev)
    from flink_ml_amd.models.feature.vector_ops import _poly_terms

    X = _dense(300, 5, 4).to(dtype)
    terms = torch.as_tensor(_poly_terms(5, 3))
    got = blas.gather_prod(_to(X, dev), terms).cpu()
    Xp = torch.cat([X.double(), torch.ones(300, 1, dtype=torch.float64)], 1)
    ref = Xp[:, terms.long()].prod(2)
    assert got.dtype == dtype and got.shape == ref.shape
    assert torch.allclose(got.double(), ref, rtol=_tol(dtype), atol=_tol(dtype))


@pytest.mark.gpu
def test_sync_check_mode_runs_kernels(monkeypatch):
    """FMLX_SYNC_CHECK: every native launch is followed by a device sync (faults are attributed to
    the launching kernel); results are unchanged."""
    _need("cuda")
    from flink_ml_amd.ops import native

    monkeypatch.setattr(native, "SYNC_CHECK", True)
    X = _dense(64, 7, 9).cuda()
    assert torch.allclose(blas.row_norm(X, 2.0).cpu(), torch.linalg.vector_norm(X.cpu(), dim=1), rtol=1e-12)
