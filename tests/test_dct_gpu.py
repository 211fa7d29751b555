"""K17: the f32-MFMA DCT kernel (ops/csrc/dct.hip) against the fp64 torch product with the same
orthonormal basis (the CPU path of models/feature/vector_ops.DCT, itself pinned to the reference's
DCT test values in tests/test_feature_vector_ops.py), for every n class: multiples of 4 (16-byte
path), odd n (scalar path), n = 1 and the 128 maximum; partial last tiles; forward and inverse."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("rows,n", [(1, 1), (63, 3), (64, 100), (1000, 100), (12_345, 100), (777, 37), (4096, 128),
                                    (129, 16), (5000, 64), (300, 127)])
@pytest.mark.parametrize("inverse", [False, True])
def test_dct_rows_matches_fp64(rows, n, inverse):
    _need_gpu()
    from flink_ml_amd.ops.dct import dct_matrix, dct_rows

    g = torch.Generator().manual_seed(rows * 131 + n)
    X = torch.rand((rows, n), generator=g, dtype=torch.float64) * 2 - 1
    M = dct_matrix(n)
    ref = X @ (M if inverse else M.t())
    got = dct_rows(X.float().cuda(), inverse).double().cpu()
    # exact-f32 MFMA: a k-ordered f32 fma chain over the f32-rounded inputs
    tol = 3e-7 * (X.abs() @ (M if inverse else M.t()).abs()) + 1e-7
    assert bool(((got - ref).abs() <= tol).all()), float((got - ref).abs().max())


def test_dct_stage_on_device_roundtrip():
    _need_gpu()
    from flink_ml_amd import Table
    from flink_ml_amd.models import DCT

    g = torch.Generator().manual_seed(0)
    X = torch.rand((10_000, 100), generator=g, dtype=torch.float32).cuda()
    t = Table({"input": X}, num_rows=10_000)
    y = DCT().set_input_col("input").set_output_col("o").transform(t)[0].column("o")
    back = DCT().set_inverse(True).set_input_col("o").set_output_col("b").transform(
        Table({"o": y}, num_rows=10_000))[0].column("b")
    np.testing.assert_allclose(back.cpu().numpy(), X.cpu().numpy(), atol=2e-6)


@pytest.mark.parametrize("rows,n", [(1, 1), (63, 3), (1000, 100), (777, 37), (4096, 128), (300, 127)])
@pytest.mark.parametrize("inverse", [False, True])
def test_dct_rows_f64_matches_fp64_product(rows, n, inverse):
    """fp64 rows (parity mode, DCT.java computes in double) on the f64-MFMA kernel, not
    a library GEMM — against the fp64 torch product to fp64 rounding."""
    _need_gpu()
    from flink_ml_amd.ops.dct import dct_matrix, dct_rows

    g = torch.Generator().manual_seed(rows * 7 + n)
    X = torch.rand((rows, n), generator=g, dtype=torch.float64) * 2 - 1
    M = dct_matrix(n)
    ref = X @ (M if inverse else M.t())
    got = dct_rows(X.cuda(), inverse).cpu()
    assert got.dtype == torch.float64
    tol = 1e-15 * (X.abs() @ (M if inverse else M.t()).abs()) * n + 1e-16
    assert bool(((got - ref).abs() <= tol).all()), float((got - ref).abs().max())


def test_dct_stage_fp64_takes_the_kernel():
    _need_gpu()
    from flink_ml_amd import Table
    from flink_ml_amd.models import DCT
    from flink_ml_amd.ops import dct as dk

    calls = []
    real = dk.dct_rows
    dk.dct_rows = lambda X, inv=False: calls.append(X.dtype) or real(X, inv)
    try:
        X = torch.rand((500, 40), dtype=torch.float64).cuda()
        out = DCT().set_input_col("i").set_output_col("o").transform(Table({"i": X}, num_rows=500))[0].column("o")
    finally:
        dk.dct_rows = real
    assert calls == [torch.float64]
    ref = X.cpu() @ dk.dct_matrix(40).t()
    np.testing.assert_allclose(out.cpu().numpy(), ref.numpy(), atol=1e-13)
