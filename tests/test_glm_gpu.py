"""GPU numerics of the fused GLM kernels vs a plain PyTorch fp32/fp64 reference of the same op."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _ref_round(X, y, w, coef, B, e, loss):
    n = X.shape[0]
    P = (n + B - 1) // B
    s = (e % P) * B
    t = min(s + B, n)
    from flink_ml_amd.ops.glm import torch_loss_and_mult

    xb = X[s:t].to(torch.float64)
    dot = xb @ coef.to(torch.float64)
    l, m = torch_loss_and_mult(loss, dot, y[s:t].to(torch.float64), w[s:t].to(torch.float64))
    return m @ xb, w[s:t].sum().item(), l.sum().item()


def _register_resident_cases():
    """(dtype, d) pairs the register-resident round kernel takes; wider rows (e.g. d=1001 or fp32
    d=3000) train through the GEMV path, covered by test_device_sgd_wide_dense_gemv_path."""
    from flink_ml_amd.ops.glm import pick_layout

    return [(dt, d) for d in (4, 100, 1000, 1001, 3000) for dt in (torch.float32, torch.bfloat16, torch.float64)
            if pick_layout(torch.empty((2, d), dtype=dt)) is not None]


@pytest.mark.parametrize("dtype,d", _register_resident_cases())
@pytest.mark.parametrize("loss", [0, 1, 2])
def test_grad_partials_match_torch(dtype, d, loss):
    _need_gpu()
    from flink_ml_amd.ops import glm as gk

    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(d * 7 + loss)
    n = 5000
    X = torch.rand((n, d), generator=g).to(dtype).to(dev)
    y = torch.randint(0, 2, (n,), generator=g).to(torch.float64)
    w = torch.rand(n, generator=g).to(torch.float64) + 0.5
    acc = torch.float64 if dtype == torch.float64 else torch.float32
    coef = (torch.randn(d, generator=g) * 0.1).to(acc)
    lay = gk.pick_layout(X)
    if lay is None:
        pytest.skip("layout not supported")
    B = 1500
    nparts = max(1, min(512, -(-B // (gk.WPB * 16))))
    partials = torch.zeros((nparts, d + 2), dtype=acc, device=dev)
    for e in (0, 3):
        state = torch.tensor([e, 1, 1, 0, 0, 0, 0, 0], dtype=torch.int32, device=dev)
        gk.grad_partials(X, y.to(dev, acc), w.to(dev, acc), coef.to(dev), B, loss, state, partials, nparts)
        torch.cuda.synchronize()
        got = partials.sum(0).double().cpu()
        ref_g, ref_w, ref_l = _ref_round(X.cpu(), y, w, coef, B, e, loss)
        tol = 1e-9 if dtype == torch.float64 else 2e-4
        scale = max(1.0, ref_g.abs().max().item())
        assert torch.allclose(got[:d], ref_g, atol=tol * scale * 10, rtol=tol), (got[:d] - ref_g).abs().max()
        assert abs(got[d].item() - ref_w) <= tol * abs(ref_w) * 10
        assert abs(got[d + 1].item() - ref_l) <= 1e-3 * abs(ref_l) + 1e-6


def test_predict_matches_torch():
    _need_gpu()
    from flink_ml_amd.ops import glm as gk

    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(3)
    for dtype in (torch.float32, torch.bfloat16, torch.float64):
        X = torch.rand((3000, 257 if dtype != torch.bfloat16 else 256), generator=g).to(dtype)
        coef = torch.randn(X.shape[1], generator=g, dtype=torch.float64) * 0.1
        for mode in (0, 1, 2):
            pred, raw = gk.predict_dense(X.to(dev), coef, mode, 0.1)
            rp, rr = gk.dots_to_outputs(X.double() @ coef, mode, 0.1)
            dot_err = 1e-2 if dtype == torch.bfloat16 else 1e-5
            if mode == 2:
                assert torch.allclose(pred.cpu(), rp, atol=dot_err)
            else:
                assert torch.allclose(raw.cpu(), rr, atol=dot_err)


@pytest.mark.parametrize("graph", [False, True])
def test_device_sgd_matches_host_reference(graph):
    _need_gpu()
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer, TorchGlmTrainer

    g = torch.Generator(device="cpu").manual_seed(11)
    n, d = 4000, 64
    X = torch.rand((n, d), generator=g, dtype=torch.float64)
    y = (X @ torch.randn(d, generator=g, dtype=torch.float64) > 0).double()
    for loss in ("logistic", "hinge", "leastsquare"):
        for reg, en in ((0.0, 0.0), (0.1, 0.0), (0.1, 1.0), (0.1, 0.5)):
            sgd = SGD(max_iter=12, learning_rate=0.1, global_batch_size=1000, tol=1e-6, reg=reg, elastic_net=en)
            ref = TorchGlmTrainer(sgd, np.zeros(d), X, y, None, loss).fit()
            dev = DeviceGlmTrainer(sgd, np.zeros(d), X.cuda(), y.cuda(), None, loss, use_graph=graph)
            got = dev.fit()
            assert np.allclose(got, ref, atol=1e-9, rtol=1e-9), (loss, reg, en, np.abs(got - ref).max())


def test_device_sgd_early_termination():
    _need_gpu()
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer, TorchGlmTrainer

    g = torch.Generator(device="cpu").manual_seed(5)
    X = torch.rand((500, 8), generator=g, dtype=torch.float64)
    y = torch.zeros(500, dtype=torch.float64)
    sgd = SGD(max_iter=100, learning_rate=1.0, global_batch_size=500, tol=0.05)
    ref = TorchGlmTrainer(sgd, np.zeros(8), X, y, None, "logistic")
    r = ref.fit()
    dev = DeviceGlmTrainer(sgd, np.zeros(8), X.cuda(), y.cuda(), None, "logistic", use_graph=True)
    got = dev.fit()
    assert dev.rounds_executed() == ref.rounds
    assert np.allclose(got, r, atol=1e-9)


def test_lr_estimator_on_gpu_goldens():
    _need_gpu()
    from flink_ml_amd import Table, Vectors
    from flink_ml_amd.config import dtype_policy
    from flink_ml_amd.models import LogisticRegression

    rows = [(Vectors.dense(x, 2, 3, 4), float(x > 10), float(1 + (i % 5))) for i, x in
            enumerate([1, 2, 3, 4, 5, 11, 12, 13, 14, 15])]
    t = Table.from_rows(rows, ["features", "label", "weight"])
    with dtype_policy("fp64"):
        m = LogisticRegression().set_weight_col("weight").fit(t)
    coef = m.get_model_data()[0].rows()[0][0].values
    assert np.allclose(coef, [0.525, -0.283, -0.425, -0.567], atol=0.01)


@pytest.mark.parametrize("dtype,d", [(torch.float32, 3000), (torch.float64, 3000), (torch.bfloat16, 5000),
                                     (torch.bfloat16, 5001), (torch.float32, 16384), (torch.float64, 1500)])
def test_device_sgd_wide_dense_fused_kernel(dtype, d):
    """Rows one wave cannot hold run on the wide-row kernel (8 waves split each row's columns;
    d = 5001 through the zero-padded copy), one fused launch per round, weighted and unweighted:
    results equal the fp64 host trainer, and tol termination is decided on the device."""
    _need_gpu()
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer, TorchGlmTrainer

    g = torch.Generator(device="cpu").manual_seed(d)
    n = 1500
    X = torch.rand((n, d), generator=g, dtype=torch.float64).to(dtype)
    y = (X.to(torch.float64) @ torch.linspace(-1, 1, d, dtype=torch.float64) > 0).double()
    w = torch.rand(n, generator=g, dtype=torch.float64) + 0.5
    # (the L1 part of the elastic net flips coefficients near 0 by ±lr·en·reg on a last-bit change of
    # a 16384-term fp32 dot: L2 only at that width)
    en = 0.5 if d <= 5001 else 0.0
    for loss in ("logistic", "hinge", "leastsquare"):
        for wt in (w, None):
            sgd = SGD(max_iter=7, learning_rate=0.05, global_batch_size=400, tol=1e-9, reg=0.1, elastic_net=en)
            ref = TorchGlmTrainer(sgd, np.zeros(d), X.to(torch.float64), y, wt, loss).fit()
            tr = DeviceGlmTrainer(sgd, np.zeros(d), X.cuda(), y.cuda(), None if wt is None else wt.cuda(), loss)
            assert tr.wide_fused and not tr.wide
            got = tr.fit()
            assert got.shape == (d,) and tr.rounds_executed() == 7
            tol = (1e-10 if dtype == torch.float64 else 1e-4) * max(1.0, np.abs(ref).max())
            assert np.abs(got - ref).max() < tol, (loss, np.abs(got - ref).max())
    # tol termination decided on the device by the wide kernel's tail
    sgd2 = SGD(max_iter=100, learning_rate=0.5, global_batch_size=n, tol=0.3)
    r2 = TorchGlmTrainer(sgd2, np.zeros(d), X.to(torch.float64), y, None, "logistic")
    c2 = r2.fit()
    t2 = DeviceGlmTrainer(sgd2, np.zeros(d), X.cuda(), y.cuda(), None, "logistic")
    g2 = t2.fit()
    assert t2.rounds_executed() == r2.rounds
    assert np.abs(g2 - c2).max() < (1e-8 if dtype == torch.float64 else 1e-4) * max(1.0, np.abs(c2).max())


@pytest.mark.parametrize("dtype,d", [(torch.float32, 40000), (torch.bfloat16, 40001)])
def test_device_sgd_wide_dense_gemv_path(dtype, d):
    """Rows beyond the wide-row kernel (8 × 64 × 8 chunks) run as two GEMVs + the device update."""
    _need_gpu()
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer, TorchGlmTrainer

    g = torch.Generator(device="cpu").manual_seed(d)
    n = 300
    X = torch.rand((n, d), generator=g, dtype=torch.float64).to(dtype)
    y = (X.to(torch.float64) @ torch.linspace(-1, 1, d, dtype=torch.float64) > 0).double()
    w = torch.rand(n, generator=g, dtype=torch.float64) + 0.5
    for loss in ("logistic", "hinge", "leastsquare"):
        sgd = SGD(max_iter=7, learning_rate=0.05, global_batch_size=100, tol=1e-9, reg=0.1, elastic_net=0.5)
        ref = TorchGlmTrainer(sgd, np.zeros(d), X.to(torch.float64), y, w, loss).fit()
        tr = DeviceGlmTrainer(sgd, np.zeros(d), X.cuda(), y.cuda(), w.cuda(), loss)
        assert tr.wide and not tr.wide_fused
        got = tr.fit()
        assert tr.rounds_executed() == 7
        tol = (1e-10 if dtype == torch.float64 else 1e-4) * max(1.0, np.abs(ref).max())
        assert np.abs(got - ref).max() < tol, (loss, np.abs(got - ref).max())


@pytest.mark.parametrize("dtype,d", [(torch.float32, 1001), (torch.float32, 2047), (torch.bfloat16, 1003),
                                     (torch.bfloat16, 4093), (torch.float64, 1023)])
def test_device_sgd_misaligned_width_padded_to_fused_kernel(dtype, d):
    """Widths that break the 16-byte row chunks (fp32 d = 1001, bf16 d % 8 != 0) train on a fused
    round kernel (one-wave, or wide-row for bf16 4093) through a zero-padded copy: the padding
    coefficients stay 0, the returned model
    has the input width, and results equal the host trainer (and the GEMV path, pad=False)."""
    _need_gpu()
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer, TorchGlmTrainer

    g = torch.Generator(device="cpu").manual_seed(d)
    n = 1300
    X = torch.rand((n, d), generator=g, dtype=torch.float64).to(dtype)
    y = (X.to(torch.float64) @ torch.linspace(-1, 1, d, dtype=torch.float64) > 0).double()
    w = torch.rand(n, generator=g, dtype=torch.float64) + 0.5
    for loss in ("logistic", "hinge"):
        sgd = SGD(max_iter=6, learning_rate=0.05, global_batch_size=400, tol=1e-9, reg=0.1, elastic_net=0.5)
        ref = TorchGlmTrainer(sgd, np.zeros(d), X.to(torch.float64), y, w, loss).fit()
        tr = DeviceGlmTrainer(sgd, np.zeros(d), X.cuda(), y.cuda(), w.cuda(), loss)
        assert not tr.wide and (tr.layout is not None or tr.wide_fused)
        assert tr.X.shape[1] % (16 // X.element_size()) == 0
        got = tr.fit()
        assert got.shape == (d,) and tr.rounds_executed() == 6
        assert float(tr.coef[d:].abs().max() if tr.X.shape[1] > d else 0.0) == 0.0
        tol = (1e-10 if dtype == torch.float64 else 1e-4) * max(1.0, np.abs(ref).max())
        assert np.abs(got - ref).max() < tol, (loss, np.abs(got - ref).max())
        gemv = DeviceGlmTrainer(sgd, np.zeros(d), X.cuda(), y.cuda(), w.cuda(), loss, pad=False)
        if gemv.wide:
            assert np.abs(gemv.fit() - got).max() < tol
