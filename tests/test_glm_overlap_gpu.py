"""Overlapped deferred SGD rounds (FMLX_GLM_OVERLAP, csrc/glm.hip overlap_wait / overlap_arrive):
consecutive launches alternate between two streams and hand off through in-kernel arrival
counts instead of a kernel boundary. Checked against the fp64 host trainer at the bench's row
width — direct launches and hipGraph replays, a fit that ends on the tolerance while further
launches are already queued (their no-op rounds still arrive), and no wait timeout."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def _data(n, d, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    Xb = torch.rand((n, d), generator=g).to(torch.bfloat16)
    y = torch.randint(0, 2, (n,), generator=g).to(torch.float64)
    return Xb, y


@pytest.mark.parametrize("graph,iters,blocks", [(False, 7, 0), (True, 25, 0), (True, 24, 512), (False, 9, 224)])
def test_overlapped_rounds_match_host(graph, iters, blocks, monkeypatch):
    _need_gpu()
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer, TorchGlmTrainer
    from flink_ml_amd.ops import glm as gk

    monkeypatch.setattr(gk, "OVERLAP", True)
    monkeypatch.setattr(gk, "GRAD_BLOCKS", blocks)
    n, d, B = 160_000, 1000, 40_000
    Xb, y = _data(n, d, 3)
    sgd = SGD(max_iter=iters, learning_rate=0.1, global_batch_size=B, tol=1e-12)
    ref = TorchGlmTrainer(sgd, np.zeros(d), Xb.to(torch.float64), y, None, "logistic").fit()
    tr = DeviceGlmTrainer(sgd, np.zeros(d), Xb.cuda(), y.cuda(), None, "logistic", use_graph=graph, check_every=5)
    assert tr.defer and tr.overlap
    got = tr.fit()
    assert tr.rounds_executed() == iters
    assert int(tr.scratch.cnt[gk.ARR_ERR].item()) == 0
    assert np.allclose(got, ref, rtol=2e-4, atol=2e-6), np.abs(got - ref).max()


def test_overlapped_rounds_stop_on_tolerance_with_launches_queued(monkeypatch):
    """The tolerance ends the iteration at round r while later launches are already queued (10
    rounds per graph): every later launch waits, sees the done word, arrives and exits; the
    coefficients are round r's and the executed count matches the host trainer."""
    _need_gpu()
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer, TorchGlmTrainer
    from flink_ml_amd.ops import glm as gk

    monkeypatch.setattr(gk, "OVERLAP", True)
    n, d, B = 60_000, 1000, 60_000
    Xb, y = _data(n, d, 5)
    sgd = SGD(max_iter=200, learning_rate=1.0, global_batch_size=B, tol=0.62)
    host = TorchGlmTrainer(sgd, np.zeros(d), Xb.to(torch.float64), y, None, "logistic")
    ref = host.fit()
    assert 2 < host.rounds < 40
    tr = DeviceGlmTrainer(sgd, np.zeros(d), Xb.cuda(), y.cuda(), None, "logistic", use_graph=True, check_every=10)
    got = tr.fit()
    assert tr.rounds_executed() == host.rounds
    assert int(tr.scratch.cnt[gk.ARR_ERR].item()) == 0
    assert np.allclose(got, ref, rtol=2e-4, atol=2e-6), np.abs(got - ref).max()
    # a further replay after the stop stays a no-op and keeps the hand-off consistent
    tr.run_rounds(20)
    torch.cuda.synchronize()
    assert tr.rounds_executed() == host.rounds
    assert int(tr.scratch.cnt[gk.ARR_ERR].item()) == 0
    assert np.array_equal(tr.coef.double().cpu().numpy(), got)
