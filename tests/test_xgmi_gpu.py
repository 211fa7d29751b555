"""xGMI one-shot all-reduce (ops/csrc/xgmi_allreduce.hip) and the fused multi-GPU SGD round
(glm.hip TAIL_XGMI), rehearsed with 2 ranks sharing cuda:0: a CPU (gloo) bootstrap exchanges the
IPC handles and the two processes map each other's uncached exchange buffers on the same device.
Kernels, tags, slot reuse, bounded waits and the rank-order sum are the code that runs across
8 GPUs; only the link is local. References: exact integer sums, and the fp64 host SGD trainer."""
import math

import numpy as np
import pytest
import torch

from tests.spmd import run_spmd

pytestmark = pytest.mark.gpu

ENV = {"FMLX_DEVICE": "cuda:0", "FMLX_XGMI": "force", "FMLX_XGMI_SPIN": str(1 << 20)}


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _allreduce_worker(rank, world, strict="0"):
    import torch

    from flink_ml_amd.parallel import xgmi

    x = xgmi.get()
    assert x is not None, "xGMI exchange did not come up"
    assert xgmi.strict_fence() == (strict == "1")
    S = world * (world + 1) // 2
    for dt in (torch.float32, torch.float64):
        for n in (1, 7, 1024, 1025, 3 * 4096 + 7, 300_000):
            for rep in range(3):  # both slots, then slot 0 again
                t = torch.arange(n, device="cuda:0", dtype=dt) * (rank + 1) + rep
                x.all_reduce_(t)
                exp = torch.arange(n, dtype=torch.float64) * S + rep * world
                assert torch.equal(t.to(torch.float64).cpu(), exp), (dt, n, rep)
    # the comm layer routes device sums through the exchange
    from flink_ml_amd.parallel import comm

    v = torch.full((513,), float(rank + 1), device="cuda:0", dtype=torch.float32)
    comm.all_reduce_sum(v)
    assert torch.all(v.cpu() == S)
    torch.cuda.synchronize()
    assert x.healthy()
    return True


@pytest.mark.parametrize("strict", ["0", "1"])
def test_xgmi_allreduce_two_ranks_one_gpu(strict):
    """Both fence modes of the hand-off (FMLX_XGMI_STRICT_FENCE)."""
    _need_gpu()
    env = dict(ENV, FMLX_XGMI_STRICT_FENCE=strict)
    assert run_spmd(_allreduce_worker, 2, strict, env=env, timeout=300) == [True, True]


def _twoshot_worker(rank, world, sizes):
    import torch

    from flink_ml_amd.parallel import comm, xgmi

    x = xgmi.get()
    assert x is not None, "xGMI exchange did not come up"
    S = world * (world + 1) // 2
    for dt in (torch.float32, torch.float64):
        for n in sizes:
            for rep in range(3):  # both slots, then slot 0 again
                t = torch.arange(n, device="cuda:0", dtype=dt) * (rank + 1) + rep
                x.all_reduce_(t, path="twoshot")
                exp = torch.arange(n, dtype=torch.float64) * S + rep * world
                assert torch.equal(t.to(torch.float64).cpu(), exp), (dt, n, rep)
    # size routing: a 4 MB feedback (dim 1M + 2) goes through the two-shot, a small one one-shot
    assert x.path(1_000_002) == "twoshot" and x.path(1000) == "oneshot" and x.path(3 << 20) == "rccl"
    v = torch.full((1_000_002,), float(rank + 1), device="cuda:0", dtype=torch.float32)
    comm.all_reduce_sum(v)
    assert torch.all(v.cpu() == S)
    # interleaved one-shot / two-shot calls keep their own tags
    for i in range(4):
        a = torch.full((5000,), float(rank + i), device="cuda:0")
        b = torch.full((200_000,), float(rank * 2 + i), device="cuda:0")
        x.all_reduce_(a, path="oneshot")
        x.all_reduce_(b, path="twoshot")
        assert torch.all(a.cpu() == sum(r + i for r in range(world)))
        assert torch.all(b.cpu() == sum(2 * r + i for r in range(world)))
    torch.cuda.synchronize()
    assert x.healthy()
    return True


@pytest.mark.parametrize("strict", ["0", "1"])
@pytest.mark.parametrize("world,sizes", [(2, (1, 1023, 1025, 2 * 1024 * 2 + 5, 300_000, 1_100_007)),
                                         (4, (1, 4097, 4 * 1024 * 3 + 1, 600_001))])
def test_xgmi_twoshot_allreduce_ranks_on_one_gpu(world, sizes, strict):
    """Two-shot (reduce-scatter + all-gather over the peer-mapped buffers): exact integer sums
    for partial chunk groups, both slots, f32/f64; routing of a 4 MB payload through it."""
    _need_gpu()
    env = dict(ENV, FMLX_XGMI_STRICT_FENCE=strict)
    assert run_spmd(_twoshot_worker, world, sizes, env=env, timeout=300) == [True] * world


def _sgd_worker(rank, world, xgmi_mode, dtype_name, defer_xgmi="1", fallback=False):
    import os

    import numpy as np
    import torch

    os.environ["FMLX_XGMI"] = xgmi_mode
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer, TorchGlmTrainer
    from flink_ml_amd.ops import glm as gk

    g = torch.Generator(device="cpu").manual_seed(100 + rank)
    n, d = 3000 + 500 * rank, 100
    X = torch.rand((n, d), generator=g, dtype=torch.float64)
    y = (X @ torch.linspace(-1, 1, d, dtype=torch.float64) > 0).double()
    w = torch.rand(n, generator=g, dtype=torch.float64) + 0.5
    out = {}
    for loss in ("logistic", "hinge", "leastsquare"):
        sgd = SGD(max_iter=8, learning_rate=0.1, global_batch_size=1600, tol=1e-9, reg=0.05, elastic_net=0.3)
        ref = TorchGlmTrainer(sgd, np.zeros(d), X, y, w, loss).fit()
        Xd = X.to(getattr(torch, dtype_name)).cuda()
        tr = DeviceGlmTrainer(sgd, np.zeros(d), Xd, y.cuda(), w.cuda(), loss, use_graph=(loss == "hinge" and xgmi_mode == "force"))
        expect = gk.TAIL_XGMI if xgmi_mode == "force" else gk.TAIL_FEEDBACK
        assert tr.mode == expect, (tr.mode, expect)
        # the in-kernel exchange runs deferred (launch e + 1's lead block completes round e)
        assert tr.defer == (xgmi_mode == "force" and defer_xgmi == "1"), tr.defer
        if fallback:  # bench.py's re-time after an xGMI timeout: RCCL/gloo feedback path
            tr.use_rccl()
            assert tr.mode == gk.TAIL_FEEDBACK and not tr.defer and tr.cw is None and tr.xg is None
        got = tr.fit()
        out[loss] = (float(np.abs(got - ref).max()), float(np.abs(ref).max()), got.tobytes())
    return out


@pytest.mark.parametrize("xgmi_mode,world,defer_xgmi,strict", [
    ("force", 2, "1", "0"), ("force", 2, "0", "0"), ("force", 4, "1", "0"), ("0", 2, "1", "0"),
    ("force", 2, "1", "1"), ("force", 4, "1", "1")])
def test_fused_sgd_round_two_ranks_matches_host(xgmi_mode, world, defer_xgmi, strict):
    _check_sgd_ranks(xgmi_mode, world, defer_xgmi, False, strict)


def test_sgd_switch_to_rccl_after_xgmi_matches_host():
    """DeviceGlmTrainer.use_rccl() (the bench's fallback left defer=1 on the feedback
    tail and the launcher returned -7) trains through the process-group all-reduce instead."""
    _check_sgd_ranks("force", 2, "1", True)


def _check_sgd_ranks(xgmi_mode, world, defer_xgmi, fallback, strict="0"):
    """TAIL_XGMI (in-kernel xGMI exchange: deferred — launch e + 1's lead block exchanges and
    applies round e — and ticketed) and TAIL_FEEDBACK (+ process-group all-reduce) reproduce the
    fp64 host trainer at 2 and 4 ranks, and every rank ends with bit-identical coefficients."""
    _need_gpu()
    env = dict(ENV, FMLX_XGMI=xgmi_mode, FMLX_GLM_DEFER_XGMI=defer_xgmi, FMLX_XGMI_STRICT_FENCE=strict)
    res = run_spmd(_sgd_worker, world, xgmi_mode, "float64", defer_xgmi, fallback, env=env, timeout=300)
    for loss in res[0]:
        err, scale, b0 = res[0][loss]
        assert err <= 1e-9 * max(1.0, scale), (loss, err)
        for r in res[1:]:
            assert b0 == r[loss][2], loss  # replicas identical


def _wide_grid_worker(rank, world):
    import numpy as np
    import torch

    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer, TorchGlmTrainer
    from flink_ml_amd.ops import glm as gk
    from flink_ml_amd.parallel.context import get_context

    g = torch.Generator(device="cpu").manual_seed(7 + rank)
    n, d = 140_000, 64
    X = torch.rand((n, d), generator=g, dtype=torch.float32).to(torch.bfloat16)
    y = (X.double() @ torch.linspace(-1, 1, d, dtype=torch.float64) > 0).double()
    sgd = SGD(max_iter=6, learning_rate=0.5, global_batch_size=2 * 70_000, tol=1e-9)
    tr = DeviceGlmTrainer(sgd, np.zeros(d), X.cuda(), y.cuda(), None, "logistic", use_graph=False)
    assert gk.round_blocks(tr.X) == 512 and get_context().sharers == world
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    assert tr.mode == gk.TAIL_XGMI and tr.nparts == cus // world, tr.nparts
    got = tr.fit()
    ref = TorchGlmTrainer(sgd, np.zeros(d), X.double(), y, None, "logistic").fit()
    return float(np.abs(got - ref).max()), float(np.abs(ref).max())


def test_two_ranks_one_gpu_512_block_shape_runs():
    """two ranks sharing one GPU at a shape whose 1-rank grid is 512 blocks (two per CU
    under the LDS pad) — every rank's grid must stay resident for the in-kernel exchange, so the
    grid is capped to CUs / sharers (measured by PCI id) instead of timing out."""
    _need_gpu()
    for err, scale in run_spmd(_wide_grid_worker, 2, env=ENV, timeout=300):
        assert err <= 1e-4 * max(1.0, scale), err


@pytest.mark.parametrize("det,blocks,unroll,defer,dma", [
    (False, 0, 0, True, None), (False, 0, 0, False, None), (False, 256, 0, True, 0), (False, 256, 2, True, 0),
    (False, 224, 4, True, 0), (False, 512, 0, True, 0), (False, 512, 0, False, 0), (True, 512, 0, True, 0),
    (True, 256, 1, True, 0), (False, 224, 2, True, 3), (False, 512, 1, True, 4), (False, 224, 2, False, 3),
    (True, 256, 2, True, 3)])
def test_fused_round_flagship_shape_matches_torch(det, blocks, unroll, defer, dma, monkeypatch):
    """Fused rounds (TAIL_UPDATE) at the bench shape, bf16 rows: the shipped default (blocks = 0 →
    round_blocks(), unroll = 0 → the shape's row loop; deferred and ticketed tails), 224 / 256 /
    512-block grids, 2 / 4 / 8 rows in flight per wave, atomic tail and the deterministic 16-group
    fixed-order tail."""
    _need_gpu()
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer, TorchGlmTrainer
    from flink_ml_amd.ops import glm as gk

    monkeypatch.setattr(gk, "DETERMINISTIC", det)
    monkeypatch.setattr(gk, "GRAD_BLOCKS", blocks)
    monkeypatch.setattr(gk, "GRAD_UNROLL", unroll)
    monkeypatch.setattr(gk, "DEFER", defer)
    gk.RoundScratch(1, 8, torch.float32, "cuda")  # applies the process default first
    gk.set_dma(gk.DMA_DEPTH if dma is None else dma)  # None: the shipped default

    g = torch.Generator(device="cpu").manual_seed(7)
    n, d, B = 200_000, 1000, 100_000
    Xb = torch.rand((n, d), generator=g).to(torch.bfloat16)
    y = torch.randint(0, 2, (n,), generator=g).to(torch.float64)
    sgd = SGD(max_iter=3, learning_rate=0.1, global_batch_size=B, tol=1e-9)
    ref = TorchGlmTrainer(sgd, np.zeros(d), Xb.to(torch.float64), y, None, "logistic").fit()
    tr = DeviceGlmTrainer(sgd, np.zeros(d), Xb.cuda(), y.cuda(), None, "logistic", use_graph=False)
    assert tr.nparts == (blocks or gk.round_blocks(tr.X)) and tr.scratch.det == det
    assert tr.defer == (defer and not det)
    try:
        got = tr.fit()
    finally:
        gk.set_dma(gk.DMA_DEPTH)
    assert tr.rounds_executed() == 3
    assert np.allclose(got, ref, rtol=2e-4, atol=2e-6), np.abs(got - ref).max()


@pytest.mark.parametrize("blocks", [256, 512])
def test_deterministic_tail_is_bitwise_reproducible(blocks, monkeypatch):
    """FMLX_DETERMINISTIC=1: two fits from the same data give bit-identical coefficients (the
    fixed-order group tree); a regression to an order-dependent reduction fails here. The default
    atomic tail is only checked to agree to rounding."""
    _need_gpu()
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer
    from flink_ml_amd.ops import glm as gk

    monkeypatch.setattr(gk, "GRAD_BLOCKS", blocks)
    g = torch.Generator(device="cpu").manual_seed(11)
    n, d, B = 120_000, 1000, 60_000
    Xb = torch.rand((n, d), generator=g).to(torch.bfloat16).cuda()
    y = torch.randint(0, 2, (n,), generator=g).to(torch.float64).cuda()

    def fit(det):
        monkeypatch.setattr(gk, "DETERMINISTIC", det)
        sgd = SGD(max_iter=6, learning_rate=0.1, global_batch_size=B, tol=0.0)
        return DeviceGlmTrainer(sgd, np.zeros(d), Xb, y, None, "logistic", use_graph=False).fit()

    a, b = fit(True), fit(True)
    assert np.array_equal(a, b)
    c = fit(False)
    assert np.allclose(a, c, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("graph,defer", [(False, True), (True, True), (False, False), (True, False)])
def test_multi_round_launch_terminates_mid_way(graph, defer, monkeypatch):
    """One host call issuing many rounds (and a replayed 16-round hipGraph) stops exactly where
    TerminateOnMaxIterOrTol says, even in the middle of the call (deferred completion: the
    launch after the last round applies its update and stops)."""
    _need_gpu()
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer, TorchGlmTrainer
    from flink_ml_amd.ops import glm as gk

    monkeypatch.setattr(gk, "DEFER", defer)

    g = torch.Generator(device="cpu").manual_seed(3)
    n, d, B = 60_000, 64, 20_000
    X = torch.rand((n, d), generator=g) - 0.5
    y = (X @ torch.linspace(-1, 1, d) > 0).to(torch.float64)
    ref_tr = TorchGlmTrainer(SGD(max_iter=40, learning_rate=2.0, global_batch_size=B, tol=0.4), np.zeros(d),
                             X.to(torch.float64), y, None, "logistic")
    ref = ref_tr.fit()
    assert 16 < ref_tr.rounds < 32, ref_tr.rounds  # stops inside the second 16-round call / graph
    sgd = SGD(max_iter=40, learning_rate=2.0, global_batch_size=B, tol=0.4)
    tr = DeviceGlmTrainer(sgd, np.zeros(d), X.cuda(), y.cuda(), None, "logistic", use_graph=graph)
    tr.rounds_per_graph = 16
    assert tr.defer == defer
    tr.run_rounds(40)
    torch.cuda.synchronize()
    assert tr.rounds_executed() == ref_tr.rounds
    assert np.allclose(tr.coef.double().cpu().numpy(), ref, rtol=1e-4, atol=1e-6)


def _timeout_worker(rank, world):
    import time

    import torch

    from flink_ml_amd.parallel import comm, xgmi

    x = xgmi.get()
    assert x is not None, "xGMI exchange did not come up"
    x.spin_limit = 2000  # a few ms of polling
    if rank == 1:
        time.sleep(3.0)  # rank 0's wait gives up long before this rank publishes
    t = torch.full((2000,), float(rank + 1), device="cuda:0")
    x.all_reduce_(t)
    torch.cuda.synchronize()
    out = {"nan": bool(torch.isnan(t).all().item()), "healthy": x.healthy()}
    try:
        comm.all_reduce_sum(torch.ones(8, device="cuda:0"))  # refuses once the error word is set
        out["raised"] = False
    except xgmi.XgmiTimeout:
        out["raised"] = True
    # bench.py's recovery: agree over the process group (no exchange check), retire the exchange,
    # and the next device all-reduce goes to the process group with exact sums
    out["agree"] = comm.all_agree(x.healthy())
    xgmi.disable()
    v = torch.full((8,), float(rank + 1), device="cuda:0")
    comm.all_reduce_sum(v)
    out["after"] = v.cpu().tolist()
    return out


def test_xgmi_timeout_poisons_and_raises():
    """a peer later than the spin limit must never yield a silent partial sum."""
    _need_gpu()
    res = run_spmd(_timeout_worker, 2, env=ENV, timeout=300)
    r0 = res[0]
    assert r0["nan"] and not r0["healthy"] and r0["raised"], r0
    assert not any(r["agree"] for r in res)
    assert all(r["after"] == [3.0] * 8 for r in res)


@pytest.mark.parametrize("rem", [0, 3])
def test_deferred_rounds_match_ticketed_tail(rem, monkeypatch):
    """Deferred completion vs the ticketed atomic tail over many graph replays with odd remainders
    (both round-number parities), stopping at max_iter: same rounds, coefficients to rounding."""
    _need_gpu()
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer
    from flink_ml_amd.ops import glm as gk

    g = torch.Generator(device="cpu").manual_seed(5)
    n, d, B = 90_000, 1000, 30_000
    Xb = torch.rand((n, d), generator=g).to(torch.bfloat16).cuda()
    y = torch.randint(0, 2, (n,), generator=g).to(torch.float32).cuda()
    out = {}
    for defer in (True, False):
        monkeypatch.setattr(gk, "DEFER", defer)
        sgd = SGD(max_iter=40 + rem, learning_rate=0.1, global_batch_size=B, tol=0.0)
        tr = DeviceGlmTrainer(sgd, np.zeros(d), Xb, y, None, "logistic", use_graph=True)
        assert tr.defer == defer
        tr.rounds_per_graph = 8
        for k in (5, 8, 1, 16, 3, 7 + rem):  # mixes graph replays and parities
            tr.run_rounds(k)
        tr.run_rounds(4)  # past max_iter: no-ops (deferred: the first one completes the last round)
        torch.cuda.synchronize()
        assert tr.rounds_executed() == 40 + rem and not tr.running()
        out[defer] = tr.coef.double().cpu().numpy()
    assert np.allclose(out[True], out[False], rtol=1e-5, atol=1e-7), np.abs(out[True] - out[False]).max()


@pytest.mark.parametrize("dtype,d,dma,unroll", [("bf16", 1000, 0, 0), ("bf16", 520, 0, 0), ("fp32", 300, 0, 0),
                                                ("bf16", 1000, 3, 0), ("bf16", 520, 2, 1), ("bf16", 1000, 4, 2),
                                                ("bf16", 1000, 2, 4)])
def test_round_covers_every_row_once(dtype, d, dma, unroll, monkeypatch):
    """The deferred round's row schedule processes every row of the round's batch exactly once
    for any batch size (fewer rows than wave slots, a partial last step, the whole set), with
    16-byte register loads and with the LDS-DMA row ring (``dma`` = ring depth in steps) at 2, 4
    and 8 rows in flight. Integer row weights make Σweight (feedback[d]) an exact,
    order-independent row census of each round; Σloss agrees with a torch evaluation."""
    _need_gpu()
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer
    from flink_ml_amd.ops import glm as gk

    monkeypatch.setattr(gk, "DEFER", True)
    monkeypatch.setattr(gk, "DETERMINISTIC", False)
    monkeypatch.setattr(gk, "GRAD_UNROLL", unroll)
    gk.RoundScratch(1, 8, torch.float32, "cuda")  # applies the process default first
    gk.set_dma(dma)
    try:
        g = torch.Generator(device="cpu").manual_seed(9)
        n = 157_003
        X = torch.rand((n, d), generator=g)
        X = X.to(torch.bfloat16) if dtype == "bf16" else X
        y = torch.randint(0, 2, (n,), generator=g).to(torch.float32)
        wt = (torch.arange(n) % 7 + 1).to(torch.float32)
        for B in (1_000, 31_337, 157_003, 100_000):
            tr = DeviceGlmTrainer(SGD(max_iter=6, learning_rate=0.1, global_batch_size=B, tol=0.0), np.zeros(d),
                                  X.cuda(), y.cuda(), wt.cuda(), "logistic", use_graph=False)
            assert tr.defer
            P = -(-n // B)
            tr._launch_round(1)  # round 0 (w = 0: every row's loss is log 2)
            for e in range(5):  # both launch parities twice
                tr._launch_round(1)  # launch e + 1 completes round e and publishes its feedback
                torch.cuda.synchronize()
                b0 = (e % P) * B
                want = float(wt[b0:min(b0 + B, n)].sum())
                got = float(tr.feedback[d].item())
                assert got == want, (B, e, got, want)
                if e == 0:
                    assert abs(float(tr.feedback[d + 1].item()) - want * math.log(2.0)) <= 1e-5 * want
    finally:
        gk.set_dma(gk.DMA_DEPTH)


def test_shipped_default_graph_fit_matches_torch(monkeypatch):
    """The shipped configuration exactly as bench.py runs it — default grid (round_blocks), default
    row loop, deferred completion, hipGraph-captured rounds — against the fp64 torch reference."""
    _need_gpu()
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer, TorchGlmTrainer
    from flink_ml_amd.ops import glm as gk

    monkeypatch.setattr(gk, "GRAD_BLOCKS", 0)
    monkeypatch.setattr(gk, "GRAD_UNROLL", 0)
    g = torch.Generator(device="cpu").manual_seed(13)
    n, d, B = 300_000, 1000, 100_000
    Xb = torch.rand((n, d), generator=g).to(torch.bfloat16)
    y = torch.randint(0, 2, (n,), generator=g).to(torch.float64)
    sgd = SGD(max_iter=7, learning_rate=0.1, global_batch_size=B, tol=0.0)
    ref = TorchGlmTrainer(sgd, np.zeros(d), Xb.to(torch.float64), y, None, "logistic").fit()
    tr = DeviceGlmTrainer(sgd, np.zeros(d), Xb.cuda(), y.cuda(), None, "logistic", use_graph=True)
    assert tr.defer and tr.nparts == gk.round_blocks(tr.X)
    got = tr.fit()
    assert tr.rounds_executed() == 7
    assert np.allclose(got, ref, rtol=2e-4, atol=2e-6), np.abs(got - ref).max()
