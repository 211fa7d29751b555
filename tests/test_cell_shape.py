"""Host-side rules of the sparse forward's cells (ops/glm.py BatchCsc._pick_cells) and the
XCD-aware block order of glm.hip glm_csr_cell_fwd_kernel, checked without a GPU: the shape the
picker chooses for the SVC north-star shard, denser rows, narrow models, and that the kernel's
blockIdx → cell map is a bijection of the grid for every grid size."""
import types

import pytest
import torch


class _Vals:
    device = None

    def __init__(self, es=4):
        self._es = es

    def element_size(self):
        return self._es


def _pick(monkeypatch, n, d, B, nnz, cus=256, es=4, splits=0, rbb=None):
    from flink_ml_amd.ops import glm as gk

    monkeypatch.setattr(torch.cuda, "get_device_properties",
                        lambda dev: types.SimpleNamespace(multi_processor_count=cus))
    monkeypatch.setattr(gk, "CELL_SPLITS", splits)
    if rbb is not None:
        monkeypatch.setattr(gk, "CELL_RBB", rbb)
    c = gk.BatchCsc.__new__(gk.BatchCsc)
    c.rbb, c.cells = 10, 0
    c._pick_cells(_Vals(es), [0, n * nnz], n, d, B)
    return c


def test_svc_shard_shape(monkeypatch):
    # 6.25M × 1M, 64 nnz, batch 100k: 98 blocks of 1024 rows × 5 splits = 490 cells (≈ 2 per CU)
    c = _pick(monkeypatch, 6_250_000, 1_000_000, 100_000, 64)
    assert (c.rbb, c.S, c.cells) == (10, 5, 490)
    assert c.CS * c.S >= 1_000_000 and c.cb == 18
    # the average cell (13.1K entries) fits the rank bits with 20 % to spare
    assert 64 * 1024 / c.S * 1.2 <= 1 << (32 - c.cb)


def test_dense_rows_take_more_splits(monkeypatch):
    c = _pick(monkeypatch, 1_000_000, 1_000_000, 100_000, 300)
    cell = 300 * (1 << c.rbb) / c.S
    assert cell * 1.2 <= min(1 << (32 - c.cb), 128 * 1024 // 4)
    assert c.S > 5


def test_narrow_model_and_explicit_splits(monkeypatch):
    c = _pick(monkeypatch, 5_100, 800, 2_000, 30)
    assert c.S <= 64 and c.cells == 2 * c.S  # 2 row blocks
    c = _pick(monkeypatch, 5_100, 5, 2_000, 3)
    assert c.S <= 5  # never more splits than columns
    c = _pick(monkeypatch, 12_345, 3_001, 5_000, 6, splits=5, rbb=10)
    assert (c.rbb, c.S, c.cells) == (10, 5, 25)


def test_fp64_cells_respect_lds(monkeypatch):
    c = _pick(monkeypatch, 1_000_000, 1_000_000, 100_000, 300, es=8)
    assert 300 * (1 << c.rbb) / c.S * 8 * 1.2 <= 128 * 1024


@pytest.mark.parametrize("grid", list(range(1, 70)) + [490, 491, 497, 588, 784, 1176])
def test_xcd_block_order_is_a_bijection(grid):
    # glm.hip glm_csr_cell_fwd_kernel: XCD x = b mod 8 holds ceil((grid - x) / 8) blocks and
    # starts at x·floor(grid/8) + min(x, grid mod 8)
    q, r = grid >> 3, grid & 7
    got = sorted((b & 7) * q + min(b & 7, r) + (b >> 3) for b in range(grid))
    assert got == list(range(grid))
    # contiguity: each XCD's cells form one range
    for x in range(8):
        gs = [(b & 7) * q + min(b & 7, r) + (b >> 3) for b in range(x, grid, 8)]
        assert gs == list(range(gs[0], gs[0] + len(gs))) if gs else True
