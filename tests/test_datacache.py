"""Native spillable data cache (reference DataCacheWriteReadTest / ReplayOperator behaviour):
records round-trip across memory and file segments, budgets force spilling, reopen from the
manifest, Table batches replay in order (dense, sparse, object columns), prefetch thread, and the
iteration runtime replays a one-pass source from the cache."""
import os

import numpy as np
import pytest
import torch

from flink_ml_amd import Table
from flink_ml_amd.parallel.datacache import CachedReplay, DataCache, TableCache
from flink_ml_amd.table import SparseColumn


def test_records_memory_then_files(tmp_path):
    c = DataCache(str(tmp_path / "c"), segment_bytes=1000, memory_budget=2500)
    recs = [np.arange(i * 10, i * 10 + 50, dtype=np.int64) for i in range(20)]  # 400 B each
    for r in recs:
        c.append(r)
    st = c.stats()
    assert st["memory_segments"] == 2 and st["file_bytes"] > 0 and st["segments"] > 2
    for i, r in enumerate(recs):
        assert np.array_equal(np.frombuffer(c.read(i), np.int64), r)
    big = np.ones(5000, np.uint8)  # larger than a segment: gets its own
    j = c.append(big)
    assert c.read(j) == big.tobytes()
    c.spill()
    assert c.stats()["memory_bytes"] == 0
    assert np.array_equal(np.frombuffer(c.read(3), np.int64), recs[3])
    c.finish()
    c.close(remove=False)
    r = DataCache.reopen(str(tmp_path / "c"))
    assert len(r) == 21 and np.array_equal(np.frombuffer(r.read(19), np.int64), recs[19])
    r.close(remove=True)
    assert not os.path.exists(str(tmp_path / "c"))


def _batches():
    g = torch.Generator().manual_seed(0)
    out = []
    for b in range(5):
        X = torch.randn(100, 8, generator=g, dtype=torch.float64)
        sp = SparseColumn.from_dense((X > 1.0).to(torch.float64))
        out.append(Table({"x": X, "y": torch.arange(100, dtype=torch.int64) + 100 * b, "s": sp,
                          "w": ["r%d" % (100 * b + i) for i in range(100)]}, num_rows=100))
    return out


@pytest.mark.parametrize("prefetch", [0, 2])
def test_table_cache_replay(tmp_path, prefetch):
    src = _batches()
    tc = TableCache(path=str(tmp_path / "t"), segment_bytes=4096, memory_budget=8192)
    for t in src:
        tc.append(t)
    for _ in range(2):
        got = list(tc.replay(prefetch=prefetch))
        assert len(got) == 5
        for a, b in zip(src, got):
            assert torch.equal(a.column("x"), b.column("x")) and torch.equal(a.column("y"), b.column("y"))
            assert torch.equal(a.column("s").to_dense(), b.column("s").to_dense())
            assert a.get_list("w") == b.get_list("w")
    tail = list(tc.replay(prefetch=prefetch, start=3))
    assert [int(t.column("y")[0]) for t in tail] == [300, 400]
    tc.finish()
    r = TableCache.reopen(str(tmp_path / "t"))
    assert torch.equal(r.load(4).column("x"), src[4].column("x"))
    r.close()


def test_cached_replay_in_bounded_iteration(tmp_path):
    from flink_ml_amd.parallel.iteration import (IterationBodyResult, IterationConfig, Iterations,
                                                 ReplayableDataStreamList)

    pulls = []

    def gen():
        for t in _batches():
            pulls.append(1)
            yield t

    stream = CachedReplay(gen(), path=str(tmp_path / "r"))

    class Body:
        def process(self, variables, streams, ctx):
            total = sum(float(t.column("x").sum()) for t in streams[0])
            r = variables[0][0]
            return IterationBodyResult([[r + 1]] if r + 1 < 4 else [[]], [[total]])

    out = Iterations.iterate_bounded_streams_until_termination(
        [[0]], ReplayableDataStreamList.replay(stream), IterationConfig(), Body())
    expected = sum(float(t.column("x").sum()) for t in _batches())
    assert out[0] == pytest.approx([expected] * 4)
    assert len(pulls) == 5  # the source was consumed once; rounds 1..3 replayed from the cache
    stream.close()


@pytest.mark.gpu
def test_table_cache_replays_to_gpu(tmp_path):
    src = _batches()
    tc = TableCache(path=str(tmp_path / "g"), memory_budget=4096)
    for t in src:
        tc.append(t)
    for a, b in zip(src, tc.replay(device="cuda")):
        assert b.column("x").is_cuda and torch.equal(a.column("x"), b.column("x").cpu())
    tc.close()
