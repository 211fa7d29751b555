"""Stream-ordering checker of the ingestion hand-off (``utils/streamcheck.py``, FMLX_STREAM_CHECK)."""
import pytest
import torch

from flink_ml_amd import Table
from flink_ml_amd.stream import StreamTable
from flink_ml_amd.utils import streamcheck


def test_checksum_detects_changes():
    g = torch.Generator().manual_seed(0)
    a = torch.rand((1000, 17), generator=g)
    b = a.clone()
    assert streamcheck.checksum(a) == streamcheck.checksum(b)
    b[123, 4] += 1.0
    assert streamcheck.checksum(a) != streamcheck.checksum(b)
    c = a.clone()
    c[[0, 1]] = c[[1, 0]]  # swapped rows: same byte sum, different position weights
    assert streamcheck.checksum(a) != streamcheck.checksum(c)
    assert streamcheck.checksum(torch.empty(0)) == (0, 0)


def test_disabled_by_default(monkeypatch):
    monkeypatch.delenv("FMLX_STREAM_CHECK", raising=False)
    assert not streamcheck.enabled()
    monkeypatch.setenv("FMLX_STREAM_CHECK", "1")
    assert streamcheck.enabled()


def _host_stream(n=40_000, d=64, rows=10_000):
    g = torch.Generator().manual_seed(1)
    t = Table({"features": torch.rand((n, d), generator=g), "label": torch.randint(0, 2, (n,), generator=g).double()})
    return t, StreamTable.from_table(t, rows)


@pytest.mark.gpu
def test_gpu_prefetch_handoffs_verified(monkeypatch):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setenv("FMLX_STREAM_CHECK", "1")
    t, st = _host_stream()
    total = 0.0
    for b in st.to_device(torch.device("cuda")):
        total += float(b.column("features").sum())  # the consumer reads every batch
    assert abs(total - float(t.column("features").double().sum())) < 1e-2 * max(1.0, abs(total))


@pytest.mark.gpu
def test_gpu_prefetch_race_is_reported(monkeypatch):
    """A consumer-side write into a handed-over copy (what a reused allocator block or a missing
    wait would look like) is reported at the next hand-off."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setenv("FMLX_STREAM_CHECK", "1")
    _, st = _host_stream()
    it = iter(st.to_device(torch.device("cuda")))
    b0 = next(it)
    b0.column("features")[5].fill_(-7.0)  # corrupt the device copy on the consumer stream
    with pytest.raises(streamcheck.StreamOrderError, match="batch 0"):
        next(it)
