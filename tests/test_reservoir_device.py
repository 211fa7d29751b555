"""Parallel reservoir sampler (ops/datagen.py reservoir_sample_device): bit-exact with the
sequential java.util.Random sampler of DataStreamUtils.SamplingOperator (javarand.cpp), including
streams where nextInt rejections shift every later draw. Runs the device algorithm on the CPU
(host-generated next(31) stream); the GPU test adds the HIP stream generator."""
import numpy as np
import pytest
import torch

from flink_ml_amd.models.kmeans import reservoir_sample_indices
from flink_ml_amd.ops import datagen


@pytest.mark.parametrize("n,k,seed", [(1, 4, 0), (4, 4, 1), (5, 4, 2), (1000, 10, 3), (100_000, 7, 4),
                                      (1_500_000, 1024, 5), (2_000_000, 3, -77), (300_000, 65536, 9)])
def test_device_reservoir_matches_sequential(n, k, seed):
    got = datagen.reservoir_sample_device(n, k, seed, "cpu").numpy()
    ref = reservoir_sample_indices(n, k, seed)
    assert np.array_equal(got, ref)


def test_next31_stream_offsets():
    a = datagen.next31_stream(11, 0, 1000, "cpu")
    b = datagen.next31_stream(11, 600, 400, "cpu")
    assert torch.equal(a[600:], b)


@pytest.mark.gpu
def test_device_reservoir_on_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    # (the candidate compaction kernel + host order up to 65536 candidates, ≈ n² / 2^32: the
    # 100k / 300k / 1M cases; 3M takes the ordered torch path)
    for n, k, seed in ((3_000_000, 1024, 1), (100_000, 10, 7), (300_000, 65536, 9), (1_000_000, 10, 2)):
        assert torch.equal(datagen.next31_stream(seed, 17, 5000, "cuda").cpu(), datagen.next31_stream(seed, 17, 5000, "cpu"))
        got = datagen.reservoir_sample_device(n, k, seed, "cuda").cpu().numpy()
        assert np.array_equal(got, reservoir_sample_indices(n, k, seed))
