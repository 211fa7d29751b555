"""Host-side helpers added in round 4: the CSR batch-bounds cache that lets a sparse fit start
without a device -> host copy (ops/glm.py ``_batch_bounds``), and the count of ranks sharing one
GPU that caps the in-kernel-exchange grid in one-GPU rehearsals (parallel/context.py
``device_sharers``)."""
import gc

import torch

from flink_ml_amd.ops import glm as gk
from flink_ml_amd.parallel.context import SPMDContext, count_sharers, device_sharers


def test_batch_bounds_cached_per_tensor_and_version():
    ip = torch.tensor([0, 2, 5, 5, 9, 12], dtype=torch.int64)
    a = gk._batch_bounds(ip, 5, 2)
    assert a == (12, [0, 5, 9, 12])
    assert gk._batch_bounds(ip, 5, 2) is a  # cached
    assert gk._batch_bounds(ip, 5, 3) == (12, [0, 5, 12])  # other batch size: its own entry
    ip[5] = 13  # in-place change bumps the version: recomputed
    assert gk._batch_bounds(ip, 5, 2) == (13, [0, 5, 9, 13])
    key = id(ip)
    del ip
    gc.collect()
    assert key not in gk._BOUNDS_CACHE  # dropped with the tensor


def test_device_sharers():
    cpu = SPMDContext(rank=0, world_size=4, device=torch.device("cpu"))
    assert device_sharers(cpu) == 1
    gpu = SPMDContext(rank=1, world_size=4, device=torch.device("cuda", 0), sharers=4)
    assert device_sharers(gpu) == 4
    assert device_sharers(SPMDContext(rank=1, world_size=4, device=torch.device("cuda", 0))) == 1
    assert device_sharers(SPMDContext(rank=0, world_size=1, device=torch.device("cuda", 0), sharers=3)) == 1
    # sharing is counted from the ranks' PCI identities, not guessed from device_count()
    ids = ["h/0000:05:00", "h/0000:05:00", "h/0000:15:00", "g/0000:05:00"]
    assert [count_sharers(ids, r) for r in range(4)] == [2, 2, 1, 1]
