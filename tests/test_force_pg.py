"""FMLX_FORCE_PG=1: a process group at WORLD_SIZE=1 (the one-GPU rehearsal of the distributed
code path, tests/test_rccl_gpu.py) — here on gloo/CPU: the context reports a distributed run and
collectives go through torch.distributed."""
import numpy as np
import torch

from tests.spmd import run_spmd


def _worker(rank, world):
    import torch.distributed as dist

    from flink_ml_amd.parallel import comm, xgmi
    from flink_ml_amd.parallel.context import get_context

    ctx = get_context()
    out = {"dist": ctx.is_distributed, "forced": ctx.forced, "world": ctx.world_size, "init": dist.is_initialized(),
           "path": xgmi.collective_path()}
    t = torch.arange(5, dtype=torch.float64)
    comm.all_reduce_sum(t)
    out["sum"] = t.tolist()
    out["gather"] = comm.all_gather_object({"r": rank})
    return out


def test_force_pg_world_one_on_gloo():
    (res,) = run_spmd(_worker, 1, env={"FMLX_FORCE_PG": "1"})
    assert res["dist"] and res["forced"] and res["init"] and res["world"] == 1
    assert res["path"] == "gloo"
    assert np.allclose(res["sum"], np.arange(5))
    assert res["gather"] == [{"r": 0}]


def test_force_pg_off_by_default():
    from flink_ml_amd.parallel.context import get_context

    assert not get_context().is_distributed
