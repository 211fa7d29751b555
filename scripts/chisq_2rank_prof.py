"""Two ranks on one GPU run ChiSqTest (flatten) over shards of an integer-valued and a float-valued
feature table (the multi-rank contingency path: catstats.global_value_label_counts); the parent
never touches the GPU. Under ``rocprofv3 --kernel-trace`` every rank writes its own database:
``scripts/kstats.py`` over them lists the kernels of that path (no torch
unique / sort kernels). Prints one JSON line per kind with the statistics rank 0 computed."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _table(kind, rank, world, n=200_000, d=8):
    import torch

    from flink_ml_amd import Table

    g = torch.Generator().manual_seed(11)
    if kind == "int":
        X = torch.randint(0, 12, (n, d), generator=g).to(torch.float64)
    else:
        X = (torch.randint(0, 40, (n, d), generator=g).to(torch.float64) * 0.37).round(decimals=3)
    y = torch.randint(0, 3, (n,), generator=g).to(torch.float64)
    s, e = rank * n // world, (rank + 1) * n // world
    return Table({"features": X[s:e].cuda(), "label": y[s:e].cuda()}, num_rows=e - s)


def _worker(rank, world, kind):
    from flink_ml_amd.models import ChiSqTest

    t = _table(kind, rank, world)
    ChiSqTest().set_flatten(True).transform(t)[0].rows()  # warm (first-use code objects)
    rows = ChiSqTest().set_flatten(True).transform(t)[0].rows()
    return [[float(v) for v in r] for r in rows[:3]]


def main():
    from tests.spmd import run_spmd

    env = {"FMLX_DEVICE": "cuda:0", "FMLX_XGMI": "0"}
    for kind in ("int", "float"):
        res = run_spmd(_worker, 2, kind, env=env, timeout=300)
        assert res[0] == res[1]
        print(json.dumps({"kind": kind, "ranks": 2, "first_rows": res[0]}), flush=True)


if __name__ == "__main__":
    main()
