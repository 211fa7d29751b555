"""Multi-process SPMD test harness (the analogue of the reference's local MiniCluster with
parallelism 4): spawns ``world`` CPU ranks over the gloo backend on 127.0.0.1 and returns
each rank's result."""
import os
import socket
import traceback

import torch.multiprocessing as mp


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, fn, args, q, env=None, backend="gloo"):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "FMLX_DEVICE": "cpu"})
    os.environ.update(env or {})
    try:
        import torch

        torch.set_num_threads(1)
        from flink_ml_amd.parallel.context import init_distributed, shutdown

        init_distributed(backend=backend, timeout_s=120)
        res = fn(rank, world, *args)
        q.put((rank, "ok", res))
        shutdown()
    except Exception:  # pragma: no cover - reported to the parent
        q.put((rank, "err", traceback.format_exc()))


def run_spmd(fn, world: int, *args, timeout: float = 180, env=None, backend="gloo"):
    """``env``: extra environment for every rank (e.g. ``{"FMLX_DEVICE": "cuda:0"}`` to put all
    ranks on one GPU with a gloo group). ``backend=None``: the context's choice (``nccl`` = RCCL
    on a GPU)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, args, q, env, backend)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            rank, status, res = q.get(timeout=timeout)
            if status != "ok":
                raise RuntimeError("rank %d failed:\n%s" % (rank, res))
            results[rank] = res
    finally:
        for p in procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
    return [results[r] for r in range(world)]
