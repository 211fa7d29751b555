"""Multi-process SPMD test harness (the analogue of the reference's local MiniCluster with
parallelism 4): spawns ``world`` CPU ranks over the gloo backend on 127.0.0.1 and returns
each rank's result."""
import datetime
import os
import traceback

import torch.distributed as dist
import torch.multiprocessing as mp


def _worker(rank, world, port, fn, args, q, env=None, backend="gloo"):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "FMLX_DEVICE": "cpu",
                       "FMLX_STORE": "127.0.0.1:%d" % port})
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
    # The parent hosts the rendezvous store on a port the kernel assigns at bind time and keeps it
    # bound until every rank is done; the ranks connect as clients (FMLX_STORE). Handing out a
    # bind-then-closed "free" port instead races other groups for the number (GPUTEST_r03).
    store = dist.TCPStore("127.0.0.1", 0, world, is_master=True, wait_for_workers=False,
                          timeout=datetime.timedelta(seconds=timeout))
    port = store.port
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
        del store
    return [results[r] for r in range(world)]
