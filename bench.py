#!/usr/bin/env python3
"""Flagship benchmark: LogisticRegression mini-batch SGD, 10M × 1K dense, bf16 features.

Config (BASELINE.json north star #2; reference ``logisticregression-benchmark.json`` widened to
1K features): maxIter/lr 0.1/tol 1e-6/reg 0, global batch 100,000 rows per GPU, synthetic
``LabeledPointWithWeightGenerator``-shaped data (features U[0,1), labels {0,1}) generated on
device, random-init-equivalent zero model (the reference's init).

One *step* = one full SGD round of the reference (``SGD.java:246-285``): fused loss+gradient
over the rank's 100k-row minibatch (HIP kernel), deterministic reduction, RCCL all-reduce of
the (d+2) feedback when N > 1, device-side termination check, model update + regularisation.
Nothing is skipped inside the timed region.

Scaling (``--scaling``): *weak* (default, the driver contract) — every GPU keeps a 100k-row local
batch (global batch = 100k·N) over its 1/N shard of the 10M-row dataset; *strong* — the
reference's own semantics, a fixed global batch of 100k rows split over the N ranks with the
remainder to the low ranks (``SGD.java:206-213``, ``logisticregression-benchmark.json``).
``value`` = total samples/s over all GPUs.

Launch: ``python bench.py --gpus N``. Without a ``WORLD_SIZE`` in the environment and N > 1 this
process is only a launcher (it never touches the GPU): it hosts the rendezvous TCPStore and
starts N fresh rank processes of this same script — one per GPU, like the reference's
``benchmark-run.sh`` → ``flink run`` at the cluster's parallelism — and exits with their status.
Under ``python -m torch.distributed.run --nproc-per-node N … bench.py --gpus N`` the ranks come
from the environment, and a ``WORLD_SIZE`` that differs from ``--gpus`` is an error.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def timed_region(tr, ctx, warmup: int, steps: int):
    """Warm-up, then EXACTLY ``steps`` SGD rounds between barrier + synchronize brackets.

    Every hipGraph the timed ``run_rounds(steps)`` replays is captured, instantiated and
    replayed once BEFORE the clock starts (``precapture`` + one priming replay each), so the
    timed region only replays graphs, whatever ``--steps``/``--warmup`` the driver passes.
    Returns (host wall seconds, device seconds measured by events around the same region).
    """
    tr.precapture(steps)
    tr.prime(steps)
    tr.run_rounds(warmup)
    torch.cuda.synchronize()
    ctx.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    tr.timing = True
    t0 = time.perf_counter()
    ev0.record()
    tr.run_rounds(steps)
    ev1.record()
    torch.cuda.synchronize()
    ctx.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    tr.timing = False
    return elapsed, ev0.elapsed_time(ev1) * 1e-3


VERIFY_ROUNDS = 3
VERIFY_RTOL = 1e-4


def verify_exchange(make, comm, rounds: int = VERIFY_ROUNDS):
    """Untimed check that the timed rounds' cross-rank combination computed the right thing
    (a silent ordering bug of the in-kernel exchange must not yield a confident number).

    Two fresh trainers of the timed configuration run ``rounds`` rounds from the same start with
    direct launches: ``a`` exactly as timed (in-kernel xGMI exchange, deferred completion when the
    timed rounds used it), ``b`` on the process group (feedback → RCCL all-reduce → update). Every
    rank then requires (1) ``a``'s coefficients bitwise identical on all ranks (each applied the same
    exchanged feedback) and (2) ``a`` ≈ ``b`` (the exchanged feedback equals the process-group sum of
    the same per-rank partials, up to summation order). Reference: the reference's own payload
    checks, ``AllReduceImpl.java:118-120,187-188``. Returns (agreed verdict, details)."""
    a = make()
    a.use_graph = False
    a.sgd.max_iter = rounds + 2  # (direct launches read it; the flush round too)
    a.run_rounds(rounds)
    a.flush()
    ca = a.coef[:a.d_model].double().cpu()
    b = make()
    b.use_rccl()
    b.use_graph = False
    b.sgd.max_iter = rounds + 2
    b.run_rounds(rounds)
    b.flush()
    cb = b.coef[:b.d_model].double().cpu()
    from flink_ml_amd.parallel.context import get_context

    me = str(get_context().rank)
    if os.environ.get("FMLX_BENCH_INJECT_EXCHANGE_ERROR") == me or (
            os.environ.get("FMLX_BENCH_INJECT_XGMI_ERROR") == me and getattr(a, "xg", None) is not None):
        ca = ca.clone()
        ca[0] += 1e-3 * (1.0 + ca.abs().max())  # test hook: a corrupted exchange on this rank
    replicas = comm.all_gather_tensor(ca)
    identical = all(torch.equal(replicas[0], c) for c in replicas)
    scale = max(float(cb.abs().max()), 1e-30)
    rel = float((ca - cb).abs().max()) / scale
    ok = comm.all_agree(bool(identical and rel <= VERIFY_RTOL))
    return ok, {"replicas_identical": identical, "rel_err_vs_process_group": rel}


def launch_ranks(n: int, argv, env=None, timeout: float = None) -> int:
    """Starts ``n`` rank processes of this script (``argv``: its arguments) on this node and
    returns the first non-zero exit status (0 if every rank succeeded).

    The parent hosts the rendezvous TCPStore on a port the kernel assigns at bind time and keeps
    it bound until the ranks are done; the ranks connect as clients (``FMLX_STORE``), so no
    bind-then-close port race. Rank r gets RANK = LOCAL_RANK = r (GPU r), WORLD_SIZE =
    LOCAL_WORLD_SIZE = n. Nothing here initialises the GPU, and the ranks are children, never an
    exec of this process. When a rank fails the others are given 30 s, then killed, so a peer
    stuck in a collective cannot hold the job.
    """
    import datetime
    import subprocess

    import torch.distributed as dist

    store = dist.TCPStore("127.0.0.1", 0, n, is_master=True, wait_for_workers=False,
                          timeout=datetime.timedelta(seconds=900))
    base = dict(os.environ if env is None else env)
    base.pop("FMLX_FORCE_PG", None)
    procs = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(store.port),
                 FMLX_STORE="127.0.0.1:%d" % store.port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=e))
    rc, t_end = 0, None if timeout is None else time.monotonic() + timeout
    try:
        live = list(procs)
        while live:
            for p in list(live):
                c = p.poll()
                if c is None:
                    continue
                live.remove(p)
                if c != 0 and rc == 0:
                    rc = c
                    grace = time.monotonic() + 30
                    t_end = grace if t_end is None else min(t_end, grace)
            if live and t_end is not None and time.monotonic() > t_end:
                for p in live:
                    p.kill()
                rc = rc or 124
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.wait()
        del store
    return 1 if rc < 0 else rc


def check_world(gpus: int, env=None) -> str:
    """'launch' (spawn ``gpus`` ranks), 'run' (this process is a rank), or raises SystemExit
    when the environment's WORLD_SIZE contradicts ``--gpus``."""
    env = os.environ if env is None else env
    if "WORLD_SIZE" not in env:
        return "launch" if gpus > 1 else "run"
    world = int(env["WORLD_SIZE"])
    if world != gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d (the launcher started a different number of ranks)"
                         % (gpus, world))
    return "run"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--rows", type=int, default=10_000_000, help="total dataset rows (sharded over GPUs)")
    ap.add_argument("--dim", type=int, default=1000)
    ap.add_argument("--batch", type=int, default=100_000,
                    help="minibatch rows: per GPU (--scaling weak) or global, split over the ranks (strong)")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"])
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32", "fp64"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check: every rank joins the process group, prints its rank/world/backend as "
                         "one JSON line and exits (runs on CPU)")
    ap.add_argument("--graph-rounds", type=int, default=0,
                    help="SGD rounds captured per hipGraph replay (0: the timed steps, at most 200, in one replay "
                         "— every graph is captured and primed before the clock starts)")
    ap.add_argument("--capture-after-data", action="store_true",
                    help="A/B: build the trainer and capture its graphs after generating the data (the GPU then "
                         "idles through the host-side capture right before the timed region)")
    ap.add_argument("--torch-profile", default="", help="after the timed region, record a torch.profiler trace of "
                                                        "extra rounds into this directory (not timed)")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if check_world(args.gpus) == "launch":
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    from flink_ml_amd.parallel.context import init_distributed
    from flink_ml_amd.parallel import comm

    ctx = init_distributed()
    world, rank = ctx.world_size, ctx.rank
    if ctx.is_distributed:
        import torch.distributed as dist

        if dist.get_world_size() != args.gpus and not ctx.forced:
            raise SystemExit("process group has %d ranks, --gpus %d" % (dist.get_world_size(), args.gpus))
    if args.dry_run:
        from flink_ml_amd.parallel import comm as _comm

        total = _comm.all_reduce_scalar(float(rank + 1), "sum") if ctx.is_distributed else 1.0
        print(json.dumps({"rank": rank, "world": world, "backend": ctx.backend if ctx.is_distributed else None,
                          "device": str(ctx.device), "rank_sum": total}), flush=True)
        return
    if ctx.device.type != "cuda":
        raise SystemExit("bench.py needs a GPU (torch.cuda.is_available() is False)")
    dev = ctx.device

    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer
    from flink_ml_amd.ops import glm as gk

    dt = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp64": torch.float64}[args.dtype]
    n_local = args.rows // world + (1 if args.rows % world > rank else 0)
    X = torch.empty((n_local, args.dim), dtype=dt, device=dev)
    # labels in the trainer's accumulation dtype, so the trainer aliases this tensor (no copy)
    y = torch.empty(n_local, dtype=torch.float64 if dt == torch.float64 else torch.float32, device=dev)

    def generate():
        # synthetic LabeledPointWithWeight data, generated directly in HBM in the compute dtype
        gen = torch.Generator(device=dev)
        gen.manual_seed(1234 + rank)
        chunk = 1 << 20
        for s in range(0, n_local, chunk):
            e = min(s + chunk, n_local)
            X[s:e] = torch.rand((e - s, args.dim), generator=gen, device=dev, dtype=torch.float32).to(dt)
        y.copy_(torch.randint(0, 2, (n_local,), generator=gen, device=dev))
        torch.cuda.synchronize()

    import numpy as np

    global_batch = args.batch * world if args.scaling == "weak" else args.batch

    # rounds the run executes: warm-up, one priming replay of every graph the timed region
    # replays (hipGraph upload / first-launch costs), the timed steps, plus one
    def make_trainer():
        sgd = SGD(max_iter=1, learning_rate=0.1, global_batch_size=global_batch, tol=1e-6)
        tr = DeviceGlmTrainer(sgd, np.zeros(args.dim), X, y, None, "logistic", use_graph=not args.no_graph)
        tr.rounds_per_graph = args.graph_rounds if args.graph_rounds > 0 else max(1, min(args.steps, 200))
        sgd.max_iter = args.warmup + tr.priming_rounds(args.steps) + args.steps + 1  # read at capture
        if args.torch_profile:
            sgd.max_iter += PROFILE_ROUNDS
        return tr

    if (world > 1 or ctx.forced) and not ctx.is_distributed:
        raise SystemExit("WORLD_SIZE=%d but the process group did not come up" % world)
    if args.capture_after_data:
        generate()
    trainer = make_trainer()
    if not args.capture_after_data:
        # set-up order: the trainer and its hipGraphs (host-side capture, milliseconds with the
        # GPU idle; kernels hold pointers, nothing reads the data) first, then the data generation,
        # so the GPU comes to the priming replay, the warm-up and the timed steps from sustained
        # load at its working clock rather than from the idle gap of the capture. The timed work is
        # the same either way (profiles/r4/lr_bench_setup_order_ab.log).
        trainer.precapture(args.steps)
        generate()
    if world > 1 and ctx.backend == "nccl" and trainer.xg is None and os.environ.get("FMLX_XGMI", "1") != "0":
        msg = "xGMI one-shot exchange did not come up (allocation, IPC mapping or self-test); rounds use RCCL"
        if os.environ.get("FMLX_REQUIRE_XGMI", "0") == "1":
            raise SystemExit(msg)
        if rank == 0:
            print("WARNING: " + msg, file=sys.stderr, flush=True)
    elapsed, kernel_s = timed_region(trainer, ctx, args.warmup, args.steps)
    # a bounded xGMI wait that gave up (a peer never arrived) means partial feedback: never
    # report it — re-time the same rounds on the RCCL path instead (decided on every rank)
    ok = trainer.xg is None or trainer.xg.healthy()
    if not comm.all_agree(ok):
        if rank == 0:
            print("xGMI exchange timed out; re-timing on the RCCL path", file=sys.stderr)
        from flink_ml_amd.parallel import xgmi

        xgmi.disable()  # every later device all-reduce (and check) goes to the process group
        trainer = make_trainer()
        trainer.use_rccl()
        elapsed, kernel_s = timed_region(trainer, ctx, args.warmup, args.steps)
    elapsed = comm.all_reduce_scalar(elapsed, "max")
    kernel_s = comm.all_reduce_scalar(kernel_s, "max")
    trainer.flush()  # untimed: deferred mode completes the last timed round in one more launch
    executed = trainer.rounds_executed()
    if executed < args.warmup + args.steps:
        raise SystemExit("SGD terminated early (%d rounds): timing would skip work" % executed)
    verified, vinfo = None, {}
    if ctx.is_distributed and world > 1:
        # the timed replicas must agree bitwise, and the exchange must equal the process-group
        # sum; otherwise re-time with the system-scope fences, and fail if that disagrees too
        final = comm.all_gather_tensor(trainer.coef[:trainer.d_model].double().cpu())
        same = comm.all_agree(all(torch.equal(final[0], c) for c in final))
        verified, vinfo = verify_exchange(make_trainer, comm)
        verified = verified and same
        vinfo["timed_replicas_identical"] = same
        if not verified and trainer.xg is not None:
            from flink_ml_amd.parallel import xgmi

            if rank == 0:
                print("exchange_verified: false (%s); re-timing with FMLX_XGMI_STRICT_FENCE=1" % vinfo,
                      file=sys.stderr, flush=True)
            xgmi.set_strict_fence(True)
            trainer = make_trainer()
            elapsed, kernel_s = timed_region(trainer, ctx, args.warmup, args.steps)
            elapsed = comm.all_reduce_scalar(elapsed, "max")
            kernel_s = comm.all_reduce_scalar(kernel_s, "max")
            trainer.flush()
            final = comm.all_gather_tensor(trainer.coef[:trainer.d_model].double().cpu())
            same = comm.all_agree(all(torch.equal(final[0], c) for c in final))
            verified, vinfo = verify_exchange(make_trainer, comm)
            verified = verified and same
            vinfo.update(timed_replicas_identical=same, strict_fence=True)
        if not verified and trainer.xg is not None:
            # the in-kernel exchange disagrees even with system-scope fences: time the process-group
            # path (feedback → RCCL all-reduce → update) instead and report THAT, verified the same
            # way — never the xGMI number
            from flink_ml_amd.parallel import xgmi

            if rank == 0:
                print("exchange_verified: false with the strict fence too (%s); re-timing on the RCCL path"
                      % vinfo, file=sys.stderr, flush=True)
            xgmi.disable()
            trainer = make_trainer()
            trainer.use_rccl()
            elapsed, kernel_s = timed_region(trainer, ctx, args.warmup, args.steps)
            elapsed = comm.all_reduce_scalar(elapsed, "max")
            kernel_s = comm.all_reduce_scalar(kernel_s, "max")
            trainer.flush()
            final = comm.all_gather_tensor(trainer.coef[:trainer.d_model].double().cpu())
            same = comm.all_agree(all(torch.equal(final[0], c) for c in final))
            verified, vinfo = verify_exchange(make_trainer, comm)
            verified = verified and same
            vinfo.update(timed_replicas_identical=same, xgmi_rejected=True)
        if not verified:
            if rank == 0:
                print(json.dumps({"exchange_verified": False, "detail": vinfo}), flush=True)
            raise SystemExit("bench.py: the cross-rank exchange disagrees with the process-group all-reduce")

    ms = elapsed / args.steps * 1e3
    samples = global_batch * args.steps
    value = samples / elapsed
    collective = "none" if not ctx.is_distributed else ("xgmi" if trainer.xg is not None else ctx.backend)
    if rank == 0:
        print("bench: world_size=%d backend=%s collective=%s gpus_per_device=%d scaling=%s"
              % (world, ctx.backend if ctx.is_distributed else "none", collective, ctx.sharers, args.scaling),
              file=sys.stderr, flush=True)
        rec = {
            "metric": "samples/sec (whole node), LogisticRegression 10M\u00d71K dense at 1/2/4/8 MI355X",
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "kernel_us_per_step": round(kernel_s / args.steps * 1e6, 2),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "exchange_verified": verified,
            "dtype": args.dtype,
            "data": "synthetic (device-generated U[0,1) features, Bernoulli labels; LabeledPointWithWeightGenerator shape)",
            "config": {
                "model": "LogisticRegression (SGD, binary logistic loss)",
                "global_batch": global_batch,
                "seq_len": None,
                "parallelism": "dp%d" % world,
                "rows": args.rows,
                "dim": args.dim,
                "per_gpu_batch": trainer.B if args.scaling == "weak" else global_batch / world,
                "world_size_observed": world,
                "backend": ctx.backend if ctx.is_distributed else None,
                "hipgraph": trainer.use_graph,
                "collective": collective,
                "collective_path": {1: "rccl all-reduce of the (d+2) feedback" if ctx.backend == "nccl" else
                                    "%s all-reduce of the (d+2) feedback" % ctx.backend,
                                    2: "none (1 GPU: the update is fused into the round kernel)",
                                    3: "in-kernel xgmi exchange"}[trainer.mode],
                "round": {1: "fused kernel + rccl all-reduce + update", 2: "one fused kernel",
                          3: "one fused kernel with in-kernel xgmi exchange"}[trainer.mode],
                "hbm_gb_per_s": round(trainer.B * args.dim * X.element_size() / (ms * 1e-3) / 1e9, 1),
                "exchange_check": vinfo or None,
            },
        }
        print(json.dumps(rec), flush=True)
    if args.torch_profile:
        from flink_ml_amd.utils import tracing

        with tracing.torch_profile(args.torch_profile):
            trainer.run_rounds(PROFILE_ROUNDS)
            torch.cuda.synchronize()


PROFILE_ROUNDS = 20

if __name__ == "__main__":
    main()
