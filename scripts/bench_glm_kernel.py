#!/usr/bin/env python3
"""A/B of SGD-round configurations in ONE process with interleaved repetitions
(cdna_hip_programming.md §5.4 rule 24): µs per round of the flagship shape for each variant.

Variants: ``u`` (rows in flight per wave = 2u), ``b`` (blocks = partial rows), ``split``
(legacy 3-launch round: grad partials → stage-1 → reduce+update) vs the fused one-launch round,
``defer`` (0: ticketed atomic tail; 1: round e − 1 completed in launch e's prologue), ``dma``
(LDS-DMA row ring depth in steps, 0 = register loads).
Usage: python scripts/bench_glm_kernel.py --configs "u=2,b=512;u=4,b=256;split=1"
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer  # noqa: E402
from flink_ml_amd.ops import glm as gk  # noqa: E402


def parse(cfgs):
    out = []
    for c in cfgs.split(";"):
        d = dict(kv.split("=") for kv in c.split(",") if kv)
        out.append({k: int(v) for k, v in d.items()})
    return out


class SplitTrainer(DeviceGlmTrainer):
    """The pre-fusion round: 3 launches (kept for the A/B)."""

    def _launch_round(self, rounds=1):
        for _ in range(rounds):
            self._split_round()

    def _split_round(self):
        s = self.sgd
        sc = self.scratch
        gk.grad_partials(self.X, self.y, self.w, self.coef, self.B, self.loss, self.state, sc.partials, sc.nparts)
        if self.mode0_only:
            return
        gk.reduce_update(sc.partials, sc.nparts, self.d, sc.stage1, self.coef, self.feedback, self.state, s.max_iter,
                         s.tol, s.learning_rate, s.reg, s.elastic_net)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--dim", type=int, default=1000)
    ap.add_argument("--batch", type=int, default=100_000)
    ap.add_argument("--rounds", type=int, default=200)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--ld", type=int, default=0, help="row pitch in elements (0: dense rows)")
    ap.add_argument("--configs", default="u=2,b=512;u=1,b=512;u=4,b=512;u=2,b=256;u=4,b=256;split=1")
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(1)
    ld = a.ld if a.ld > 0 else a.dim
    X = torch.empty((a.rows, ld), dtype=torch.bfloat16, device=dev)[:, :a.dim]
    for s in range(0, a.rows, 1 << 20):
        e = min(s + (1 << 20), a.rows)
        X[s:e] = torch.rand((e - s, a.dim), generator=g, device=dev).to(torch.bfloat16)
    y = torch.randint(0, 2, (a.rows,), generator=g, device=dev).float()
    cfgs = parse(a.configs)
    res = {json.dumps(c): [] for c in cfgs}
    for rep in range(a.reps):
        for c in cfgs:
            gk.GRAD_UNROLL = c.get("u", 0)
            gk.GRAD_BLOCKS = c.get("b", 512)
            gk.set_tuning(c.get("pad", -1), c.get("nt", -1))
            gk.DETERMINISTIC = bool(c.get("det", 0))
            gk.DEFER = bool(c.get("defer", 1))
            gk.set_tail_tuning(c.get("reps", 4), bool(c.get("t2", 0)))
            gk.set_dma(c.get("dma", 0))
            sgd = SGD(max_iter=10 ** 8, learning_rate=0.1, global_batch_size=a.batch, tol=0.0)
            cls = SplitTrainer if (c.get("split") or c.get("m0")) else DeviceGlmTrainer
            tr = cls(sgd, np.zeros(a.dim), X, y, None, "logistic", use_graph=True)
            tr.mode0_only = bool(c.get("m0"))
            if cls is SplitTrainer:  # the split round needs the block-partials scratch
                tr.scratch = gk.RoundScratch(tr.nparts, a.dim, torch.float32, dev, det=True)
                tr.defer, tr.cw = False, None
            tr.rounds_per_graph = c.get("R", 10)
            tr.run_rounds(20)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tr.run_rounds(a.rounds)
            torch.cuda.synchronize()
            us = (time.perf_counter() - t0) / a.rounds * 1e6
            # deferred rounds: the last launch's round completes in the next launch
            assert c.get("m0") or tr.rounds_executed() == 20 + a.rounds - int(tr.defer)
            res[json.dumps(c)].append(us)
    gb = a.batch * a.dim * 2 / 1e9
    for k, v in res.items():
        med = statistics.median(v)
        print(json.dumps({"config": json.loads(k), "ld": ld, "us_per_round_median": round(med, 2),
                          "us_min": round(min(v), 2), "samples_per_s": round(a.batch / med * 1e6),
                          "batch_TB_per_s": round(gb / med * 1e6 / 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
