"""BinaryClassificationEvaluator (reference ``LIB/evaluation/binaryclassification``).

The reference range-partitions the scores (sampled boundaries), sorts every partition, exchanges
per-partition summaries and then computes, in one pass over the descending scores,
AUC by the tie-averaged rank sum and the trapezoid sums for area under PR and Lorenz curves plus
KS (``BinaryClassificationEvaluator.java:103-460``).

MI355X-native version of the same plan (K21):
* range partition = sampled boundaries + a stable counting sort of the rows by target rank
  (``groupsort.hip``) + one ``all_to_all_v`` of (score, label, weight);
* local descending sort on the device: a stable LSD radix sort of 64-bit score keys over only the
  bits that differ (``radix.hip``; ties keep arrival order as in the reference);
* the per-partition summaries are an all-gather of two counts;
* every metric comes out of one scan of the sorted rows (``binclass.hip``: cumulative TP/FP,
  tie-group bounds for the averaged AUC ranks, PR / Lorenz trapezoids, KS max, fixed-order
  partial sums) and the partial sums / max are all-reduced.
The torch formulation below (``cumsum`` / ``unique_consecutive``) is the CPU reference.
"""
from __future__ import annotations

import math
from typing import List

import numpy as np
import torch

from .. import config
from ..api.stage import AlgoOperator
from ..common.param import HasLabelCol, HasRawPredictionCol, HasWeightCol
from ..io import read_write as rw
from ..param.param import ParamValidators, StringArrayParam
from ..parallel import comm
from ..table import SparseColumn, Table
from .feature.common import get_world_distributed

AREA_UNDER_ROC, AREA_UNDER_PR, AREA_UNDER_LORENZ, KS = "areaUnderROC", "areaUnderPR", "areaUnderLorenz", "ks"
NUM_SAMPLE_FOR_RANGE_PARTITION = 100


def parse_samples(t: Table, label_col: str, raw_col: str, weight_col):
    """(score, isPositive, weight) on the compute device (``ParseSample``)."""
    dev = config.compute_device()
    c = t.column(raw_col)
    if isinstance(c, torch.Tensor):
        score = (c[:, 1] if c.dim() == 2 else c).to(dev, torch.float64)
    elif isinstance(c, SparseColumn):
        score = c.to_dense(torch.float64, device=dev)[:, 1]
    else:
        score = torch.tensor([float(v.get(1)) if hasattr(v, "get") else float(v) for v in c], dtype=torch.float64,
                             device=dev)
    pos = t.scalars(label_col, dtype=torch.float64, device=dev) == 1.0
    w = t.scalars(weight_col, dtype=torch.float64, device=dev) if weight_col else torch.ones_like(score)
    return score, pos, w


def _range_partition(score, pos, w):
    """Sample boundaries like ``getBoundaryRange`` and route rows so that rank r holds the r-th
    score range (higher rank = higher scores); returns this rank's rows."""
    from ..parallel.context import get_context

    ctx = get_context()
    n = score.numel()
    g = torch.Generator().manual_seed(1234567 + ctx.rank)
    if n:
        samp = score.cpu()[torch.randint(0, n, (NUM_SAMPLE_FOR_RANGE_PARTITION,), generator=g)]
    else:
        samp = torch.full((NUM_SAMPLE_FOR_RANGE_PARTITION,), float(np.finfo(np.float64).max), dtype=torch.float64)
    allsamp = torch.sort(torch.cat(comm.all_gather_tensor(samp))).values
    bounds = allsamp[torch.arange(ctx.world_size) * NUM_SAMPLE_FOR_RANGE_PARTITION].to(score.device)
    # part = max i > 0 with score > bounds[i], else 0 (AppendTaskId)
    part = torch.clamp(torch.searchsorted(bounds, score, right=False) - 1, min=0)
    part = torch.where(score > bounds[0], part, torch.zeros_like(part))
    if score.is_cuda:
        from ..ops.kmeans import group_by_key

        order, offsets, _ = group_by_key(part, ctx.world_size, stable=True)  # groupsort.hip counting sort
        counts = torch.diff(offsets).cpu().tolist()
    else:
        order = torch.argsort(part, stable=True)
        counts = torch.bincount(part, minlength=ctx.world_size).cpu().tolist()
    packed = torch.stack([score, pos.to(torch.float64), w], dim=1)[order]
    chunks = list(torch.split(packed, counts))
    recv = comm.all_to_all_v(chunks)
    got = torch.cat([r.to(score.device) for r in recv]) if recv else packed[:0]
    return got[:, 0], got[:, 1] > 0.5, got[:, 2]


def compute_metrics(score: torch.Tensor, pos: torch.Tensor, w: torch.Tensor) -> dict:
    dist = get_world_distributed()
    if dist:
        score, pos, w = _range_partition(score, pos, w)
    if score.is_cuda:
        return _device_metrics(score.contiguous(), pos, w, dist)
    order = torch.argsort(-score, stable=True)
    s, p, wt = score[order], pos[order], w[order]
    n_pos, n_neg = int(p.sum()), int((~p).sum())
    if dist:
        from ..parallel.context import get_context

        ctx = get_context()
        summ = comm.all_gather_object((n_pos, n_neg))
        before_t = sum(summ[r][0] for r in range(ctx.rank + 1, ctx.world_size))
        before_f = sum(summ[r][1] for r in range(ctx.rank + 1, ctx.world_size))
        tot_t = sum(x[0] for x in summ)
        tot_f = sum(x[1] for x in summ)
    else:
        before_t = before_f = 0
        tot_t, tot_f = n_pos, n_neg
    total = tot_t + tot_f
    dev = s.device
    n = s.numel()
    # ---- AUC: tie groups get their average ascending rank (AccumulateMultiScoreOperator)
    if n:
        ranks = (total - (before_t + before_f) - torch.arange(n, device=dev)).to(torch.float64)
        _, inv, cnt = torch.unique_consecutive(s, return_inverse=True, return_counts=True)
        G = cnt.numel()
        rsum = torch.zeros(G, dtype=torch.float64, device=dev).index_add_(0, inv, ranks)
        pw = torch.zeros(G, dtype=torch.float64, device=dev).index_add_(0, inv, torch.where(p, wt, torch.zeros_like(wt)))
        nw = torch.zeros(G, dtype=torch.float64, device=dev).index_add_(0, inv, torch.where(p, torch.zeros_like(wt), wt))
        auc_parts = torch.stack([(rsum / cnt.to(torch.float64) * pw).sum(), pw.sum(), nw.sum()])
    else:
        auc_parts = torch.zeros(3, dtype=torch.float64, device=dev)
    # ---- PR / Lorenz / KS: prefix sums of unweighted counts (updateBinaryMetrics)
    if n:
        cp = before_t + torch.cumsum(p.to(torch.float64), 0)
        cn = before_f + torch.cumsum((~p).to(torch.float64), 0)
        cp0 = torch.cat([torch.tensor([float(before_t)], dtype=torch.float64, device=dev), cp[:-1]])
        cn0 = torch.cat([torch.tensor([float(before_f)], dtype=torch.float64, device=dev), cn[:-1]])

        def rates(a, b):
            tpr = a / tot_t if tot_t else torch.ones_like(a)
            fpr = b / tot_f if tot_f else torch.ones_like(b)
            prec = torch.where(a + b == 0, torch.ones_like(a), a / torch.clamp(a + b, min=1))
            prate = (a + b) / total
            return tpr, fpr, prec, prate

        tpr, fpr, prec, prate = rates(cp, cn)
        tpr0, _, prec0, prate0 = rates(cp0, cn0)
        lorenz = ((prate - prate0) * (tpr + tpr0) / 2).sum()
        pr = ((tpr - tpr0) * (prec + prec0) / 2).sum()
        ks = torch.abs(fpr - tpr).max()
    else:
        lorenz = pr = ks = torch.zeros((), dtype=torch.float64, device=dev)
    sums = torch.cat([auc_parts, torch.stack([lorenz, pr])])
    if dist:
        sums = comm.all_reduce_sum(sums)
        ks = comm.all_reduce(ks.reshape(1).clone(), "max")[0]
    acc, P, N, lorenz, pr = sums.cpu().tolist()
    auc = (acc - P * (P + 1) / 2) / (P * N) if P > 0 and N > 0 else float("nan")
    return {AREA_UNDER_ROC: auc, AREA_UNDER_PR: pr, AREA_UNDER_LORENZ: lorenz, KS: float(ks)}


def _device_metrics(score: torch.Tensor, pos: torch.Tensor, w: torch.Tensor, dist: bool) -> dict:
    """The same metrics through the native sort + scan (ops/sorting.py)."""
    from ..ops import sorting

    n = score.numel()
    n_pos = int(pos.sum()) if n else 0
    n_neg = n - n_pos
    before_t = before_f = 0
    tot_t, tot_f = n_pos, n_neg
    if dist:
        from ..parallel.context import get_context

        ctx = get_context()
        summ = comm.all_gather_object((n_pos, n_neg))
        before_t = sum(summ[r][0] for r in range(ctx.rank + 1, ctx.world_size))
        before_f = sum(summ[r][1] for r in range(ctx.rank + 1, ctx.world_size))
        tot_t = sum(x[0] for x in summ)
        tot_f = sum(x[1] for x in summ)
    total = tot_t + tot_f
    keys, rows = sorting.sort_scores_desc(score, pos)
    unit = bool((w == 1).all()) if n else True
    m = sorting.binary_metrics(keys, rows, None if unit else w, before_t, before_f, tot_t, tot_f)
    # Σ_g avg_rank_g·PW_g with avg_rank = total − before − (gs + ge)/2 (local positions gs..ge)
    sums = torch.stack([(total - before_t - before_f) * m[1] - 0.5 * m[0], m[1], m[2], m[3], m[4]])
    ks = m[5]
    if dist:
        sums = comm.all_reduce_sum(sums)
        ks = comm.all_reduce(ks.reshape(1).clone(), "max")[0]
    acc, P, N, lorenz, pr = sums.cpu().tolist()
    auc = (acc - P * (P + 1) / 2) / (P * N) if P > 0 and N > 0 else float("nan")
    return {AREA_UNDER_ROC: auc, AREA_UNDER_PR: pr, AREA_UNDER_LORENZ: lorenz, KS: float(ks)}


@rw.register_stage
class BinaryClassificationEvaluator(AlgoOperator, HasLabelCol, HasRawPredictionCol, HasWeightCol):
    JAVA_CLASS_NAME = "org.apache.flink.ml.evaluation.binaryclassification.BinaryClassificationEvaluator"
    AREA_UNDER_ROC, AREA_UNDER_PR, AREA_UNDER_LORENZ, KS = AREA_UNDER_ROC, AREA_UNDER_PR, AREA_UNDER_LORENZ, KS
    METRICS_NAMES = StringArrayParam("metricsNames", "Names of output metrics.", (AREA_UNDER_ROC, AREA_UNDER_PR),
                                     ParamValidators.is_sub_set(AREA_UNDER_ROC, AREA_UNDER_PR, KS, AREA_UNDER_LORENZ))

    def transform(self, *inputs) -> List[Table]:
        score, pos, w = parse_samples(inputs[0], self.get(self.LABEL_COL), self.get(self.RAW_PREDICTION_COL),
                                      self.get(self.WEIGHT_COL))
        m = compute_metrics(score, pos, w)
        names = self.get(self.METRICS_NAMES)
        return [Table({k: torch.tensor([m[k]], dtype=torch.float64) for k in names}, num_rows=1).as_replicated()]
