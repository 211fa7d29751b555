"""Statistical hypothesis tests (reference ``LIB/stats/{anovatest,chisqtest,fvaluetest}``).

Each test reduces the rank's partition to fixed-size sufficient statistics on the device, then
one all-reduce combines them:

* ANOVATest — per-class feature sums as a one-hot GEMM (fp64, deterministic, no atomics) plus
  column sum / Σx²; F = MSB / MSW, p = 1 - F_cdf(F; C-1, N-C)  (``ANOVATest.java:120-200``).
* FValueTest — label/feature moments, then the centred cross-moment (y - ȳ)ᵀ(X - x̄) as one GEMV;
  corr² → F with (1, N-2) dof (``FValueTest.java:150-260``).
* ChiSqTest — per-feature contingency tables [#values, #labels] (on the GPU: the catstats
  kernels, across ranks one all-reduce of the table — ``catstats.global_value_label_counts``);
  Pearson statistic, dof = (V-1)(L-1), p-value and statistic rounded HALF_UP to 11
  decimals like ``ChiSqTest.java:440-455``.

Distribution CDFs come from scipy (commons-math3 in the reference).
"""
from __future__ import annotations

from decimal import ROUND_HALF_UP, Decimal
from typing import List, Tuple

import numpy as np
import torch
from scipy import stats as sps

from .. import config
from ..api.stage import AlgoOperator
from ..common.param import HasFeaturesCol, HasFlatten, HasLabelCol
from ..io import read_write as rw
from ..linalg.vectors import DenseVector
from ..ops import features as fo
from ..parallel import comm
from ..parallel import datastream as ds
from ..table import SparseColumn, Table
from .feature.common import get_world_distributed


def features_and_labels(t: Table, features_col: str, label_col: str,
                        keep_dtype: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
    """Dense features [n, d] (fp64, or the stored dtype on the GPU with ``keep_dtype`` — the
    reduction kernels accumulate in fp64 themselves) and fp64 labels on the compute device."""
    c = t.column(features_col)
    if isinstance(c, SparseColumn):
        X = c.to_dense(torch.float64, device=config.compute_device())
    else:
        X = config.features_for_compute(t, features_col, allow_sparse=False)
        if not (keep_dtype and X.device.type == "cuda"):
            X = X.to(torch.float64)
    lab = t.column(label_col)
    if isinstance(lab, list) and any(v is None for v in lab):
        raise ValueError("Input data must contain label value.")
    y = t.scalars(label_col, dtype=torch.float64, device=X.device)
    return X, y


def global_sorted_unique(v: torch.Tensor) -> torch.Tensor:
    """Sorted union of the ranks' distinct values (labels / categories): a keyed distinct over
    the values' bit patterns (all-to-all to the key owners, all-gather of their results)."""
    if v.is_cuda:
        from ..ops import catstats

        u = catstats.sorted_unique(v)  # native histogram / sorted distinct (no library sort)
        if get_world_distributed():
            # the ranks' distinct lists all-gathered and their union taken by the same native
            # distinct pass (no keyed shuffle, no library sort)
            u = catstats.sorted_unique(torch.cat([g.to(v.device) for g in comm.all_gather_tensor(u)]))
        return u.to(v.dtype)
    u = torch.unique(v)
    if get_world_distributed():
        k, _ = ds.global_distinct(ds.float_keys(u))
        u = torch.sort(ds.keys_to_float(k)).values.to(device=v.device, dtype=v.dtype)
    return u


def value_label_counts(X: torch.Tensor, li: torch.Tensor, L: int):
    """(feature, value, label) counts over all ranks as ONE keyed reduce — the keyed
    aggregations of ``ChiSqTest.java:127-130`` and ``NaiveBayes.java:95-103``: keys
    (j, value bits, label) are summed rank-locally, shuffled to their owner rank
    (``datastream.reduce_by_key_tensor``) and the owners' results gathered.

    Returns (vals, flat, Vn): per feature the sorted distinct values (float64 tensors), the
    counts as one flat float64 array with feature j's [V_j, L] block (value-major) at offset
    Σ_{i<j} V_i·L, and V_j per feature."""
    n, d = X.shape
    dev = X.device
    jj = torch.arange(d, device=dev, dtype=torch.int64)[None, :].expand(n, d)
    keys = torch.stack([jj, ds.float_keys(X).reshape(n, d), li.to(torch.int64)[:, None].expand(n, d)], -1)
    uk, cnt = ds.global_distinct(keys.reshape(-1, 3))
    jb, inv = torch.unique(uk[:, :2], dim=0, return_inverse=True)
    fl = ds.keys_to_float(jb[:, 1])
    o1 = torch.argsort(fl, stable=True)
    o2 = o1[torch.argsort(jb[o1, 0], stable=True)]  # (feature, value) order
    U = jb.shape[0]
    rank = torch.empty(U, dtype=torch.int64, device=uk.device)
    rank[o2] = torch.arange(U, device=uk.device)
    Vn = torch.bincount(jb[:, 0], minlength=d)
    start = torch.cumsum(Vn, 0) - Vn
    vidx = rank[inv] - start[uk[:, 0]]
    flat = torch.zeros(U * L, dtype=torch.float64, device=uk.device)
    flat[(start[uk[:, 0]] + vidx) * L + uk[:, 2]] = cnt.to(torch.float64)
    vals = list(torch.split(fl[o2], Vn.tolist())) if d else []
    return [v.to(dev) for v in vals], flat.cpu().numpy(), Vn.cpu().numpy()


def class_sums(X: torch.Tensor, ci: torch.Tensor, C: int, chunk: int = 1 << 20) -> torch.Tensor:
    """Σ rows of X per class as onehotᵀ·X in fp64 row chunks (deterministic, MFMA/BLAS path)."""
    out = torch.zeros((C, X.shape[1]), dtype=torch.float64, device=X.device)
    ar = torch.arange(C, device=X.device)
    for s in range(0, X.shape[0], chunk):
        oh = (ci[s:s + chunk, None] == ar[None, :]).to(torch.float64)
        out += oh.t() @ X[s:s + chunk]
    return out


def _reduce(t: torch.Tensor) -> torch.Tensor:
    return comm.all_reduce_sum(t) if get_world_distributed() else t


def _result_table(idx_name: str, stat_name: str, flat_names, p, dof, stat, flatten: bool, dof_kind=int) -> Table:
    d = len(p)
    if flatten:
        return Table({flat_names[0]: torch.arange(d, dtype=torch.int64), flat_names[1]: torch.tensor(p, dtype=torch.float64),
                      flat_names[2]: torch.tensor(dof, dtype=torch.int64), flat_names[3]: torch.tensor(stat, dtype=torch.float64)},
                     num_rows=d).as_replicated()
    return Table({idx_name: [DenseVector(np.asarray(p, dtype=np.float64))],
                  "degreesOfFreedom": [[dof_kind(x) for x in dof]],
                  stat_name: [DenseVector(np.asarray(stat, dtype=np.float64))]}, num_rows=1).as_replicated()


class _TestParams(HasFeaturesCol, HasLabelCol, HasFlatten):
    pass


@rw.register_stage
class ANOVATest(AlgoOperator, _TestParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.stats.anovatest.ANOVATest"

    def compute(self, t: Table):
        X, y = features_and_labels(t, self.get(self.FEATURES_COL), self.get(self.LABEL_COL), keep_dtype=True)
        cls = global_sorted_unique(y)
        C, d = cls.numel(), X.shape[1]
        ci = torch.searchsorted(cls, y)
        if C <= fo.MAX_GROUPS:
            S, tot, totsq = fo.group_colstats(X, ci, C)
        else:
            Xd = X.to(torch.float64)
            S, tot, totsq = class_sums(Xd, ci, C), Xd.sum(0), (Xd * Xd).sum(0)
        if ci.is_cuda:
            from ..ops import catstats

            cls_n = catstats.label_counts(ci, C).to(torch.float64)
        else:
            cls_n = torch.bincount(ci, minlength=C).to(torch.float64)
        packed = torch.cat([S.reshape(-1), cls_n, tot, totsq])
        packed = _reduce(packed).cpu().numpy()
        S = packed[:C * d].reshape(C, d)
        cnt = packed[C * d:C * d + C]
        tot, totsq = packed[C * d + C:C * d + C + d], packed[C * d + C + d:]
        n = cnt.sum()
        dfb, dfw = C - 1, int(n) - C
        if dfb <= 0:
            raise ValueError("Num of classes should be positive.")
        if dfw <= 0:
            raise ValueError("Num of samples should be greater than num of classes.")
        with np.errstate(invalid="ignore", divide="ignore"):
            sq = tot * tot
            ss_tot = totsq - sq / n
            between = (S * S / cnt[:, None]).sum(0) - sq / n
            within = ss_tot - between
            f = (between / dfb) / (within / dfw)
            p = 1.0 - sps.f.cdf(f, dfb, dfw)
        return p, [dfb + dfw] * d, f

    def transform(self, *inputs):
        p, dof, f = self.compute(inputs[0])
        return [_result_table("pValues", "fValues", ("featureIndex", "pValue", "degreeOfFreedom", "fValue"), p, dof, f,
                              self.get(self.FLATTEN))]


@rw.register_stage
class FValueTest(AlgoOperator, _TestParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.stats.fvaluetest.FValueTest"

    def compute(self, t: Table):
        X, y = features_and_labels(t, self.get(self.FEATURES_COL), self.get(self.LABEL_COL), keep_dtype=True)
        d = X.shape[1]
        ym = _reduce(torch.stack([torch.tensor(float(y.numel()), dtype=torch.float64, device=y.device), y.sum(),
                                  (y * y).sum()]))
        n = float(ym[0])
        my = ym[1] / n
        sy = torch.sqrt((ym[2] / n - my * my) * n / (n - 1))
        yc = y - my
        S, sx_, sxx = fo.group_colstats(X, None, 1, yc)
        mom = _reduce(torch.cat([S[0], yc.sum()[None], sx_, sxx]))
        mx = mom[d + 1:2 * d + 1] / n
        sx = torch.sqrt((mom[2 * d + 1:] / n - mx * mx) * n / (n - 1))
        # Σ (y-ȳ)(x-x̄) = Σ (y-ȳ)x − x̄ Σ (y-ȳ)
        cov = (mom[:d] - mx * mom[d]) / (n - 1)
        dof = int(n) - 2
        corr = cov / (sy * sx)
        f = (corr * corr / (1 - corr * corr) * dof).cpu().numpy()
        with np.errstate(invalid="ignore"):
            p = 1.0 - sps.f.cdf(f, 1, dof)
        return p, [dof] * d, f

    def transform(self, *inputs):
        p, dof, f = self.compute(inputs[0])
        return [_result_table("pValues", "fValues", ("featureIndex", "pValue", "degreeOfFreedom", "fValue"), p, dof, f,
                              self.get(self.FLATTEN))]


def _round11(v: float) -> float:
    if v != v or v in (float("inf"), float("-inf")):
        return v
    return float(Decimal(v).quantize(Decimal("1e-11"), rounding=ROUND_HALF_UP))


@rw.register_stage
class ChiSqTest(AlgoOperator, _TestParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.stats.chisqtest.ChiSqTest"

    def compute(self, t: Table):
        X, y = features_and_labels(t, self.get(self.FEATURES_COL), self.get(self.LABEL_COL), keep_dtype=True)
        labels = global_sorted_unique(y)
        L, d = labels.numel(), X.shape[1]
        li = torch.searchsorted(labels, y)
        if X.is_cuda:
            # native contingency tables (ops/catstats.py: integer table or sorted-column distinct;
            # across ranks one all-reduce of the table, after a union of the ranks' value lists)
            from ..ops import catstats

            if get_world_distributed():
                counts, vals_np, slots = catstats.global_value_label_counts(X, li.to(torch.int32), L)
            else:
                counts, vals_np, slots = catstats.value_label_counts(X, li, L)
            vals = [torch.as_tensor(v) for v in vals_np]
            flat = np.concatenate([counts[j][:, slots[j]].T.reshape(-1) for j in range(d)]).astype(np.float64) \
                if d else np.zeros(0)
        elif get_world_distributed():
            # (CPU ranks) distinct values and contingency counts in one keyed shuffle
            vals, flat, _ = value_label_counts(X.to(torch.float64), li, L)
        else:
            vals = [torch.unique(X[:, j]) for j in range(d)]
            tables = []
            for j in range(d):
                vi = torch.searchsorted(vals[j], X[:, j].contiguous())
                tables.append(torch.bincount(vi * L + li, minlength=vals[j].numel() * L).to(torch.float64))
            flat = torch.cat(tables).cpu().numpy() if tables else np.zeros(0)
        p_out, dof_out, stat_out, off = [], [], [], 0
        for j in range(d):
            V = vals[j].numel()
            obs = flat[off:off + V * L].reshape(V, L)
            off += V * L
            n = obs.sum()
            exp = np.outer(obs.sum(1), obs.sum(0)) / n
            stat = float(((obs - exp) ** 2 / exp).sum())
            dof = (V - 1) * (L - 1)
            if dof == 0:
                stat, p = 0.0, 1.0
            else:
                p = 1.0 - float(sps.chi2.cdf(stat, dof))
            p_out.append(_round11(p))
            dof_out.append(dof)
            stat_out.append(_round11(stat))
        return p_out, dof_out, stat_out

    def transform(self, *inputs):
        p, dof, s = self.compute(inputs[0])
        return [_result_table("pValues", "statistics", ("featureIndex", "pValue", "degreeOfFreedom", "statistic"), p,
                              dof, s, self.get(self.FLATTEN))]
