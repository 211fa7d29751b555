"""NaiveBayes / NaiveBayesModel, multinomial over categorical feature values
(reference ``LIB/classification/naivebayes/{NaiveBayes,NaiveBayesModel,NaiveBayesModelData}.java``).

fit: the per-(label, feature, value) counts the reference builds with two keyed mapPartitions
(C11/K22) are, per feature column, one ``bincount`` over (value-index, label-index) on the device;
the tables of all columns are all-reduced in one call. Then, as in ``GenerateModelFunction``:

    theta[l][j][v] = log(count(l, j, v) + s) − log(n_l + s·|V_j|)
    pi[l]          = log(n_l·d + s) − log(n·d + L·s)

predict: every feature value becomes a column index into one flattened [L, ΣV_j] log-probability
table, so a block of rows is a single gather + sum over features; argmax with the reference's
first-max rule. An unseen feature value raises (the reference fails with an NPE).
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np
import torch

from .. import config
from ..api.stage import Estimator
from ..common.param import HasFeaturesCol, HasLabelCol, HasPredictionCol
from ..io import read_write as rw
from ..io import serialization as ser
from ..linalg.vectors import DenseVector
from ..param.param import FloatParam, ParamValidators, StringParam
from ..parallel import comm
from ..table import SparseColumn, Table
from ..utils.java import java_double_hash, java_hashmap_order
from .base import ModelWithData
from .feature.common import get_world_distributed
from .linear import rw_update
from .stats import features_and_labels, global_sorted_unique, value_label_counts


class NaiveBayesModelParams(HasFeaturesCol, HasPredictionCol):
    MODEL_TYPE = StringParam("modelType", "The model type.", "multinomial", ParamValidators.in_array("multinomial"))


class NaiveBayesParams(NaiveBayesModelParams, HasLabelCol):
    SMOOTHING = FloatParam("smoothing", "The smoothing parameter.", 1.0, ParamValidators.gt_eq(0.0))


def _ordered(m: Dict[float, float]) -> Dict[float, float]:
    return {k: m[k] for k in java_hashmap_order(list(m.keys()), java_double_hash)}


@rw.register_stage
class NaiveBayesModel(ModelWithData, NaiveBayesModelParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.classification.naivebayes.NaiveBayesModel"
    MODEL_DATA_COLUMNS = ("theta", "piArray", "labels")

    @staticmethod
    def encode_record(out, row):
        theta, pi, labels = row
        ser.write_dense_vector(out, labels)
        ser.write_dense_vector(out, pi)
        out.write_int(len(theta))
        out.write_int(len(theta[0]))
        for maps in theta:
            for m in maps:
                ser.write_map(out, _ordered(m), lambda o, k: o.write_double(k), lambda o, v: o.write_double(v))

    @staticmethod
    def decode_record(inp):
        labels = ser.read_dense_vector(inp)
        pi = ser.read_dense_vector(inp)
        nl, nf = inp.read_int(), inp.read_int()
        theta = [[ser.read_map(inp, lambda i: i.read_double(), lambda i: i.read_double()) for _ in range(nf)]
                 for _ in range(nl)]
        return (theta, pi, labels)

    @classmethod
    def make_model_data_table(cls, rows):
        return Table({"theta": [r[0] for r in rows], "piArray": [r[1] for r in rows], "labels": [r[2] for r in rows]},
                     num_rows=len(rows))

    def _build_state(self, rows):
        theta, pi, labels = rows[0]
        dev = config.compute_device()
        nl, nf = len(theta), len(theta[0])
        vals, offs, flat_cols = [], [0], []
        for j in range(nf):
            v = sorted(theta[0][j].keys())
            vals.append(torch.tensor(v, dtype=torch.float64, device=dev))
            flat_cols.append(np.array([[theta[i][j].get(x, np.nan) for x in v] for i in range(nl)]).reshape(nl, -1))
            offs.append(offs[-1] + len(v))
        table = torch.from_numpy(np.concatenate(flat_cols, axis=1) if flat_cols else np.zeros((nl, 0))).to(dev)
        return (vals, torch.tensor(offs[:-1], dtype=torch.int64, device=dev), table,
                torch.as_tensor(np.asarray(pi.values), device=dev), torch.as_tensor(np.asarray(labels.values),
                                                                                   device=dev))

    def transform(self, *inputs):
        t = inputs[0]
        vals, offs, table, pi, labels = self._model_state()
        c = t.column(self.get(self.FEATURES_COL))
        X = c.to_dense(torch.float64, device=table.device) if isinstance(c, SparseColumn) else \
            config.features_for_compute(t, self.get(self.FEATURES_COL), allow_sparse=False).to(table.device,
                                                                                                torch.float64)
        n, d = X.shape
        if d > len(vals):
            raise ValueError("The input vector has %d features, the model has %d." % (d, len(vals)))
        cols = torch.empty((n, d), dtype=torch.int64, device=X.device)
        for j in range(d):
            pos = torch.clamp(torch.searchsorted(vals[j], X[:, j].contiguous()), max=vals[j].numel() - 1)
            if not bool((vals[j][pos] == X[:, j]).all()):
                raise RuntimeError("Feature %d of the input contains a value unseen in training." % j)
            cols[:, j] = offs[j] + pos
        probs = table[:, cols].sum(dim=2).t() + pi[None, :] if d else pi[None, :].expand(n, -1)
        pred = labels[torch.argmax(probs, dim=1)]  # first max, like findMaxProbLabel
        return [t.with_column(self.get(self.PREDICTION_COL), pred.to(torch.float64))]


def _label_value_counts(X: torch.Tensor, li: torch.Tensor, L: int, dist: bool):
    """Per (feature, label, distinct value) counts (NaiveBayes.java:97-200's three keyed
    aggregations) as one device histogram. Returns counts [d, L, Vmax] (numpy), per-feature sorted
    distinct values and their slots in the last axis, and per-label row counts.

    Small non-negative integer features (the categorical case) index the histogram directly
    (one all-reduce of the dense histogram across ranks); anything else goes through one
    column-wise sort + batched searchsorted on one rank, and through the keyed (feature, value,
    label) shuffle of ``stats.value_label_counts`` across ranks."""
    n, d = X.shape
    dev = X.device
    if X.is_cuda:
        return _label_value_counts_device(X, li, L, dist)
    n_lab = torch.bincount(li, minlength=L).to(torch.float64)
    if n:
        flags = torch.stack([-X.min(), X.max(), (X != torch.round(X)).any().to(X.dtype)]).to(torch.float64)
    else:
        flags = torch.tensor([-0.0, -1.0, 0.0], dtype=torch.float64, device=dev)
    if dist:
        flags = comm.all_reduce(flags, "max")
    neg_min, vmax_f, non_int = flags.tolist()
    if non_int == 0 and -neg_min >= 0 and (vmax_f + 1) * L * d <= (1 << 27):
        Vmax = int(vmax_f) + 1
        jj = torch.arange(d, device=dev, dtype=torch.int64)[None, :]
        key = (jj * L + li[:, None]) * Vmax + X.to(torch.int64)
        cnt = torch.bincount(key.reshape(-1), minlength=d * L * Vmax).to(torch.float64)
        if dist:
            both = comm.all_reduce_sum(torch.cat([cnt, n_lab]))
            cnt, n_lab = both[:-L], both[-L:]
        counts = cnt.reshape(d, L, Vmax).cpu().numpy()
        present = counts.sum(1) > 0
        slots = [np.nonzero(present[j])[0] for j in range(d)]
        return counts, [sl.astype(np.float64) for sl in slots], slots, n_lab.cpu().numpy()
    if dist:
        # (feature, value, label) counts and the distinct values in one keyed shuffle
        vals_t, flat, Vn = value_label_counts(X, li, L)
        Vmax = max(1, int(Vn.max()) if d else 1)
        counts = np.zeros((d, L, Vmax), dtype=np.float64)
        off = 0
        for j in range(d):
            V = int(Vn[j])
            counts[j, :, :V] = flat[off:off + V * L].reshape(V, L).T
            off += V * L
        n_lab = comm.all_reduce_sum(n_lab)
        return (counts, [v.cpu().numpy() for v in vals_t], [np.arange(int(Vn[j])) for j in range(d)],
                n_lab.cpu().numpy())
    Xt = X.t().contiguous()
    S = torch.sort(Xt, dim=1).values if n else Xt
    start = torch.ones_like(S, dtype=torch.bool)
    if n > 1:
        start[:, 1:] = S[:, 1:] != S[:, :-1]
    pos = torch.cumsum(start.to(torch.int64), dim=1) - 1
    Vn = (pos[:, -1] + 1).cpu().numpy() if n else np.zeros(d, dtype=np.int64)
    Vmax = max(1, int(Vn.max()) if d else 1)
    table = torch.full((d, Vmax), float("inf"), dtype=torch.float64, device=dev)
    # every element of a run writes the same value to its slot; padding stays +inf
    table.scatter_(1, pos, S.to(torch.float64))
    codes = torch.searchsorted(table, Xt.to(torch.float64))
    jj = torch.arange(d, device=dev, dtype=torch.int64)[:, None]
    key = (jj * L + li[None, :]) * Vmax + codes
    cnt = torch.bincount(key.reshape(-1), minlength=d * L * Vmax).to(torch.float64)
    table_np = table.cpu().numpy()
    slots = [np.arange(int(Vn[j])) for j in range(d)]
    return (cnt.reshape(d, L, Vmax).cpu().numpy(), [table_np[j, :int(Vn[j])] for j in range(d)], slots,
            n_lab.cpu().numpy())


def _label_value_counts_device(X: torch.Tensor, li: torch.Tensor, L: int, dist: bool):
    """``_label_value_counts`` through the native contingency kernels (ops/catstats.py): integer
    features with a table of at most 2^27 cells (the categorical case; value range from the global
    min / max) are counted by one pass of ``cs_hist`` into [d, L, V] and all-reduced as one dense
    table; other values take the sorted-column distinct pass on one rank and the keyed shuffle of
    ``catstats.global_value_label_counts`` (native union of the ranks' value lists) across ranks."""
    from ..ops import catstats

    n, d = X.shape
    dev = X.device
    n_lab = catstats.label_counts(li, L).to(torch.float64)
    mn, mx, non = catstats.flags(X) if n else (float("inf"), float("-inf"), False)
    if dist:
        f = comm.all_reduce(torch.tensor([-mn, mx, float(non)], dtype=torch.float64, device=dev), "max").tolist()
        mn, mx, non = -f[0], f[1], f[2] != 0.0
    if not non and mx >= mn and (mx - mn + 1) * L * d <= catstats.MAX_TABLE:
        vmin, V = int(mn), int(mx - mn) + 1
        cnt = catstats.int_table(X, li, L, vmin, V).to(torch.float64)
        if dist:
            both = comm.all_reduce_sum(torch.cat([cnt.reshape(-1), n_lab]))
            cnt, n_lab = both[:-L].reshape(d, L, V), both[-L:]
        counts = cnt.cpu().numpy()
        present = counts.sum(1) > 0
        slots = [np.nonzero(present[j])[0] for j in range(d)]
        return counts, [(sl + vmin).astype(np.float64) for sl in slots], slots, n_lab.cpu().numpy()
    if dist:
        counts, vals, slots = catstats.global_value_label_counts(X, li, L)
        return counts, vals, slots, comm.all_reduce_sum(n_lab).cpu().numpy()
    counts, vals, slots = catstats.value_label_counts(X, li, L, int_range=None)
    return counts.astype(np.float64), vals, slots, n_lab.cpu().numpy()


def _labels_integral(y: torch.Tensor) -> bool:
    """No label with a fractional part (NaN counts as one, ±inf does not: y != round(y)). On the
    GPU one library reduction answers it for finite labels (torch's compare / round / any kernels
    load their code objects lazily: ~16 ms inside the first fit of a process)."""
    if y.is_cuda:
        from ..ops import catstats

        if not catstats.flags(y)[2]:
            return True
    return not bool((y != torch.round(y)).any())


@rw.register_stage
class NaiveBayes(Estimator, NaiveBayesParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.classification.naivebayes.NaiveBayes"

    def fit(self, *inputs):
        t = inputs[0]
        lab = t.column(self.get(self.LABEL_COL))
        if isinstance(lab, list) and any(v is None for v in lab):
            raise ValueError("Input data should contain label value.")
        fc = t.column(self.get(self.FEATURES_COL))
        if isinstance(fc, list) and len({v.size() for v in fc}) > 1:
            raise ValueError("Feature vectors should be of equal length.")
        # on the GPU the stored dtype stays (the contingency kernels read f32 or f64 themselves)
        X, y = features_and_labels(t, self.get(self.FEATURES_COL), self.get(self.LABEL_COL), keep_dtype=True)
        if not _labels_integral(y):
            raise ValueError("Label value should be indexed number.")
        s = self.get(self.SMOOTHING)
        dist = get_world_distributed()
        if dist:
            try:
                comm.check_equal_across_ranks(int(X.shape[1]), "feature vector length")
            except ValueError:
                raise ValueError("Feature vectors should be of equal length.") from None
        labels = global_sorted_unique(y)
        L, d = labels.numel(), X.shape[1]
        li = torch.searchsorted(labels, y)  # binary search per row
        counts, vals, slots, n_l = _label_value_counts(X, li, L, dist)
        labels_np = labels.cpu().numpy()
        # the reference's model lists labels in HashMap<Double, _> order
        order = [int(np.searchsorted(labels_np, v)) for v in java_hashmap_order(labels_np.tolist(), java_double_hash)]
        n_total = n_l.sum()
        pi_log = np.log(n_total * d + L * s)
        theta: List[List[Dict[float, float]]] = []
        for li_ in order:
            row = []
            for j in range(d):
                V = vals[j].size
                logs = np.log(counts[j, li_, slots[j]] + s) - np.log(n_l[li_] + s * V)
                row.append(dict(zip(vals[j].tolist(), logs.tolist())))
            theta.append(row)
        pi = DenseVector(np.array([np.log(n_l[i] * d + s) - pi_log for i in order]))
        md = (theta, pi, DenseVector(labels_np[order].astype(np.float64)))
        m = NaiveBayesModel().set_model_data(NaiveBayesModel.make_model_data_table([md]))
        rw_update(m, self)
        return m
