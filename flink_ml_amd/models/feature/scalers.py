"""Scalers and variance-based selection (reference ``LIB/feature/{standardscaler,minmaxscaler,
maxabsscaler,robustscaler,variancethresholdselector}``).

fit = one fused column-statistics pass over the rank's HBM-resident partition (``colstats.hip``,
K15) + one all-reduce of the fixed-size statistics; transform = one fused per-column affine
kernel (``affine_cols``, K16). Sparse inputs stay sparse where the reference keeps them sparse
(MaxAbsScaler, StandardScaler without centering).
"""
from __future__ import annotations

import numpy as np
import torch

from ...api.stage import Estimator
from ...common.param import HasInputCol, HasOutputCol, HasRelativeError
from ...io import read_write as rw
from ...io import serialization as ser
from ...ops import features as fo
from ...param.param import BooleanParam, FloatParam, ParamValidators
from ...parallel import comm
from ...table import SparseColumn, Table
from ..base import ModelWithData
from ..linear import rw_update
from .common import (all_reduce_stats, dec_dense, dense_input, dense_vec, enc_dense, select_by_indices,
                     sparse_map_values, vector_input)


def _stats(table: Table, col: str) -> dict:
    X = dense_input(table, col)
    return all_reduce_stats(fo.column_stats(X))


def _t(v, dev):
    return torch.as_tensor(v.values if hasattr(v, "values") else v, dtype=torch.float64, device=dev)


# ------------------------------------------------------------------------------- StandardScaler
class StandardScalerParams(HasInputCol, HasOutputCol):
    WITH_MEAN = BooleanParam("withMean", "Whether centers the data with mean before scaling.", False)
    WITH_STD = BooleanParam("withStd", "Whether scales the data with standard deviation.", True)


@rw.register_stage
class StandardScalerModel(ModelWithData, StandardScalerParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.standardscaler.StandardScalerModel"
    MODEL_DATA_COLUMNS = ("mean", "std")

    @staticmethod
    def encode_record(out, row):
        enc_dense(out, row[0])
        enc_dense(out, row[1])

    @staticmethod
    def decode_record(inp):
        return (dec_dense(inp), dec_dense(inp))

    def transform(self, *inputs):
        t = inputs[0]
        mean, std = self.model_data_rows()[0]
        X = vector_input(t, self.get(self.INPUT_COL))
        dev = X.values.device if isinstance(X, SparseColumn) else X.device
        sd = _t(std, "cpu")  # [d] scale formed on the host, one copy to the device
        scale = torch.where(sd == 0, torch.zeros_like(sd), 1.0 / torch.where(sd == 0, torch.ones_like(sd), sd)).to(dev)
        with_mean, with_std = self.get(self.WITH_MEAN), self.get(self.WITH_STD)
        if isinstance(X, SparseColumn) and not with_mean:
            out = sparse_map_values(X, lambda v, i: v * scale[i]) if with_std else X
        else:
            if isinstance(X, SparseColumn):
                X = X.to_dense(torch.float64)
            out = fo.affine_cols(X, _t(mean, dev) if with_mean else None, scale if with_std else None)
        return [t.with_column(self.get(self.OUTPUT_COL), out)]


@rw.register_stage
class StandardScaler(Estimator, StandardScalerParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.standardscaler.StandardScaler"

    def fit(self, *inputs):
        s = _stats(inputs[0], self.get(self.INPUT_COL))
        n = s["count"]
        if n == 0:
            raise RuntimeError("The training set is empty.")
        # the [d] finalisation on the host (same IEEE fp64 ops): on the device each of these small
        # elementwise ops loads its torch code object at first use (~70 ms each in a fresh process)
        mean = s["sum"].cpu() / n
        if n > 1:
            std = torch.sqrt((s["sumsq"].cpu() - n * mean * mean) / (n - 1))
        else:
            std = torch.zeros_like(mean)
        m = StandardScalerModel().set_model_data(
            StandardScalerModel.make_model_data_table([(dense_vec(mean), dense_vec(std))]))
        rw_update(m, self)
        return m


# ------------------------------------------------------------------------------- MinMaxScaler
class MinMaxScalerParams(HasInputCol, HasOutputCol):
    MIN = FloatParam("min", "Lower bound of the output feature range.", 0.0, ParamValidators.not_null())
    MAX = FloatParam("max", "Upper bound of the output feature range.", 1.0, ParamValidators.not_null())


@rw.register_stage
class MinMaxScalerModel(ModelWithData, MinMaxScalerParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.minmaxscaler.MinMaxScalerModel"
    MODEL_DATA_COLUMNS = ("minVector", "maxVector")

    @staticmethod
    def encode_record(out, row):
        enc_dense(out, row[0])
        enc_dense(out, row[1])

    @staticmethod
    def decode_record(inp):
        return (dec_dense(inp), dec_dense(inp))

    def transform(self, *inputs):
        t = inputs[0]
        mn, mx = self.model_data_rows()[0]
        X = dense_input(t, self.get(self.INPUT_COL))
        lo, hi = self.get(self.MIN), self.get(self.MAX)
        mnv, mxv = _t(mn, "cpu"), _t(mx, "cpu")  # [d] scale / offset formed on the host
        const = (mnv - mxv).abs() < 1.0e-5
        rng = torch.where(const, torch.ones_like(mnv), mxv - mnv)
        scale = torch.where(const, torch.zeros_like(mnv), (hi - lo) / rng)
        offset = torch.where(const, torch.full_like(mnv, (hi + lo) / 2), lo - mnv * scale)
        scale, offset = scale.to(X.device), offset.to(X.device)
        return [t.with_column(self.get(self.OUTPUT_COL), fo.affine_cols(X, None, scale, offset))]


@rw.register_stage
class MinMaxScaler(Estimator, MinMaxScalerParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.minmaxscaler.MinMaxScaler"

    def fit(self, *inputs):
        s = _stats(inputs[0], self.get(self.INPUT_COL))
        if s["count"] == 0:
            raise RuntimeError("The training set is empty.")
        m = MinMaxScalerModel().set_model_data(
            MinMaxScalerModel.make_model_data_table([(dense_vec(s["min"]), dense_vec(s["max"]))]))
        rw_update(m, self)
        return m


# ------------------------------------------------------------------------------- MaxAbsScaler
@rw.register_stage
class MaxAbsScalerModel(ModelWithData, HasInputCol, HasOutputCol):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.maxabsscaler.MaxAbsScalerModel"
    MODEL_DATA_COLUMNS = ("maxVector",)

    @staticmethod
    def encode_record(out, row):
        enc_dense(out, row[0])

    @staticmethod
    def decode_record(inp):
        return (dec_dense(inp),)

    def transform(self, *inputs):
        t = inputs[0]
        (mx,) = self.model_data_rows()[0]
        X = vector_input(t, self.get(self.INPUT_COL))
        dev = X.values.device if isinstance(X, SparseColumn) else X.device
        m = _t(mx, "cpu")  # [d] scale formed on the host
        scale = torch.where(m != 0, 1.0 / torch.where(m != 0, m, torch.ones_like(m)), torch.ones_like(m)).to(dev)
        if isinstance(X, SparseColumn):
            out = sparse_map_values(X, lambda v, i: v * scale[i])
        else:
            out = fo.affine_cols(X, None, scale)
        return [t.with_column(self.get(self.OUTPUT_COL), out)]


@rw.register_stage
class MaxAbsScaler(Estimator, HasInputCol, HasOutputCol):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.maxabsscaler.MaxAbsScaler"

    def fit(self, *inputs):
        t = inputs[0]
        X = vector_input(t, self.get(self.INPUT_COL))
        if isinstance(X, SparseColumn):
            d = X.size
            mx = torch.zeros(d, dtype=torch.float64, device=X.values.device)
            if X.values.numel():
                mx = mx.scatter_reduce(0, X.indices.long(), X.values.to(torch.float64).abs(), "amax")
        else:
            st = fo.column_stats(X)
            # (the [d] max-abs on the host: a device torch.maximum / abs would load their code
            # objects at first use, ~100 ms in a fresh process)
            mx = torch.maximum(st["max"].cpu().abs(), st["min"].cpu().abs()) if X.shape[0] else torch.zeros(
                X.shape[1], dtype=torch.float64)
        mx = comm.all_reduce(mx.clone(), "max")
        m = MaxAbsScalerModel().set_model_data(MaxAbsScalerModel.make_model_data_table([(dense_vec(mx),)]))
        rw_update(m, self)
        return m


# ------------------------------------------------------------------------------- RobustScaler
def exact_quantiles(X: torch.Tensor, ps, rel_err: float) -> torch.Tensor:
    """Per-column quantiles with the reference QuantileSummary query semantics on exact data
    (``QuantileSummary.java:237-364``): p <= relErr -> min, p >= 1-relErr -> max, otherwise the
    element of 1-based rank ceil(p·n); NaNs ignored. Exact ranks satisfy the GK ε bound. Computed by
    a distributed radix select (``ops/quantile.py``) — the shards never leave their ranks."""
    from ...ops.quantile import column_quantiles

    return column_quantiles(X, ps, rel_err, distributed=get_distributed())


def get_distributed():
    from ...parallel.context import get_context

    return get_context().is_distributed


class RobustScalerModelParams(HasInputCol, HasOutputCol):
    WITH_CENTERING = BooleanParam("withCentering", "Whether to center the data with median before scaling.", False)
    WITH_SCALING = BooleanParam("withScaling", "Whether to scale the data to quantile range.", True)


class RobustScalerParams(RobustScalerModelParams, HasRelativeError):
    LOWER = FloatParam("lower", "Lower quantile to calculate quantile range.", 0.25,
                       ParamValidators.in_range(0.0, 1.0, False, False))
    UPPER = FloatParam("upper", "Upper quantile to calculate quantile range.", 0.75,
                       ParamValidators.in_range(0.0, 1.0, False, False))


@rw.register_stage
class RobustScalerModel(ModelWithData, RobustScalerModelParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.robustscaler.RobustScalerModel"
    MODEL_DATA_COLUMNS = ("medians", "ranges")

    @staticmethod
    def encode_record(out, row):
        enc_dense(out, row[0])
        enc_dense(out, row[1])

    @staticmethod
    def decode_record(inp):
        return (dec_dense(inp), dec_dense(inp))

    def transform(self, *inputs):
        t = inputs[0]
        med, rng = self.model_data_rows()[0]
        X = dense_input(t, self.get(self.INPUT_COL))
        if X.shape[0] and X.shape[1] != med.size():
            raise ValueError("Number of features must be %d but got %d." % (med.size(), X.shape[1]))
        r = _t(rng, "cpu")  # [d] scale formed on the host
        scale = torch.where(r == 0, torch.zeros_like(r), 1.0 / torch.where(r == 0, torch.ones_like(r), r)).to(X.device)
        out = fo.affine_cols(X, _t(med, X.device) if self.get(self.WITH_CENTERING) else None,
                             scale if self.get(self.WITH_SCALING) else None)
        return [t.with_column(self.get(self.OUTPUT_COL), out)]


@rw.register_stage
class RobustScaler(Estimator, RobustScalerParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.robustscaler.RobustScaler"

    def fit(self, *inputs):
        if self.get(self.LOWER) >= self.get(self.UPPER):
            raise ValueError("lower must be smaller than upper")
        X = dense_input(inputs[0], self.get(self.INPUT_COL))
        if comm.all_reduce_scalar(float(X.shape[0]), "sum") == 0:
            raise RuntimeError("The training set is empty.")
        q = exact_quantiles(X, [0.5, self.get(self.LOWER), self.get(self.UPPER)], self.get(self.RELATIVE_ERROR))
        m = RobustScalerModel().set_model_data(
            RobustScalerModel.make_model_data_table([(dense_vec(q[0]), dense_vec(q[2] - q[1]))]))
        rw_update(m, self)
        return m


# ------------------------------------------------------------------------------- VarianceThresholdSelector
class VarianceThresholdSelectorParams(HasInputCol, HasOutputCol):
    VARIANCE_THRESHOLD = FloatParam("varianceThreshold",
                                    "Features with a variance not greater than this threshold will be removed.", 0.0,
                                    ParamValidators.gt_eq(0.0))


@rw.register_stage
class VarianceThresholdSelectorModel(ModelWithData, HasInputCol, HasOutputCol):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.variancethresholdselector.VarianceThresholdSelectorModel"
    MODEL_DATA_COLUMNS = ("numOfFeatures", "indices")

    @staticmethod
    def encode_record(out, row):
        out.write_int(int(row[0]))
        ser.write_int_array(out, row[1])

    @staticmethod
    def decode_record(inp):
        return (inp.read_int(), list(ser.read_int_array(inp)))

    @classmethod
    def make_model_data_table(cls, rows):
        return Table({"numOfFeatures": torch.tensor([int(r[0]) for r in rows]), "indices": [list(r[1]) for r in rows]},
                     num_rows=len(rows))

    def transform(self, *inputs):
        t = inputs[0]
        nf, idx = self.model_data_rows()[0]
        idx = sorted(int(i) for i in idx)
        X = vector_input(t, self.get(self.INPUT_COL))
        d = X.size if isinstance(X, SparseColumn) else X.shape[1]
        if t.num_rows and d != nf:
            raise ValueError("%s has %d features, but VarianceThresholdSelector is expecting %d features as input."
                             % (self.get(self.INPUT_COL), d, nf))
        return [t.with_column(self.get(self.OUTPUT_COL), select_by_indices(X, idx))]


@rw.register_stage
class VarianceThresholdSelector(Estimator, VarianceThresholdSelectorParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.variancethresholdselector.VarianceThresholdSelector"

    def fit(self, *inputs):
        s = _stats(inputs[0], self.get(self.INPUT_COL))
        n = s["count"]
        if n == 0:
            raise RuntimeError("The training set is empty.")
        sm, sq = s["sum"].cpu(), s["sumsq"].cpu()  # [d] on the host (no first-use torch kernel loads)
        var = sq / n - (sm / n) * (sm / n)
        idx = torch.nonzero(var > self.get(self.VARIANCE_THRESHOLD)).reshape(-1).tolist()
        m = VarianceThresholdSelectorModel().set_model_data(
            VarianceThresholdSelectorModel.make_model_data_table([(int(s["sum"].shape[0]), idx)]))
        rw_update(m, self)
        return m
