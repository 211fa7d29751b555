"""UnivariateFeatureSelector (reference ``LIB/feature/univariatefeatureselector``).

Fit runs the matching hypothesis test (ChiSq for categorical/categorical, ANOVA for
continuous/categorical, F-value for continuous/continuous — all device reductions, see
``models/stats.py``) and selects feature indices from the p-values with the reference's
numTopFeatures / percentile / fpr / fdr / fwe rules (``UnivariateFeatureSelector.java:200-290``).
The model keeps the indices (``IntPrimitiveArraySerializer`` record) and transforms by gathering
the selected columns (sparse inputs stay sparse).
"""
from __future__ import annotations

from typing import List

import numpy as np
import torch

from ...api.stage import Estimator
from ...common.param import HasFeaturesCol, HasLabelCol, HasOutputCol
from ...io import read_write as rw
from ...io import serialization as ser
from ...param.param import FloatParam, ParamValidators, StringParam
from ...table import SparseColumn, Table
from ..base import ModelWithData
from ..linear import rw_update
from .common import select_by_indices, vector_input

CATEGORICAL, CONTINUOUS = "categorical", "continuous"
NUM_TOP_FEATURES, PERCENTILE, FPR, FDR, FWE = "numTopFeatures", "percentile", "fpr", "fdr", "fwe"


class UnivariateFeatureSelectorModelParams(HasFeaturesCol, HasOutputCol):
    pass


class UnivariateFeatureSelectorParams(UnivariateFeatureSelectorModelParams, HasLabelCol):
    CATEGORICAL, CONTINUOUS = CATEGORICAL, CONTINUOUS
    NUM_TOP_FEATURES, PERCENTILE, FPR, FDR, FWE = NUM_TOP_FEATURES, PERCENTILE, FPR, FDR, FWE
    FEATURE_TYPE = StringParam("featureType", "The feature type.", None,
                               ParamValidators.in_array(CATEGORICAL, CONTINUOUS))
    LABEL_TYPE = StringParam("labelType", "The label type.", None, ParamValidators.in_array(CATEGORICAL, CONTINUOUS))
    SELECTION_MODE = StringParam("selectionMode", "The feature selection mode.", NUM_TOP_FEATURES,
                                 ParamValidators.in_array(NUM_TOP_FEATURES, PERCENTILE, FPR, FDR, FWE))
    SELECTION_THRESHOLD = FloatParam(
        "selectionThreshold", "The upper bound of the features that selector will select. If not set, it will be "
        "replaced with a meaningful value according to different selection modes at runtime. When the mode is "
        "numTopFeatures, it will be replaced with 50; when the mode is percentile, it will be replaced with 0.1; "
        "otherwise, it will be replaced with 0.05.", None)


def select_indices(p_values, mode: str, threshold: float) -> List[int]:
    """The reference ``SelectIndicesFromPValuesOperator.endInput`` rules (ties by index)."""
    pv = [(float(p), i) for i, p in enumerate(p_values)]
    n = len(pv)
    ordered = sorted(pv, key=lambda t: (t[0], t[1]))
    if mode == NUM_TOP_FEATURES:
        return [i for _, i in ordered[:min(n, int(threshold))]]
    if mode == PERCENTILE:
        return [i for _, i in ordered[:min(n, int(n * threshold))]]
    if mode == FPR:
        return [i for p, i in pv if p < threshold]
    if mode == FDR:
        max_index = -1
        for k, (p, _) in enumerate(ordered):
            if p < (threshold / n) * (k + 1):
                max_index = max(max_index, k)
        return [i for _, i in ordered[:max_index + 1]]
    if mode == FWE:
        return [i for p, i in pv if p < threshold / n]
    raise RuntimeError("Unknown Selection Mode: %s" % mode)


@rw.register_stage
class UnivariateFeatureSelectorModel(ModelWithData, UnivariateFeatureSelectorModelParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.univariatefeatureselector.UnivariateFeatureSelectorModel"
    MODEL_DATA_COLUMNS = ("indices",)

    @staticmethod
    def encode_record(out, row):
        ser.write_int_array(out, np.asarray(row[0], dtype=np.int32))

    @staticmethod
    def decode_record(inp):
        return ([int(x) for x in ser.read_int_array(inp)],)

    @classmethod
    def make_model_data_table(cls, rows):
        return Table({"indices": [[int(x) for x in r[0]] for r in rows]}, num_rows=len(rows))

    def transform(self, *inputs):
        t = inputs[0]
        idx = sorted(int(i) for i in self.model_data_rows()[0][0])
        out_col = self.get(self.OUTPUT_COL)
        if not idx:
            return [t.with_column(out_col, torch.zeros((t.num_rows, 0), dtype=torch.float64))]
        X = vector_input(t, self.get(self.FEATURES_COL))
        d = X.size if isinstance(X, SparseColumn) else X.shape[1]
        if t.num_rows and d <= idx[-1]:
            raise ValueError("Input %d features, but UnivariateFeatureSelector is expecting at least %d features as "
                             "input." % (d, idx[-1] + 1))
        return [t.with_column(out_col, select_by_indices(X, idx))]


@rw.register_stage
class UnivariateFeatureSelector(Estimator, UnivariateFeatureSelectorParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.univariatefeatureselector.UnivariateFeatureSelector"

    def _threshold(self) -> float:
        th = self.get(self.SELECTION_THRESHOLD)
        mode = self.get(self.SELECTION_MODE)
        if th is None:
            return 50.0 if mode == NUM_TOP_FEATURES else (0.1 if mode == PERCENTILE else 0.05)
        if mode == NUM_TOP_FEATURES:
            if not (th >= 1 and float(int(th)) == th):
                raise ValueError("SelectionThreshold needs to be a positive Integer for selection mode "
                                 "numTopFeatures, but got %s." % th)
        elif not (0 <= th <= 1):
            raise ValueError("SelectionThreshold needs to be in the range [0, 1] for selection mode %s, but got %s."
                             % (mode, th))
        return th

    def fit(self, *inputs):
        from ..stats import ANOVATest, ChiSqTest, FValueTest

        ft, lt = self.get(self.FEATURE_TYPE), self.get(self.LABEL_TYPE)
        if ft == CATEGORICAL and lt == CATEGORICAL:
            test = ChiSqTest()
        elif ft == CONTINUOUS and lt == CATEGORICAL:
            test = ANOVATest()
        elif ft == CONTINUOUS and lt == CONTINUOUS:
            test = FValueTest()
        else:
            raise ValueError("Unsupported combination: featureType=%s, labelType=%s." % (ft, lt))
        threshold = self._threshold()
        test.set_features_col(self.get(self.FEATURES_COL)).set_label_col(self.get(self.LABEL_COL))
        p_values = test.compute(inputs[0])[0]
        idx = select_indices(p_values, self.get(self.SELECTION_MODE), threshold)
        m = UnivariateFeatureSelectorModel().set_model_data(UnivariateFeatureSelectorModel.make_model_data_table(
            [(idx,)]))
        rw_update(m, self)
        return m
