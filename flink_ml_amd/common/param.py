"""Shared ``Has*`` parameter mixins (reference ``LIB/common/param/*.java``; names, defaults and
validators identical so metadata JSON round-trips with the reference)."""
from __future__ import annotations

from ..param.param import (BooleanParam, FloatParam, IntParam, LongParam, ParamValidators as V, StringArrayParam,
                           StringParam, WindowsParam, WithParams)
from ..utils.java import java_string_hash
from .window import GlobalWindows


class HasFeaturesCol(WithParams):
    FEATURES_COL = StringParam("featuresCol", "Features column name.", "features", V.not_null())


class HasLabelCol(WithParams):
    LABEL_COL = StringParam("labelCol", "Label column name.", "label", V.not_null())


class HasPredictionCol(WithParams):
    PREDICTION_COL = StringParam("predictionCol", "Prediction column name.", "prediction", V.not_null())


class HasRawPredictionCol(WithParams):
    RAW_PREDICTION_COL = StringParam("rawPredictionCol", "Raw prediction column name.", "rawPrediction")


class HasWeightCol(WithParams):
    WEIGHT_COL = StringParam("weightCol", "Weight column name.", None)


class HasMaxIter(WithParams):
    MAX_ITER = IntParam("maxIter", "Maximum number of iterations.", 20, V.gt(0))


class HasTol(WithParams):
    TOL = FloatParam("tol", "Convergence tolerance for iterative algorithms.", 1e-6, V.gt_eq(0))


class HasLearningRate(WithParams):
    LEARNING_RATE = FloatParam("learningRate", "Learning rate of optimization method.", 0.1, V.gt(0))


class HasGlobalBatchSize(WithParams):
    GLOBAL_BATCH_SIZE = IntParam("globalBatchSize", "Global batch size of training algorithms.", 32, V.gt(0))


class HasReg(WithParams):
    REG = FloatParam("reg", "Regularization parameter.", 0.0, V.gt_eq(0.0))


class HasElasticNet(WithParams):
    ELASTIC_NET = FloatParam("elasticNet", "ElasticNet parameter.", 0.0, V.in_range(0.0, 1.0))


class HasMultiClass(WithParams):
    MULTI_CLASS = StringParam("multiClass", "Classification type.", "auto",
                              V.in_array("auto", "binomial", "multinomial"))


class HasDistanceMeasure(WithParams):
    DISTANCE_MEASURE = StringParam("distanceMeasure", "Distance measure.", "euclidean",
                                   V.in_array("euclidean", "manhattan", "cosine"))


class HasSeed(WithParams):
    SEED = LongParam("seed", "The random seed.", None)

    def get_seed(self) -> int:
        s = self.get(self.SEED)
        if s is not None:
            return s
        java = getattr(type(self), "JAVA_CLASS_NAME", None) or type(self).__name__
        return java_string_hash(java)

    getSeed = get_seed


class HasDecayFactor(WithParams):
    DECAY_FACTOR = FloatParam("decayFactor", "The forgetfulness of the previous centroids.", 0.0, V.in_range(0, 1))


class HasBatchStrategy(WithParams):
    COUNT_STRATEGY = "count"
    BATCH_STRATEGY = StringParam("batchStrategy", "Strategy to create mini batch from online train data.",
                                 "count", V.in_array("count"))


class HasNumFeatures(WithParams):
    NUM_FEATURES = IntParam("numFeatures", "The number of features. It will be the length of the output vector.",
                            262144, V.gt(0))


class HasHandleInvalid(WithParams):
    ERROR_INVALID = "error"
    SKIP_INVALID = "skip"
    KEEP_INVALID = "keep"
    HANDLE_INVALID = StringParam("handleInvalid", "Strategy to handle invalid entries.", "error",
                                 V.in_array("error", "skip", "keep"))


class HasInputCol(WithParams):
    INPUT_COL = StringParam("inputCol", "Input column name.", "input", V.not_null())


class HasOutputCol(WithParams):
    OUTPUT_COL = StringParam("outputCol", "Output column name.", "output", V.not_null())


class HasInputCols(WithParams):
    INPUT_COLS = StringArrayParam("inputCols", "Input column names.", None, V.non_empty_array())


class HasOutputCols(WithParams):
    OUTPUT_COLS = StringArrayParam("outputCols", "Output column names.", None, V.non_empty_array())


class HasCategoricalCols(WithParams):
    CATEGORICAL_COLS = StringArrayParam("categoricalCols", "Categorical column names.", (), V.not_null())


class HasRelativeError(WithParams):
    RELATIVE_ERROR = FloatParam("relativeError", "The relative target precision for the approximate quantile algorithm.",
                                0.001, V.in_range(0, 1))


class HasFlatten(WithParams):
    FLATTEN = BooleanParam("flatten", "If false, the returned table contains only a single row, otherwise, one row per feature.",
                           False)


class HasWindows(WithParams):
    WINDOWS = WindowsParam("windows", "Windowing strategy that determines how to create mini-batches from input data.",
                           GlobalWindows.get_instance(), V.not_null())
