"""Benchmark data generators (reference ``flink-ml-benchmark/.../datagenerator``).

Every generator is a ``WithParams`` with the reference's params (seed, colNames, numValues,
vectorDim, arraySize, numDistinctValues, featureArity, labelArity, arity) and produces this rank's
partition: rank r of P draws ``numValues/P`` (+1 for r < numValues % P) rows from
``java.util.Random(Tuple2.of(seed, r).hashCode())`` — the reference's ``RowGenerator`` with the
rank as the subtask index. Numeric rows are generated on the device with the bit-exact jump-ahead
LCG kernel (``ops/datagen.py``); string rows are materialised on the host.
"""
from __future__ import annotations

from typing import List

import numpy as np
import torch

from .. import config
from ..common.param import HasSeed
from ..io import read_write as rw
from ..linalg.vectors import DenseVector
from ..ops.datagen import java_rows
from ..param.param import IntParam, LongParam, ParamValidators, StringArrayArrayParam, WithParams
from ..parallel.context import get_context
from ..table import StringArrayColumn, StringColumn, Table
from ..utils.java import _i32, java_long_hash

_PKG = "org.apache.flink.ml.benchmark.datagenerator."


def task_seed(seed: int, task: int) -> int:
    """``Tuple2.of(Long seed, Integer task).hashCode()``."""
    return _i32(31 * java_long_hash(int(seed)) + int(task))


def task_rows(num_values: int, task: int, num_tasks: int) -> int:
    div, mod = divmod(int(num_values), num_tasks)
    return div + 1 if mod > task else div


def _check_names(names, k: int) -> None:
    if names is None or len(names) != 1 or len(names[0]) != k:
        raise ValueError("colNames must hold exactly one table with %d column(s), got %r" % (k, names))


class DataGenerator(HasSeed):
    JAVA_CLASS_NAME = None

    def get_data(self) -> List[Table]:
        raise NotImplementedError

    getData = get_data


class HasVectorDim(WithParams):
    VECTOR_DIM = IntParam("vectorDim", "Dimension of vector-typed data to be generated.", 1, ParamValidators.gt(0))


class HasArraySize(WithParams):
    ARRAY_SIZE = IntParam("arraySize", "Number of elements in the generated array.", 1, ParamValidators.gt(0))


class HasNumDistinctValues(WithParams):
    NUM_DISTINCT_VALUES = IntParam("numDistinctValues", "Number of distinct values of the data to be generated.", 10,
                                   ParamValidators.gt(0))


class InputDataGenerator(DataGenerator):
    NUM_VALUES = LongParam("numValues", "Number of data to be generated.", 10, ParamValidators.gt(0))
    COL_NAMES = StringArrayArrayParam("colNames", "A 2D array of strings. Each string array element represents the "
                                      "column names of a data table.", None)

    def _task(self):
        ctx = get_context()
        return ctx.rank, ctx.world_size, task_rows(self.get(self.NUM_VALUES), ctx.rank, ctx.world_size), \
            task_seed(self.get_seed(), ctx.rank)

    def _rows(self, ops, nvec, vec_dtype=None, int_codes=False):
        _, _, n, seed = self._task()
        dev = config.compute_device()
        if vec_dtype is None:
            vec_dtype = torch.float64 if dev.type == "cpu" else config.compute_dtype()
        return java_rows(seed, n, ops, nvec, device=dev, vec_dtype=vec_dtype, int_codes=int_codes)


@rw.register_stage
class DenseVectorGenerator(InputDataGenerator, HasVectorDim):
    JAVA_CLASS_NAME = _PKG + "common.DenseVectorGenerator"

    def get_data(self):
        names = self.get(self.COL_NAMES)
        _check_names(names, 1)
        vec, _ = self._rows([0] * self.get(self.VECTOR_DIM), self.get(self.VECTOR_DIM))
        return [Table({names[0][0]: vec}, num_rows=vec.shape[0])]


@rw.register_stage
class DenseVectorArrayGenerator(InputDataGenerator, HasVectorDim, HasArraySize):
    JAVA_CLASS_NAME = _PKG + "common.DenseVectorArrayGenerator"

    def get_data(self):
        names = self.get(self.COL_NAMES)
        a, d = self.get(self.ARRAY_SIZE), self.get(self.VECTOR_DIM)
        vec, _ = self._rows([0] * (a * d), a * d, vec_dtype=torch.float64)
        arr = vec.reshape(-1, a, d)
        return [Table({names[0][0]: arr}, num_rows=arr.shape[0])]


@rw.register_stage
class DoubleGenerator(InputDataGenerator):
    JAVA_CLASS_NAME = _PKG + "common.DoubleGenerator"
    ARITY = IntParam("arity", "Arity of the generated double values. If set to positive value, each feature would be "
                     "an integer in range [0, arity - 1]. If set to zero, each feature would be a continuous double "
                     "in range [0, 1).", 0, ParamValidators.gt_eq(0))

    def get_data(self):
        names = self.get(self.COL_NAMES)
        k = len(names[0])
        _, sc = self._rows([self.get(self.ARITY)] * k, 0)
        return [Table({c: sc[:, i].contiguous() for i, c in enumerate(names[0])}, num_rows=sc.shape[0])]


@rw.register_stage
class LabeledPointWithWeightGenerator(InputDataGenerator, HasVectorDim):
    JAVA_CLASS_NAME = _PKG + "common.LabeledPointWithWeightGenerator"
    FEATURE_ARITY = IntParam("featureArity", "Arity of each feature. If set to positive value, each feature would be "
                             "an integer in range [0, arity - 1]. If set to zero, each feature would be a continuous "
                             "double in range [0, 1).", 2, ParamValidators.gt_eq(0))
    LABEL_ARITY = IntParam("labelArity", "Arity of label. If set to positive value, the label would be an integer in "
                           "range [0, arity - 1]. If set to zero, the label would be a continuous double in range "
                           "[0, 1).", 2, ParamValidators.gt_eq(0))

    def get_data(self):
        names = self.get(self.COL_NAMES)
        _check_names(names, 3)
        d = self.get(self.VECTOR_DIM)
        fa = self.get(self.FEATURE_ARITY)
        ops = [fa] * d + [self.get(self.LABEL_ARITY), 0]
        # categorical features stay exact in fp64/fp32; continuous ones use the compute dtype
        vec_dtype = None if fa == 0 else (torch.float64 if config.compute_device().type == "cpu" else torch.float32)
        vec, sc = self._rows(ops, d, vec_dtype)
        f, l, w = names[0]
        return [Table({f: vec, l: sc[:, 0].contiguous(), w: sc[:, 1].contiguous()}, num_rows=vec.shape[0])]


@rw.register_stage
class RandomStringGenerator(InputDataGenerator, HasNumDistinctValues):
    JAVA_CLASS_NAME = _PKG + "common.RandomStringGenerator"

    def get_data(self):
        names = self.get(self.COL_NAMES)
        k = len(names[0])
        _, sc = self._rows([self.get(self.NUM_DISTINCT_VALUES)] * k, 0, int_codes=True)
        vocab = [str(i) for i in range(self.get(self.NUM_DISTINCT_VALUES))]
        # dictionary-encoded, device-resident strings (rows materialise as str on demand)
        return [Table({c: StringColumn(sc[:, i].contiguous().to(torch.int32), vocab) for i, c in enumerate(names[0])},
                      num_rows=sc.shape[0])]


@rw.register_stage
class RandomStringArrayGenerator(InputDataGenerator, HasNumDistinctValues, HasArraySize):
    JAVA_CLASS_NAME = _PKG + "common.RandomStringArrayGenerator"

    def get_data(self):
        names = self.get(self.COL_NAMES)
        k, a = len(names[0]), self.get(self.ARRAY_SIZE)
        _, sc = self._rows([self.get(self.NUM_DISTINCT_VALUES)] * (k * a), 0, int_codes=True)
        codes = sc.reshape(sc.shape[0], k, a)
        vocab = [str(i) for i in range(self.get(self.NUM_DISTINCT_VALUES))]
        # dictionary-encoded, device-resident string arrays (rows materialise as lists on demand)
        return [Table({c: StringArrayColumn.from_dense_codes(codes[:, i, :].contiguous(), vocab)
                       for i, c in enumerate(names[0])}, num_rows=codes.shape[0])]


@rw.register_stage
class KMeansModelDataGenerator(DataGenerator, HasVectorDim, HasArraySize):
    JAVA_CLASS_NAME = _PKG + "clustering.KMeansModelDataGenerator"

    def get_data(self):
        g = DenseVectorArrayGenerator()
        from ..param.param import update_existing_params

        update_existing_params(g, self.get_param_map())
        g.set_num_values(1).set_col_names([["centroids"]])
        from ..parallel.context import get_context

        # the single model row comes from task 0
        ctx = get_context()
        seed = task_seed(g.get_seed(), 0)
        a, d = self.get(self.ARRAY_SIZE), self.get(self.VECTOR_DIM)
        vec, _ = java_rows(seed, 1, [0] * (a * d), a * d, device="cpu")
        cents = [DenseVector(r) for r in vec.reshape(a, d).numpy()]
        from ..models.kmeans import KMeansModel

        return [KMeansModel.make_model_data_table([(cents, DenseVector(np.zeros(a)))])]
