"""Stage API (reference ``flink-ml-core/.../api/*.java``; Python ``pyflink/ml/core/api.py:31-114``).

* ``Stage`` — has params, ``save(path)`` and a class-level ``load(path)``.
* ``AlgoOperator.transform(*tables) -> List[Table]``.
* ``Transformer`` — an AlgoOperator whose outputs are row-aligned with its input.
* ``Estimator.fit(*tables) -> Model``.
* ``Model`` — a Transformer with ``set_model_data(*tables)`` / ``get_model_data()``.

Tables are per-rank partitions (see ``flink_ml_amd.table``); ``fit`` is an SPMD call —
every rank calls it on its own partition and they cooperate through collectives.
"""
from __future__ import annotations

from typing import List

from ..io import read_write as rw
from ..param.param import WithParams
from ..table import Table


class Stage(WithParams):
    JAVA_CLASS_NAME: str = None

    def save(self, path: str) -> None:
        rw.save_metadata(self, path)

    @classmethod
    def load(cls, path: str):
        stage = rw.load_stage_param(path)
        if not isinstance(stage, cls):
            raise RuntimeError("Loaded stage %s is not a %s" % (type(stage).__name__, cls.__name__))
        return stage

    def __repr__(self):
        return "%s(%s)" % (type(self).__name__, ", ".join(
            "%s=%r" % (p.name, v) for p, v in self.get_param_map().items()))


class AlgoOperator(Stage):
    def transform(self, *inputs: Table) -> List[Table]:
        raise NotImplementedError


class Transformer(AlgoOperator):
    pass


class Model(Transformer):
    def set_model_data(self, *inputs: Table):
        raise NotImplementedError("%s does not support set_model_data" % type(self).__name__)

    def get_model_data(self) -> List[Table]:
        raise NotImplementedError("%s does not support get_model_data" % type(self).__name__)

    setModelData = set_model_data
    getModelData = get_model_data


class Estimator(Stage):
    def fit(self, *inputs: Table) -> Model:
        raise NotImplementedError
