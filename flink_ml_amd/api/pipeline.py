"""Pipeline / PipelineModel (reference ``flink-ml-core/.../builder/Pipeline.java:79-107``,
``PipelineModel.java:63-68``).

``Pipeline.fit`` fits every Estimator in order and transforms the tables only while a later
Estimator still needs them (``Pipeline.java:100-103``). Tables stay device-resident between
stages, so a Pipeline is a chain of kernel launches with no host round trip.
"""
from __future__ import annotations

from typing import List, Sequence

from ..io import read_write as rw
from ..table import Table
from .stage import AlgoOperator, Estimator, Model, Stage


@rw.register_stage
class PipelineModel(Model):
    JAVA_CLASS_NAME = "org.apache.flink.ml.builder.PipelineModel"

    def __init__(self, stages: Sequence[Stage] = ()):
        super().__init__()
        self.stages: List[Stage] = list(stages)

    def transform(self, *inputs: Table) -> List[Table]:
        tables = list(inputs)
        for s in self.stages:
            tables = s.transform(*tables)
        return tables

    def save(self, path: str) -> None:
        rw.save_pipeline(self, self.stages, path)

    @classmethod
    def load(cls, path: str) -> "PipelineModel":
        return PipelineModel(rw.load_pipeline(path, cls.JAVA_CLASS_NAME))

    def get_stages(self) -> List[Stage]:
        return self.stages


@rw.register_stage
class Pipeline(Estimator):
    JAVA_CLASS_NAME = "org.apache.flink.ml.builder.Pipeline"

    def __init__(self, stages: Sequence[Stage] = ()):
        super().__init__()
        self.stages: List[Stage] = list(stages)

    def fit(self, *inputs: Table) -> PipelineModel:
        last_est = -1
        for i, s in enumerate(self.stages):
            if isinstance(s, Estimator):
                last_est = i
        model_stages = []
        tables = list(inputs)
        for i, s in enumerate(self.stages):
            if isinstance(s, AlgoOperator):
                ms = s
            else:
                ms = s.fit(*tables)
            model_stages.append(ms)
            if i < last_est:
                tables = ms.transform(*tables)
        return PipelineModel(model_stages)

    def save(self, path: str) -> None:
        rw.save_pipeline(self, self.stages, path)

    @classmethod
    def load(cls, path: str) -> "Pipeline":
        return Pipeline(rw.load_pipeline(path, cls.JAVA_CLASS_NAME))

    def get_stages(self) -> List[Stage]:
        return self.stages
