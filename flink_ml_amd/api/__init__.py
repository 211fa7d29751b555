from .stage import AlgoOperator, Estimator, Model, Stage, Transformer  # noqa: F401
from .pipeline import Pipeline, PipelineModel  # noqa: F401
from .graph import Graph, GraphBuilder, GraphModel, TableId  # noqa: F401
