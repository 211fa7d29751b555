"""``feature.stringindexer`` stages."""
from flink_ml_amd.models import StringIndexer, StringIndexerModel, IndexToStringModel  # noqa: F401

__all__ = ['StringIndexer', 'StringIndexerModel', 'IndexToStringModel']
