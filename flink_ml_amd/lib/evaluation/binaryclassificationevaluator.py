"""``evaluation.binaryclassificationevaluator`` stages."""
from flink_ml_amd.models import BinaryClassificationEvaluator  # noqa: F401

__all__ = ['BinaryClassificationEvaluator']
