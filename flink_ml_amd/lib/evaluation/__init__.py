"""``evaluation`` stages (reference ``pyflink.ml.lib.evaluation``)."""
from .binaryclassificationevaluator import BinaryClassificationEvaluator  # noqa: F401
