"""``classification.naivebayes`` stages."""
from flink_ml_amd.models import NaiveBayes, NaiveBayesModel  # noqa: F401

__all__ = ['NaiveBayes', 'NaiveBayesModel']
