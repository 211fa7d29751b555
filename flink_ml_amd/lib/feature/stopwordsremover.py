"""``feature.stopwordsremover`` stages."""
from flink_ml_amd.models import StopWordsRemover  # noqa: F401

__all__ = ['StopWordsRemover']
