"""``feature.ngram`` stages."""
from flink_ml_amd.models import NGram  # noqa: F401

__all__ = ['NGram']
