"""``feature.tokenizer`` stages."""
from flink_ml_amd.models import Tokenizer  # noqa: F401

__all__ = ['Tokenizer']
