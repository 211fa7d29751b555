"""``feature.regextokenizer`` stages."""
from flink_ml_amd.models import RegexTokenizer  # noqa: F401

__all__ = ['RegexTokenizer']
