"""``feature.countvectorizer`` stages."""
from flink_ml_amd.models import CountVectorizer, CountVectorizerModel  # noqa: F401

__all__ = ['CountVectorizer', 'CountVectorizerModel']
