"""``feature.kbinsdiscretizer`` stages."""
from flink_ml_amd.models import KBinsDiscretizer, KBinsDiscretizerModel  # noqa: F401

__all__ = ['KBinsDiscretizer', 'KBinsDiscretizerModel']
