"""``classification.linearsvc`` stages."""
from flink_ml_amd.models import LinearSVC, LinearSVCModel  # noqa: F401

__all__ = ['LinearSVC', 'LinearSVCModel']
