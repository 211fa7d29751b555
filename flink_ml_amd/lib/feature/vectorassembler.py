"""``feature.vectorassembler`` stages."""
from flink_ml_amd.models import VectorAssembler  # noqa: F401

__all__ = ['VectorAssembler']
