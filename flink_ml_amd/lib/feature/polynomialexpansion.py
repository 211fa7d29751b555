"""``feature.polynomialexpansion`` stages."""
from flink_ml_amd.models import PolynomialExpansion  # noqa: F401

__all__ = ['PolynomialExpansion']
