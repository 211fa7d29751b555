"""``regression.linearregression`` stages."""
from flink_ml_amd.models import LinearRegression, LinearRegressionModel  # noqa: F401

__all__ = ['LinearRegression', 'LinearRegressionModel']
