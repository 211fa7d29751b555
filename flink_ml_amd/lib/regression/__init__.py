"""``regression`` stages (reference ``pyflink.ml.lib.regression``)."""
from .linearregression import LinearRegression, LinearRegressionModel  # noqa: F401
