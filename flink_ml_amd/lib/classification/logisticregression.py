"""``classification.logisticregression`` stages."""
from flink_ml_amd.models import LogisticRegression, LogisticRegressionModel, OnlineLogisticRegression, OnlineLogisticRegressionModel  # noqa: F401

__all__ = ['LogisticRegression', 'LogisticRegressionModel', 'OnlineLogisticRegression', 'OnlineLogisticRegressionModel']
