"""``classification`` stages (reference ``pyflink.ml.lib.classification``)."""
from .knn import KNN, KNNModel  # noqa: F401
from .linearsvc import LinearSVC, LinearSVCModel  # noqa: F401
from .logisticregression import LogisticRegression, LogisticRegressionModel, OnlineLogisticRegression, OnlineLogisticRegressionModel  # noqa: F401
from .naivebayes import NaiveBayes, NaiveBayesModel  # noqa: F401
