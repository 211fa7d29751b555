"""Algorithm library (reference flink-ml-lib): importing this package registers every stage."""
from . import linear  # noqa: F401
from .linear import (LinearRegression, LinearRegressionModel, LinearSVC, LinearSVCModel,  # noqa: F401
                     LogisticRegression, LogisticRegressionModel)
from . import kmeans  # noqa: F401,E402
from .kmeans import KMeans, KMeansModel  # noqa: F401,E402
from . import online  # noqa: F401,E402
from .online import (OnlineKMeans, OnlineKMeansModel, OnlineLogisticRegression,  # noqa: F401,E402
                     OnlineLogisticRegressionModel)
from . import feature  # noqa: F401,E402
from .feature import *  # noqa: F401,F403,E402
from . import stats  # noqa: F401,E402
from .stats import ANOVATest, ChiSqTest, FValueTest  # noqa: F401,E402
from . import knn, naive_bayes  # noqa: F401,E402
from .knn import Knn, KnnModel  # noqa: F401,E402
from .naive_bayes import NaiveBayes, NaiveBayesModel  # noqa: F401,E402
from . import evaluation  # noqa: F401,E402
from .evaluation import BinaryClassificationEvaluator  # noqa: F401,E402
from . import agglomerative  # noqa: F401,E402
from .agglomerative import AgglomerativeClustering  # noqa: F401,E402
# reference Python API spellings (pyflink.ml.lib.classification.knn)
KNN, KNNModel = Knn, KnnModel  # noqa: E305
