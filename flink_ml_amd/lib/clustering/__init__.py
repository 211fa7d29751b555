"""``clustering`` stages (reference ``pyflink.ml.lib.clustering``)."""
from .agglomerativeclustering import AgglomerativeClustering  # noqa: F401
from .kmeans import KMeans, KMeansModel, OnlineKMeans, OnlineKMeansModel  # noqa: F401
