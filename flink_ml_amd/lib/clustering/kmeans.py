"""``clustering.kmeans`` stages."""
from flink_ml_amd.models import KMeans, KMeansModel, OnlineKMeans, OnlineKMeansModel  # noqa: F401

__all__ = ['KMeans', 'KMeansModel', 'OnlineKMeans', 'OnlineKMeansModel']
