"""Distance measures (reference ``CORE/common/distance/*.java``): ``DistanceMeasure.get_instance``
by name, point-to-point ``distance`` on ``VectorWithNorm`` and ``find_closest`` (Euclidean with
the norm lower-bound pruning of ``EuclideanDistanceMeasure.java:53-73``).

The batched forms used by KMeans / OnlineKMeans / KMeansModel run as HIP kernels
(``ops/csrc/kmeans.hip``); ``find_closest_batch`` exposes that path for whole matrices.
"""
from __future__ import annotations

import math
from typing import Sequence

import numpy as np
import torch

from ..linalg import DenseVector, Vector


class VectorWithNorm:
    """A vector with its cached L2 norm (reference ``CORE/linalg/VectorWithNorm.java``)."""

    def __init__(self, vector: Vector, l2_norm: float = None):
        self.vector = vector
        arr = vector.to_array() if hasattr(vector, "to_array") else np.asarray(vector, dtype=np.float64)
        self._arr = np.asarray(arr, dtype=np.float64)
        self.l2_norm = float(np.linalg.norm(self._arr)) if l2_norm is None else float(l2_norm)

    def __eq__(self, other):
        return isinstance(other, VectorWithNorm) and np.array_equal(self._arr, other._arr) \
            and self.l2_norm == other.l2_norm


class DistanceMeasure:
    NAME = None

    @staticmethod
    def get_instance(name: str) -> "DistanceMeasure":
        if name not in _INSTANCES:
            raise ValueError("distanceMeasure %s is not recognized. Supported options: 'euclidean, manhattan, "
                             "cosine'." % name)
        return _INSTANCES[name]

    def distance(self, v1: VectorWithNorm, v2: VectorWithNorm) -> float:
        raise NotImplementedError

    def find_closest(self, centroids: Sequence[VectorWithNorm], point: VectorWithNorm) -> int:
        best, best_d = -1, float("inf")
        for i, c in enumerate(centroids):
            d = self.distance(c, point)
            if d < best_d:
                best, best_d = i, d
        return best

    def find_closest_batch(self, X: torch.Tensor, centroids: torch.Tensor) -> torch.Tensor:
        """Closest centroid for every row of X (device kernel on GPU tensors)."""
        from ..ops import kmeans as kk

        if X.device.type == "cuda":
            cb = kk.CentroidBuffers(centroids.shape[0], centroids.shape[1], X.device,
                                    torch.float64 if X.dtype == torch.float64 else torch.float32)
            cb.set(centroids)
            return kk.assign(X, cb, self.NAME).to(torch.int64)
        return kk.torch_assign(X, centroids, self.NAME)


class EuclideanDistanceMeasure(DistanceMeasure):
    NAME = "euclidean"

    @staticmethod
    def _sq(v1: VectorWithNorm, v2: VectorWithNorm) -> float:
        return max(0.0, v1.l2_norm * v1.l2_norm + v2.l2_norm * v2.l2_norm - 2.0 * float(np.dot(v1._arr, v2._arr)))

    def distance(self, v1, v2):
        return math.sqrt(self._sq(v1, v2))

    def find_closest(self, centroids, point):
        best_sq, best = float("inf"), 0
        for i, c in enumerate(centroids):
            lb = (point.l2_norm - c.l2_norm) ** 2
            if lb >= best_sq:
                continue
            d = self._sq(point, c)
            if d < best_sq:
                best_sq, best = d, i
        return best


class ManhattanDistanceMeasure(DistanceMeasure):
    NAME = "manhattan"

    def distance(self, v1, v2):
        if v1._arr.size != v2._arr.size:
            raise ValueError("vectors must have the same size")
        return float(np.abs(v1._arr - v2._arr).sum())


class CosineDistanceMeasure(DistanceMeasure):
    NAME = "cosine"

    def distance(self, v1, v2):
        if not (v1.l2_norm > 0 and v2.l2_norm > 0):
            raise ValueError("Consine distance is not defined for zero-length vectors.")
        return 1.0 - float(np.dot(v1._arr, v2._arr)) / v1.l2_norm / v2.l2_norm


_INSTANCES = {c.NAME: c() for c in (EuclideanDistanceMeasure, ManhattanDistanceMeasure, CosineDistanceMeasure)}
