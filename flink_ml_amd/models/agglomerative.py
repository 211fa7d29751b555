"""AgglomerativeClustering (reference ``LIB/clustering/agglomerativeclustering``).

Per window (``windowAllAndProcess``, all rows of a window on one rank, like the reference's
parallelism-1 operator):

1. pairwise distances of the window's points on the device — one GEMM for euclidean/cosine
   (``‖a‖² + ‖b‖² − 2a·b`` clamped at 0, exactly ``EuclideanDistanceMeasure``), ``cdist(p=1)``
   for manhattan — copied to the host as the condensed upper triangle;
2. the NN-chain merge loop in native C++ (``csrc/host/nnchain.cpp``), which reproduces the
   reference's HashSet scan order and Lance–Williams updates;
3. merges sorted by distance (stable), relabelled, cut by ``numClusters`` or
   ``distanceThreshold`` and turned into cluster ids with the reference's union-find and
   first-seen remapping.

Outputs: the input rows + ``predictionCol`` (int), and the merge table
(clusterId1, clusterId2, distance, sizeOfMergedCluster).
"""
from __future__ import annotations

import ctypes
from typing import List, Optional

import numpy as np
import torch

from .. import config
from ..api.stage import AlgoOperator
from ..common.param import HasDistanceMeasure, HasFeaturesCol, HasPredictionCol, HasWindows
from ..io import read_write as rw
from ..ops import native
from ..param.param import BooleanParam, FloatParam, IntParam, ParamValidators, StringParam
from ..parallel.datastream import window_all_and_process
from ..table import SparseColumn, Table

LINKAGE_WARD, LINKAGE_COMPLETE, LINKAGE_SINGLE, LINKAGE_AVERAGE = "ward", "complete", "single", "average"
_LINKAGE_CODE = {LINKAGE_WARD: 0, LINKAGE_COMPLETE: 1, LINKAGE_AVERAGE: 2, LINKAGE_SINGLE: 3}

native.register_host_sigs({"fmlx_nnchain": ([ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p],
                                             ctypes.c_int64)})


native.register_kernel_sigs({"fmlx_pairwise_euclid_f64": [ctypes.c_void_p, ctypes.c_long, ctypes.c_int,
                                                             ctypes.c_long, ctypes.c_void_p, ctypes.c_long,
                                                             ctypes.c_int, ctypes.c_void_p]})


def _euclid_device(X: torch.Tensor, condensed: bool) -> torch.Tensor:
    X = X.contiguous()
    n, d = X.shape
    out = torch.empty(n * (n - 1) // 2 if condensed else (n, n), dtype=torch.float64, device=X.device)
    if out.numel():
        native.call("fmlx_pairwise_euclid_f64", native.ptr(X), n, d, max(d, 1), native.ptr(out), n, int(condensed),
                    native.stream_ptr(X.device))
    return out


def condensed_distances(X: torch.Tensor, metric: str) -> np.ndarray:
    """The upper triangle of the distance matrix, row by row (what the NN-chain core reads), on
    the host. Euclidean on the GPU writes it directly (half the copy, no index pass)."""
    X = X.to(torch.float64)
    n = X.shape[0]
    if metric == "euclidean" and X.device.type == "cuda" and 1 < n <= 16 * 65535:
        return _euclid_device(X, True).cpu().numpy()
    pair = pairwise_distances(X, metric).cpu().numpy()
    return np.ascontiguousarray(pair[np.triu_indices(n, 1)], dtype=np.float64)


def pairwise_distances(X: torch.Tensor, metric: str) -> torch.Tensor:
    """Full [n, n] fp64 distance matrix with the reference DistanceMeasure formulas. Euclidean on
    the GPU is one library kernel (csrc/blas.hip pairwise_euclid_f64_kernel): a GEMM plus clamp /
    sqrt passes through torch would also load their code objects lazily, ~60 ms inside the first
    fit of a process."""
    X = X.to(torch.float64)
    if metric == "euclidean" and X.device.type == "cuda" and 0 < X.shape[0] <= 16 * 65535:
        return _euclid_device(X, False)
    if metric == "manhattan":
        return torch.cdist(X, X, p=1)
    sq = (X * X).sum(1)
    dots = X @ X.t()
    if metric == "cosine":
        nrm = torch.sqrt(sq)
        if bool((nrm <= 0).any()):
            raise ValueError("Consine distance is not defined for zero-length vectors.")
        return 1 - dots / nrm[:, None] / nrm[None, :]
    return torch.sqrt(torch.clamp(sq[:, None] + sq[None, :] - 2.0 * dots, min=0.0))


def nn_chain(pair: np.ndarray, n: int, linkage: str):
    """Merges (a, b, merged, dist) in discovery order and node sizes via the native core. ``pair``
    is the full [n, n] matrix or its condensed upper triangle."""
    cond = np.ascontiguousarray(pair if pair.ndim == 1 else pair[np.triu_indices(n, 1)], dtype=np.float64)
    m = max(n - 1, 0)
    a = np.zeros(m, dtype=np.int64)
    b = np.zeros(m, dtype=np.int64)
    merged = np.zeros(m, dtype=np.int64)
    dist = np.zeros(m, dtype=np.float64)
    sizes = np.zeros(max(2 * n - 1, 1), dtype=np.int64)
    lib = native.host()
    got = lib.fmlx_nnchain(cond.ctypes.data if cond.size else None, n, _LINKAGE_CODE[linkage], a.ctypes.data,
                           b.ctypes.data, merged.ctypes.data, dist.ctypes.data, sizes.ctypes.data)
    if got < 0:
        raise RuntimeError("nn-chain failed")
    return a[:got], b[:got], merged[:got], dist[:got], sizes


def _union_find_labels(chain, num_points: int) -> np.ndarray:
    parent = np.full(max(2 * num_points - 1, 1), -1, dtype=np.int64)
    next_label = num_points

    def find(x):
        p = x
        while parent[x] != -1:
            x = parent[x]
        while parent[p] != x and parent[p] != -1:
            p2 = parent[p]
            parent[p] = x
            p = p2
        return x

    for a, b in chain:
        ra, rb = find(a), find(b)
        parent[ra] = next_label
        parent[rb] = next_label
        next_label += 1
    return np.array([find(i) for i in range(num_points)], dtype=np.int64)


class AgglomerativeClusteringParams(HasDistanceMeasure, HasFeaturesCol, HasPredictionCol, HasWindows):
    LINKAGE_WARD, LINKAGE_COMPLETE, LINKAGE_SINGLE, LINKAGE_AVERAGE = (LINKAGE_WARD, LINKAGE_COMPLETE, LINKAGE_SINGLE,
                                                                       LINKAGE_AVERAGE)
    NUM_CLUSTERS = IntParam("numClusters", "The max number of clusters to create.", 2)
    DISTANCE_THRESHOLD = FloatParam("distanceThreshold", "Threshold to decide whether two clusters should be merged.",
                                    None)
    LINKAGE = StringParam("linkage", "Criterion for computing distance between two clusters.", LINKAGE_WARD,
                          ParamValidators.in_array(LINKAGE_WARD, LINKAGE_COMPLETE, LINKAGE_AVERAGE, LINKAGE_SINGLE))
    COMPUTE_FULL_TREE = BooleanParam("computeFullTree", "Whether computes the full tree after convergence.", False,
                                     ParamValidators.not_null())


@rw.register_stage
class AgglomerativeClustering(AlgoOperator, AgglomerativeClusteringParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.clustering.agglomerativeclustering.AgglomerativeClustering"

    def _cluster_window(self, t: Table, merges_out: list) -> Optional[Table]:
        n = t.num_rows
        if n == 0:
            return None
        c = t.column(self.get(self.FEATURES_COL))
        dev = config.compute_device()
        X = c.to_dense(torch.float64, device=dev) if isinstance(c, SparseColumn) else \
            config.features_for_compute(t, self.get(self.FEATURES_COL), allow_sparse=False).to(dev, torch.float64)
        pair = condensed_distances(X, self.get(self.DISTANCE_MEASURE))
        a, b, merged, dist, sizes = nn_chain(pair, n, self.get(self.LINKAGE))
        order = np.argsort(dist, kind="stable")
        chain = [[int(a[i]), int(b[i]), int(merged[i]), float(dist[i])] for i in order]
        # reOrderNnChain: renumber merged clusters in sorted order
        next_id = len(chain) + 1
        mapping = {}
        for item in chain:
            item[0] = mapping.get(item[0], item[0])
            item[1] = mapping.get(item[1], item[1])
            mapping[item[2]] = next_id
            next_id += 1
        thr = self.get(self.DISTANCE_THRESHOLD)
        stopped = sum(1 for it in chain if it[3] <= thr) if thr is not None else n - self.get(self.NUM_CLUSTERS)
        stopped = max(0, min(stopped, len(chain)))
        labels = _union_find_labels([(it[0], it[1]) for it in chain[:stopped]], len(chain) + 1)
        remap, ids = {}, np.empty(n, dtype=np.int64)
        for i in range(n):
            ids[i] = remap.setdefault(int(labels[i]), len(remap))
        if self.get(self.COMPUTE_FULL_TREE):
            stopped = len(chain)
        for it in chain[:stopped]:
            c1, c2 = min(it[0], it[1]), max(it[0], it[1])
            merges_out.append((c1, c2, it[3], int(sizes[c1] + sizes[c2])))
        return t.with_column(self.get(self.PREDICTION_COL), torch.from_numpy(ids.astype(np.int32)))

    def transform(self, *inputs) -> List[Table]:
        nc, thr = self.get(self.NUM_CLUSTERS), self.get(self.DISTANCE_THRESHOLD)
        if not ((nc is None) != (thr is None)):
            raise ValueError("One of param numCluster and distanceThreshold should be null.")
        if self.get(self.LINKAGE) == LINKAGE_WARD and self.get(self.DISTANCE_MEASURE) != "euclidean":
            raise ValueError("%s was provided as distance measure while linkage was ward. Ward only works with "
                             "euclidean." % self.get(self.DISTANCE_MEASURE))
        merges: list = []
        t = inputs[0]
        out = window_all_and_process(t, self.get(self.WINDOWS), lambda w: self._cluster_window(w, merges))
        if out is None:
            cols = {n: [] for n in t.column_names}
            cols[self.get(self.PREDICTION_COL)] = torch.zeros(0, dtype=torch.int32)
            out = Table(cols, num_rows=0)
        merge_table = Table({"clusterId1": torch.tensor([m[0] for m in merges], dtype=torch.int64),
                             "clusterId2": torch.tensor([m[1] for m in merges], dtype=torch.int64),
                             "distance": torch.tensor([m[2] for m in merges], dtype=torch.float64),
                             "sizeOfMergedCluster": torch.tensor([m[3] for m in merges], dtype=torch.int64)},
                            num_rows=len(merges))
        return [out, merge_table]
