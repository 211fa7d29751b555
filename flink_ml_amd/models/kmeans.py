"""KMeans / KMeansModel (reference ``LIB/clustering/kmeans/KMeans.java``, ``KMeansModel.java``,
``KMeansModelData.java``).

fit: random init by the reference's two-level reservoir sample (``KMeans.java:310-327`` →
``DataStreamUtils.sample``, per-partition ``java.util.Random(seed)`` then a parallelism-1 pass)
then ``maxIter`` Lloyd rounds (``TerminateOnMaxIter``). Each round on MI355X: fused MFMA
distance + argmin kernel over the HBM-resident partition, deterministic ordered chunk sums,
ONE RCCL all-reduce of ``[k·D sums | k counts]`` (replacing the gather-to-one reduce + broadcast,
C3 in SURVEY §2.2), and a finalize kernel that also prepares the next round's bf16 centroids.
Empty clusters become NaN centroids exactly like ``BLAS.scal(1/0)`` in the reference.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from .. import config
from ..api.stage import Estimator
from ..common.param import HasDistanceMeasure, HasFeaturesCol, HasMaxIter, HasPredictionCol, HasSeed
from ..io import read_write as rw
from ..io import serialization as ser
from ..linalg.vectors import DenseVector
from ..ops import kmeans as kk
from ..ops import native
from ..param.param import IntParam, ParamValidators, StringParam
from ..parallel import comm
from ..parallel.context import get_context
from ..table import SparseColumn, Table
from ..utils import graphs, tracing
from .base import ModelWithData
from .linear import rw_update

native.register_host_sigs({"fmlx_reservoir_sample": ([ctypes.c_int64, ctypes.c_int32, ctypes.c_int64,
                                                      ctypes.c_void_p], ctypes.c_int)})


def reservoir_sample_indices(n: int, k: int, seed: int) -> np.ndarray:
    """Positions chosen by ``SamplingOperator`` (java.util.Random reservoir), in slot order."""
    out = np.zeros(max(min(n, k), 0), dtype=np.int64)
    if n == 0 or k == 0:
        return out
    cnt = native.host().fmlx_reservoir_sample(int(n), int(k), int(seed), out.ctypes.data)
    return out[:cnt]


def sample_rows(X: torch.Tensor, k: int, seed: int) -> np.ndarray:
    """``DataStreamUtils.sample``: reservoir per rank (only the k chosen rows leave the device),
    gather in rank order, reservoir again over the union."""
    draw_dev = X.device if X.device.type == "cuda" else config.compute_device()
    if draw_dev.type == "cuda":
        # the n-long draw stream in parallel on the device (bit-exact; ops/datagen.py); only the
        # k chosen rows leave HBM (a host-resident out-of-core partition: the draw still runs on
        # the GPU, the k rows are gathered on the host)
        from ..ops.datagen import reservoir_sample_device

        idx = reservoir_sample_device(int(X.shape[0]), k, seed, draw_dev)
    else:
        idx = torch.as_tensor(reservoir_sample_indices(int(X.shape[0]), k, seed))
    local = X[idx.to(X.device)].to(torch.float64).cpu().numpy() if len(idx) else np.zeros((0, X.shape[1]))
    gathered = comm.all_gather_object(local)
    allrows = np.concatenate([g for g in gathered if g.shape[0] > 0], axis=0) if any(
        g.shape[0] for g in gathered) else np.zeros((0, X.shape[1]))
    return allrows[reservoir_sample_indices(allrows.shape[0], k, seed)]


class KMeansModelParams(HasDistanceMeasure, HasFeaturesCol, HasPredictionCol):
    K = IntParam("k", "The max number of clusters to create.", 2, ParamValidators.gt(1))


class KMeansParams(HasSeed, HasMaxIter, KMeansModelParams):
    INIT_MODE = StringParam("initMode", "The initialization algorithm. Supported options: 'random'.", "random",
                            ParamValidators.in_array("random"))


def _encode_kmeans(out, row):
    cents, weights = row[0], row[1]
    out.write_int(len(cents))
    for c in cents:
        ser.write_dense_vector(out, c.to_dense() if hasattr(c, "to_dense") else DenseVector(c))
    ser.write_dense_vector(out, weights.to_dense() if hasattr(weights, "to_dense") else DenseVector(weights))


def _decode_kmeans(inp):
    k = inp.read_int()
    cents = [ser.read_dense_vector(inp) for _ in range(k)]
    return (cents, ser.read_dense_vector(inp))


def kmeans_model_data_table(centroids: np.ndarray, weights: np.ndarray) -> Table:
    return Table({"centroids": [[DenseVector(c) for c in centroids]],
                  "weights": [DenseVector(weights)]}, num_rows=1)


@rw.register_stage
class KMeansModel(ModelWithData, KMeansModelParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.clustering.kmeans.KMeansModel"
    MODEL_DATA_COLUMNS = ("centroids", "weights")
    encode_record = staticmethod(_encode_kmeans)
    decode_record = staticmethod(_decode_kmeans)

    @classmethod
    def make_model_data_table(cls, rows):
        r = rows[0]
        return Table({"centroids": [list(r[0])], "weights": [r[1]]}, num_rows=1)

    def _build_state(self, rows):
        cents, weights = rows[-1][0], rows[-1][1]
        C = np.stack([c.to_array() for c in cents]) if len(cents) else np.zeros((0, 0))
        return torch.as_tensor(C, dtype=torch.float64), torch.as_tensor(weights.to_array(), dtype=torch.float64)

    def centroids(self) -> np.ndarray:
        return self._model_state()[0].numpy()

    def transform(self, *inputs: Table):
        t = inputs[0]
        C, _ = self._model_state()
        if C.shape[0] > self.get(self.K):
            raise ValueError("number of centroids %d exceeds k=%d" % (C.shape[0], self.get(self.K)))
        X = config.features_for_compute(t, self.get(self.FEATURES_COL), allow_sparse=False)
        metric = self.get(self.DISTANCE_MEASURE)
        if X.device.type == "cuda":
            cb = kk.CentroidBuffers(C.shape[0], C.shape[1], X.device,
                                    torch.float64 if X.dtype == torch.float64 else torch.float32)
            cb.set(C)
            pred = kk.assign(X, cb, metric).to(torch.int64)
        else:
            pred = kk.torch_assign(X, C, metric)
        return [t.with_column(self.get(self.PREDICTION_COL), pred)]


@rw.register_stage
class KMeans(Estimator, KMeansParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.clustering.kmeans.KMeans"

    def fit(self, *inputs: Table) -> KMeansModel:
        t = inputs[0]
        fcol = self.get(self.FEATURES_COL)
        Xh = config.host_features_if_oversized(t, fcol)  # larger than FMLX_HBM_BUDGET: stays on the host
        X = Xh if Xh is not None else config.features_for_compute(t, fcol, allow_sparse=False)
        k = self.get(self.K)
        metric = self.get(self.DISTANCE_MEASURE)
        init = sample_rows(X, k, self.get_seed())
        if Xh is not None:
            from ..common.outofcore import hbm_budget, streamed_kmeans

            cents, weights = streamed_kmeans(Xh, init, self.get(self.MAX_ITER), metric, config.compute_device(),
                                             hbm_budget(config.compute_device()))
        else:
            cents, weights = kmeans_lloyd(X, init, self.get(self.MAX_ITER), metric)
        model = KMeansModel().set_model_data(kmeans_model_data_table(cents, weights))
        rw_update(model, self)
        return model


def _graph_ok(ck, log: bool) -> bool:
    """A KMeans round can be replayed from a hipGraph: no per-round host work (checkpoints,
    round logs) and a capturable collective (single rank, or RCCL / the xGMI kernel)."""
    import os

    ctx = get_context()
    return (os.environ.get("FMLX_HIPGRAPH", "1") == "1" and not ck.interval and not log
            and (not ctx.is_distributed or ctx.backend == "nccl"))


def kmeans_lloyd(X: torch.Tensor, init: np.ndarray, max_iter: int, metric: str):
    """``maxIter`` Lloyd rounds; returns (centroids [k,D] f64, weights [k] f64)."""
    from ..parallel.checkpoint import AlgorithmCheckpoint, fault_point

    kc, D = init.shape
    ck = AlgorithmCheckpoint("kmeans")
    start, restored = 0, ck.restore()
    if restored is not None:
        start, st = restored
        init, counts0 = st["centroids"].numpy(), st["weights"]
    if X.device.type == "cuda":
        acc = torch.float64 if X.dtype == torch.float64 else torch.float32
        cb = kk.CentroidBuffers(kc, D, X.device, acc)
        cb.set(torch.as_tensor(init))
        if restored is not None:
            cb.weights.copy_(counts0.to(cb.weights.dtype))
        rnd = kk.KMeansRound(X, kc, metric)
        log = tracing.rounds_enabled()
        if _graph_ok(ck, log) and max_iter - start >= 3:
            # the round is host-sync free: run it once eagerly (warm-up), capture ONE round into a
            # hipGraph and replay it for the remaining rounds (one submission per round)
            with tracing.range("kmeans.fit"):
                fault_point(start)
                payload = rnd.run(cb)
                comm.all_reduce_sum(payload)
                rnd.finalize(cb, payload)

                def one_round():
                    p = rnd.run(cb)
                    comm.all_reduce_sum(p)
                    rnd.finalize(cb, p)

                g = graphs.capture(one_round, X.device)
                # the capture did not execute the round: replay max_iter - start - 1 times
                for e in range(start + 1, max_iter):
                    fault_point(e)
                    g.replay()
            out = cb.cent.to(torch.float64).cpu().numpy(), cb.weights.cpu().numpy()
            comm.check_collectives()
            return out
        with tracing.range("kmeans.fit"):
            for e in range(start, max_iter):
                fault_point(e)
                with tracing.range("kmeans.round"):
                    if log:
                        evs = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                        evs[0].record()
                    payload = rnd.run(cb)
                    if log:
                        evs[1].record()
                    comm.all_reduce_sum(payload)
                    if log:
                        evs[2].record()
                    rnd.finalize(cb, payload)
                if log:
                    evs[2].synchronize()
                    tracing.log_round(kind="kmeans", rank=get_context().rank, epoch=e,
                                      kernel_ms=round(evs[0].elapsed_time(evs[1]), 4),
                                      collective_ms=round(evs[1].elapsed_time(evs[2]), 4),
                                      bytes=int(payload.numel() * payload.element_size()))
                ck.maybe_save(e + 1, lambda: {"centroids": cb.cent.to(torch.float64), "weights": cb.weights})
        out = cb.cent.to(torch.float64).cpu().numpy(), cb.weights.cpu().numpy()
        comm.check_collectives()  # after the host sync: no round used a partial xGMI exchange
        return out
    C = torch.as_tensor(init, dtype=torch.float64)
    counts = counts0.to(torch.float64) if restored is not None else torch.zeros(kc, dtype=torch.float64)
    for e in range(start, max_iter):
        fault_point(e)
        payload = comm.all_reduce_sum(kk.torch_round_payload(X, C, metric))
        C, counts = kk.torch_finalize(payload, kc, D)
        ck.maybe_save(e + 1, lambda: {"centroids": C, "weights": counts})
    return C.numpy(), counts.numpy()
