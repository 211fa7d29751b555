"""Out-of-core bounded training: partitions larger than the HBM budget.

The reference caches every training partition in operator state that spills to disk and then
iterates over it: ``SGD.java:297-300,331-336`` (``trainDataState``), ``KMeans.java:242-248``
(``ListStateWithCache``), with the spill mechanics of
``ITER/datacache/nonkeyed/DataCacheWriter.java:101-107,169-178``. Here the same three-level cache
is HBM → host memory → disk:

* ``BatchStore`` cuts a host-resident partition into the trainer's row batches. The leading batches
  that fit the HBM budget (``FMLX_HBM_BUDGET``, bytes, suffixes K/M/G/T) are copied to the device
  once and stay there; the others go into the native ``DataCache`` (``parallel/datacache.py``) —
  memory segments up to its host budget (``FMLX_HOST_CACHE_BUDGET``), files under
  ``FMLX_DATA_CACHE_PATH`` beyond it. Memory segments are pinned in place
  (``hipHostRegister``), so a cached batch is DMA'd straight from the cache, with no staging copy.
* ``BatchRing`` streams the non-resident batches through a ring of device slots on a dedicated
  copy stream: the copy of batch b waits only for the round that last used its slot (a
  device-side event wait), the round that reads it waits only for its copy, so H2D copies of
  coming batches run under the current rounds' kernels. File-segment batches are read into a
  pinned staging buffer of the slot first (host side, after that slot's previous copy finished).
* ``StreamedGlmTrainer`` runs the fused SGD round kernel (``DeviceGlmTrainer``) on each round's
  batch wherever it lives: round e visits batch e mod P exactly as ``SGD.java:263-268`` does.
  The termination check never drains the pipeline: the device state is copied to pinned memory
  asynchronously and read at the next check interval if that copy has landed.
* ``streamed_kmeans`` runs Lloyd iterations over the same store: every iteration visits all
  batches (assign + ordered cluster sums per batch, payloads added in batch order), then one
  all-reduce and the centroid update (``KMeans.java:285-296``).
"""
from __future__ import annotations

import os
import re
from typing import List, Optional

import numpy as np
import torch

from ..ops import native
from ..parallel.datacache import DataCache


def parse_bytes(v: Optional[str]) -> Optional[int]:
    """'12G' / '512M' / '1000000' → bytes (None / '' → None)."""
    if v is None or str(v).strip() == "":
        return None
    m = re.fullmatch(r"\s*([0-9.]+)\s*([kKmMgGtT]?)[iI]?[bB]?\s*", str(v))
    if not m:
        raise ValueError("bad byte size %r" % v)
    mult = {"": 1, "k": 1 << 10, "m": 1 << 20, "g": 1 << 30, "t": 1 << 40}[m.group(2).lower()]
    return int(float(m.group(1)) * mult)


def hbm_budget() -> Optional[int]:
    """FMLX_HBM_BUDGET: device bytes a bounded fit may keep resident (None: unlimited)."""
    return parse_bytes(os.environ.get("FMLX_HBM_BUDGET"))


def host_cache_budget() -> int:
    return parse_bytes(os.environ.get("FMLX_HOST_CACHE_BUDGET")) or (64 << 30)


RING_SLOTS = int(os.environ.get("FMLX_OOC_RING", "3"))


class BatchStore:
    """Row batches of a host partition: the leading ``resident`` ones on the device, the rest in a
    DataCache (pinned memory segments, then files)."""

    def __init__(self, X: torch.Tensor, B: int, device, budget: Optional[int], ring: int = RING_SLOTS,
                 host_budget: Optional[int] = None, cache_path: Optional[str] = None,
                 segment_bytes: Optional[int] = None):
        if X.dim() != 2:
            raise ValueError("dense row batches only")
        self.X, self.B, self.device = X, max(1, int(B)), torch.device(device)
        self.n, self.d = int(X.shape[0]), int(X.shape[1])
        self.dtype = X.dtype
        self.es = X.element_size()
        self.P = max(1, -(-self.n // self.B)) if self.n else 0
        self.batch_bytes = self.B * self.d * self.es
        if budget is None:
            R = self.P
        else:
            R = max(0, min(self.P, budget // max(1, self.batch_bytes) - ring))
        self.R = R
        on_dev = self.device.type == "cuda"
        # resident prefix: one device tensor, filled chunk by chunk from (pinned) host memory
        rows = min(self.n, R * self.B)
        self.resident = torch.empty((rows, self.d), dtype=self.dtype, device=self.device)
        for s in range(0, rows, self.B):
            e = min(rows, s + self.B)
            self.resident[s:e].copy_(X[s:e], non_blocking=False)
        self.cache = None
        self.recs: List[int] = []
        self._registered: List[int] = []
        if R < self.P:
            kw = {"memory_budget": host_budget if host_budget is not None else host_cache_budget()}
            if segment_bytes:
                kw["segment_bytes"] = segment_bytes
            self.cache = DataCache(path=cache_path, **kw)
            for b in range(R, self.P):
                s, e = b * self.B, min(self.n, (b + 1) * self.B)
                self.recs.append(self.cache.append(X[s:e].contiguous().view(torch.uint8).reshape(-1).numpy()))
            if on_dev:
                for p, cap in self.cache.memory_segments():  # DMA straight from the cache
                    if native.kernels().fmlx_host_register(p, cap) == 0:
                        self._registered.append(p)

    def rows(self, b: int) -> int:
        return min(self.n, (b + 1) * self.B) - b * self.B

    def is_resident(self, b: int) -> bool:
        return b < self.R

    def resident_view(self, b: int) -> torch.Tensor:
        return self.resident[b * self.B: b * self.B + self.rows(b)]

    def record(self, b: int) -> int:
        return self.recs[b - self.R]

    def stats(self) -> dict:
        st = {"batches": self.P, "resident": self.R, "streamed": self.P - self.R, "batch_bytes": self.batch_bytes}
        if self.cache is not None:
            st.update({"cache_" + k: v for k, v in self.cache.stats().items()})
        return st

    def close(self) -> None:
        for p in self._registered:
            native.kernels().fmlx_host_unregister(p)
        self._registered = []
        if self.cache is not None:
            self.cache.close()
            self.cache = None


class BatchRing:
    """Device slots the non-resident batches are streamed into (see the module docstring)."""

    def __init__(self, store: BatchStore, slots: int = RING_SLOTS):
        from ..utils import graphs

        self.store = store
        dev = store.device
        self.K = max(2, int(slots))
        self.slots = [torch.empty((store.B, store.d), dtype=store.dtype, device=dev) for _ in range(self.K)]
        self.staging = [None] * self.K  # pinned host buffers for file-segment batches (lazily)
        self.copy_stream = graphs.aux_stream(dev, "ooc-h2d")
        self.copied = [torch.cuda.Event() for _ in range(self.K)]
        self.freed = [torch.cuda.Event() for _ in range(self.K)]
        self.staged = [torch.cuda.Event() for _ in range(self.K)]  # last copy out of staging[s]
        self.used = [False] * self.K
        self.next = 0
        self.h2d_bytes = 0

    def fetch(self, b: int) -> torch.Tensor:
        """Slot holding batch ``b``; the current stream waits for its copy."""
        from ..utils import hostsync

        st = self.store
        s = self.next
        self.next = (s + 1) % self.K
        slot = self.slots[s]
        rows = st.rows(b)
        nbytes = rows * st.d * st.es
        rec = st.record(b)
        src = st.cache.record_ptr(rec)
        if src is None:  # file segment: into this slot's pinned staging buffer first
            if self.staging[s] is None:
                self.staging[s] = torch.empty(st.batch_bytes, dtype=torch.uint8, pin_memory=True)
            if self.used[s]:
                hostsync.wait_event(self.staged[s])  # its previous copy out of staging is done
            st.cache.read_into(rec, self.staging[s])
            src = self.staging[s].data_ptr()
        cs = self.copy_stream
        if self.used[s]:
            cs.wait_event(self.freed[s])  # the round that last read this slot has run
        native.call("fmlx_memcpy_h2d", slot.data_ptr(), src, nbytes, cs.cuda_stream)
        self.copied[s].record(cs)
        self.staged[s].record(cs)
        self.h2d_bytes += nbytes
        torch.cuda.current_stream(st.device).wait_event(self.copied[s])
        self.used[s] = True
        self._cur = s
        return slot[:rows]

    def release(self) -> None:
        """The current stream's work that reads the last fetched slot is queued."""
        self.freed[self._cur].record(torch.cuda.current_stream(self.store.device))


class StreamedGlmTrainer:
    """SGD over a host partition that does not fit the HBM budget (see the module docstring)."""

    def __init__(self, sgd, init_coef, X: torch.Tensor, y: torch.Tensor, weight, loss: str, device,
                 budget: Optional[int], check_every: int = 8, **store_kw):
        from ..parallel.context import get_context
        from .optimizer import DeviceGlmTrainer, local_batch_size

        ctx = get_context()
        self.sgd = sgd
        dev = torch.device(device)
        self.device = dev
        B = local_batch_size(sgd.global_batch_size, ctx.rank, ctx.world_size)
        self.store = BatchStore(X, max(1, B), dev, budget, **store_kw)
        self.ring = BatchRing(self.store) if self.store.R < self.store.P else None
        acc = torch.float64 if X.dtype == torch.float64 else torch.float32
        self.y = y.to(device=dev, dtype=acc).reshape(-1).contiguous()
        self.w = weight.to(device=dev, dtype=acc).reshape(-1).contiguous() if weight is not None else None
        # the inner trainer owns coefficients, device state, scratch and the fused kernel; it is
        # pointed at one batch per launch (n = that batch's rows, so the kernel's batch is the view)
        first = self.store.resident_view(0) if self.store.R else self.ring.slots[0]
        w0 = self.w[:first.shape[0]] if self.w is not None else None
        # (pad=False: the inner trainer is re-pointed at ring slots of the unpadded width)
        self.inner = DeviceGlmTrainer(sgd, init_coef, first, self.y[:first.shape[0]], w0, loss, use_graph=False,
                                      check_every=check_every, pad=False)
        self.check_every = max(1, int(check_every))

    def _round(self, e: int) -> None:
        st, tr = self.store, self.inner
        b = e % st.P if st.P else 0
        if st.P == 0:
            Xb = st.resident
            lo = 0
        elif st.is_resident(b):
            Xb = st.resident_view(b)
            lo = b * st.B
        else:
            Xb = self.ring.fetch(b)
            lo = b * st.B
        tr.X = Xb
        tr.n = Xb.shape[0]
        tr.y = self.y[lo:lo + Xb.shape[0]]
        if self.w is not None:
            tr.w = self.w[lo:lo + Xb.shape[0]]
        tr._launch_round(1)
        tr._launched += 1
        if self.ring is not None and st.P and not st.is_resident(b):
            self.ring.release()

    def fit(self) -> np.ndarray:
        from ..utils import hostsync, tracing

        with tracing.range("sgd.fit.streamed"):
            for e in range(self.sgd.max_iter):
                self._round(e)
                if (e + 1) % self.check_every == 0 and self.inner._poll_stopped():
                    break
            self.inner.flush()
        coef = hostsync.to_host(self.inner.coef).to(torch.float64).numpy()
        self.inner.check_exchange()
        return coef

    def rounds_executed(self) -> int:
        return self.inner.rounds_executed()

    def close(self) -> None:
        self.store.close()


# rows per KMeans batch of the out-of-core Lloyd loop (FMLX_OOC_KMEANS_ROWS)
KMEANS_BATCH_ROWS = int(os.environ.get("FMLX_OOC_KMEANS_ROWS", str(1 << 21)))


def streamed_kmeans(X: torch.Tensor, init: np.ndarray, max_iter: int, metric: str, device,
                    budget: Optional[int], batch_rows: int = 0, **store_kw):
    """Lloyd iterations over a host partition larger than the HBM budget: every iteration visits
    all row batches (resident ones in place, the others streamed through the ring), each batch runs
    assign → stable grouping → ordered gather-sums (ops/kmeans.KMeansRound), the batches' [sums |
    counts] payloads are added in batch order (deterministic), then one all-reduce and the centroid
    update, as ``KMeans.java:285-296`` reduces its CentroidsUpdateAccumulator. Returns
    (centroids [k, D] f64, weights [k] f64)."""
    from ..ops import kmeans as kk
    from ..parallel import comm
    from ..utils import hostsync, tracing

    dev = torch.device(device)
    kc, D = init.shape
    store = BatchStore(X, batch_rows or KMEANS_BATCH_ROWS, dev, budget, **store_kw)
    ring = BatchRing(store) if store.R < store.P else None
    acc = torch.float64 if X.dtype == torch.float64 else torch.float32
    cb = kk.CentroidBuffers(kc, D, dev, acc)
    cb.set(torch.as_tensor(init))
    rounds = {}  # one KMeansRound per (base pointer, rows): resident views and ring slots

    def round_for(Xb: torch.Tensor):
        key = (Xb.data_ptr(), Xb.shape[0])
        r = rounds.get(key)
        if r is None:
            r = rounds[key] = kk.KMeansRound(Xb, kc, metric)
        return r

    total = torch.zeros(kc * D + kc, dtype=acc, device=dev)
    try:
        with tracing.range("kmeans.fit.streamed"):
            for _ in range(max_iter):
                total.zero_()
                rnd = None
                for b in range(store.P):
                    Xb = store.resident_view(b) if store.is_resident(b) else ring.fetch(b)
                    rnd = round_for(Xb)
                    total.add_(rnd.run(cb))
                    if not store.is_resident(b):
                        ring.release()
                comm.all_reduce_sum(total)
                if rnd is None:
                    rnd = round_for(store.resident)
                rnd.finalize(cb, total)
        cent = hostsync.to_host(cb.cent).to(torch.float64).numpy()
        weights = hostsync.to_host(cb.weights).numpy()
        comm.check_collectives()
        return cent, weights
    finally:
        store.close()
