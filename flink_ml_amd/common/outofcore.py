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


# (tests: (free, total) device bytes that stand in for hipMemGetInfo in the default budget)
_FREE_OVERRIDE: Optional[tuple] = None
MARGIN_MIN = 4 << 30      # the default budget leaves at least this much of the device free …
MARGIN_FRAC = 0.10        # … or this fraction of its capacity (kernels' scratch, the trainers' buffers)


def hbm_budget(device=None) -> Optional[int]:
    """Device bytes a bounded fit may keep resident: ``FMLX_HBM_BUDGET`` when set; otherwise, on a
    GPU, the device's free memory minus a margin (max(4 GiB, 10 % of its capacity)) — so a
    partition larger than what is free streams by itself, as the reference's data cache spills
    without being asked (``DataCacheWriter.java:101-107,169-178``), instead of failing to
    allocate. None (unlimited) without a GPU."""
    env = parse_bytes(os.environ.get("FMLX_HBM_BUDGET"))
    if env is not None:
        return env
    if _FREE_OVERRIDE is not None:
        free, total = _FREE_OVERRIDE
    else:
        dev = torch.device(device) if device is not None else None
        if dev is None:
            from ..config import compute_device

            dev = compute_device()
        if dev.type != "cuda":
            return None
        free, total = torch.cuda.mem_get_info(dev)
    return max(0, int(free) - max(MARGIN_MIN, int(MARGIN_FRAC * total)))


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


    # (BatchRing interface: byte slots, the bytes of a record, a typed view of a filled slot)
    def slot_bytes(self) -> int:
        return self.batch_bytes

    def record_bytes(self, b: int) -> int:
        return self.rows(b) * self.d * self.es

    def view(self, slot: torch.Tensor, b: int):
        rows = self.rows(b)
        return slot[:rows * self.d * self.es].view(self.dtype).view(rows, self.d)


def _align(x: int, a: int = 16) -> int:
    return -(-x // a) * a


class SparseBatchStore:
    """CSR row batches of a host partition (``SparseColumn``) under an HBM budget — the sparse
    counterpart of ``BatchStore`` (bounded LinearSVC / LR on 1M-wide features): the leading batches
    that fit stay on the device as ONE CSR (indptr rebased to 0; a batch is an indptr window over
    the shared indices / values), the others become DataCache records [indptr rebased (rows + 1)
    int64 | indices int32 | values], streamed through the same ring."""

    def __init__(self, X, B: int, device, budget: Optional[int], ring: int = RING_SLOTS,
                 host_budget: Optional[int] = None, cache_path: Optional[str] = None,
                 segment_bytes: Optional[int] = None):
        ip = X.indptr.to(torch.int64)
        self.indices_h = X.indices.to(torch.int32)
        self.values_h = X.values
        self.size = X.size
        self.B, self.device = max(1, int(B)), torch.device(device)
        self.n = len(X)
        self.dtype = X.values.dtype
        self.es = X.values.element_size()
        self.P = max(1, -(-self.n // self.B)) if self.n else 0
        self.base = int(ip[0]) if self.n else 0
        self.ip_h = ip - self.base
        bnd = [int(self.ip_h[min(self.n, b * self.B)]) for b in range(self.P + 1)]
        self.bounds = bnd
        self.nnz_max = max([bnd[b + 1] - bnd[b] for b in range(self.P)] + [0])
        per = [self.record_bytes(b) for b in range(self.P)]
        if budget is None:
            R = self.P
        else:
            left = budget - ring * self.slot_bytes()
            R = 0
            while R < self.P and left >= per[R]:
                left -= per[R]
                R += 1
        self.R = R
        rows, nz = min(self.n, R * self.B), bnd[R] if self.P else 0
        self.r_indptr = self.ip_h[:rows + 1].to(self.device)
        o = self.base
        self.r_indices = self.indices_h[o:o + nz].to(self.device)
        self.r_values = self.values_h[o:o + nz].to(self.device)
        self.cache = None
        self.recs: List[int] = []
        self._registered: List[int] = []
        if R < self.P:
            kw = {"memory_budget": host_budget if host_budget is not None else host_cache_budget()}
            if segment_bytes:
                kw["segment_bytes"] = segment_bytes
            self.cache = DataCache(path=cache_path, **kw)
            for b in range(R, self.P):
                self.recs.append(self.cache.append(self._record(b)))
            if self.device.type == "cuda":
                for p, cap in self.cache.memory_segments():
                    if native.kernels().fmlx_host_register(p, cap) == 0:
                        self._registered.append(p)

    def _layout(self, rows: int, nz: int):
        o_idx = _align((rows + 1) * 8)
        o_val = _align(o_idx + nz * 4)
        return o_idx, o_val, o_val + nz * self.es

    def _record(self, b: int) -> np.ndarray:
        r0, rows = b * self.B, self.rows(b)
        j0, j1 = self.bounds[b], self.bounds[b + 1]
        o_idx, o_val, total = self._layout(rows, j1 - j0)
        buf = np.zeros(total, dtype=np.uint8)
        buf[:(rows + 1) * 8] = (self.ip_h[r0:r0 + rows + 1] - j0).numpy().view(np.uint8)
        buf[o_idx:o_idx + (j1 - j0) * 4] = self.indices_h[self.base + j0:self.base + j1].numpy().view(np.uint8)
        v = self.values_h[self.base + j0:self.base + j1].contiguous()
        buf[o_val:total] = v.view(torch.uint8).numpy()
        return buf

    def rows(self, b: int) -> int:
        return min(self.n, (b + 1) * self.B) - b * self.B

    def is_resident(self, b: int) -> bool:
        return b < self.R

    def resident_view(self, b: int):
        """(indptr window, indices, values) of a resident batch (absolute offsets)."""
        r0 = b * self.B
        return self.r_indptr[r0:r0 + self.rows(b) + 1], self.r_indices, self.r_values

    def record(self, b: int) -> int:
        return self.recs[b - self.R]

    def slot_bytes(self) -> int:
        return self._layout(self.B, self.nnz_max)[2]

    def record_bytes(self, b: int) -> int:
        return self._layout(self.rows(b), self.bounds[b + 1] - self.bounds[b])[2]

    def view(self, slot: torch.Tensor, b: int):
        rows, nz = self.rows(b), self.bounds[b + 1] - self.bounds[b]
        o_idx, o_val, total = self._layout(rows, nz)
        return (slot[:(rows + 1) * 8].view(torch.int64), slot[o_idx:o_idx + nz * 4].view(torch.int32),
                slot[o_val:total].view(self.dtype))

    def stats(self) -> dict:
        st = {"batches": self.P, "resident": self.R, "streamed": self.P - self.R, "slot_bytes": self.slot_bytes(),
              "sparse": True}
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

    def __init__(self, store, slots: int = RING_SLOTS):
        from ..utils import graphs

        self.store = store
        dev = store.device
        self.K = max(2, int(slots))
        self.slots = [torch.empty(max(1, store.slot_bytes()), dtype=torch.uint8, device=dev) for _ in range(self.K)]
        self.staging = [None] * self.K  # pinned host buffers for file-segment batches (lazily)
        self.copy_stream = graphs.aux_stream(dev, "ooc-h2d")
        self.copied = [torch.cuda.Event() for _ in range(self.K)]
        self.freed = [torch.cuda.Event() for _ in range(self.K)]
        self.staged = [torch.cuda.Event() for _ in range(self.K)]  # last copy out of staging[s]
        self.used = [False] * self.K
        self.next = 0
        self.h2d_bytes = 0

    def fetch(self, b: int):
        """Batch ``b`` in a device slot (the store's typed view); the current stream waits for its
        copy."""
        from ..utils import hostsync

        st = self.store
        s = self.next
        self.next = (s + 1) % self.K
        slot = self.slots[s]
        nbytes = st.record_bytes(b)
        rec = st.record(b)
        src = st.cache.record_ptr(rec)
        if src is None:  # file segment: into this slot's pinned staging buffer first
            if self.staging[s] is None:
                self.staging[s] = torch.empty(max(1, st.slot_bytes()), dtype=torch.uint8, pin_memory=True)
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
        return st.view(slot, b)

    def release(self) -> None:
        """The current stream's work that reads the last fetched slot is queued."""
        self.freed[self._cur].record(torch.cuda.current_stream(self.store.device))


class StreamedGlmTrainer:
    """SGD over a host partition that does not fit the HBM budget (see the module docstring)."""

    def __init__(self, sgd, init_coef, X: torch.Tensor, y: torch.Tensor, weight, loss: str, device,
                 budget: Optional[int], check_every: int = 8, **store_kw):
        from ..parallel.context import get_context
        from .optimizer import DeviceGlmTrainer, local_batch_size

        from ..table import SparseColumn

        ctx = get_context()
        self.sgd = sgd
        dev = torch.device(device)
        self.device = dev
        B = local_batch_size(sgd.global_batch_size, ctx.rank, ctx.world_size)
        self.sparse = isinstance(X, SparseColumn)
        if self.sparse:
            acc = torch.float64 if X.values.dtype == torch.float64 else torch.float32
            X = SparseColumn(X.indptr, X.indices, X.values.to(acc), X.size)
            self.store = SparseBatchStore(X, max(1, B), dev, budget, **store_kw)
        else:
            acc = torch.float64 if X.dtype == torch.float64 else torch.float32
            self.store = BatchStore(X, max(1, B), dev, budget, **store_kw)
        self.ring = BatchRing(self.store) if self.store.R < self.store.P else None
        self.y = y.to(device=dev, dtype=acc).reshape(-1).contiguous()
        self.w = weight.to(device=dev, dtype=acc).reshape(-1).contiguous() if weight is not None else None
        # the inner trainer owns coefficients, device state, scratch and the fused kernel; it is
        # pointed at one batch per launch (n = that batch's rows, so the kernel's batch is the view)
        if self.store.P == 0:
            first = self.store.resident if not self.sparse else self.store.resident_view(0)
        elif self.store.R:
            first = self.store.resident_view(0)
        else:
            first = self.store.view(self.ring.slots[0], 0)
        if self.sparse:
            ip, ix, vv = first
            rows0 = int(ip.shape[0]) - 1
            first = SparseColumn(ip, ix, vv, X.size)
            # every batch runs the single-visit bucket round, its buffers sized for the largest batch
            kw = {"bucket_nnz": (max(1, self.store.nnz_max), self.store.bounds[-1] / max(1, self.store.n))}
        else:
            rows0 = int(first.shape[0])
            kw = {"pad": False}  # (the inner trainer is re-pointed at ring slots of the unpadded width)
        w0 = self.w[:rows0] if self.w is not None else None
        self.inner = DeviceGlmTrainer(sgd, init_coef, first, self.y[:rows0], w0, loss, use_graph=False,
                                      check_every=check_every, **kw)
        self.check_every = max(1, int(check_every))

    def _round(self, e: int) -> None:
        st, tr = self.store, self.inner
        b = e % st.P if st.P else 0
        if st.P == 0:
            Xb = st.resident if not self.sparse else st.resident_view(0)
            lo = 0
        elif st.is_resident(b):
            Xb = st.resident_view(b)
            lo = b * st.B
        else:
            Xb = self.ring.fetch(b)
            lo = b * st.B
        if self.sparse:
            tr.indptr, tr.indices, tr.values = Xb
            rows = int(Xb[0].shape[0]) - 1
        else:
            tr.X = Xb
            rows = int(Xb.shape[0])
        tr.n = rows
        tr.y = self.y[lo:lo + rows]
        if self.w is not None:
            tr.w = self.w[lo:lo + rows]
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
        coef = hostsync.to_host(self.inner.coef[:self.inner.d_model]).to(torch.float64).numpy()
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
