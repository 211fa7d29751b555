"""One-shot small-message all-reduce over xGMI peer memory (``ops/csrc/xgmi_allreduce.hip``).

SURVEY §5 ("Distributed communication backend") / §7.4 hard part 6: the reference's per-round
payloads — SGD feedback ``double[dim+2]`` (``LIB/common/optimizer/SGD.java:252``, reduced by
``CORE/common/datastream/AllReduceImpl.java:54-302``), KMeans ``[k·dim ‖ k]``
(``LIB/clustering/kmeans/KMeans.java:166-173``), OnlineLR ``[grad ‖ weightSum]`` — are 0.8 KB to
0.5 MB: latency bound, where a ring all-reduce pays 2·(P−1) dependent link hops.

Here every rank exports ONE uncached exchange buffer through a dmabuf IPC handle
(``hipIpcGetMemHandle``), maps every peer's buffer (``hipIpcOpenMemHandle``), and an all-reduce
is one kernel per rank that publishes its chunk, waits for the peers' tags and sums the P
records in rank order — bit-identical on every rank, all P−1 xGMI links pulled at once. The
fused SGD round kernel (``glm.hip``, mode ``TAIL_XGMI``) uses the same buffers for its feedback
exchange, so a multi-GPU SGD round is still ONE kernel launch per rank.

Enablement is collective, so ranks never disagree on the path: world sizes 2..8 on a ``nccl``
(RCCL) group, every rank allocates and maps every peer, and a self-test against exact expected
sums passes on ALL ranks; otherwise collectives stay on RCCL. ``FMLX_XGMI=0`` disables the path;
``FMLX_XGMI=force`` also enables it on a gloo group (several ranks sharing one GPU: how the GPU
test rehearses it on a one-GPU box). Every device-side wait is bounded. A wait that gives up
writes NaN instead of a partial sum and raises an error word that lives in host-mapped coherent
memory, so the host reads it with no device sync: ``comm.all_reduce`` checks it before every
xGMI launch and algorithms check it at their host sync points (``check()``); either raises
``XgmiTimeout`` instead of returning numbers computed from a partial exchange.
"""
from __future__ import annotations

import ctypes
import os
import threading
import warnings
from typing import Optional

import torch
import torch.distributed as dist

from ..ops import native
from ..ops.native import c_int, c_long, c_void_p
from .context import get_context

native.register_kernel_sigs({
    "fmlx_xar_total_bytes": ([], c_long),
    "fmlx_xar_chunk": [],
    "fmlx_xar_max_blocks": [],
    "fmlx_xar_max_ranks": [],
    "fmlx_xar_gen_size": [],
    "fmlx_xar_glm_max": [],
    "fmlx_xar_handle_size": [],
    "fmlx_xar_alloc": [c_long, c_void_p, c_void_p],
    "fmlx_xar_open": [c_void_p, c_void_p],
    "fmlx_xar_close": [c_void_p],
    "fmlx_xar_free": [c_void_p],
    "fmlx_host_flags_alloc": [c_int, c_void_p, c_void_p],
    "fmlx_host_flags_free": [c_void_p],
    "fmlx_xar_allreduce": [c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_long, c_void_p, c_void_p, c_void_p,
                           c_long, c_void_p],
    "fmlx_xar_allreduce2": [c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_long, c_void_p, c_void_p, c_void_p,
                            c_long, c_void_p],
    "fmlx_xar_twoshot_max": ([], c_long),
    "fmlx_xar_strict_fence": [],
    "fmlx_xar_set_strict_fence": [c_int],
})


def strict_fence() -> bool:
    """True when the exchange's hand-off uses system-scope release/acquire fences
    (``FMLX_XGMI_STRICT_FENCE=1``, read once per process by the kernel library)."""
    return bool(native.kernels().fmlx_xar_strict_fence())


def set_strict_fence(on: bool) -> None:
    """Switches the system-scope fences on / off for every exchange launched from now on (kernels
    already captured into hipGraphs keep the mode they were captured with)."""
    native.kernels().fmlx_xar_set_strict_fence(int(bool(on)))

# polls (each ≈ one xGMI round trip + s_sleep) before a wait gives up: several seconds, far
# beyond any lockstep drift between ranks, far below a hang
DEFAULT_SPIN = int(os.environ.get("FMLX_XGMI_SPIN", str(1 << 22)))
# payload routing: one-shot pull up to MAX_ONESHOT_ELEMS (latency-bound: one cross-rank wait),
# two-shot (reduce-scatter + all-gather over the peer buffers, 2·(P−1)/P·n per rank on xGMI
# instead of (P−1)·n) up to MAX_TWOSHOT_ELEMS, RCCL above. A 512 KB KMeans payload (k = 1024,
# D = 128) and the 4 MB sparse-SVC feedback (dim 1M) take the two-shot.
MAX_ONESHOT_ELEMS = int(os.environ.get("FMLX_XGMI_MAX_ELEMS", str(1 << 17)))
MAX_TWOSHOT_ELEMS = int(os.environ.get("FMLX_XGMI_TWOSHOT_MAX", str(2 << 20)))


class XgmiTimeout(RuntimeError):
    """A bounded xGMI wait gave up: some peer never arrived (its outputs were poisoned)."""


class HostFlags:
    """int32 words in host-mapped coherent memory, written by kernels, read by the host with no
    device synchronisation (a plain load of pinned host memory)."""

    def __init__(self, n: int = 1):
        lib = native.kernels()
        h, d = c_void_p(), c_void_p()
        rc = lib.fmlx_host_flags_alloc(int(n), ctypes.byref(h), ctypes.byref(d))
        if rc != 0:
            raise RuntimeError("hipHostMalloc of the status words failed (%d)" % rc)
        self.lib, self.n = lib, n
        self.host, self.dev = h.value, d.value
        self._view = (ctypes.c_int32 * n).from_address(self.host)

    def get(self, i: int = 0) -> int:
        return int(self._view[i])

    def clear(self, i: int = 0) -> None:
        self._view[i] = 0

    def close(self) -> None:
        if self.host:
            self.lib.fmlx_host_flags_free(c_void_p(self.host))
            self.host = None


class XgmiComm:
    """Peer-mapped exchange buffers of one process group (one instance per process)."""

    def __init__(self, handles_group=None, spin_limit: int = DEFAULT_SPIN):
        ctx = get_context()
        if not ctx.is_gpu:
            raise RuntimeError("the xGMI exchange needs a GPU")
        lib = native.kernels()
        self.lib = lib
        self.world, self.rank = ctx.world_size, ctx.rank
        self.device = ctx.device
        self.chunk = lib.fmlx_xar_chunk()
        self.max_elems = self.chunk * lib.fmlx_xar_max_blocks()
        self.twoshot_max = int(lib.fmlx_xar_twoshot_max())
        self.glm_max = lib.fmlx_xar_glm_max()
        self.spin_limit = int(spin_limit)
        self._base = None
        self._opened = []
        hs = lib.fmlx_xar_handle_size()
        handle = ctypes.create_string_buffer(hs)
        base = c_void_p()
        rc = -1
        try:
            with torch.cuda.device(self.device):
                rc = lib.fmlx_xar_alloc(lib.fmlx_xar_total_bytes(), ctypes.byref(base), handle)
        except Exception:  # pragma: no cover - reported collectively below
            rc = -1
        mine = bytes(handle.raw) if rc == 0 else None
        if rc == 0:
            self._base = base.value
        handles = [None] * self.world
        dist.all_gather_object(handles, mine, group=handles_group)  # every rank takes part
        if any(h is None for h in handles):
            self.close()
            raise RuntimeError("xGMI exchange buffer allocation failed on some rank")
        ptrs = []
        ok = True
        for r, h in enumerate(handles):
            if r == self.rank:
                ptrs.append(self._base)
                continue
            p = c_void_p()
            if ok and lib.fmlx_xar_open(ctypes.create_string_buffer(h, len(h)), ctypes.byref(p)) == 0 and p.value:
                ptrs.append(p.value)
                self._opened.append(p.value)
            else:
                ok = False
                ptrs.append(0)
        self.map_ok = ok
        self.peers = torch.tensor(ptrs, dtype=torch.int64, device=self.device)  # device pointer table
        self.gen = torch.zeros(lib.fmlx_xar_gen_size(), dtype=torch.int32, device=self.device)
        self.err = HostFlags(1)

    # -- kernel plumbing --------------------------------------------------------------------------
    def kernel_args(self):
        """(peers, world, rank, gen, err, spin_limit) as passed to the HIP launchers."""
        return (self.peers.data_ptr(), self.world, self.rank, self.gen.data_ptr(), self.err.dev,
                self.spin_limit)

    def path(self, n: int) -> str:
        """'oneshot', 'twoshot' or 'rccl' for an n-element payload."""
        if n <= min(self.max_elems, MAX_ONESHOT_ELEMS):
            return "oneshot"
        if n <= min(self.twoshot_max, MAX_TWOSHOT_ELEMS):
            return "twoshot"
        return "rccl"

    def accepts(self, t: torch.Tensor) -> bool:
        """Payloads up to ``FMLX_XGMI_TWOSHOT_MAX`` (default 2M elements = 8 MB fp32): one-shot
        pull up to ``FMLX_XGMI_MAX_ELEMS`` (128K), two-shot above; beyond that RCCL's pipelined
        ring/tree wins on bandwidth."""
        return (t.is_cuda and t.device == self.device and t.dtype in (torch.float32, torch.float64)
                and t.is_contiguous() and self.path(t.numel()) != "rccl")

    def all_reduce_(self, t: torch.Tensor, state: Optional[torch.Tensor] = None, path: Optional[str] = None) -> torch.Tensor:
        """In-place sum over the group (same shape on every rank), stream-ordered on the current
        stream and capturable in a hipGraph. ``state``: optional SGD round state predicating the call.
        ``path``: force 'oneshot' / 'twoshot' (tests); default by size."""
        self.check()  # an earlier exchange of this group gave up: its peers' tags no longer line up
        dt = 0 if t.dtype == torch.float32 else 1
        kind = path or self.path(t.numel())
        fn = "fmlx_xar_allreduce2" if kind == "twoshot" else "fmlx_xar_allreduce"
        native.call(fn, dt, self.peers.data_ptr(), self.world, self.rank, t.data_ptr(),
                    t.data_ptr(), t.numel(), self.gen.data_ptr(), self.err.dev, native.ptr(state),
                    self.spin_limit, native.stream_ptr(t.device))
        return t

    def healthy(self) -> bool:
        """False once any exchange of this group gave up (no device sync: host-mapped word;
        kernels still in flight are seen once they finish)."""
        return self.err.get() == 0

    def check(self) -> None:
        if self.err.get() != 0:
            raise XgmiTimeout("xGMI exchange timed out on rank %d: a peer never arrived; results of the "
                              "affected collectives were poisoned (NaN)" % self.rank)

    def self_test(self) -> bool:
        """Exact-integer sums through both slots, partial and multi-block chunks, f32 and f64."""
        W = self.world
        ok = True
        for dt in (torch.float32, torch.float64):
            for n, kind in ((1, "oneshot"), (1000, "oneshot"), (3 * self.chunk + 5, "oneshot"),
                            (1, "twoshot"), ((2 * W + 1) * self.chunk + 7, "twoshot")):
                for rep in range(2):
                    t = torch.arange(n, device=self.device, dtype=dt) * (self.rank + 1) + (self.rank + rep)
                    self.all_reduce_(t, path=kind)
                    exp = (torch.arange(n, dtype=torch.float64) * (W * (W + 1) // 2)
                           + (W * (W - 1) // 2 + rep * W))
                    ok = ok and bool(torch.equal(t.to(torch.float64).cpu(), exp))
        torch.cuda.synchronize(self.device)
        return ok and self.healthy()

    def close(self) -> None:
        if getattr(self, "err", None) is not None:
            self.err.close()
        for p in self._opened:
            self.lib.fmlx_xar_close(c_void_p(p))
        self._opened = []
        if self._base:
            self.lib.fmlx_xar_free(c_void_p(self._base))
            self._base = None


_COMM: Optional[XgmiComm] = None
_TRIED = False
_LOCK = threading.Lock()


def _all_ok(flag: bool, ctx) -> bool:
    dev = ctx.device if ctx.backend == "nccl" else torch.device("cpu")
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(int(t.item()))


def get() -> Optional[XgmiComm]:
    """The process-wide xGMI exchange, or None when collectives stay on RCCL. The first call is
    collective (every rank of the group must make it) — ``init_distributed`` makes it eagerly."""
    global _COMM, _TRIED
    if _TRIED:
        return _COMM
    with _LOCK:
        if _TRIED:
            return _COMM
        _TRIED = True
        ctx = get_context()
        mode = os.environ.get("FMLX_XGMI", "1").lower()
        if mode in ("0", "off", "false", "no") or not ctx.is_distributed or not ctx.is_gpu:
            return None
        if ctx.backend != "nccl" and mode != "force":
            return None
        if ctx.world_size > native.kernels().fmlx_xar_max_ranks():
            return None
        comm = None
        try:
            comm = XgmiComm()
            ok = comm.map_ok
        except Exception as e:  # allocation failed somewhere: every rank saw it in the gather
            warnings.warn("xGMI exchange unavailable (%s); collectives stay on RCCL" % e)
            return None
        if not _all_ok(ok, ctx):
            comm.close()
            return None
        ok = comm.self_test() and os.environ.get("FMLX_XGMI_INJECT_FAIL", "0") != "1"  # test hook
        if not _all_ok(ok, ctx):
            warnings.warn("xGMI all-reduce self-test failed; collectives stay on RCCL")
            comm.close()
            return None
        _COMM = comm
        return _COMM


def collective_path() -> str:
    """What a device all-reduce of this process runs on: 'none' (no process group), 'xgmi' (the
    one-shot exchange is up), or the process group's backend ('nccl' = RCCL, 'gloo')."""
    ctx = get_context()
    if not ctx.is_distributed:
        return "none"
    return "xgmi" if get() is not None else str(ctx.backend)


def check() -> None:
    """Raises ``XgmiTimeout`` if any xGMI exchange of this process gave up. Cheap (no device sync);
    algorithms call it at their host sync points, after the device work they waited for."""
    if _COMM is not None:
        _COMM.check()


def disable() -> None:
    """Retires the exchange for the rest of the process group's life (after a bounded wait gave
    up, its peers' tags no longer line up): later device all-reduces go to the process group.
    Collective in effect — every rank must call it at the same point (``comm.all_agree`` first)."""
    global _COMM, _TRIED
    with _LOCK:
        if _COMM is not None:
            try:
                torch.cuda.synchronize(_COMM.device)
            finally:
                _COMM.close()
        _COMM = None
        _TRIED = True


def reset() -> None:
    """Forgets the exchange (process-group teardown)."""
    global _COMM, _TRIED
    with _LOCK:
        if _COMM is not None:
            try:
                torch.cuda.synchronize(_COMM.device)
            finally:
                _COMM.close()
        _COMM = None
        _TRIED = False
