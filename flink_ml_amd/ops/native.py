"""Loader for the in-tree native libraries (ctypes, flat C ABI).

The HIP kernels are plain ``extern "C"`` launchers that take device pointers and a
``hipStream_t``; we launch them onto torch's *current* HIP stream, so they order correctly
with torch ops and RCCL collectives and can be captured into a hipGraph
(``torch.cuda.CUDAGraph``) together with them.

Debugging: ``FMLX_SYNC_CHECK=1`` synchronises the device after every native launch and reports an
asynchronous fault under the name of the kernel that caused it (the HIP analogue of a blocking
launch mode; slow, off by default).

Policy: on a GPU host the native library is REQUIRED — ``kernels()`` raises if it is
missing (no silent eager fallback). On CPU-only hosts the ops layer runs its torch reference
implementation (same semantics, fp64), which is what the CPU test-suite exercises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must be imported first: our .so binds to torch's libamdhip64.so.7)

from . import build as _build

_LOCK = threading.Lock()
_KLIB = None
_HLIB = None
# one-time cost of loading every code object of the kernel library at library load (host ms;
# None: not done — no GPU, or FMLX_PRELOAD=0), and the number of code objects
PRELOAD_MS = None
PRELOAD_OBJECTS = 0
BKT_LIMITS = None  # the bucket round's compile-time limits (ops/glm.py _bkt_limits), read at load
PRELOAD_STAGES = {}  # ms per stage of the library load (code objects, pinned blocks, dry launches, pool)

DT_F32, DT_F64, DT_BF16, DT_F16, DT_I32, DT_I64 = 0, 1, 2, 3, 4, 5

_TORCH2DT = {
    torch.float32: DT_F32,
    torch.float64: DT_F64,
    torch.bfloat16: DT_BF16,
    torch.float16: DT_F16,
    torch.int32: DT_I32,
    torch.int64: DT_I64,
}

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_long = ctypes.c_long
c_ulonglong = ctypes.c_ulonglong
c_double = ctypes.c_double
c_float = ctypes.c_float

# name -> argtypes (restype is always int: hipError_t, 0 == success)
_KERNEL_SIGS = {
    # glm.hip
    "fmlx_glm_grad_partials": [c_int, c_int, c_int, c_int, c_void_p, c_long, c_void_p, c_void_p, c_void_p, c_long, c_int,
                               c_long, c_int, c_void_p, c_void_p, c_int, c_void_p],
    "fmlx_glm_round": [c_int, c_int, c_int, c_int, c_void_p, c_long, c_void_p, c_void_p, c_void_p, c_long, c_int,
                       c_long, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                       c_int, c_double,
                       c_double, c_double, c_double, c_void_p, c_int, c_int, c_void_p, c_void_p, c_long, c_int, c_int,
                       c_int, c_int, c_void_p, c_void_p],
    "fmlx_glm_round_wide": [c_int, c_int, c_int, c_void_p, c_long, c_void_p, c_void_p, c_void_p, c_long, c_int, c_long,
                            c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, c_double, c_double,
                            c_double, c_double, c_void_p],
    "fmlx_glm_set_tuning": [c_long, c_int],
    "fmlx_glm_set_tail_tuning": [c_int, c_int],
    "fmlx_glm_set_trace": ([c_void_p], None),
    "fmlx_glm_cnt_elems": [],
    "fmlx_glm_set_dma": [c_int],
    "fmlx_glm_acc_elems": ([c_int], c_long),
    "fmlx_glm_reduce_update": [c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                               c_double, c_double, c_double, c_double, c_void_p],
    "fmlx_glm_reduce": [c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "fmlx_glm_update": [c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_double, c_double, c_double, c_double,
                        c_void_p],
    "fmlx_glm_predict": [c_int, c_int, c_int, c_void_p, c_long, c_long, c_int, c_void_p, c_int, c_double, c_void_p,
                         c_void_p, c_void_p],
    "fmlx_glm_grad_csr": [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_int, c_long,
                          c_int, c_void_p, c_void_p, c_void_p],
    "fmlx_glm_csr_predict": [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_void_p, c_void_p],
    "fmlx_glm_set_csc_tuning": [c_int, c_int],
    "fmlx_glm_set_cell_xcd": ([c_int], None),
    "fmlx_glm_wl_elems": [],
    "fmlx_glm_csc_round": [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_int,
                           c_long, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                           c_int, c_double, c_double, c_double, c_double, c_void_p, c_void_p, c_int, c_int, c_int,
                           c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                           c_void_p, c_void_p, c_void_p],
    # glm_sparse.hip: single-visit bucket round
    "fmlx_glm_bkt_limits": [c_void_p],
    "fmlx_glm_sparse_set_trace": ([c_void_p], None),
    "fmlx_glm_bkt_round": [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_int,
                           c_long, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_double, c_double, c_double,
                           c_double, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                           c_long, c_void_p, c_void_p, c_void_p, c_int, c_void_p],
    "fmlx_glm_bkt_set_trace": ([c_void_p, c_long], None),
    "fmlx_glm_bkt_count_all": [c_void_p, c_void_p, c_long, c_long, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_int, c_long, c_void_p],
    # sort.hip
    "fmlx_sorted_bounds": [c_void_p, c_long, c_int, c_void_p, c_void_p],
    "fmlx_seg_sort_scratch": ([c_void_p, c_int, c_int, c_int], c_long),
    "fmlx_seg_sort64": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                        c_long, c_void_p, c_void_p, c_long, c_void_p],
    "fmlx_seg_sort32": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                        c_long, c_void_p],
    # csc_build.hip
    "fmlx_csc_keys64": [c_void_p, c_void_p, c_void_p, c_long, c_long, c_long, c_int, c_long, c_void_p, c_void_p,
                        c_int, c_void_p],
    "fmlx_csc_keys": [c_void_p, c_void_p, c_long, c_long, c_long, c_int, c_long, c_void_p, c_void_p, c_void_p,
                      c_void_p],
    "fmlx_csc_fill": [c_int, c_void_p, c_long, c_long, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "fmlx_csc_sort_split": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                            c_long, c_void_p, c_void_p, c_long, c_void_p, c_long, c_int, c_void_p],
    "fmlx_csc_colptr": [c_void_p, c_long, c_int, c_int, c_void_p, c_long, c_void_p, c_void_p],
    "fmlx_csc_tiles": [c_void_p, c_long, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_long,
                       c_void_p],
    "fmlx_csc_tiles_scratch": ([c_int, c_int], c_long),
    "fmlx_csc_tile_keys": [c_int, c_void_p, c_long, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                           c_void_p, c_long, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "fmlx_csc_tile_store": [c_int, c_void_p, c_void_p, c_long, c_long, c_int, c_int, c_void_p, c_void_p, c_void_p,
                            c_void_p],
    "fmlx_cell_keys": [c_int, c_void_p, c_void_p, c_void_p, c_long, c_long, c_long, c_long, c_int, c_int, c_int, c_int,
                       c_void_p, c_void_p, c_void_p],
    "fmlx_cell_rekey": [c_void_p, c_long, c_int, c_int, c_void_p, c_void_p],
    "fmlx_cell_store": [c_int, c_void_p, c_void_p, c_long, c_long, c_void_p, c_int, c_long, c_void_p, c_int, c_int,
                        c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "fmlx_cell_bounds": [c_void_p, c_long, c_int, c_void_p, c_int, c_int, c_long, c_int, c_void_p, c_void_p],
    # blas.hip set-up helpers
    "fmlx_fill32": [c_void_p, c_long, ctypes.c_uint, c_void_p],
    "fmlx_csr_batch_bounds": [c_void_p, c_long, c_long, c_long, c_void_p, c_void_p],
    "fmlx_host_register": [c_void_p, c_long],
    "fmlx_host_unregister": [c_void_p],
    "fmlx_memcpy_h2d": [c_void_p, c_void_p, c_long, c_void_p],
}

_HOST_SIGS = {}


def register_kernel_sigs(sigs: dict) -> None:
    _KERNEL_SIGS.update(sigs)
    if _KLIB is not None:
        _apply_sigs(_KLIB, sigs)


def register_host_sigs(sigs: dict) -> None:
    _HOST_SIGS.update(sigs)
    if _HLIB is not None:
        _apply_sigs(_HLIB, sigs, restype=None)


def _apply_sigs(lib, sigs, restype=c_int):
    for name, spec in sigs.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        if isinstance(spec, tuple):
            fn.argtypes, fn.restype = spec
        else:
            fn.argtypes = spec
            fn.restype = restype


def gpu_available() -> bool:
    from ..parallel.context import get_context

    return get_context().device.type == "cuda"


def kernel_lib_path() -> str:
    return _build.KERNEL_LIB


def kernels():
    """The HIP kernel library (raises if missing: never a silent fallback on GPU)."""
    global _KLIB
    if _KLIB is not None:
        return _KLIB
    with _LOCK:
        if _KLIB is None:
            path = _build.KERNEL_LIB
            if not os.path.exists(path):
                if os.environ.get("FMLX_AUTOBUILD", "1") == "1":
                    _build.build_kernels()
                else:
                    raise RuntimeError("native kernel library missing: %s (run python -m flink_ml_amd.ops.build)" % path)
            _build.check_fresh("kernels")  # never load a binary built from other sources
            lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
            _apply_sigs(lib, _KERNEL_SIGS)
            _preload(lib)
            _KLIB = lib
    return _KLIB


def _preload(lib) -> None:
    """Loads every code object of the library now (one empty anchor-kernel launch per
    translation unit, csrc/common.h FMLX_DEFINE_PRELOAD) instead of lazily inside the first fit
    that launches one of its kernels; the one-time cost goes to PRELOAD_MS."""
    global PRELOAD_MS, PRELOAD_OBJECTS
    if os.environ.get("FMLX_PRELOAD", "1") == "0" or not torch.cuda.is_available():
        return
    import time

    fn = getattr(lib, "fmlx_preload_all", None)
    if fn is None:
        return
    fn.argtypes, fn.restype = [c_void_p], c_int
    t0 = time.perf_counter()
    k = fn(torch.cuda.current_stream().cuda_stream)
    PRELOAD_MS = (time.perf_counter() - t0) * 1e3
    PRELOAD_STAGES["code_objects"] = round(PRELOAD_MS, 2)
    if k < 0:
        raise RuntimeError("preloading the kernel library's code objects failed (%d)" % k)
    from ..utils import hostsync

    t1 = time.perf_counter()
    hostsync.warm(torch.cuda.current_device())  # pinned read-back block + first-use imports
    PRELOAD_STAGES["pinned_readback"] = round((time.perf_counter() - t1) * 1e3, 2)
    t1 = time.perf_counter()
    warm = getattr(lib, "fmlx_glm_sparse_warm", None)  # every sparse-round kernel launched once, dry
    if warm is not None:
        warm.argtypes, warm.restype = [c_void_p], c_int
        if warm(torch.cuda.current_stream().cuda_stream) != 0:
            raise RuntimeError("warming the sparse round kernels failed")
        torch.cuda.current_stream().synchronize()
    PRELOAD_STAGES["sparse_warm_launches"] = round((time.perf_counter() - t1) * 1e3, 2)
    torch.cuda.get_device_properties(torch.cuda.current_device())  # (first call: runtime queries)
    # the bucket round's compile-time limits, read here (a first fit paid ~50 µs for the first call
    # of the entry point); through ``lib``: kernels() holds its lock until this returns
    # (no package import here: a module imported inside this lock could register signatures that
    # _apply_sigs has already passed)
    global BKT_LIMITS
    import numpy as np

    lim = np.zeros(8, dtype=np.int32)
    lib.fmlx_glm_bkt_limits(lim.ctypes.data)
    BKT_LIMITS = lim
    # one device segment for torch's caching allocator, freed at once: the trainers' buffers of a
    # first fit are then carved out of it instead of each new size paying a hipMalloc inside the fit
    # (a fresh hipMalloc is tens to hundreds of µs of GPU-idle host time)
    pool = int(os.environ.get("FMLX_DEVICE_POOL_MB", "2048")) << 20
    t1 = time.perf_counter()
    if pool > 0:
        seg = torch.empty(pool, dtype=torch.uint8, device=torch.cuda.current_device())
        del seg
    PRELOAD_STAGES["device_pool"] = round((time.perf_counter() - t1) * 1e3, 2)
    PRELOAD_MS = (time.perf_counter() - t0) * 1e3
    PRELOAD_OBJECTS = k


def host():
    """The host-side C++ runtime library (hashing, caches, sketches)."""
    global _HLIB
    if _HLIB is not None:
        return _HLIB
    with _LOCK:
        if _HLIB is None:
            # FMLX_HOST_LIB: an alternative build of the host runtime (the ASan/UBSan one in tests)
            path = os.environ.get("FMLX_HOST_LIB") or _build.HOST_LIB
            if not os.path.exists(path):
                _build.build_host()
            if path == _build.HOST_LIB:
                _build.check_fresh("host")
            lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
            _apply_sigs(lib, _HOST_SIGS, restype=None)
            _HLIB = lib
    return _HLIB


def zeros(shape, dtype, device) -> torch.Tensor:
    """``torch.zeros`` on the GPU through the library's own (preloaded) fill kernel: torch's fill
    kernels load their code object lazily on first use (tens of ms inside a fit)."""
    t = torch.empty(shape, dtype=dtype, device=device)
    nbytes = t.numel() * t.element_size()
    if t.device.type != "cuda":
        return t.zero_()
    if nbytes % 4:
        return t.zero_()
    call("fmlx_fill32", t.data_ptr(), nbytes // 4, 0, stream_ptr(t.device))
    return t


def zeros_many(specs, device):
    """Several zero-filled device tensors carved out of ONE allocation with ONE fill launch (each
    launch from Python costs ~15 µs of host time that a short fit's GPU idles through): ``specs`` =
    [(shape, dtype), ...] → list of tensors (256-byte aligned views)."""
    offs, total = [], 0
    for shape, dtype in specs:
        n = 1
        for x in (shape if isinstance(shape, (tuple, list)) else (shape,)):
            n *= int(x)
        es = torch.empty(0, dtype=dtype).element_size()
        offs.append((total, n, dtype, shape))
        total += -(-max(1, n * es) // 256) * 256
    blob = zeros((total // 4,), torch.int32, device)
    raw = blob.view(torch.uint8)
    out = []
    for off, n, dtype, shape in offs:
        es = torch.empty(0, dtype=dtype).element_size()
        out.append(raw[off:off + n * es].view(dtype).reshape(shape))
    return out


def fill_i32(t: torch.Tensor, value: int) -> torch.Tensor:
    """In-place fill of a contiguous int32 CUDA tensor (library kernel)."""
    call("fmlx_fill32", t.data_ptr(), t.numel(), int(value) & 0xFFFFFFFF, stream_ptr(t.device))
    return t


def ptr(t) -> int:
    if t is None:
        return None
    return t.data_ptr()


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def dtype_code(dtype: torch.dtype) -> int:
    return _TORCH2DT[dtype]


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError("HIP launch %s failed with error %d" % (what, rc))


SYNC_CHECK = os.environ.get("FMLX_SYNC_CHECK", "0") == "1"


def call(name: str, *args) -> None:
    rc = getattr(kernels(), name)(*args)
    check(rc, name)
    if SYNC_CHECK and torch.cuda.is_available() and not torch.cuda.is_current_stream_capturing():
        try:
            torch.cuda.synchronize()
        except RuntimeError as e:
            raise RuntimeError("native kernel %s failed asynchronously: %s" % (name, e)) from e
