"""Row-wise orthonormal DCT-II / DCT-III on the f32 MFMA (``csrc/dct.hip``)."""
from __future__ import annotations

import ctypes
import functools
import math

import torch

from . import native
from .native import c_int, c_long, c_void_p

native.register_kernel_sigs({
    "fmlx_dct_basis_shape": [c_int, c_void_p, c_void_p],
    "fmlx_dct_rows": [c_void_p, c_long, c_int, c_void_p, c_void_p, c_int, c_void_p],
})

MAX_N = 128


@functools.lru_cache(maxsize=32)
def dct_matrix(n: int) -> torch.Tensor:
    """Orthonormal DCT-II basis M [n, n] (rows = frequencies), fp64 on the host."""
    k = torch.arange(n, dtype=torch.float64)[:, None]
    i = torch.arange(n, dtype=torch.float64)[None, :]
    m = torch.cos(math.pi * (2 * i + 1) * k / (2 * n))
    m[0] *= math.sqrt(1.0 / n)
    m[1:] *= math.sqrt(2.0 / n)
    return m


@functools.lru_cache(maxsize=64)
def _padded_basis(n: int, inverse: bool, device: str) -> torch.Tensor:
    kp, nps = ctypes.c_int(), ctypes.c_int()
    if native.kernels().fmlx_dct_basis_shape(n, ctypes.byref(kp), ctypes.byref(nps)) != 0:
        raise ValueError("DCT size %d outside 1..%d" % (n, MAX_N))
    M = dct_matrix(n)
    Bm = M if inverse else M.t()  # Y = X·Bm: forward X·Mᵀ, inverse X·M
    out = torch.zeros((kp.value, nps.value), dtype=torch.float32)
    out[:n, :n] = Bm.to(torch.float32)
    return out.to(device)


def dct_rows(X: torch.Tensor, inverse: bool = False) -> torch.Tensor:
    """DCT of every row of a CUDA f32 matrix [rows, n ≤ 128] (exact-f32 MFMA; one read and one
    write of the rows)."""
    rows, n = X.shape
    X = X.contiguous()
    Y = torch.empty_like(X)
    B = _padded_basis(n, bool(inverse), str(X.device))
    cus = torch.cuda.get_device_properties(X.device).multi_processor_count
    native.call("fmlx_dct_rows", native.ptr(X), rows, n, native.ptr(B), native.ptr(Y), cus,
                native.stream_ptr(X.device))
    return Y
