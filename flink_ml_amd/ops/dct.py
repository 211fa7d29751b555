"""Row-wise orthonormal DCT-II / DCT-III on the f32 MFMA (``csrc/dct.hip``): the
even/odd butterfly splits the n × n product into two ⌈n/2⌉-sized ones."""
from __future__ import annotations

import ctypes
import functools
import math

import torch

from . import native
from .native import c_int, c_long, c_void_p

native.register_kernel_sigs({
    "fmlx_dct_basis_shape": [c_int, c_void_p, c_void_p],
    "fmlx_dct_rows": [c_void_p, c_long, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p],
    "fmlx_dct_rows_f64": [c_void_p, c_long, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p],
})


def set_diag(diag: int = 0, per_cu: int = 0) -> None:
    """Diagnostics of the kernel's pipeline (1: skip the MFMAs, 2: skip the tile loads, 4: skip the
    stores; per_cu: cap on blocks per CU). Results are wrong while diag != 0."""
    fn = native.kernels().fmlx_dct_set_diag
    fn.restype = None
    fn(int(diag), int(per_cu))

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
def _padded_basis(n: int, inverse: bool, device: str, dtype: torch.dtype = torch.float32) -> torch.Tensor:
    """Both half bases of the even/odd butterfly as the kernel reads its MFMA B fragments:
    [2][KP/4][4][16][nt8], element [p][q][hh][r][c] = B_p[4q + hh][16c + r] with B_p[kk][o] =
    M[2o + p][kk] (forward: k' = o, i = kk) or M[2kk + p][o] (inverse: k' = kk, i = o)."""
    kp, nt8 = ctypes.c_int(), ctypes.c_int()
    if native.kernels().fmlx_dct_basis_shape(n, ctypes.byref(kp), ctypes.byref(nt8)) != 0:
        raise ValueError("DCT size %d outside 1..%d" % (n, MAX_N))
    M = dct_matrix(n)
    KP, NT8 = kp.value, nt8.value
    h = (n + 1) // 2
    halves = []
    for p in (0, 1):
        rows = M[p::2, :h]  # M[2k' + p][i], i < h
        B = rows.t() if not inverse else rows  # forward: [i][k'];  inverse: [k'][i]
        P = torch.zeros((KP, 16 * NT8), dtype=dtype)
        P[:B.shape[0], :B.shape[1]] = B.to(dtype)
        halves.append(P.reshape(KP // 4, 4, NT8, 16).permute(0, 1, 3, 2).contiguous())
    return torch.stack(halves).contiguous().to(device)


def dct_rows(X: torch.Tensor, inverse: bool = False) -> torch.Tensor:
    """DCT of every row of a CUDA f32 or f64 matrix [rows, n ≤ 128] (exact-f32 / f64 MFMA; one
    read and one write of the rows)."""
    rows, n = X.shape
    X = X.contiguous()
    Y = torch.empty_like(X)
    f64 = X.dtype == torch.float64
    B = _padded_basis(n, bool(inverse), str(X.device), torch.float64 if f64 else torch.float32)
    cus = torch.cuda.get_device_properties(X.device).multi_processor_count
    native.call("fmlx_dct_rows_f64" if f64 else "fmlx_dct_rows", native.ptr(X), rows, n, native.ptr(B), native.ptr(Y),
                int(bool(inverse)), cus, native.stream_ptr(X.device))
    return Y
