"""Python bindings for the GLM kernels (``csrc/glm.hip``) plus torch reference versions.

The reference versions define the semantics and run on CPU (tests, parity mode); on a GPU
the HIP launchers are used and there is no fallback.
"""
from __future__ import annotations

import math
import os
import weakref
from typing import Optional, Tuple

import numpy as np
import torch

from . import native

LOSS_CODES = {"logistic": 0, "hinge": 1, "leastsquare": 2, "ftrl": 3}
MAX_CPL = 8
WPB = 8
# row loop of the round kernel (A/B knob): 0 = default for the shape (U = 2 up to 32 bytes per
# lane, else 1), U > 0 = 2·U rows in flight per wave. (The grouped loop, -4 / -8, measured slower
# on the flagship shape — 40.6 / 42.2 vs 37.9 µs — and was removed in round 4.)
GRAD_UNROLL = int(os.environ.get("FMLX_GLM_UNROLL", "0"))
# 512 blocks x 8 waves = 4 waves per SIMD (the 128-VGPR cap of the flagship layout): interleaved
# A/B at 10M x 1000 bf16 on one MI355X, 3 repeats (profiles/r2/lr_grid_ab_1gpu.log): 41.0 µs per
# round vs 43.4 (256), 43.5 (384), 48.4 (768), 48.2 (1024). Accumulator replicas 2/4/8 and one
# contiguous run of rows per wave instead of the interleaved rows measured within 1-2 % (the
# latter slower): scripts/bench_glm_kernel.py, round-2 log in profiles/r2/INDEX.md
# round 3: 0 = by shape (round_blocks). Rows of 32 bytes per lane (bf16 d 513-1024, the flagship
# 1000) take 4 rows in flight per wave on 224 blocks (28 per XCD): 37.31 us per round vs 38.56 on
# 256 blocks and 39.75 for U=1 on 512, interleaved on one MI355X (profiles/r3/lr_unroll_grid_*,
# lr_unroll2_grid_*; bench.py 39.5 vs 40.8 us per step)
GRAD_BLOCKS = int(os.environ.get("FMLX_GLM_BLOCKS", "0"))


def round_blocks(X) -> int:
    """Grid of the fused round for rows ``X`` (FMLX_GLM_BLOCKS / GRAD_BLOCKS > 0 overrides)."""
    if GRAD_BLOCKS > 0:
        return GRAD_BLOCKS
    lay = pick_layout(X) if X is not None else None
    if lay is not None and GRAD_UNROLL == 0 and lay[0] * lay[1] * X.element_size() == 32:
        return 224
    if lay is not None and (lay[0] * lay[1] * X.element_size() > 32 or X.dtype == torch.float64):
        return 256  # over 128 VGPRs (csrc/glm.hip glm_min_waves): one block per CU
    return 512


# rows streamed once per pass use non-temporal loads when the data set exceeds the 256 MiB
# Infinity Cache (otherwise rounds re-read it from there)
NT_MIN_BYTES = 256 << 20


def set_tuning(lds_pad: int = -1, nt: int = -1) -> None:
    """A/B knobs of the round kernel (-1 = automatic): extra LDS per block (caps blocks per CU)
    and non-temporal row loads."""
    native.call("fmlx_glm_set_tuning", int(lds_pad), int(nt))


def set_tail_tuning(acc_reps: int = 4, ticket2: bool = False) -> None:
    """A/B knobs of the atomic round tail: accumulator replicas (block b adds into replica
    b mod reps) and two-level arrival tickets."""
    native.call("fmlx_glm_set_tail_tuning", int(acc_reps), int(bool(ticket2)))


# LDS-DMA row ring of the fused round (csrc/glm.hip, DEPTH): bf16 rows of d 513–1024 stream into a
# per-wave LDS ring by global_load_lds (DEPTH − 1 steps of U rows in flight through the math).
# FMLX_GLM_DMA = ring depth in steps (0 = 16-byte register loads).
DMA_DEPTH = int(os.environ.get("FMLX_GLM_DMA", "0"))


def set_dma(depth: int) -> None:
    """Ring depth of the fused round's LDS-DMA row path (0 = off; 2–4 steps)."""
    if native.kernels().fmlx_glm_set_dma(int(depth)) != 0:
        raise ValueError("depth must be 0, 2, 3 or 4")


def set_trace(buf: Optional[torch.Tensor]) -> None:
    """Diagnostics: fused-round launches write per-block {start, rows done, atomics drained, hw
    id} s_memrealtime stamps (100 MHz) into ``buf`` (int64 [blocks, 4]); None switches off."""
    native.kernels().fmlx_glm_set_trace(native.ptr(buf))


def set_bkt_trace(buf: Optional[torch.Tensor]) -> None:
    """Diagnostics: the bucket round's forward writes per-block phase stamps (s_memrealtime, 100 MHz:
    entry, bookkeeping loaded, products staged, loss done, records staged, stores issued) into
    ``buf`` (int64 [blocks, 8]; blocks past its rows write nothing); None switches off."""
    if buf is None:
        native.kernels().fmlx_glm_bkt_set_trace(None, 0)
    else:
        assert buf.dtype == torch.int64 and buf.dim() == 2 and buf.shape[1] == 8 and buf.is_contiguous()
        native.kernels().fmlx_glm_bkt_set_trace(native.ptr(buf), int(buf.shape[0]))


def pick_layout(X: torch.Tensor, rounds: bool = True) -> Optional[Tuple[int, int]]:
    """(epc, cpl) for the register-resident path, or None if d is too wide / misaligned.
    ``rounds=False``: the prediction kernel's limit (no gradient registers: bf16 up to 8 chunks)."""
    if X.dim() != 2:
        return None
    n, d = X.shape
    es = X.element_size()
    ld = X.stride(0)
    if X.stride(1) != 1:
        return None
    base = X.data_ptr()
    for vb in (16, 8, 4, 2):
        epc = vb // es
        if epc < 1:
            continue
        if d % epc == 0 and (ld * es) % vb == 0 and base % vb == 0:
            break
    else:
        return None
    nch = d // epc
    cpl = 1
    while cpl * 64 < nch:
        cpl *= 2
    if cpl > MAX_CPL or (rounds and es == 2 and cpl > 4):
        # (bf16 rows of 2049–4096: the one-wave kernel needs > 256 VGPRs there and spills — 1.9
        # TB/s vs 5 TB/s on the wide-row kernel, profiles/r5/glm_widths*.jsonl)
        return None
    return epc, cpl


WIDE_WAVES = 8  # csrc/glm.hip glm_round_wide_kernel: waves splitting a row's columns
WIDE_FUSED = os.environ.get("FMLX_GLM_WIDE_FUSED", "1") == "1"  # 0: wide rows take the GEMV path (A/B)


def pick_wide_layout(X: torch.Tensor) -> Optional[Tuple[int, int]]:
    """(epc, cpl) of the wide-row round kernel (16-byte chunks, a row's chunks split over 8
    waves, cpl chunks per lane of a slice), or None (misaligned, or wider than 8 × 64 × 8 chunks:
    bf16 32768, fp32 16384, fp64 8192)."""
    if X.dim() != 2 or X.stride(1) != 1:
        return None
    es = X.element_size()
    epc = 16 // es
    d = X.shape[1]
    if d % epc or (X.stride(0) * es) % 16 or X.data_ptr() % 16:
        return None
    per = -(-(d // epc) // WIDE_WAVES)
    for cpl in (1, 2, 4, 8):
        if 64 * cpl >= per:
            return epc, cpl
    return None


def wide_blocks_per_cu(X) -> int:
    """Blocks of the wide-row kernel per CU: 2 for one chunk per lane (measured: bf16 4096 0.184
    vs 0.295 ms per round), else 1 (bf16 8192 at two chunks: 0.352 with 2 per CU vs 0.342)."""
    lay = pick_wide_layout(X)
    return 2 if lay is not None and lay[1] <= 1 else 1


def glm_round_wide(X, y, wt, coef, B: int, loss: int, state, scratch: "RoundScratch", mode: int, feedback,
                   max_iter: int, tol: float, lr: float, reg: float, en: float) -> None:
    """One round of the wide-row kernel (atomic tail; TAIL_UPDATE or TAIL_FEEDBACK)."""
    epc, cpl = pick_wide_layout(X)
    native.call("fmlx_glm_round_wide", native.dtype_code(X.dtype), epc, cpl, native.ptr(X), X.stride(0), native.ptr(y),
                native.ptr(wt), native.ptr(coef), X.shape[0], X.shape[1], B, loss, native.ptr(state), scratch.nparts,
                mode, native.ptr(scratch.cnt), native.ptr(scratch.acc), native.ptr(feedback), int(max_iter), float(tol),
                float(lr), float(reg), float(en), native.stream_ptr(X.device))


def pad_columns(X: torch.Tensor) -> Optional[torch.Tensor]:
    """A copy of X whose rows are zero-padded to a whole number of 16-byte chunks, when that makes
    it fit the register-resident round kernel (misaligned widths: fp32 d = 1001, bf16 d % 8 ≠ 0,
    a row stride that breaks 16-byte alignment); None when even the padded row is too wide or the
    copy does not fit in free device memory. The padding columns are zero, so their gradient is
    zero and their coefficients stay 0 through every update (SGD step and regularisation)."""
    if X.dim() != 2 or not X.is_cuda:
        return None
    n, d = X.shape
    epc = 16 // X.element_size()
    dp = -(-d // epc) * epc
    nch = dp // epc
    cpl = 1
    while cpl * 64 < nch:
        cpl *= 2
    # the wide-row kernel only runs where the trainer would pick it (a padded copy for
    # the GEMV path doubled the partition's HBM for no speedup)
    wide_ok = not DETERMINISTIC and WIDE_FUSED
    if cpl > MAX_CPL and (not wide_ok or -(-nch // WIDE_WAVES) > 64 * 8):  # neither fused kernel
        return None
    need = n * dp * X.element_size()
    free, _ = torch.cuda.mem_get_info(X.device)
    if need > 0.8 * free:
        return None
    Xp = torch.empty((n, dp), dtype=X.dtype, device=X.device)
    Xp[:, d:].zero_()
    Xp[:, :d].copy_(X)
    return Xp if pick_layout(Xp) is not None or wide_ok and pick_wide_layout(Xp) is not None else None


def grad_partials(X, y, wt, coef, B: int, loss: int, state, partials, nblocks: int) -> None:
    epc, cpl = pick_layout(X)
    native.call("fmlx_glm_grad_partials", native.dtype_code(X.dtype), epc, cpl, GRAD_UNROLL, native.ptr(X), X.stride(0),
                native.ptr(y), native.ptr(wt), native.ptr(coef), X.shape[0], X.shape[1], B, loss,
                native.ptr(state), native.ptr(partials), nblocks, native.stream_ptr(X.device))


def stage1_rows(nparts: int) -> int:
    return (nparts + 31) // 32


# fused-round tails (csrc/glm.hip): what the last block of the round does after the reduction
TAIL_PARTIALS, TAIL_FEEDBACK, TAIL_UPDATE, TAIL_XGMI = 0, 1, 2, 3
TAIL_MAX_BLOCKS = 512         # deterministic (fixed-order) tail
TAIL_MAX_BLOCKS_ATOMIC = 2048  # float-atomic tail
# FMLX_DETERMINISTIC=1: fixed-order in-kernel reduction (bit-reproducible run to run); default:
# float atomics into one accumulator (shorter round tail; last bits vary with arrival order)
DETERMINISTIC = os.environ.get("FMLX_DETERMINISTIC", "0") == "1"
# 1-GPU fused rounds complete round e − 1 in the prologue of launch e (no arrival ticket / serial
# last-block tail; csrc/glm.hip defer_prologue)
DEFER = os.environ.get("FMLX_GLM_DEFER", "1") == "1"
# the same across ranks over the in-kernel xGMI exchange (TAIL_XGMI)
DEFER_XGMI = os.environ.get("FMLX_GLM_DEFER_XGMI", "1") == "1"


def defer_supported(d: int, acc: torch.dtype) -> bool:
    """Deferred completion needs the flat atomic tail ([WPB][d] LDS image ≤ 64 KiB) and the
    row-at-a-time loop."""
    es = 8 if acc == torch.float64 else 4
    return DEFER and not DETERMINISTIC and WPB * d * es <= 64 * 1024


def max_round_blocks() -> int:
    return TAIL_MAX_BLOCKS if DETERMINISTIC else TAIL_MAX_BLOCKS_ATOMIC


_dma_applied = False


class RoundScratch:
    """Device scratch of one fused round: block partials / group rows (deterministic tail), the
    atomic accumulator, arrival tickets (all zero-initialised; the kernel re-arms them)."""

    def __init__(self, nparts: int, d: int, acc: torch.dtype, device, det: bool = None):
        global _dma_applied
        if not _dma_applied:
            set_dma(DMA_DEPTH)
            _dma_applied = True
        self.nparts = nparts
        self.det = DETERMINISTIC if det is None else bool(det)
        if self.det:
            self.partials = native.zeros((nparts, d + 2), acc, device)
            self.stage1 = native.zeros((stage1_rows(nparts), d + 2), acc, device)
        else:
            self.partials = native.zeros((1, d + 2), acc, device)
            self.stage1 = None
        # atomic tail: ACC_MAX_REPS replicas of the [d+2] accumulator on whole 256-B lines
        self.acc = native.zeros(int(native.kernels().fmlx_glm_acc_elems(d)), acc, device)
        # 64 group + 1 top tickets
        self.cnt = native.zeros(int(native.kernels().fmlx_glm_cnt_elems()), torch.int32, device)


def glm_round(X, y, wt, coef, B: int, loss: int, state, scratch: RoundScratch, mode: int, feedback=None,
              max_iter: int = 1, tol: float = 0.0, lr: float = 0.0, reg: float = 0.0, en: float = 0.0,
              xg=None, rounds: int = 1, defer: bool = False, parity: int = 0, cw=None) -> None:
    """``rounds`` SGD rounds (loss+gradient over the round's batch, fixed-order reduction and — by
    mode — feedback output, update, or xGMI exchange + update), each ONE kernel launch predicated
    on the device running flag (one host call issues all ``rounds`` launches).

    ``defer``: 1-GPU TAIL_UPDATE with the atomic tail only — launch e completes round e − 1 in its
    prologue; launch i of the call reads its round number from state word ``(parity + i) & 1``
    and ``cw`` is the [2, d] coefficient ring."""
    epc, cpl = pick_layout(X)
    flags = 1 if X.shape[0] * X.stride(0) * X.element_size() > NT_MIN_BYTES else 0
    if xg is not None:
        peers, world, rank, gen, err, spin = xg.kernel_args()
    else:
        peers, world, rank, gen, err, spin = None, 1, 0, None, None, 0
    native.call("fmlx_glm_round", native.dtype_code(X.dtype), epc, cpl, GRAD_UNROLL, native.ptr(X), X.stride(0),
                native.ptr(y), native.ptr(wt), native.ptr(coef), X.shape[0], X.shape[1], B, loss, native.ptr(state),
                native.ptr(scratch.partials), scratch.nparts, mode, int(scratch.det), native.ptr(scratch.cnt),
                native.ptr(scratch.acc), native.ptr(scratch.stage1), native.ptr(feedback), int(max_iter), float(tol), float(lr), float(reg),
                float(en), peers, world, rank, gen, err, int(spin), flags, int(rounds), int(bool(defer)), int(parity),
                native.ptr(cw), native.stream_ptr(X.device))


def reduce_update(partials, nparts: int, d: int, stage1, coef, feedback, state, max_iter, tol, lr, reg, en) -> None:
    native.call("fmlx_glm_reduce_update", int(coef.dtype == torch.float64), native.ptr(partials), nparts, d,
                native.ptr(stage1), native.ptr(coef), native.ptr(feedback), native.ptr(state), max_iter, tol, lr, reg, en,
                native.stream_ptr(coef.device))


def reduce_only(partials, nparts: int, d: int, stage1, feedback, state) -> None:
    native.call("fmlx_glm_reduce", int(feedback.dtype == torch.float64), native.ptr(partials), nparts, d,
                native.ptr(stage1), native.ptr(feedback), native.ptr(state), native.stream_ptr(feedback.device))


def update(feedback, d: int, coef, state, max_iter, tol, lr, reg, en) -> None:
    native.call("fmlx_glm_update", int(coef.dtype == torch.float64), native.ptr(feedback), d, native.ptr(coef),
                native.ptr(state), max_iter, tol, lr, reg, en, native.stream_ptr(coef.device))


def grad_csr(indptr, idx, val, y, wt, coef, n, d, B, loss, state, grad) -> None:
    native.call("fmlx_glm_grad_csr", int(val.dtype == torch.float64), native.ptr(indptr), native.ptr(idx),
                native.ptr(val), native.ptr(y), native.ptr(wt), native.ptr(coef), n, d, B, loss,
                native.ptr(state), native.ptr(grad), native.stream_ptr(val.device))


# sparse rounds through per-batch transposes (csrc/glm.hip glm_csc_bwd_kernel)
CSC_MAX_BYTES = 8 << 30  # the column-major copies of a partition: at most this much
CSC_RUN_MAX = 16  # consecutive batches transposed per sort
TRANSPOSE = True  # False: the transposed layout is never built (the atomic-scatter fallback; tests)
# fp32 copies over 11–20 column bits: high-bits pass + bucket-local pass (0: two LSD passes + colptr)
CSC_BUCKET = True


SEG_SORT_DIGIT_BITS = 10  # radix.hip RS_MAX_DIGIT_BITS


def seg_sort_passes(key_bits: int) -> int:
    """Digit passes of ``seg_sort`` (digits of <= 10 bits, balanced)."""
    return -(-int(key_bits) // SEG_SORT_DIGIT_BITS)


def seg_sort_scratch(bounds, key_bits: int) -> int:
    import numpy as np

    b = np.ascontiguousarray(np.asarray(bounds, dtype=np.int64))
    need = int(native.kernels().fmlx_seg_sort_scratch(b.ctypes.data, len(bounds) - 1, int(key_bits),
                                                             SEG_SORT_DIGIT_BITS))
    if need < 0:
        raise ValueError("seg_sort: bad segment table (S=%d, key_bits=%d)" % (len(bounds) - 1, key_bits))
    return max(need, 1)


def seg_sort(keys: torch.Tensor, vals: torch.Tensor, bounds, kbase, key_bits: int, keys_alt=None, vals_alt=None,
             scratch=None, split=None):
    """Stable segmented LSD radix sort (csrc/radix.hip, no library sort) of int32 ``keys`` with
    int32 / int64 payloads ``vals``: segment s = positions [bounds[s], bounds[s + 1]) is sorted by
    the low ``key_bits`` bits of (key − kbase[s]); equal keys keep their input order. The passes
    ping-pong between (keys, vals) and (keys_alt, vals_alt), so the inputs are overwritten; the
    sorted pair ends in the alt buffers when ``seg_sort_passes(key_bits)`` is odd. Returns the
    sorted (keys, vals). Pre-allocated ``keys_alt`` / ``vals_alt`` / ``scratch`` (int32,
    ``seg_sort_scratch``) make the call allocation-free (hipGraph capture). ``split`` = (lo, hi,
    offset), int64 payloads only: the last pass writes the payloads' low / high 32-bit words to
    lo[offset + i] / hi[offset + i] (int32 / 32-bit tensors) instead of the payload buffers."""
    import numpy as np

    S = len(bounds) - 1
    b = np.ascontiguousarray(np.asarray(bounds, dtype=np.int64))
    kb = np.ascontiguousarray(np.asarray(kbase, dtype=np.int32))
    lib = native.kernels()
    if scratch is None:
        scratch = torch.empty(seg_sort_scratch(bounds, key_bits), dtype=torch.int32, device=keys.device)
    k2 = torch.empty_like(keys) if keys_alt is None else keys_alt
    v2 = torch.empty_like(vals) if vals_alt is None else vals_alt
    args = (native.ptr(keys), native.ptr(vals), native.ptr(k2), native.ptr(v2), b.ctypes.data, kb.ctypes.data, S,
            int(key_bits), SEG_SORT_DIGIT_BITS, native.ptr(scratch), scratch.numel())
    if vals.element_size() == 8:
        lo, hi, off = split if split is not None else (None, None, 0)
        rc = lib.fmlx_seg_sort64(*args, native.ptr(lo), native.ptr(hi), int(off), native.stream_ptr(keys.device))
    else:
        if split is not None:
            raise ValueError("seg_sort: split output needs int64 payloads")
        rc = lib.fmlx_seg_sort32(*args, native.stream_ptr(keys.device))
    if rc < 0:
        raise RuntimeError("fmlx_seg_sort failed: %d" % rc)
    return (k2, v2) if rc == 1 else (keys, vals)


_BOUNDS_CACHE = {}  # id(indptr) -> (weak reference, {(n, B, version): (nnz, bounds)})
_ROW_MAX = {}  # id(indptr) -> {(n, B, version): the longest row} (filled with the bounds)
_BOUNDS_PENDING = {}  # id(indptr) -> (weak reference, key, pinned host buffer, completion event)


def prefetch_batch_bounds(indptr: torch.Tensor, n: int, B: int) -> None:
    """Queues the device → host read of :func:`_batch_bounds` without waiting for it, so the host's
    next set-up work (allocations, fill launches) runs while the kernel and the copy complete; the
    later ``_batch_bounds`` call only collects it (a first fit's ~0.14 ms blocking read)."""
    if not indptr.is_cuda or n <= 0 or B <= 0:
        return
    key = (n, B, indptr._version)
    ent = _BOUNDS_CACHE.get(id(indptr))
    if ent is not None and ent[0]() is indptr and key in ent[1]:
        return
    pend = _BOUNDS_PENDING.get(id(indptr))
    if pend is not None and pend[0]() is indptr and pend[1] == key:
        return
    P = (n + B - 1) // B
    out = torch.empty(P + 3, dtype=torch.int64, device=indptr.device)
    native.call("fmlx_csr_batch_bounds", native.ptr(indptr.contiguous()), n, B, P, native.ptr(out),
                native.stream_ptr(indptr.device))
    host = torch.empty(P + 3, dtype=torch.int64, pin_memory=True)
    host.copy_(out, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(indptr.device))
    ref = weakref.ref(indptr, lambda _r, i=id(indptr): _BOUNDS_PENDING.pop(i, None))
    _BOUNDS_PENDING[id(indptr)] = (ref, key, host, ev, out)


def batch_row_max(indptr: torch.Tensor, n: int, B: int) -> Optional[int]:
    """The longest row of the partition, read together with :func:`_batch_bounds` (None before)."""
    return _ROW_MAX.get(id(indptr), {}).get((n, B, indptr._version))


def _batch_bounds(indptr: torch.Tensor, n: int, B: int):
    """(nnz, [indptr[min(b·B, n)] for b = 0 … P]) of a CSR partition, read from the device once
    per (indptr, n, B) and kept while the tensor lives unmodified: a fit over the same data then
    starts without a device → host copy (every whole fit paid two blocking ones here)."""
    key = (n, B, indptr._version)
    ent = _BOUNDS_CACHE.get(id(indptr))
    if ent is not None and ent[0]() is indptr and key in ent[1]:
        return ent[1][key]
    from ..utils import hostsync

    P = (n + B - 1) // B
    if indptr.is_cuda:
        # one library kernel + one polled copy (no torch index / arange / cat kernels: their code
        # objects load lazily, tens of ms inside the first fit of a process)
        prefetch_batch_bounds(indptr, n, B)
        _ref, _key, host, ev, _out = _BOUNDS_PENDING.pop(id(indptr))
        hostsync.wait_event(ev)
        both = host.tolist()
    else:
        sel = torch.arange(0, P + 1).mul_(B).clamp_(max=n)
        lens = indptr[1:n + 1] - indptr[:n]
        both = torch.cat([indptr[-1:], indptr[sel], lens.max().reshape(1) if n else indptr[:1] * 0]).tolist()
    val = (int(both[0]), both[1:P + 2])
    if ent is None or ent[0]() is not indptr:
        _ROW_MAX[id(indptr)] = {}

        def _forget(_r, i=id(indptr)):
            _BOUNDS_CACHE.pop(i, None)
            _ROW_MAX.pop(i, None)

        ref = weakref.ref(indptr, _forget)
        ent = (ref, {})
        _BOUNDS_CACHE[id(indptr)] = ent
    ent[1][key] = val
    _ROW_MAX.setdefault(id(indptr), {})[key] = int(both[P + 2])
    return val


# the column-major copy's packed payload (column low bits above a 22-bit batch row: no key array
# out of the high-bits pass); CSC_PACK = False forces the unpacked bucket pass (batches > 2^22 rows
# take it anyway) — tests cover both
CSC_PACK = True


TILE_HEAVY_DIV = 8  # heavy column: > ET / this entries
# a fit tiles its batches when it visits each at least this often (the tiling costs about as much
# as TILE_MIN_VISITS rounds save: ~0.15 ms per 6.4M-entry batch vs ~13 µs per round, svc shape)
TILE_MIN_VISITS = 16
# fits visiting each batch fewer than TILE_MIN_VISITS times take the single-visit bucket round
# (BucketRound) instead of any per-batch transpose; BUCKETS = False: the transposed rounds (tests)
BUCKETS = True
TILE_SPREAD = True  # tile size from the batch and CU count
# the forward over row-block × column-split cells (glm.hip glm_csr_cell_fwd_kernel): float atomics
# in LDS, so off under FMLX_DETERMINISTIC=1 (the one-row-per-lane-group forward is bit-stable)
CELLS = True
CELL_RBB = None  # rows per row block 2^this ≤ 2^11 (None: 10 or 11, by the cell shape rules)
CELL_SPLITS = 0  # column slices per row block (0: auto)
CSC_TILE = -1  # light-tile entry capacity of the tiled backward (-1: by dtype, 0: untiled layout)
CELL_LDS_MAX = 128 * 1024  # LDS slots of the largest cell (bytes; larger: the row-group forward)


def csc_tile_entries(B: int, f64: bool) -> int:
    """Entry capacity ET of a light column tile of the tiled backward (0 = untiled layout): the
    LDS slot array of one block (128 KiB: 32768 fp32 / 16384 fp64 slots by default; CSC_TILE
    overrides, 0 disables), bounded so that the packed erow (batch row | slot << row bits) fits
    32 bits."""
    want = int(CSC_TILE)
    if want == 0:
        return 0
    least = 16 if want > 0 else 1024  # (small explicit tiles: tests)
    if want < 0:
        want = 16384 if f64 else 32768
    rb = max(1, int(B - 1).bit_length())
    et = min(want, 1 << (32 - rb) if rb < 32 else 1)
    return et if et >= least else 0


class BatchCsc:
    """Per-batch column-major copy of a CSR partition for atomic-free sparse SGD gradients.

    Batch b is the row range [b·B, min((b+1)·B, n)) (the trainer's slicing); its non-zeros keep
    their CSR positions [indptr[bB], indptr[bB+B]) but are re-ordered by column (stable, so rows
    stay ascending within a column) and carry the batch-relative row id. ``colptr[b]`` is the
    dense int32 column pointer of batch b. Costs one extra copy of the partition plus P·(d+1)·4
    bytes; ``alloc`` returns None when that exceeds ``CSC_MAX_BYTES`` or a batch has ≥ 2^31
    non-zeros (the trainer then keeps the atomic scatter kernel).

    Batches are transposed lazily (``ensure``): a fit transposes only the batches its rounds
    visit, before the rounds are launched (SGD.java:263-268 visits batch e mod P in round e), so
    a short fit over a large partition does not pay for the whole partition. The storage is
    allocated at the first ``ensure`` for the leading ``cap`` batches only (a fit of
    ``max_rounds`` < P rounds from round 0 visits batches 0 … max_rounds − 1, whose entries are the
    CSR prefix [0, indptr[max_rounds·B])); a batch beyond it re-allocates the whole partition,
    copies what was built and bumps ``version`` (device pointers changed: captured hipGraphs
    must be re-captured).
    """

    def __init__(self, G: int, bounds, indptr, indices, values, n: int, d: int, B: int, cap: int):
        self.G = G
        self.bounds, self.P = bounds, len(bounds) - 1
        self._src = (indptr, indices, values)
        self.n, self.d, self.B = n, d, B
        self.built = [False] * self.P
        self.cap = 0  # leading batches the storage covers (0: not allocated yet)
        self._want = max(1, min(cap, self.P))
        self.colptr = self.erow = self.evals = None
        self.version = 0
        # row-sorted column tiles (glm.hip glm_csc_tile_bwd_kernel; CUDA partitions only)
        self.ET = csc_tile_entries(B, values.dtype == torch.float64) if values.device.type == "cuda" else 0
        # a column of more than EL entries is a tile of its own (block-strided sum); light tiles
        # start inside one EB-entry bucket, so they hold ≤ EB + EL = ET entries (≈ EB on average)
        self.EL = max(1, self.ET // TILE_HEAVY_DIV)
        self.EB = max(1, self.ET - self.EL)
        self.rb = max(1, int(B - 1).bit_length())
        self.pb = max(1, int(self.ET - 1).bit_length())
        if self.ET:
            most = max(bounds[i + 1] - bounds[i] for i in range(self.P)) if self.P else 0
            if TILE_SPREAD and values.device.type == "cuda":
                # a block runs one tile, so the round takes one tile's time: cut the largest batch
                # into about one tile per CU (fewer, fuller tiles leave CUs idle)
                cus = torch.cuda.get_device_properties(values.device).multi_processor_count
                self.EB = min(self.EB, max(1024, -(-most // max(1, cus - 2))))  # (EB + EL ≤ ET kept)
            self.tstride = min(d, most // self.EB + 2 * (most // self.EL) + 1) + 1
        else:
            self.tstride = 0
        self.tiles = self.ntiles = None
        # forward cells: entries of batch rows [rb·2^CELL_RBB, …) × columns [s·CS, (s+1)·CS),
        # column-sorted per cell, packed (column − s·CS) | row-major rank << cb; roff: first entry
        # of every (cell, row); cmax: entries of the largest built cell (the kernel's LDS slots)
        self.cells = self.cmax = 0
        self.rbb = max(1, min(11, CELL_RBB or 10))  # (_pick_cells)
        self.cent = self.cval = self.roff = self.cpart = self.ccnt = None
        if CELLS and not DETERMINISTIC and values.device.type == "cuda" and self.P and d > 0:
            self._pick_cells(values, bounds, n, d, B)
        self.rstride = (self.cells << self.rbb) + 1

    def _pick_cells(self, values, bounds, n: int, d: int, B: int) -> None:
        """Row-block size 2^rbb and column splits S of the forward cells. About two 1024-thread
        cells per CU, all in one wave (a third cell on some CUs costs more than it spreads: 686
        cells 71.8 µs vs 490 cells 62.4 µs per round; 1024-row blocks beat 2048 at the same
        count, 62.7 vs 64.3 — profiles/r5/svc_cell_forward_ab.jsonl), with the average cell 20 %
        under its rank bits (2^(32 − column bits)) and the LDS; denser rows take more splits."""
        cus = torch.cuda.get_device_properties(values.device).multi_processor_count
        avg_row = bounds[-1] / max(1, n)
        es = values.element_size()
        rows = min(B, n)
        fallback = None
        for rbb in ((CELL_RBB,) if CELL_RBB else (10, 11)):
            nrb = -(-rows // (1 << rbb))
            S = CELL_SPLITS if CELL_SPLITS > 0 else max(1, 2 * cus // nrb)
            while True:
                S = max(1, min(S, 64, d))
                CS = -(-d // S)
                cb = max(1, int(CS - 1).bit_length())
                cell = avg_row * min(rows, 1 << rbb) / S
                fits = cb + rbb <= 32 and cell * 1.2 <= min(1 << (32 - cb), CELL_LDS_MAX // es)
                if fits or CELL_SPLITS > 0 or S >= min(64, d):
                    break
                S += 1
            cellbits = max(1, int(nrb * S - 1).bit_length())
            if not (cb + rbb <= 32 and cb + cellbits <= 32 and nrb * S < 2 ** 20):
                continue
            cand = (rbb, S, CS, cb, nrb * S)
            if fits and (CELL_SPLITS > 0 or S == max(1, min(2 * cus // nrb, 64, d))):
                fallback = cand
                break
            fallback = fallback or cand
        if fallback is not None:
            self.rbb, self.S, self.CS, self.cb, self.cells = fallback

    @staticmethod
    def pick_group(avg_nnz: float) -> int:
        g = 4
        while g < 64 and g < avg_nnz / 2:
            g *= 2
        return g

    @staticmethod
    def alloc(indptr, indices, values, n: int, d: int, B: int, max_rounds: Optional[int] = None):
        """Checks the size limits and returns an (empty) BatchCsc, or None. ``max_rounds``: the
        rounds the fit can run from round 0 (sizes the first allocation)."""
        if not TRANSPOSE or n <= 0 or B <= 0:
            return None
        P = (n + B - 1) // B
        nnz, bounds = _batch_bounds(indptr, n, B)
        extra = P * (d + 1) * 4 + nnz * (4 + values.element_size())
        if CELLS and values.device.type == "cuda":
            extra += nnz * (4 + values.element_size())  # (the forward's cell copy)
        if extra > CSC_MAX_BYTES:
            return None
        if max(bounds[i + 1] - bounds[i] for i in range(P)) >= 2 ** 31:
            return None
        csc = BatchCsc(BatchCsc.pick_group(nnz / max(n, 1)), bounds, indptr, indices, values, n, d, B,
                       P if max_rounds is None else int(max_rounds))
        if (csc.ET or csc.cells) and max_rounds is not None and max_rounds < TILE_MIN_VISITS * P:
            csc.untiled()  # too few visits per batch to pay back the tiling / cell sorts
        return csc

    def untiled(self) -> None:
        """Keeps the plain column-major layout and the row-group forward (before any batch is
        built)."""
        assert self.cap == 0
        self.ET = self.EL = self.EB = self.tstride = 0
        self.cells, self.rstride = 0, 1

    @staticmethod
    def build(indptr, indices, values, n: int, d: int, B: int):
        """Allocates and transposes every batch up front."""
        csc = BatchCsc.alloc(indptr, indices, values, n, d, B)
        if csc is not None:
            csc.ensure(range(csc.P))
        return csc

    def _storage(self, need: int) -> None:
        """Storage for at least the leading ``need`` batches (grows to the whole partition)."""
        if need <= self.cap:
            return
        cap = self._want if self.cap == 0 and need <= self._want else self.P
        values = self._src[2]
        dev = values.device
        ne = self.bounds[cap]
        colptr = torch.empty((cap, self.d + 1), dtype=torch.int32, device=dev)
        erow = torch.empty(max(ne, 1), dtype=torch.int32, device=dev)
        evals = torch.empty(max(ne, 1), dtype=values.dtype, device=dev)
        tiles = ntiles = None
        if self.ET:
            tiles = torch.empty((cap, self.tstride, 2), dtype=torch.int32, device=dev)
            ntiles = torch.empty(cap, dtype=torch.int32, device=dev)
        cent = cval = roff = None
        if self.cells:
            cent = torch.empty(max(ne, 1), dtype=torch.int32, device=dev)
            cval = torch.empty(max(ne, 1), dtype=values.dtype, device=dev)
            roff = torch.empty((cap, self.rstride), dtype=torch.int32, device=dev)
            if self.cpart is None:
                acc = torch.float64 if values.dtype == torch.float64 else torch.float32
                self.cpart = torch.empty(self.cells << self.rbb, dtype=acc, device=dev)
                self.ccnt = torch.zeros(self.cells // self.S, dtype=torch.int32, device=dev)
        if self.cap:
            old = self.bounds[self.cap]
            colptr[:self.cap] = self.colptr
            erow[:old] = self.erow[:old]
            evals[:old] = self.evals[:old]
            if tiles is not None:
                tiles[:self.cap] = self.tiles
                ntiles[:self.cap] = self.ntiles
            if cent is not None:
                cent[:old] = self.cent[:old]
                cval[:old] = self.cval[:old]
                roff[:self.cap] = self.roff
            self.version += 1
        self.colptr, self.erow, self.evals, self.cap = colptr, erow, evals, cap
        self.tiles, self.ntiles = tiles, ntiles
        self.cent, self.cval, self.roff = cent, cval, roff

    def ensure(self, batches) -> None:
        """Transposes the listed batches that are not yet (idempotent; never inside a capture).
        Runs of consecutive batches are transposed together: ONE stable sort of int32 keys
        (batch slot · d + column) over the run's non-zeros — entries of a batch stay in its own
        CSR range, columns ascend inside it and rows ascend inside a column — then the row ids,
        values and column pointers straight from the sorted order (csrc/csc_build.hip)."""
        indptr, indices, values = self._src
        n, d, B = self.n, self.d, self.B
        todo = [b for b in sorted(set(int(x) % self.P for x in batches)) if not self.built[b]]
        if not todo:
            return
        self._storage(todo[-1] + 1)
        max_slots = max(1, min(CSC_RUN_MAX, (2 ** 31 - 1) // max(d, 1)))
        runs, cur = [], [todo[0]]
        for b in todo[1:]:
            if b == cur[-1] + 1 and len(cur) < max_slots:
                cur.append(b)
            else:
                runs.append(cur)
                cur = [b]
        runs.append(cur)
        for run in runs:
            for b in run:
                self.built[b] = True
            b0, b1 = run[0], run[-1] + 1
            j0, j1 = self.bounds[b0], self.bounds[b1]
            if j1 == j0:
                self.colptr[b0:b1].zero_()
                continue
            r0, r1 = b0 * B, min(b1 * B, n)
            if values.device.type == "cuda":
                self._transpose_native(b0, len(run), r0, r1, j0, j1)
                if self.ET:
                    self._tile(b0, len(run), j0, j1)
                if self.cells:
                    self._cells(b0, len(run), r0, r1, j0, j1)
            else:
                self._transpose_torch(b0, len(run), r0, r1, j0, j1)

    def _tile(self, b0, slots, j0, j1) -> None:
        """Cuts the run's batches into column tiles and re-orders every tile's entries by row
        (csc_build.hip csc_tiles / csc_tile_keys / radix sort / csc_tile_store)."""
        import numpy as np

        from . import sorting

        values = self._src[2]
        dev = values.device
        m, d = j1 - j0, self.d
        f64 = int(values.dtype == torch.float64)
        stream = native.stream_ptr(dev)
        lib = native.kernels()
        cnt = torch.empty(max(1, int(lib.fmlx_csc_tiles_scratch(slots, d))), dtype=torch.int32, device=dev)
        native.call("fmlx_csc_tiles", native.ptr(self.colptr), b0, slots, d, self.EB, self.EL, native.ptr(self.tiles),
                    self.tstride, native.ptr(self.ntiles), native.ptr(cnt), cnt.numel(), stream)
        bstart = torch.from_numpy(np.asarray(self.bounds[b0:b0 + slots], dtype=np.int64)).to(dev)
        keys = torch.empty(m, dtype=sorting.U64, device=dev)
        pay = torch.empty(m, dtype=torch.int32, device=dev)
        native.call("fmlx_csc_tile_keys", f64, native.ptr(self.colptr), b0, slots, d, native.ptr(self.tiles),
                    self.tstride, native.ptr(self.ntiles), native.ptr(bstart), native.ptr(self.erow),
                    native.ptr(self.evals), j0, self.rb, self.pb, self.EL, native.ptr(keys), native.ptr(pay), stream)
        tb = max(1, int(self.tstride - 1).bit_length())
        seg = [self.bounds[b0 + s] - j0 for s in range(slots + 1)]
        keys, pay = sorting.sort_u64(keys, pay, seg, self.pb, self.pb + self.rb + tb)
        src = self.evals[j0:j1].clone() if f64 else None
        native.call("fmlx_csc_tile_store", f64, native.ptr(keys), native.ptr(pay), m, j0, self.rb, self.pb,
                    native.ptr(src), native.ptr(self.erow), native.ptr(self.evals), stream)

    def _cells(self, b0, slots, r0, r1, j0, j1) -> None:
        """The run's batches as forward cells (csc_build.hip): keys in row-major cell order, a
        stable radix sort on the (cell, row) bits, the row offsets, a re-key to (cell, column) with
        the row-major position riding along, a second stable sort, and the packed entries. Turns
        the cells off (the row-group forward takes over) when a cell outgrows its rank bits or the
        LDS."""
        import numpy as np

        from . import sorting

        indptr, indices, values = self._src
        dev = values.device
        m = j1 - j0
        f64 = int(values.dtype == torch.float64)
        stream = native.stream_ptr(dev)
        cellbits = max(1, int(self.cells - 1).bit_length())
        keys = torch.empty(m, dtype=sorting.U64, device=dev)
        pay = torch.empty(m, dtype=torch.int32, device=dev)
        native.call("fmlx_cell_keys", f64, native.ptr(indptr), native.ptr(indices), native.ptr(values), r0, r1, self.B,
                    j0, self.rbb, self.S, self.CS, self.cb, native.ptr(keys), native.ptr(pay), stream)
        seg = [self.bounds[b0 + s] - j0 for s in range(slots + 1)]
        starts = np.ascontiguousarray(np.asarray(seg, dtype=np.int64))
        keys, pay = sorting.sort_u64(keys, pay, seg, self.cb, self.cb + self.rbb + cellbits)
        native.call("fmlx_cell_bounds", native.ptr(keys), m, self.cb, starts.ctypes.data, slots,
                    self.cells << self.rbb, b0, self.rstride, native.ptr(self.roff), stream)
        kb = torch.empty_like(keys)
        native.call("fmlx_cell_rekey", native.ptr(keys), m, self.rbb, self.cb, native.ptr(kb), stream)
        del keys
        kb, pay = sorting.sort_u64(kb, pay, seg, 32, 32 + self.cb + cellbits)
        src = values[j0:j1] if f64 else None
        native.call("fmlx_cell_store", f64, native.ptr(kb), native.ptr(pay), m, j0, starts.ctypes.data, slots, b0,
                    native.ptr(self.roff), self.rstride, self.rbb, self.cb, native.ptr(src), native.ptr(self.cent),
                    native.ptr(self.cval), stream)
        # the largest cell of the run (one host read per build run)
        cs = self.roff[b0:b0 + slots, :self.rstride - 1:1 << self.rbb]
        nxt = torch.cat([cs[:, 1:], self.roff[b0:b0 + slots, -1:]], 1)
        big = int((nxt - cs).max()) if m else 0
        es = values.element_size()
        if big > (1 << (32 - self.cb)) or big * es > CELL_LDS_MAX:
            self._cells_off()
            return
        self.cmax = max(self.cmax, big)

    def _cells_off(self) -> None:
        self.cells, self.rstride, self.cmax = 0, 1, 0
        self.cent = self.cval = self.roff = self.cpart = self.ccnt = None
        self.version += 1  # (captured rounds must be re-captured without the cells)

    def _transpose_native(self, b0, slots, r0, r1, j0, j1) -> None:
        import numpy as np

        indptr, indices, values = self._src
        dev = values.device
        m, d = j1 - j0, self.d
        stream = native.stream_ptr(dev)
        # one segment per batch of the run, sorted by column (key − slot·d: ceil(log2 d) bits,
        # two 10-bit passes for 1M columns) — the batches' entries are already contiguous
        seg = [self.bounds[b0 + s] - j0 for s in range(slots + 1)]
        kbase = [s * d for s in range(slots)]
        bits = max(1, int(d - 1).bit_length())
        starts = np.ascontiguousarray(np.asarray(seg, dtype=np.int64))  # batch starts, run-relative
        if values.dtype == torch.float32 and CSC_BUCKET and 11 <= bits <= 20:
            # (value bits, row) as one 64-bit payload; the sort's keys are the CSR columns
            # themselves (segment = batch, so no slot offset): a stable pass on the high column
            # bits, then one block per (batch, 1024-column) bucket writes rows / values in column
            # order and the column pointers — no key array, no sorted keys
            # a batch of ≤ 2^22 rows: the column's low 10 bits ride in the payload (bits 22..31 above
            # the row), so the high-bits pass writes no keys and the bucket pass reads none
            pack = int(CSC_PACK and self.B <= (1 << 22))
            pay = torch.empty(m, dtype=torch.int64, device=dev)
            native.call("fmlx_csc_keys64", native.ptr(indptr), native.ptr(indices), native.ptr(values), r0, r1, self.B,
                        d, j0, None, native.ptr(pay), pack, stream)
            cols = indices[j0:j1]
            # held (no aliasing); packed: no key leaves the high-bits pass, so no key buffer
            key_alt, pay_alt = (cols if pack else torch.empty_like(cols)), torch.empty_like(pay)
            sc = torch.empty(seg_sort_scratch(seg, bits), dtype=torch.int32, device=dev)
            kb = np.zeros(slots, dtype=np.int32)
            rc = native.kernels().fmlx_csc_sort_split(
                native.ptr(cols), native.ptr(pay), native.ptr(key_alt), native.ptr(pay_alt), starts.ctypes.data,
                kb.ctypes.data, slots, bits, d, native.ptr(sc), sc.numel(), native.ptr(self.erow),
                native.ptr(self.evals), j0, native.ptr(self.colptr), b0, pack, stream)
            if rc != 0:
                raise RuntimeError("fmlx_csc_sort_split failed: %d" % rc)
            return
        key = torch.empty(m, dtype=torch.int32, device=dev)
        if values.dtype == torch.float32:
            # (value bits, row) as one 64-bit payload through the sort, then a sequential split
            pay = torch.empty(m, dtype=torch.int64, device=dev)
            native.call("fmlx_csc_keys64", native.ptr(indptr), native.ptr(indices), native.ptr(values), r0, r1, self.B,
                        d, j0, native.ptr(key), native.ptr(pay), 0, stream)
            # the last pass writes (row, value bits) straight into erow / evals (no unpack pass)
            keys_out, _ = seg_sort(key, pay, seg, kbase, bits, split=(self.erow, self.evals, j0))
        else:
            rel = torch.empty(m, dtype=torch.int32, device=dev)
            iota = torch.empty(m, dtype=torch.int32, device=dev)
            native.call("fmlx_csc_keys", native.ptr(indptr), native.ptr(indices), r0, r1, self.B, d, j0,
                        native.ptr(key), native.ptr(rel), native.ptr(iota), stream)
            keys_out, order = seg_sort(key, iota, seg, kbase, bits)
            native.call("fmlx_csc_fill", 1, native.ptr(order), m, j0, native.ptr(rel), native.ptr(values),
                        native.ptr(self.erow), native.ptr(self.evals), stream)
        native.call("fmlx_csc_colptr", native.ptr(keys_out), m, slots, d, starts.ctypes.data, b0,
                    native.ptr(self.colptr), stream)

    def _transpose_torch(self, b0, slots, r0, r1, j0, j1) -> None:
        indptr, indices, values = self._src
        dev = values.device
        d, B = self.d, self.B
        lens = indptr[r0 + 1:r1 + 1] - indptr[r0:r1]
        rows = torch.arange(r0, r1, device=dev, dtype=torch.int64)
        slot = torch.div(rows - r0, B, rounding_mode="floor")
        rel = (rows - r0 - slot * B).to(torch.int32)  # batch-relative row id
        ent_slot = torch.repeat_interleave(slot.to(torch.int32), lens, output_size=j1 - j0)
        key = ent_slot * d + indices[j0:j1]
        order, starts = _stable_order(key, slots * d)
        self.erow[j0:j1] = torch.repeat_interleave(rel, lens, output_size=j1 - j0)[order]
        self.evals[j0:j1] = values[j0:j1][order]
        # batch s of the run starts at starts[s·d]; its column c at starts[s·d + c]
        S = starts[:-1].view(slots, d)
        self.colptr[b0:b0 + slots, :d] = S - S[:, :1]
        self.colptr[b0:b0 + slots, d] = starts[d::d] - S[:, 0]

    def ensure_rounds(self, first_epoch: int, k: int) -> None:
        """Transposes the batches of rounds first_epoch … first_epoch + k − 1."""
        if all(self.built):
            return
        self.ensure(range(first_epoch, first_epoch + min(k, self.P)))


def _stable_order(key: torch.Tensor, bound: int):
    """Stable argsort of int32 keys in [0, bound) and the bucket starts of the sorted keys
    (int32 [bound + 1]: first position of a key >= c). On the GPU an LSD radix sort over only the
    ceil(log2 bound) key bits with int32 payloads (radix.hip ``seg_sort``) and one boundary
    kernel; torch elsewhere."""
    m = key.numel()
    if key.device.type != "cuda" or m == 0:
        order = torch.sort(key, stable=True).indices
        starts = torch.zeros(bound + 1, dtype=torch.int32, device=key.device)
        starts[1:] = torch.cumsum(torch.bincount(key.long(), minlength=bound), 0).to(torch.int32)
        return order, starts
    bits = max(1, int(bound - 1).bit_length())
    iota = torch.arange(m, dtype=torch.int32, device=key.device)
    keys_out, order = seg_sort(key.clone(), iota, [0, m], [0], bits)
    starts = torch.empty(bound + 1, dtype=torch.int32, device=key.device)
    native.call("fmlx_sorted_bounds", native.ptr(keys_out), m, int(bound), native.ptr(starts),
                native.stream_ptr(key.device))
    return order.long(), starts


def wl_elems() -> int:
    return int(native.kernels().fmlx_glm_wl_elems())


def set_csc_tuning(fwd_cap: int = 0, bwd_cap: int = 0) -> None:
    """Grid caps of the sparse forward / backward kernels (0 = default; A/B knob)."""
    native.kernels().fmlx_glm_set_csc_tuning(int(fwd_cap), int(bwd_cap))


def csc_round(csc: BatchCsc, indptr, idx, val, y, wt, coef, n, d, B, loss, state, mult, wl, fb, fuse: bool,
              max_iter, tol, lr, reg, en) -> None:
    if csc.cap == 0:
        raise RuntimeError("BatchCsc.ensure must run before the first round")
    native.call("fmlx_glm_csc_round", int(val.dtype == torch.float64), csc.G, native.ptr(indptr), native.ptr(idx),
                native.ptr(val), native.ptr(y), native.ptr(wt), native.ptr(coef), n, d, B, loss, native.ptr(state),
                native.ptr(mult), native.ptr(wl), native.ptr(csc.colptr), native.ptr(csc.erow), native.ptr(csc.evals),
                native.ptr(fb), int(fuse), max_iter, tol, lr, reg, en, native.ptr(csc.tiles), native.ptr(csc.ntiles),
                csc.tstride, csc.rb, csc.EL, csc.ET, native.ptr(csc.cent), native.ptr(csc.cval), native.ptr(csc.roff),
                csc.rstride, csc.rbb, getattr(csc, "S", 0), getattr(csc, "CS", 0), getattr(csc, "cb", 0), csc.cells, csc.cmax,
                native.ptr(csc.cpart), native.ptr(csc.ccnt), native.stream_ptr(val.device))


_BKT_LIMITS = None


def _bkt_limits():
    """The bucket round kernels' compile-time limits (csrc/glm_sparse.hip fmlx_glm_bkt_limits), read once
    (at library load: native._preload)."""
    global _BKT_LIMITS
    if _BKT_LIMITS is None and native.BKT_LIMITS is not None:
        _BKT_LIMITS = native.BKT_LIMITS
    if _BKT_LIMITS is None:
        lim = np.zeros(8, dtype=np.int32)
        native.kernels().fmlx_glm_bkt_limits(lim.ctypes.data)
        _BKT_LIMITS = lim
    return _BKT_LIMITS


class BucketRound:
    """Device buffers of the single-visit sparse round (csrc/glm_sparse.hip glm_bkt_*): per round,
    the batch's entries are counted per column slice of 2^csb columns, written by the forward into
    their slice's bucket as (column in slice, m_row·x) and summed per slice in LDS by the backward —
    nothing is precomputed per batch, so a fit that visits each batch once (the reference's
    LinearSVC benchmark: SGD.java:263-268 over 100k-row batches) pays no transpose. Buffers: the
    largest batch's entries (an 8-byte (column, value) record each; fp64 16), a [d] accumulator for slices summed in several
    chunks, and the [forward blocks][slices] count / offset matrices."""

    CHUNK = 32768  # backward entries per work item (a slice of more is summed in chunks; fp64: ≤ 16384)

    SLOT_BYTES_MAX = 256 << 20  # the one-time counts of a fit's batches: at most this much

    RB_HEADROOM = 1.1  # rows per forward block leave this factor of the mean row length free

    def __init__(self, indptr, values, n: int, d: int, B: int, G: int, most: Optional[int] = None,
                 avg: Optional[float] = None, batches: int = 0, zero_bufs=None):
        lim = _bkt_limits()
        dev = values.device
        es = values.element_size()
        nt, nb_max = int(lim[0]), int(lim[2])
        _ecap = int(lim[3] if es == 8 else lim[1])
        chunk_max = int(lim[5] if es == 8 else lim[4])
        rec_bytes = int(lim[7] if es == 8 else lim[6])
        self.G = G
        self.d = d
        # ~256 slices (the backward's parallelism), at most nb_max; ≤ 4096 columns per slice (the
        # backward's column counters share the LDS with a chunk of values)
        csb = BucketRound.slice_bits(d)
        self.csb = csb
        self.nb = -(-d // (1 << csb))
        if self.nb > nb_max:
            raise ValueError("too many column slices")
        longest = None
        if most is None:
            nnz, bounds = _batch_bounds(indptr, n, B)
            most = max(bounds[i + 1] - bounds[i] for i in range(len(bounds) - 1))
            avg = nnz / max(1, n)
            longest = batch_row_max(indptr, n, B)
        # forward rows per block: one staged piece of ECAP entries — exactly, when every row has the
        # same length; else with 10 % headroom, so a block whose rows run longer than average rarely
        # overflows into the multi-piece path (56 rows of Poisson(64) lengths exceed 3584 entries in
        # half the blocks; their mean exceeding 1.1·64 is a 5-sigma event)
        uniform = longest is not None and longest <= avg
        self.rb = max(1, min(4096, int(_ecap / (max(avg, 1.0) * (1.0 if uniform else self.RB_HEADROOM)))))
        self.chunk = min(self.CHUNK, chunk_max)
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        # as many backward blocks as the LDS lets share the CUs (a block loops over the work items,
        # so a grid of #slices covers evenly loaded slices with one arrival per block)
        blds = self.chunk * es + ((1 << csb) + 1 + 3 * self.nb + 2) * 4
        self.bwd_blocks = max(1, min(cus * max(1, (160 << 10) // blds), self.nb))
        fblocks = -(-max(1, min(B, n)) // self.rb)
        # batches > 0: the fit visits batches 0 … batches − 1; their per-(block, slice) counts and
        # offsets are made once, before the first round (count_all), when they fit SLOT_BYTES_MAX;
        # otherwise every round counts its own batch
        self.mstride = fblocks * self.nb
        self.slots = batches if 0 < batches and 3 * batches * self.mstride * 4 <= self.SLOT_BYTES_MAX else 0
        self.counted = False
        i32 = dict(dtype=torch.int32, device=dev)
        S = max(1, self.slots)
        # one allocation: counts [S][nb][blocks], record offsets and staging offsets [S][blocks][nb],
        # bucket totals [S][nb] and starts [S][nb + 1]
        m = S * self.mstride
        ints = torch.empty(3 * m + S * (2 * self.nb + 1), **i32)
        self.cntm, self.offm, self.lofs = ints[:m], ints[m:2 * m], ints[2 * m:3 * m]
        self.tot, self.bst = ints[3 * m:3 * m + S * self.nb], ints[3 * m + S * self.nb:]
        # (zero_bufs: the caller's one zero-filled allocation for `done` and `acc`)
        # done: [nb] chunk arrivals, then the backward's [8] group + [1] top arrival tickets
        self.done, self.acc = zero_bufs if zero_bufs is not None else \
            native.zeros_many([((self.nb + 16,), torch.int32), ((d,), values.dtype)], dev)
        self.rec = torch.empty(max(1, most) * rec_bytes, dtype=torch.uint8, device=dev)

    def count_all(self, indptr, idx, n: int, B: int) -> None:
        """The one-time counts of the fit's batches (no-op per round mode / already made)."""
        if self.slots and not self.counted:
            native.call("fmlx_glm_bkt_count_all", native.ptr(indptr), native.ptr(idx), n, B, self.csb, self.nb, self.rb,
                        native.ptr(self.cntm), native.ptr(self.offm), native.ptr(self.lofs), native.ptr(self.tot),
                        native.ptr(self.bst), self.slots, self.mstride, native.stream_ptr(idx.device))
            self.counted = True

    SLICE_COLS = 256  # columns per slice ≈ d / this, as a power of two in [2^6, 2^12]

    @staticmethod
    def slice_bits(d: int) -> int:
        return min(12, max(6, int(math.ceil(math.log2(max(1.0, d / float(BucketRound.SLICE_COLS)))))))

    @staticmethod
    def nb_for(d: int, es: int = 4) -> int:
        """Column slices of a BucketRound for width d (its `done` counters: this + 16)."""
        return -(-d // (1 << BucketRound.slice_bits(d)))

    @staticmethod
    def alloc(indptr, values, n: int, d: int, B: int, most: Optional[int] = None, avg: Optional[float] = None,
              batches: int = 0, zero_bufs=None):
        """A BucketRound, or None where the kernels' limits rule it out (too many slices).
        ``most`` / ``avg``: the largest batch's entries and the mean row length, when the caller
        knows them (the out-of-core trainer points one BucketRound at every streamed batch)."""
        if n <= 0 or B <= 0 or d <= 0 or values.device.type != "cuda":
            return None
        if avg is None:
            nnz, _ = _batch_bounds(indptr, n, B)
            avg = nnz / max(1, n)
        try:
            return BucketRound(indptr, values, n, d, B, BatchCsc.pick_group(avg), most=most, avg=avg, batches=batches,
                               zero_bufs=zero_bufs)
        except ValueError:
            return None


def bkt_round(bk: BucketRound, indptr, idx, val, y, wt, coef, n, d, B, loss, state, wl, fb, fuse: bool,
              max_iter, tol, lr, reg, en) -> None:
    if bk.slots and not bk.counted:
        raise RuntimeError("BucketRound.count_all must run before the first round")
    rc = native.kernels().fmlx_glm_bkt_round(
        int(val.dtype == torch.float64), bk.G, native.ptr(indptr), native.ptr(idx), native.ptr(val), native.ptr(y),
        native.ptr(wt), native.ptr(coef), n, d, B, loss, native.ptr(state), native.ptr(wl), native.ptr(fb), int(fuse),
        max_iter, float(tol), float(lr), float(reg), float(en), bk.csb, bk.rb, bk.chunk, native.ptr(bk.cntm),
        native.ptr(bk.offm), native.ptr(bk.lofs), native.ptr(bk.tot), native.ptr(bk.bst), bk.slots, bk.mstride,
        native.ptr(bk.done), native.ptr(bk.rec),
        native.ptr(bk.acc), bk.bwd_blocks, native.stream_ptr(val.device))
    if rc != 0:
        raise RuntimeError("fmlx_glm_bkt_round failed: %d" % rc)


# ---------------------------------------------------------------------------------------------
# prediction
# ---------------------------------------------------------------------------------------------
MODE_LR, MODE_SVC, MODE_LINREG = 0, 1, 2


def predict_dense(X: torch.Tensor, coef: torch.Tensor, mode: int, threshold: float = 0.0):
    """Returns (prediction[n] f64, raw[n,2] f64 or None)."""
    n = X.shape[0]
    if X.device.type == "cuda":
        lay = pick_layout(X, rounds=False)
        if lay is not None and X.dtype in (torch.float32, torch.float64, torch.bfloat16):
            acc = torch.float64 if X.dtype == torch.float64 else torch.float32
            c = coef.to(device=X.device, dtype=acc).contiguous()
            pred = torch.empty(n, dtype=torch.float64, device=X.device)
            raw = torch.empty((n, 2), dtype=torch.float64, device=X.device)
            native.call("fmlx_glm_predict", native.dtype_code(X.dtype), lay[0], lay[1], native.ptr(X), X.stride(0),
                        n, X.shape[1], native.ptr(c), mode, float(threshold), native.ptr(pred), native.ptr(raw),
                        native.stream_ptr(X.device))
            return pred, (raw if mode != MODE_LINREG else None)
        dot = (X.to(torch.float64) @ coef.to(device=X.device, dtype=torch.float64))
    else:
        dot = X.to(torch.float64) @ coef.to(dtype=torch.float64, device=X.device)
    return dots_to_outputs(dot, mode, threshold)


def predict_csr(indptr, idx, val, coef, n, mode: int, threshold: float = 0.0):
    if val.device.type == "cuda":
        acc = torch.float64 if val.dtype == torch.float64 else torch.float32
        c = coef.to(device=val.device, dtype=acc).contiguous()
        dots = torch.empty(n, dtype=torch.float64, device=val.device)
        native.call("fmlx_glm_csr_predict", int(acc == torch.float64), native.ptr(indptr), native.ptr(idx),
                    native.ptr(val.to(acc)), native.ptr(c), n, native.ptr(dots), native.stream_ptr(val.device))
    else:
        counts = indptr[1:] - indptr[:-1]
        rows = torch.repeat_interleave(torch.arange(n), counts)
        dots = torch.zeros(n, dtype=torch.float64)
        dots.index_add_(0, rows, val.to(torch.float64) * coef.to(torch.float64)[idx.long()])
    return dots_to_outputs(dots, mode, threshold)


def dots_to_outputs(dot: torch.Tensor, mode: int, threshold: float):
    dot = dot.to(torch.float64)
    if mode == MODE_LR:
        p = 1.0 - 1.0 / (1.0 + torch.exp(dot))
        return (dot >= 0).to(torch.float64), torch.stack([1.0 - p, p], dim=1)
    if mode == MODE_SVC:
        return (dot >= threshold).to(torch.float64), torch.stack([dot, -dot], dim=1)
    return dot, None


# ---------------------------------------------------------------------------------------------
# torch reference of the per-row loss / multiplier (LIB/common/lossfunc/*.java)
# ---------------------------------------------------------------------------------------------
def torch_loss_and_mult(loss: int, dot, y, wt):
    if loss == 0:
        ys = 2 * y - 1
        z = -dot * ys
        l = wt * torch.nn.functional.softplus(z)
        m = wt * (-ys / (torch.exp(dot * ys) + 1))
    elif loss == 1:
        ys = 2 * y - 1
        h = 1 - ys * dot
        pos = h > 0
        l = torch.where(pos, wt * h, torch.zeros_like(h))
        m = torch.where(pos, -ys * wt, torch.zeros_like(h))
    else:
        r = dot - y
        l = wt * 0.5 * r * r
        m = r * wt
    return l, m


def torch_regularize(coef: torch.Tensor, reg: float, en: float, lr: float) -> None:
    if reg == 0:
        return
    if en == 0:
        coef.mul_(1 - lr * reg)
    elif en == 1:
        coef.sub_(lr * en * reg * torch.sign(coef))
    else:
        coef.sub_(lr * (en * reg * torch.sign(coef) + (1 - en) * reg * coef))
