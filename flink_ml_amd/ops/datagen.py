"""Bit-exact ``java.util.Random`` row streams for the benchmark data generators.

``java_rows(seed, n, ops, nvec)`` reproduces, for one task, the values a reference
``RowGenerator`` subclass draws: ``ops[j] == 0`` is ``nextDouble()`` and ``ops[j] == b > 0`` is
``nextInt(b)``. On the GPU every row jumps to its first draw (``csrc/datagen.hip``); on the CPU the
same jump-ahead runs vectorised in numpy (uint64 arithmetic keeps the low 48 bits exact).
Rejected ``nextInt`` draws (non power-of-two bounds, ~1e-9 per draw) are detected, the offending
row is replayed sequentially on the host and the rest of the rows are regenerated at the shifted
offset — the result is always the exact reference stream.
"""
from __future__ import annotations

from typing import Sequence, Tuple

import numpy as np
import torch

from . import native
from .native import c_int, c_long, c_void_p

_MULT = 0x5DEECE66D
_ADD = 0xB
_MASK = (1 << 48) - 1

native.register_kernel_sigs({
    "fmlx_java_int_draws": [native.c_ulonglong, native.c_ulonglong, c_long, c_int, c_void_p, c_void_p, c_void_p],
    "fmlx_u8_zero_positions": [c_void_p, c_long, c_long, c_void_p, c_void_p, c_void_p],
    "fmlx_remove_positions_i32": [c_void_p, c_void_p, c_int, c_void_p, c_long, c_void_p],
    "fmlx_java_rows": [c_int, native.c_ulonglong, native.c_ulonglong, c_long, c_long, c_void_p, c_void_p, c_int, c_int,
                       c_int, c_void_p, c_void_p, c_void_p, c_void_p],
})


def scramble(seed: int) -> int:
    return (int(seed) ^ _MULT) & _MASK


def _jump_host(x: int, k: int) -> int:
    A, C, a, c = 1, 0, _MULT, _ADD
    while k:
        if k & 1:
            A, C = (A * a) & _MASK, (C * a + c) & _MASK
        c, a = (c * a + c) & _MASK, (a * a) & _MASK
        k >>= 1
    return (A * x + C) & _MASK


def _draws_per_row(ops: Sequence[int]) -> int:
    return sum(2 if o == 0 else 1 for o in ops)


def _replay_row(state: int, ops: Sequence[int]) -> Tuple[list, int]:
    """Sequential reference draws for one row from LCG ``state``; returns (values, draws used)."""
    used = 0
    vals = []

    def nxt(bits):
        nonlocal state, used
        state = (state * _MULT + _ADD) & _MASK
        used += 1
        v = state >> (48 - bits)
        return v - (1 << bits) if v >= (1 << (bits - 1)) and bits == 32 else v

    for op in ops:
        if op == 0:
            vals.append(((nxt(26) << 27) + nxt(27)) * (1.0 / (1 << 53)))
        elif op & (op - 1) == 0:
            vals.append(float((op * nxt(31)) >> 31))
        else:
            while True:
                u = nxt(31)
                r = u % op
                if u - r + op - 1 < (1 << 31):
                    vals.append(float(r))
                    break
    return vals, used


def _cpu_rows(x0: int, start: int, n: int, ops, nvec, vec: np.ndarray, scal: np.ndarray, row0: int) -> int:
    """numpy jump-ahead generation of rows [row0, row0+n); returns first rejecting row or -1."""
    dpr = _draws_per_row(ops)
    M, MASK = np.uint64(_MULT), np.uint64(_MASK)
    k = np.uint64(start) + np.arange(n, dtype=np.uint64) * np.uint64(dpr)
    A = np.ones(n, dtype=np.uint64)
    C = np.zeros(n, dtype=np.uint64)
    a, c = _MULT, _ADD
    kk = k.copy()
    with np.errstate(over="ignore"):
        while kk.any():
            bit = (kk & np.uint64(1)).astype(bool)
            A = np.where(bit, (A * np.uint64(a)) & MASK, A)
            C = np.where(bit, (C * np.uint64(a) + np.uint64(c)) & MASK, C)
            c, a = (c * a + c) & _MASK, (a * a) & _MASK
            kk >>= np.uint64(1)
        s = (A * np.uint64(x0) + C) & MASK
        reject = np.full(n, False)

        def nxt(bits):
            nonlocal s
            s = (s * M + np.uint64(_ADD)) & MASK
            return (s >> np.uint64(48 - bits)).astype(np.int64)

        nv = nvec
        for j, op in enumerate(ops):
            if op == 0:
                v = ((nxt(26) << 27) + nxt(27)).astype(np.float64) * (1.0 / (1 << 53))
            else:
                u = nxt(31)
                if op & (op - 1) == 0:
                    v = ((op * u) >> 31).astype(np.float64)
                else:
                    r = u % op
                    reject |= (u - r + op - 1) >= (1 << 31)
                    v = r.astype(np.float64)
            if j < nv:
                vec[row0:row0 + n, j] = v
            else:
                scal[row0:row0 + n, j - nv] = v
    bad = np.nonzero(reject)[0]
    return int(bad[0]) if bad.size else -1


INT_DRAWS_REJECT_CAP = 1 << 16  # rejected draws per window the positional compaction takes


def _compact_accepted(r: torch.Tensor, ok: torch.Tensor, count: int, rem: int, dst: torch.Tensor):
    """Copies the first min(rem, accepted) accepted draws of ``r`` to ``dst`` with the
    rare-rejection kernels (csrc/datagen.hip); returns how many, or None when the window holds more
    than INT_DRAWS_REJECT_CAP rejections (the caller takes the boolean-mask path)."""
    dev, cap = r.device, INT_DRAWS_REJECT_CAP
    buf = torch.zeros(cap + 1, dtype=torch.int64, device=dev)  # positions | counter
    stream = native.stream_ptr(dev)
    native.call("fmlx_u8_zero_positions", native.ptr(ok), count, cap, native.ptr(buf), native.ptr(buf[cap:]), stream)
    h = buf.cpu().numpy()
    nrej = int(h[cap])
    if nrej > cap:
        return None
    rej = np.sort(h[:nrej])
    take = min(rem, count - nrej)
    q = torch.from_numpy(rej - np.arange(nrej, dtype=np.int64)).to(dev) if nrej else buf[:1]
    native.call("fmlx_remove_positions_i32", native.ptr(r), native.ptr(q), nrej, native.ptr(dst), take, stream)
    return take


def java_uniform_int_rows(seed: int, n: int, k: int, bound: int, device) -> torch.Tensor:
    """[n, k] int32 of ``k`` successive ``Random.nextInt(bound)`` per row (rows back to back in one
    ``java.util.Random(seed)`` stream), on the device for any bound: raw draws and their rejection
    test in parallel (``fmlx_java_int_draws``), then the accepted ones compacted by a prefix sum —
    the same values as the sequential rejection loop, without a host round trip per rejection
    (bounds like 1,000,000 reject ~1 draw in 4,400)."""
    need = n * k
    x0 = scramble(seed)
    p_rej = ((1 << 31) % bound) / float(1 << 31)
    out = torch.empty(need, dtype=torch.int32, device=device)
    got, pos = 0, 0
    while got < need:
        rem = need - got
        count = int(rem / max(1e-9, 1.0 - p_rej)) + 64 + int(4 * (rem * p_rej) ** 0.5)
        r = torch.empty(count, dtype=torch.int32, device=device)
        ok = torch.empty(count, dtype=torch.uint8, device=device)
        native.call("fmlx_java_int_draws", x0, pos, count, bound, native.ptr(r), native.ptr(ok), native.stream_ptr(device))
        take = _compact_accepted(r, ok, count, rem, out[got:]) if r.is_cuda else None
        if take is None:
            acc = r[ok.bool()]
            take = min(rem, acc.numel())
            out[got:got + take] = acc[:take]
        if take == rem:
            break
        got += take
        pos += count
    return out.view(n, k)


def java_rows(seed: int, n: int, ops: Sequence[int], nvec: int, device=None, vec_dtype=torch.float64,
              int_codes: bool = False):
    """Rows of one generator task: (vec [n, nvec] in ``vec_dtype``, scalars [n, len(ops)-nvec] fp64).
    ``int_codes``: scalars that are all nextInt(b) draws of one bound may come back as int32 (the
    string generators' dictionary codes: no fp64 round trip of the whole draw stream)."""
    device = torch.device(device) if device is not None else torch.device("cpu")
    ops = [int(o) for o in ops]
    if nvec == 0 and ops and len(set(ops)) == 1 and ops[0] > 0 and ops[0] & (ops[0] - 1) != 0 and n > 0:
        # every draw is nextInt(b) with the same non-power-of-two b: compact accepted draws on the
        # device, or run the sequential Random on the host (native) — no per-rejection restarts
        if device.type == "cuda":
            codes = java_uniform_int_rows(seed, n, len(ops), ops[0], device)
            return torch.empty((n, 0), dtype=vec_dtype, device=device), codes if int_codes else codes.to(torch.float64)
        import ctypes

        native.register_host_sigs({"fmlx_java_next_ints": [ctypes.c_int64, ctypes.c_int64, ctypes.c_int32,
                                                           ctypes.c_void_p]})
        out = np.empty(n * len(ops), dtype=np.int32)
        native.host().fmlx_java_next_ints(int(seed), out.size, int(ops[0]), out.ctypes.data)
        return (torch.empty((n, 0), dtype=vec_dtype),
                torch.from_numpy(out.reshape(n, len(ops)) if int_codes else out.reshape(n, len(ops)).astype(np.float64)))
    ns = len(ops) - nvec
    dpr = _draws_per_row(ops)
    x0 = scramble(seed)
    start, row0 = 0, 0
    if device.type == "cuda":
        vec = torch.empty((n, nvec), dtype=vec_dtype, device=device)
        scal = torch.empty((n, max(ns, 0)), dtype=torch.float64, device=device)
        ops_t = torch.tensor(ops, dtype=torch.int32, device=device)
        offs = np.concatenate([[0], np.cumsum([2 if o == 0 else 1 for o in ops])[:-1]]).astype(np.int32)
        off_t = torch.from_numpy(offs).to(device)
        flag = torch.empty(1, dtype=torch.int64, device=device)
        while row0 < n:
            flag.fill_(-1)  # 0xFFFF... as unsigned
            native.call("fmlx_java_rows", native.dtype_code(vec_dtype), x0, start, row0, n - row0, native.ptr(ops_t),
                        native.ptr(off_t), len(ops), nvec, dpr, native.ptr(vec), native.ptr(scal) if ns else None, native.ptr(flag),
                        native.stream_ptr(device))
            bad = int(flag.item())
            if bad < 0:
                break
            r = row0 + bad
            vals, used = _replay_row(_jump_host(x0, start + bad * dpr), ops)
            if nvec:
                vec[r] = torch.tensor(vals[:nvec], dtype=torch.float64, device=device).to(vec_dtype)
            if ns:
                scal[r] = torch.tensor(vals[nvec:], dtype=torch.float64, device=device)
            start += bad * dpr + used
            row0 = r + 1
        return vec, scal
    vec_np = np.empty((n, nvec), dtype=np.float64)
    scal_np = np.empty((n, max(ns, 0)), dtype=np.float64)
    while row0 < n:
        bad = _cpu_rows(x0, start, n - row0, ops, nvec, vec_np, scal_np, row0)
        if bad < 0:
            break
        r = row0 + bad
        vals, used = _replay_row(_jump_host(x0, start + bad * dpr), ops)
        vec_np[r, :nvec] = vals[:nvec]
        scal_np[r, :] = vals[nvec:]
        start += bad * dpr + used
        row0 = r + 1
    return torch.from_numpy(vec_np).to(vec_dtype), torch.from_numpy(scal_np)


# ---------------------------------------------------------------------------------------------
# reservoir sampling (DataStreamUtils.SamplingOperator, DataStreamUtils.java:633-704) on device
# ---------------------------------------------------------------------------------------------
native.register_kernel_sigs({
    "fmlx_java_next31": [native.c_ulonglong, native.c_ulonglong, c_long, c_void_p, c_void_p],
    "fmlx_reservoir_final": [native.c_ulonglong, c_long, c_int, c_void_p, c_long, c_void_p, c_void_p],
    "fmlx_reservoir_candidates": [c_void_p, c_long, c_int, c_long, c_void_p, c_void_p, c_void_p, c_void_p],
})
_host_sigs_done = False


def _host_sigs():
    global _host_sigs_done
    if not _host_sigs_done:
        import ctypes

        native.register_host_sigs({
            "fmlx_reservoir_rejections": ([ctypes.c_int64, ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p],
                                          ctypes.c_int64),
            "fmlx_java_next31": [ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p],
        })
        _host_sigs_done = True


def next31_stream(seed: int, start: int, count: int, device) -> torch.Tensor:
    """Raw ``next(31)`` values of ``new Random(seed)`` at positions [start, start + count) (int32)."""
    out = torch.empty(max(int(count), 0), dtype=torch.int32, device=device)
    if count <= 0:
        return out
    if out.device.type == "cuda":
        native.call("fmlx_java_next31", scramble(seed), int(start), int(count), native.ptr(out),
                    native.stream_ptr(out.device))
    else:
        _host_sigs()
        native.host().fmlx_java_next31(int(seed), int(start), int(count), out.data_ptr())
    return out


RESERVOIR_CAND_HOST_SORT_MAX = 1 << 16  # candidates ordered on the host after the compaction kernel


def _reservoir_candidates(u: torch.Tensor, npos: int, k: int):
    """[positions | values] of the stream's candidate positions in position order (int32 [2, c],
    host), from the unordered compaction kernel plus a host sort; None when there are more than
    RESERVOIR_CAND_HOST_SORT_MAX (the caller takes the ordered torch path)."""
    cap = RESERVOIR_CAND_HOST_SORT_MAX
    buf = torch.empty(2 * cap + 2, dtype=torch.int32, device=u.device)  # cp | cu | u64 counter
    buf[2 * cap:].zero_()
    native.call("fmlx_reservoir_candidates", native.ptr(u), npos, k, cap, native.ptr(buf), native.ptr(buf[cap:]),
                native.ptr(buf[2 * cap:]), native.stream_ptr(u.device))
    h = buf.cpu().numpy()
    c = int(h[2 * cap:].view(np.uint64)[0])
    if c > cap:
        return None
    cp, cu = h[:c], h[cap:cap + c]
    order = np.argsort(cp, kind="stable")
    return np.stack([cp[order], cu[order]])


def reservoir_sample_device(n: int, k: int, seed: int, device) -> torch.Tensor:
    """Positions ``SamplingOperator`` keeps (a java.util.Random(seed) reservoir of size k over n
    elements), in reservoir-slot order — bit-exact with the sequential sampler
    (``javarand.cpp fmlx_reservoir_sample``), but with the n-long draw stream on the device:

      1. draw i (i = k .. n−1) is ``nextInt(i + 1)``; without rejections it reads stream position
         p = i − k. The raw next(31) stream is generated in parallel (jump-ahead, datagen.hip);
      2. only positions with u ≥ 2^31 − n can be rejected draws (≈ n / 2^31 of them); those
         candidates are scanned in order on the host (``fmlx_reservoir_rejections``) — the only
         sequential step, over a few percent of the stream;
      3. every position p then knows its draw i = p + k − R(p) (R = rejections before p), and the
         slot it writes; the last writer of every slot wins (a max-reduction by i).
    Returns int64 [min(n, k)] on ``device``."""
    n, k = int(n), int(k)
    dev = torch.device(device)
    if n <= 0 or k <= 0:
        return torch.zeros(0, dtype=torch.int64, device=dev)
    if n <= k:
        return torch.arange(n, dtype=torch.int64, device=dev)
    _host_sigs()
    m = n - k
    npos = m + m * n // (1 << 31) + 65536
    while True:
        u = next31_stream(seed, 0, npos, dev)
        # position p can only hold a rejected draw if u_p ≥ 2^31 − b for its bound b ≤ p + k + 1
        # (b shrinks with the rejections before p): ≈ half as many candidates as u ≥ 2^31 − n
        both = _reservoir_candidates(u, npos, k) if dev.type == "cuda" else None
        if both is None:
            pos = torch.arange(npos, dtype=torch.int64, device=dev)
            cand = torch.nonzero(u.to(torch.int64) + pos >= (1 << 31) - k - 1).view(-1)
            del pos
            both = torch.stack([cand.to(torch.int32), u[cand]])  # one D2H copy of [positions | values]
            both = both.cpu().numpy()
        cand_p, cand_u = np.ascontiguousarray(both[0]), np.ascontiguousarray(both[1])
        rej = np.zeros(max(len(cand_p), 1), dtype=np.int64)
        done = np.zeros(1, dtype=np.int32)
        nrej = int(native.host().fmlx_reservoir_rejections(n, k, npos, cand_p.ctypes.data, cand_u.ctypes.data,
                                                           len(cand_p), rej.ctypes.data, done.ctypes.data))
        if done[0]:
            break
        npos = npos * 3 // 2  # the stream ran out before the last draw: regenerate longer
    end = m + nrej  # positions consumed by draws k .. n−1
    if dev.type == "cuda":
        # one fused pass: the stream regenerated by jump-ahead, R(p) by binary search, atomicMax
        # per slot (no n-long int64 temporaries)
        del u
        rejt = torch.as_tensor(rej[:nrej], dtype=torch.int64).to(dev) if nrej else torch.zeros(1, dtype=torch.int64,
                                                                                               device=dev)
        out32 = torch.arange(k, dtype=torch.int32, device=dev)
        native.call("fmlx_reservoir_final", scramble(seed), end, k, native.ptr(rejt), nrej, native.ptr(out32),
                    native.stream_ptr(dev))
        return out32.to(torch.int64)
    u = u[:end].to(torch.int64)
    p = torch.arange(end, dtype=torch.int64, device=dev)
    rejt = torch.as_tensor(rej[:nrej], dtype=torch.int64, device=dev)
    R = torch.searchsorted(rejt, p) if nrej else torch.zeros_like(p)
    ok = torch.ones(end, dtype=torch.bool, device=dev)
    if nrej:
        ok[rejt] = False
    i = p + k - R
    b = i + 1
    pow2 = (b & (b - 1)) == 0
    slot = torch.where(pow2, (b * u) >> 31, u % b)
    sel = ok & (slot < k)
    out = torch.arange(k, dtype=torch.int64, device=dev)
    out.scatter_reduce_(0, slot[sel], i[sel], "amax")
    return out
