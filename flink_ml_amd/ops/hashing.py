"""murmur3_32 (Guava semantics) bindings: host C++ for host-resident string batches
(``csrc/host/murmur3.cpp``) and a device kernel for large pre-encoded batches (``csrc/hash.hip``)."""
from __future__ import annotations

import ctypes
import struct
from typing import List, Sequence

import numpy as np
import torch

from . import native

native.register_host_sigs({
    "fmlx_murmur3_chars": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p], None),
    "fmlx_murmur3_ints": ([ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p], None),
    "fmlx_murmur3_longs": ([ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p], None),
})
native.register_kernel_sigs({
    "fmlx_murmur3_chars_device": [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p],
})


def encode_utf16(strings: Sequence[str]):
    """Flat UTF-16 code units + int64 offsets (Java char semantics)."""
    enc = [s.encode("utf-16-le", "surrogatepass") for s in strings]
    lens = np.fromiter((len(b) // 2 for b in enc), dtype=np.int64, count=len(enc))
    offsets = np.zeros(len(enc) + 1, dtype=np.int64)
    np.cumsum(lens, out=offsets[1:])
    units = np.frombuffer(b"".join(enc), dtype=np.uint16) if enc else np.zeros(0, np.uint16)
    return np.ascontiguousarray(units), offsets


def hash_strings(strings: Sequence[str]) -> np.ndarray:
    units, offsets = encode_utf16(strings)
    out = np.zeros(len(strings), dtype=np.int32)
    if len(strings):
        native.host().fmlx_murmur3_chars(units.ctypes.data if units.size else None, offsets.ctypes.data,
                                         len(strings), out.ctypes.data)
    return out


def hash_ints(v) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(v, dtype=np.int32))
    out = np.zeros(a.shape[0], dtype=np.int32)
    if a.size:
        native.host().fmlx_murmur3_ints(a.ctypes.data, a.shape[0], out.ctypes.data)
    return out


def hash_longs(v) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(v, dtype=np.int64))
    out = np.zeros(a.shape[0], dtype=np.int32)
    if a.size:
        native.host().fmlx_murmur3_longs(a.ctypes.data, a.shape[0], out.ctypes.data)
    return out


def hash_object(obj) -> int:
    """HashingTF.hash (HashingTF.java:165-190)."""
    if obj is None:
        return 0
    if isinstance(obj, (bool, np.bool_)):
        return int(hash_ints([1 if obj else 0])[0])
    if isinstance(obj, (int, np.integer)):
        if -(1 << 31) <= int(obj) < (1 << 31):
            return int(hash_ints([int(obj)])[0])
        return int(hash_longs([int(obj)])[0])
    if isinstance(obj, (float, np.floating)):
        bits = struct.unpack(">q", struct.pack(">d", float(obj)))[0] if obj == obj else 0x7FF8000000000000
        return int(hash_longs([bits])[0])
    if isinstance(obj, str):
        return int(hash_strings([obj])[0])
    raise TypeError("HashingTF does not support type %s of input data." % type(obj).__name__)


def hash_strings_device(strings: Sequence[str], mod: int, mode: int, device) -> torch.Tensor:
    """Bucket index of every string computed on the GPU (mode 0: HashingTF, 1: FeatureHasher)."""
    units, offsets = encode_utf16(strings)
    u = torch.from_numpy(units.view(np.int16).copy()).to(device)
    o = torch.from_numpy(offsets).to(device)
    idx = torch.empty(len(strings), dtype=torch.int32, device=device)
    native.call("fmlx_murmur3_chars_device", native.ptr(u) if u.numel() else None, native.ptr(o), len(strings), mod,
                mode, None, native.ptr(idx), native.stream_ptr(device))
    return idx


def non_negative_mod(h: np.ndarray, mod: int) -> np.ndarray:
    r = np.fmod(h.astype(np.int64), mod)
    return np.where(r < 0, r + mod, r)


native.register_host_sigs({
    "fmlx_hash_prefixed_doubles": [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                   ctypes.c_int32],
    "fmlx_java_double_strings": [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p],
})


def hash_prefixed_doubles(prefix: str, vals: np.ndarray, nthreads: int = 0) -> np.ndarray:
    """murmur3_32(prefix + Double.toString(v)) for every value (native, multi-threaded)."""
    import os

    vals = np.ascontiguousarray(vals, dtype=np.float64)
    units = np.frombuffer(prefix.encode("utf-16-le"), dtype=np.uint16).copy()
    out = np.empty(vals.shape[0], dtype=np.int32)
    if vals.shape[0]:
        nt = nthreads or min(16, os.cpu_count() or 1)
        native.host().fmlx_hash_prefixed_doubles(units.ctypes.data if units.size else None, int(units.size),
                                                 vals.ctypes.data, int(vals.shape[0]), out.ctypes.data, int(nt))
    return out


native.register_kernel_sigs({
    "fmlx_hash_prefixed_doubles_dev": [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p],
})
_RYU_TABLES = {}


def ryu_tables(device):
    """The shortest-digits kernel's 128-bit multipliers, computed exactly with Python integers:
    ``inv[q] = ⌊2^(bitlen(5^q) − 1 + 125) / 5^q⌋ + 1`` (q < 342) and ``pow[i] = 5^i`` scaled to 125
    significant bits (i < 326), each as (low, high) 64-bit words."""
    key = str(device)
    if key not in _RYU_TABLES:
        mask = (1 << 64) - 1
        inv, pw = [], []
        for q in range(342):
            p = 5 ** q
            v = (1 << (p.bit_length() - 1 + 125)) // p + 1
            inv += [v & mask, v >> 64]
        for i in range(326):
            p = 5 ** i
            sh = p.bit_length() - 125
            v = p >> sh if sh >= 0 else p << -sh
            pw += [v & mask, v >> 64]

        def dev(words):
            return torch.from_numpy(np.array(words, dtype=np.uint64).view(np.int64)).to(device)

        _RYU_TABLES[key] = (dev(inv), dev(pw))
    return _RYU_TABLES[key]


def hash_prefixed_doubles_device(prefix: str, vals: torch.Tensor) -> torch.Tensor:
    """murmur3_32(prefix + Double.toString(v)) for every value of a device tensor, computed on the
    device (``csrc/javastr.hip``) — the same bits as ``hash_prefixed_doubles``."""
    vals = vals.to(torch.float64).contiguous()
    dev = vals.device
    units = torch.from_numpy(np.frombuffer(prefix.encode("utf-16-le"), dtype=np.uint16).astype(np.int16)).to(dev)
    out = torch.empty(vals.shape[0], dtype=torch.int32, device=dev)
    inv, pw = ryu_tables(dev)
    if vals.shape[0]:
        native.call("fmlx_hash_prefixed_doubles_dev", native.ptr(units) if units.numel() else None, int(units.numel()),
                    native.ptr(vals), int(vals.shape[0]), native.ptr(inv), native.ptr(pw), native.ptr(out),
                    native.stream_ptr(dev))
    return out


def java_double_strings(vals) -> list:
    """``Double.toString`` of every value (native)."""
    vals = np.ascontiguousarray(vals, dtype=np.float64)
    n = vals.shape[0]
    chars = np.empty(max(n, 1) * 32, dtype=np.uint8)
    ends = np.empty(n, dtype=np.int64)
    if n:
        native.host().fmlx_java_double_strings(vals.ctypes.data, n, chars.ctypes.data, ends.ctypes.data)
    b = chars.tobytes()
    out, s = [], 0
    for e in ends.tolist():
        out.append(b[s:e].decode("ascii"))
        s = e
    return out
