"""SPMD equivalents of ``DataStreamUtils`` (reference ``CORE/common/datastream/DataStreamUtils.java``).

In the reference each helper is a small dataflow sub-graph (partial operator per subtask, then
a parallelism-1 operator, network shuffles in between). Here each is a local computation on the
rank's partition plus at most one collective:

==========================  ============================================================
reference                   here
==========================  ============================================================
``allReduceSum`` (:102)     ``all_reduce_sum`` — RCCL all-reduce of a device tensor
``mapPartition`` (:115)     ``map_partition`` — apply fn to the whole local partition
``reduce`` (:132-143)       ``reduce`` — local fold, all-gather, fold in rank order
keyed ``reduce`` (:155)     ``reduce_by_key`` — per-key local folds, all-gather, merge (host
                              objects); ``reduce_by_key_tensor`` — device keys/values: local
                              segment reduce, hash-partitioned all-to-all, owner-side merge;
                              ``reduce_strings_by_key`` — string keys (code-unit tensors)
``aggregate`` (:182-199)    ``aggregate`` — local accumulator, all-gather, merge in rank order
``sample`` (:212-227)       ``sample`` — reservoir per rank (java.util.Random), gather, again
``generateBatchData``       ``generate_batch_data`` — deterministic per-rank split of a global
  (:571-628)                  mini-batch from the rank's stream shard
``windowAllAndProcess``     ``window_all_and_process`` — cut the partition into windows and
  (:262-303)                  process each window on rank 0's gathered data
==========================  ============================================================
"""
from __future__ import annotations

from typing import Any, Callable, Iterable, Iterator, List, Optional, Sequence

import numpy as np
import torch

from ..common.window import CountTumblingWindows, EndOfStreamWindows, GlobalWindows, Windows
from ..table import Table
from . import comm
from .context import get_context


def all_reduce_sum(t: torch.Tensor) -> torch.Tensor:
    """``DataStreamUtils.allReduceSum``: element-wise sum of one array per rank (equal lengths)."""
    comm.check_equal_across_ranks(int(t.numel()), "all-reduce array length")
    return comm.all_reduce_sum(t)


def map_partition(partition, fn: Callable):
    return fn(partition)


def reduce(value: Any, fn: Callable[[Any, Any], Any]):
    """Folds one value per rank with ``fn`` in rank order; every rank gets the result.
    ``value=None`` marks an empty partition."""
    vals = [v for v in comm.all_gather_object(value) if v is not None]
    if not vals:
        return None
    acc = vals[0]
    for v in vals[1:]:
        acc = fn(acc, v)
    return acc


def reduce_by_key(pairs: Sequence, fn: Callable[[Any, Any], Any]) -> dict:
    """Keyed ``DataStreamUtils.reduce`` (``DataStreamUtils.java:155``): folds the values of every
    key with ``fn``. Each rank folds its own (key, value) pairs, the partial maps are exchanged
    and merged in rank order; every rank gets the full result (the keyed shuffle of the
    reference becomes one all-gather of per-key partials)."""
    local: dict = {}
    for k, v in pairs:
        local[k] = fn(local[k], v) if k in local else v
    out: dict = {}
    for part in comm.all_gather_object(local):
        for k, v in part.items():
            out[k] = fn(out[k], v) if k in out else v
    return out


def _unique_rows(keys: torch.Tensor):
    """Sorted unique keys (rows, lexicographic, for [n, m] keys) and the inverse map."""
    if keys.dim() == 1:
        return torch.unique(keys, return_inverse=True)
    return torch.unique(keys, dim=0, return_inverse=True)


def _segment_reduce(keys: torch.Tensor, values: torch.Tensor, op: str):
    uk, inv = _unique_rows(keys)
    shape = (uk.shape[0],) + tuple(values.shape[1:])
    if op == "sum":
        out = torch.zeros(shape, dtype=values.dtype, device=values.device).index_add_(0, inv, values)
    elif op in ("min", "max"):
        idx = inv.view(-1, *([1] * (values.dim() - 1))).expand_as(values)
        out = torch.empty(shape, dtype=values.dtype, device=values.device).scatter_reduce_(
            0, idx, values, "amin" if op == "min" else "amax", include_self=False)
    else:
        raise ValueError("op must be sum, min or max")
    return uk, out


def key_owner(keys: torch.Tensor, world: int) -> torch.Tensor:
    """Owner rank of every key (``keyBy`` partitioning): a 64-bit mix of the key's columns mod
    ``world`` — the same on every rank and for every world size's own partitioning."""
    h = keys if keys.dim() == 1 else keys[:, 0]
    h = h.to(torch.int64)
    if keys.dim() == 2:
        for c in range(1, keys.shape[1]):
            h = h * 0x100000001B3 + keys[:, c].to(torch.int64)  # wraps in two's complement
    h = h ^ (h >> 29)
    h = h * 0x2545F4914F6CDD1D
    h = h ^ (h >> 32)
    return torch.remainder(h, world)


def reduce_by_key_tensor(keys: torch.Tensor, values: torch.Tensor, op: str = "sum", gather: bool = False):
    """Keyed ``DataStreamUtils.reduce`` (``DataStreamUtils.java:155``) for device data: integer
    ``keys`` ([n], or [n, m] multi-column keys compared as rows) and ``values`` [n, ...] stay on
    the device. Each rank folds its own rows per key (sort-unique + index_add / scatter_reduce),
    sends every partial to the key's owner rank (``key_owner`` — the keyBy shuffle) in ONE
    all-to-all, and the owner folds what it receives. Returns this rank's (sorted keys, reduced
    values) — every key lives on exactly one rank, like the reference's keyed reduce output;
    ``gather=True`` all-gathers the full result (sorted keys) instead.
    ``op`` is an associative, commutative reduction: sum, min or max."""
    if keys.dim() not in (1, 2) or values.shape[0] != keys.shape[0]:
        raise ValueError("keys [n] or [n, m] and values [n, ...] expected")
    keys = keys.to(torch.int64)
    uk, part = _segment_reduce(keys, values, op)
    ctx = get_context()
    if not ctx.is_distributed:
        return uk, part
    P = ctx.world_size
    owner = key_owner(uk, P)
    order = torch.argsort(owner, stable=True)
    uk, part, owner = uk[order], part[order], owner[order]
    counts = torch.bincount(owner, minlength=P).tolist()
    k_in = comm.all_to_all_v(list(torch.split(uk, counts)))
    v_in = comm.all_to_all_v(list(torch.split(part, counts)))
    mk, mv = _segment_reduce(torch.cat(k_in), torch.cat(v_in), op)
    if gather:
        ak = torch.cat(comm.all_gather_tensor(mk))
        av = torch.cat(comm.all_gather_tensor(mv))
        sk, inv = _unique_rows(ak)  # keys are unique across owners: a permutation
        out = torch.empty_like(av)
        out[inv] = av
        return sk, out
    return mk, mv


def float_keys(x: torch.Tensor) -> torch.Tensor:
    """int64 keys of float64 values: one key per distinct value.

    - every NaN maps to the one canonical pattern 0x7ff8000000000000, as ``Double.equals`` /
      ``doubleToLongBits`` treat all NaNs as one value (VectorIndexer.java:96-106's HashSet);
    - −0.0 is folded into +0.0. This deliberately differs from ``Double.equals``: the models
      that consume these keys look values up by float comparison (VectorIndexerModel's sorted
      category search, ChiSqTest's value order), where −0.0 == +0.0, so keeping two keys would
      give a category no input can ever hit. Parity with the reference on −0.0 is unpinned (no
      reference fixture holds −0.0)."""
    x = x.to(torch.float64).contiguous() + 0.0
    k = x.view(torch.int64)
    return torch.where(torch.isnan(x), torch.full_like(k, 0x7FF8000000000000), k)


def keys_to_float(k: torch.Tensor) -> torch.Tensor:
    return k.to(torch.int64).contiguous().view(torch.float64)


def global_distinct(keys: torch.Tensor):
    """Distinct keys over all ranks (sorted; rows for [n, m] keys) with their global counts, on
    every rank: one keyed reduce (all-to-all to the owners) + an all-gather of the owners'
    results."""
    ones = torch.ones(keys.shape[0], dtype=torch.float64, device=keys.device)
    return reduce_by_key_tensor(keys, ones, "sum", gather=True)


def _np_to_tensor(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a))


def reduce_strings_by_key(table, sums: np.ndarray, firsts: np.ndarray):
    """Keyed merge of per-rank string maps (StringIndexer / CountVectorizer vocabularies,
    ``StringIndexer.java:110-114`` keyBy + reduce): ``table`` (utils.strtable.StrTable) holds this
    rank's strings, ``sums`` [n, k] their counters (summed per string), ``firsts`` [n] their
    first-seen positions in the rank's data. Rows of one string are routed to the owner of its
    64-bit content hash in one all-to-all of the tables (code units as tensors), the owner
    merges equal strings (exact comparison: hash collisions stay apart), and the owners' results
    are all-gathered. Returns (StrTable, sums, order key) on every rank, ordered by the global
    first-seen key (rank, local first position) — the insertion order of the reference's merged
    map when partitions are merged in rank order."""
    from ..utils.strtable import StrTable

    sums = np.asarray(sums, dtype=np.float64).reshape(len(table), -1)
    firsts = np.asarray(firsts, dtype=np.int64)
    ctx = get_context()
    key = firsts + (np.int64(ctx.rank) << np.int64(40))

    def merge_local(tab, sm, ky):
        rep = tab.first_of_equal()
        if len(tab) and not np.array_equal(rep, np.arange(len(tab))):
            uniq, inv = np.unique(rep, return_inverse=True)
            s2 = np.zeros((uniq.shape[0], sm.shape[1]), dtype=np.float64)
            np.add.at(s2, inv, sm)
            k2 = np.full(uniq.shape[0], np.iinfo(np.int64).max, dtype=np.int64)
            np.minimum.at(k2, inv, ky)
            return tab.take(uniq), s2, k2
        return tab, sm, ky

    table, sums, key = merge_local(table, sums, key)
    if ctx.is_distributed:
        P = ctx.world_size
        owner = (table.hash64().view(np.uint64) % np.uint64(P)).astype(np.int64)
        order = np.argsort(owner, kind="stable")
        tab = table.take(order)
        sm, ky, ow = sums[order], key[order], owner[order]
        cnt = np.bincount(ow, minlength=P)
        bounds = np.concatenate([[0], np.cumsum(cnt)])
        ubounds = tab.offs[bounds]
        lens = np.diff(tab.offs)
        units = tab.units.astype(np.int32)
        u_in = comm.all_to_all_v([_np_to_tensor(units[ubounds[r]:ubounds[r + 1]]) for r in range(P)])
        l_in = comm.all_to_all_v([_np_to_tensor(lens[bounds[r]:bounds[r + 1]]) for r in range(P)])
        s_in = comm.all_to_all_v([_np_to_tensor(sm[bounds[r]:bounds[r + 1]]) for r in range(P)])
        k_in = comm.all_to_all_v([_np_to_tensor(ky[bounds[r]:bounds[r + 1]]) for r in range(P)])

        def table_of(u_parts, l_parts):
            u = np.concatenate([p.numpy() for p in u_parts]).astype(np.uint16) if u_parts else np.zeros(0, np.uint16)
            ln = np.concatenate([p.numpy() for p in l_parts]) if l_parts else np.zeros(0, np.int64)
            offs = np.zeros(ln.shape[0] + 1, dtype=np.int64)
            np.cumsum(ln, out=offs[1:])
            return StrTable(u, offs)

        mine = table_of(u_in, l_in)
        msum = np.concatenate([p.numpy().reshape(-1, sums.shape[1]) for p in s_in])
        mkey = np.concatenate([p.numpy() for p in k_in])
        mine, msum, mkey = merge_local(mine, msum, mkey)
        # every rank gets the whole merged map
        g_units = comm.all_gather_tensor(_np_to_tensor(mine.units.astype(np.int32)))
        g_lens = comm.all_gather_tensor(_np_to_tensor(np.diff(mine.offs)))
        g_sums = comm.all_gather_tensor(_np_to_tensor(msum))
        g_keys = comm.all_gather_tensor(_np_to_tensor(mkey))
        table = table_of(g_units, g_lens)
        sums = np.concatenate([p.numpy().reshape(-1, msum.shape[1]) for p in g_sums])
        key = np.concatenate([p.numpy() for p in g_keys])
    if key.shape[0] > 1 and not bool(np.all(key[1:] >= key[:-1])):
        order = np.argsort(key, kind="stable")
        table, sums, key = table.take(order), sums[order], key[order]
    return table, sums, key


def set_managed_memory_weight(stream, weight: int):
    """``DataStreamUtils.setManagedMemoryWeight`` (``:237-249``): in the reference it sizes the
    managed memory of the operator caching the stream. Partitions here are HBM-resident tensors
    (spilling, if any, is the data cache's job: ``parallel/datacache.py``), so it is a no-op that
    returns the stream."""
    if weight < 0:
        raise ValueError("managed memory weight must be non-negative")
    return stream


class AggregateFunction:
    """``org.apache.flink.api.common.functions.AggregateFunction`` shape."""

    def create_accumulator(self):
        raise NotImplementedError

    def add(self, value, acc):
        raise NotImplementedError

    def get_result(self, acc):
        return acc

    def merge(self, a, b):
        raise NotImplementedError


def aggregate(values: Iterable, fn: AggregateFunction, local_acc=None):
    """Local accumulation then merge of the per-rank accumulators in rank order."""
    if local_acc is None:
        local_acc = fn.create_accumulator()
        for v in values:
            local_acc = fn.add(v, local_acc)
    accs = comm.all_gather_object(local_acc)
    acc = accs[0]
    for a in accs[1:]:
        acc = fn.merge(acc, a)
    return fn.get_result(acc)


def sample(rows: Sequence, k: int, seed: int) -> list:
    """``DataStreamUtils.sample``: reservoir with ``java.util.Random(seed)`` per rank, then again
    over the rank-ordered union (``SamplingOperator``, DataStreamUtils.java:633-704)."""
    from ..models.kmeans import reservoir_sample_indices

    local = [rows[i] for i in reservoir_sample_indices(len(rows), k, seed)]
    union = [r for part in comm.all_gather_object(local) for r in part]
    return [union[i] for i in reservoir_sample_indices(len(union), k, seed)]


def generate_batch_data(stream: Iterable, global_batch_size: int) -> Iterator:
    """Yields this rank's share of each global mini-batch: ``globalBatch/P`` items, the remainder
    going to the low ranks (``DataStreamUtils.generateBatchData`` splits a countWindowAll batch
    the same way). A trailing partial batch is dropped, like the count window."""
    ctx = get_context()
    b = global_batch_size // ctx.world_size + (1 if global_batch_size % ctx.world_size > ctx.rank else 0)
    if isinstance(stream, Table):
        for s in range(0, stream.num_rows - b + 1, max(b, 1)):
            yield stream.slice(s, s + b)
        return
    buf = []
    for item in stream:
        if isinstance(item, Table):
            yield item
            continue
        buf.append(item)
        if len(buf) == b:
            yield buf
            buf = []


def window_all_and_process(table: Table, windows: Windows, fn: Callable[[Table], Table],
                           time_col: Optional[str] = None) -> Table:
    """Applies ``fn`` to every window of the (globally gathered) input; the result is produced on
    rank 0 (parallelism-1 semantics of ``windowAll``) and is empty on other ranks."""
    ctx = get_context()
    if time_col is None:
        time_col = getattr(table, "time_col", None)
    parts = comm.all_gather_object(table.to("cpu")) if ctx.is_distributed else [table]
    full = Table.concat(parts) if len(parts) > 1 else parts[0]
    if ctx.rank != 0:
        return None
    outs = []
    if isinstance(windows, (GlobalWindows, EndOfStreamWindows)) or windows is None:
        outs.append(fn(full))
    elif isinstance(windows, CountTumblingWindows):
        n = windows.size
        for s in range(0, full.num_rows - n + 1, n):
            outs.append(fn(full.slice(s, s + n)))
    else:
        # time windows: tumbling by a timestamp column (ms), sessions by gaps
        if time_col is None:
            outs.append(fn(full))
        else:
            ts = np.asarray(full.scalars(time_col, dtype=torch.float64).cpu().numpy())
            order = np.argsort(ts, kind="stable")
            full = full.take(torch.as_tensor(order))
            ts = ts[order]
            if hasattr(windows, "size"):
                keys = np.floor(ts / windows.size)
                bounds = np.nonzero(np.diff(keys))[0] + 1
            else:
                bounds = np.nonzero(np.diff(ts) >= windows.gap)[0] + 1
            starts = np.concatenate([[0], bounds])
            ends = np.concatenate([bounds, [len(ts)]])
            for s, e in zip(starts, ends):
                outs.append(fn(full.slice(int(s), int(e))))
    outs = [o for o in outs if o is not None]
    return Table.concat(outs) if outs else None
