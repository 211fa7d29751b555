"""MinHashLSH / MinHashLSHModel (reference ``LIB/feature/lsh/{LSH,LSHModel,MinHashLSH,
MinHashLSHModel,MinHashLSHModelData}.java``).

* fit: the input dimension (all vector sizes must agree) and ``java.util.Random(seed)``
  coefficients a_k = 1 + nextInt(P-1), b_k = nextInt(P-1) exactly like ``generateModelData``.
* transform: one ``minhash.hip`` launch over the CSR nonzero pattern → a [n, tables, funcs]
  fp64 tensor column (each row reads back as ``DenseVector[]``).
* approx_nearest_neighbors: bucket filter (any table whose signature equals the key's), device
  Jaccard distances from sorted-key membership, per-rank top-k then a global top-k; each rank
  returns its own rows of the global answer.
* approx_similarity_join: on one rank, a join on (table, signature) via ``unique(dim=0)`` group ids,
  deduplicated candidate pairs, Jaccard distance <= threshold; across ranks the reference's keyed
  join (``_keyed_similarity_join``: signature entries all-to-all'ed to their key owners, pairs to
  their A row's rank, B sets fetched on demand) — a broadcast of B only for non-numeric ids.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np
import torch

from ... import config
from ...api.stage import Estimator
from ...common.param import HasInputCol, HasOutputCol, HasSeed
from ...io import read_write as rw
from ...io import serialization as ser
from ...linalg.vectors import Vector
from ...ops import lsh as lsh_ops
from ...param.param import IntParam, ParamValidators
from ...parallel import comm
from ...table import SparseColumn, Table
from ...utils.java import JavaRandom
from ..base import ModelWithData
from ..linear import rw_update
from .common import get_world_distributed, vector_input

HASH_PRIME = lsh_ops.HASH_PRIME


class LSHModelParams(HasInputCol, HasOutputCol):
    pass


class LSHParams(LSHModelParams):
    NUM_HASH_TABLES = IntParam("numHashTables", "Number of hash tables.", 1, ParamValidators.gt_eq(1))
    NUM_HASH_FUNCTIONS_PER_TABLE = IntParam("numHashFunctionsPerTable", "Number of hash functions per table.", 1,
                                            ParamValidators.gt_eq(1))


def generate_model_data(num_tables: int, num_funcs: int, dim: int, seed: int):
    if dim > HASH_PRIME:
        raise ValueError("The input vector dimension %d exceeds the threshold %d." % (dim, HASH_PRIME))
    rnd = JavaRandom(seed)
    a, b = [], []
    for _ in range(num_tables * num_funcs):
        a.append(1 + rnd.next_int(HASH_PRIME - 1))
        b.append(rnd.next_int(HASH_PRIME - 1))
    return (num_tables, num_funcs, a, b)


def _sets(X) -> SparseColumn:
    return lsh_ops.to_csr_sets(X)


def _row_keys(sets: SparseColumn) -> Tuple[torch.Tensor, torch.Tensor]:
    """(row id per nnz, sorted key row*d + col) for membership tests."""
    dev = sets.values.device
    rows = torch.repeat_interleave(torch.arange(len(sets), device=dev), (sets.indptr[1:] - sets.indptr[:-1]).to(dev))
    return rows, rows * sets.size + sets.indices.to(dev).long()


def _pair_jaccard(sa: SparseColumn, sb: SparseColumn, ia: torch.Tensor, ib: torch.Tensor) -> torch.Tensor:
    """Jaccard distance of set pairs (sa[ia[p]], sb[ib[p]]), vectorised over all nnz of the A side."""
    dev = ia.device
    if ia.numel() == 0:
        return torch.zeros(0, dtype=torch.float64, device=dev)
    a_ptr, b_ptr = sa.indptr.to(dev), sb.indptr.to(dev)
    la = (a_ptr[ia + 1] - a_ptr[ia])
    lb = (b_ptr[ib + 1] - b_ptr[ib])
    # expand every pair by its A-side nnz, look the column up in B's row-keyed sorted index
    pid = torch.repeat_interleave(torch.arange(ia.numel(), device=dev), la)
    off = torch.arange(pid.numel(), device=dev) - torch.repeat_interleave(torch.cumsum(la, 0) - la, la)
    cols = sa.indices.to(dev).long()[a_ptr[ia][pid] + off]
    d = max(sa.size, sb.size)
    _, bkeys = _row_keys(SparseColumn(sb.indptr, sb.indices, sb.values, d))
    bkeys_sorted, _ = torch.sort(bkeys)
    q = ib[pid] * d + cols
    pos = torch.clamp(torch.searchsorted(bkeys_sorted, q), max=max(bkeys_sorted.numel() - 1, 0))
    hit = (bkeys_sorted[pos] == q) if bkeys_sorted.numel() else torch.zeros_like(q, dtype=torch.bool)
    inter = torch.zeros(ia.numel(), dtype=torch.float64, device=dev).index_add_(0, pid, hit.to(torch.float64))
    union = (la + lb).to(torch.float64) - inter
    if bool((union <= 0).any()):
        raise ValueError("The union of two input sets must have at least 1 elements")
    return 1.0 - inter / union


@rw.register_stage
class MinHashLSHModel(ModelWithData, LSHModelParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.lsh.MinHashLSHModel"
    MODEL_DATA_COLUMNS = ("numHashTables", "numHashFunctionsPerTable", "randCoefficientA", "randCoefficientB")

    @staticmethod
    def encode_record(out, row):
        out.write_int(int(row[0]))
        out.write_int(int(row[1]))
        ser.write_int_array(out, np.asarray(row[2], dtype=np.int32))
        ser.write_int_array(out, np.asarray(row[3], dtype=np.int32))

    @staticmethod
    def decode_record(inp):
        return (inp.read_int(), inp.read_int(), [int(x) for x in ser.read_int_array(inp)],
                [int(x) for x in ser.read_int_array(inp)])

    @classmethod
    def make_model_data_table(cls, rows):
        return Table({"numHashTables": torch.tensor([int(r[0]) for r in rows], dtype=torch.int64),
                      "numHashFunctionsPerTable": torch.tensor([int(r[1]) for r in rows], dtype=torch.int64),
                      "randCoefficientA": [list(r[2]) for r in rows], "randCoefficientB": [list(r[3]) for r in rows]},
                     num_rows=len(rows))

    def _params(self):
        nt, nf, a, b = self.model_data_rows()[0]
        return int(nt), int(nf), list(a), list(b)

    def hash_function(self, X) -> torch.Tensor:
        """Signatures [n, tables, funcs] (fp64) of a dense tensor or SparseColumn."""
        nt, nf, a, b = self._params()
        return lsh_ops.minhash(X, a, b).reshape(-1, nt, nf)

    def _hashes_of(self, t: Table) -> torch.Tensor:
        oc = self.get(self.OUTPUT_COL)
        if t.has_column(oc) and isinstance(t.column(oc), torch.Tensor) and t.column(oc).dim() == 3:
            return t.column(oc)
        return self.hash_function(vector_input(t, self.get(self.INPUT_COL)))

    def transform(self, *inputs):
        t = inputs[0]
        return [t.with_column(self.get(self.OUTPUT_COL), self._hashes_of(t))]

    # ------------------------------------------------------------------------ similarity search
    def approx_nearest_neighbors(self, dataset: Table, key: Vector, k: int, dist_col: str = "distCol") -> Table:
        dev = config.compute_device()
        H = self._hashes_of(dataset).to(dev)
        sets = _sets(vector_input(dataset, self.get(self.INPUT_COL))).to(dev)
        ks = key.to_sparse() if hasattr(key, "to_sparse") else key
        kset = SparseColumn(torch.tensor([0, len(ks.indices)], dtype=torch.int64, device=dev),
                            torch.as_tensor(np.asarray(ks.indices, dtype=np.int32), device=dev),
                            torch.ones(len(ks.indices), dtype=torch.float64, device=dev), ks.size())
        kh = self.hash_function(kset.to(dev))[0]
        cand = (H == kh[None]).all(dim=2).any(dim=1)
        idx = torch.nonzero(cand, as_tuple=True)[0]
        dist = _pair_jaccard(kset, sets, torch.zeros_like(idx), idx)
        order = torch.argsort(dist, stable=True)[:k]
        loc_idx, loc_dist = idx[order], dist[order]
        if get_world_distributed():
            from ...parallel.context import get_context

            me = get_context().rank
            # global top-k over the ranks' local top-k: (distance, rank, row) tensors gathered,
            # ordered by distance then rank then row
            mine = torch.stack([loc_dist.to(torch.float64), torch.full_like(loc_dist, float(me), dtype=torch.float64),
                                loc_idx.to(torch.float64)], 1)
            allc = torch.cat(comm.all_gather_tensor(mine)).cpu()
            o = np.lexsort((allc[:, 2].numpy(), allc[:, 1].numpy(), allc[:, 0].numpy()))[:k]
            top = allc[torch.as_tensor(o, dtype=torch.int64)]
            sel = top[top[:, 1] == me]
            chosen = list(zip(sel[:, 2].to(torch.int64).tolist(), sel[:, 0].tolist()))
        else:
            chosen = list(zip(loc_idx.cpu().tolist(), loc_dist.cpu().tolist()))
        rows = [i for i, _ in chosen]
        out = dataset.with_column(self.get(self.OUTPUT_COL), H).take(rows)
        return out.with_column(dist_col, torch.tensor([d for _, d in chosen], dtype=torch.float64))

    approxNearestNeighbors = approx_nearest_neighbors

    def approx_similarity_join(self, dataset_a: Table, dataset_b: Table, threshold: float, id_col: str,
                               dist_col: str = "distCol") -> Table:
        dev = config.compute_device()
        ha = self._hashes_of(dataset_a).to(dev)
        hb = self._hashes_of(dataset_b).to(dev)
        sa = _sets(vector_input(dataset_a, self.get(self.INPUT_COL))).to(dev)
        sb = _sets(vector_input(dataset_b, self.get(self.INPUT_COL))).to(dev)
        ids_b = dataset_b.get_list(id_col)
        if get_world_distributed():
            ids_a = dataset_a.get_list(id_col)
            # every rank must take the same branch (they issue different collectives): agree on
            # it; an empty partition votes "numeric" 
            mine = 1.0 if _numeric_ids(ids_a) and _numeric_ids(ids_b) else 0.0
            if comm.all_reduce_scalar(mine, "min") > 0.5:
                return _keyed_similarity_join(ha, hb, sa, sb, ids_a, ids_b, threshold, dist_col)
            # non-numeric ids: broadcast join (every rank sees all of B)
            parts = comm.all_gather_object((hb.cpu(), sb.to("cpu"), ids_b))
            hb = torch.cat([p[0] for p in parts]).to(dev)
            sb = SparseColumn.concat([p[1] for p in parts]).to(dev)
            ids_b = [x for p in parts for x in p[2]]
        na, nb = ha.shape[0], hb.shape[0]
        pairs = []
        for tb in range(ha.shape[1]):
            allk = torch.cat([ha[:, tb], hb[:, tb]])
            _, g = torch.unique(allk, dim=0, return_inverse=True)
            ga, gb = g[:na], g[na:]
            ob = torch.argsort(gb, stable=True)
            gbs = gb[ob]
            lo = torch.searchsorted(gbs, ga)
            hi = torch.searchsorted(gbs, ga, right=True)
            cnt = hi - lo
            ia = torch.repeat_interleave(torch.arange(na, device=dev), cnt)
            off = torch.arange(ia.numel(), device=dev) - torch.repeat_interleave(torch.cumsum(cnt, 0) - cnt, cnt)
            ib = ob[lo[ia] + off]
            pairs.append(ia * nb + ib)
        keys = torch.unique(torch.cat(pairs)) if pairs else torch.zeros(0, dtype=torch.int64, device=dev)
        ia, ib = torch.div(keys, nb, rounding_mode="floor"), keys % nb if nb else keys
        dist = _pair_jaccard(sa, sb, ia, ib)
        keep = dist <= threshold
        ia, ib, dist = ia[keep].cpu().tolist(), ib[keep].cpu().tolist(), dist[keep].cpu()
        ids_a = dataset_a.get_list(id_col)
        return Table({"datasetA.id": [ids_a[i] for i in ia], "datasetB.id": [ids_b[j] for j in ib], dist_col: dist},
                     num_rows=len(ia))

    approxSimilarityJoin = approx_similarity_join


def _numeric_ids(ids) -> bool:
    return all(isinstance(v, (int, float, np.integer, np.floating)) and not isinstance(v, bool) for v in ids)


def _gather_rows(sets: SparseColumn, rows: torch.Tensor):
    """Row lengths and concatenated column indices of ``sets[rows]``."""
    ptr = sets.indptr.to(rows.device)
    ln = ptr[rows + 1] - ptr[rows]
    pid = torch.repeat_interleave(torch.arange(rows.numel(), device=rows.device), ln)
    off = torch.arange(pid.numel(), device=rows.device) - torch.repeat_interleave(torch.cumsum(ln, 0) - ln, ln)
    return ln, sets.indices.to(rows.device).long()[ptr[rows][pid] + off]


def _keyed_similarity_join(ha, hb, sa: SparseColumn, sb: SparseColumn, ids_a, ids_b, threshold: float,
                           dist_col: str) -> Table:
    """``approxSimilarityJoin`` across ranks as the reference's keyed join (LSHModel.java:201-258:
    both sides keyed by (table, signature), co-grouped, candidate pairs deduplicated, distances):

    1. every (table, signature) entry of A and B goes to the owner of its key (one all-to-all);
       each owner pairs the A and B entries of every key it owns;
    2. candidate pairs go to the rank holding their A row (all-to-all) and are deduplicated there;
    3. the B sets (and ids) those pairs need are fetched from B's ranks (request / response
       all-to-alls) and the Jaccard distances computed next to the A rows.
    Each rank returns the pairs of its own A rows."""
    from ...parallel import datastream as ds
    from ...parallel.context import get_context

    ctx = get_context()
    P, me = ctx.world_size, ctx.rank
    dev = ha.device

    def entries(h, side):
        n, T, F = h.shape
        hk = ds.float_keys(h).reshape(n, T, F)
        tb = torch.arange(T, device=dev, dtype=torch.int64)[None, :, None].expand(n, T, 1)
        keys = torch.cat([tb, hk], 2).reshape(n * T, F + 1)
        row = torch.arange(n, device=dev, dtype=torch.int64)[:, None].expand(n, T).reshape(-1)
        meta = torch.stack([torch.full_like(row, side), torch.full_like(row, me), row], 1)
        return keys, meta

    ka, ma = entries(ha, 0)
    kb, mb = entries(hb, 1)
    keys, meta = torch.cat([ka, kb]), torch.cat([ma, mb])
    own = ds.key_owner(keys, P)
    o = torch.argsort(own, stable=True)
    cnt = torch.bincount(own, minlength=P).tolist()
    keys = torch.cat(comm.all_to_all_v(list(torch.split(keys[o], cnt))))
    meta = torch.cat(comm.all_to_all_v(list(torch.split(meta[o], cnt))))
    # 1. co-group the owned keys: A entries × B entries of every group
    if keys.shape[0]:
        _, g = torch.unique(keys, dim=0, return_inverse=True)
    else:
        g = torch.zeros(0, dtype=torch.int64, device=dev)
    isa = meta[:, 0] == 0
    ga, gb = g[isa], g[~isa]
    ea, eb = meta[isa], meta[~isa]
    ob = torch.argsort(gb, stable=True)
    gbs = gb[ob]
    lo = torch.searchsorted(gbs, ga)
    hi = torch.searchsorted(gbs, ga, right=True)
    c = hi - lo
    ia = torch.repeat_interleave(torch.arange(ga.numel(), device=dev), c)
    off = torch.arange(ia.numel(), device=dev) - torch.repeat_interleave(torch.cumsum(c, 0) - c, c)
    jb = ob[lo[ia] + off]
    pairs = torch.stack([ea[ia, 1], ea[ia, 2], eb[jb, 1], eb[jb, 2]], 1)  # a_rank, a_row, b_rank, b_row
    # 2. to the A row's rank, deduplicated (a pair can share several tables)
    own = pairs[:, 0]
    o = torch.argsort(own, stable=True)
    cnt = torch.bincount(own, minlength=P).tolist()
    pairs = torch.cat(comm.all_to_all_v(list(torch.split(pairs[o], cnt))))
    pairs = torch.unique(pairs[:, 1:], dim=0) if pairs.shape[0] else pairs[:, 1:]
    arow, brank, brow = pairs[:, 0], pairs[:, 1], pairs[:, 2]
    # 3. the B rows these pairs need: request from their ranks, answer with sets and ids
    need = torch.unique(torch.stack([brank, brow], 1), dim=0) if brow.numel() else torch.zeros(
        (0, 2), dtype=torch.int64, device=dev)
    cnt = torch.bincount(need[:, 0], minlength=P).tolist()
    req = comm.all_to_all_v(list(torch.split(need[:, 1].contiguous(), cnt)))  # rows others need from me
    # integer ids (Java longs, possibly above 2^53) travel as int64 when every rank's are integers
    ints = comm.all_reduce_scalar(1.0 if all(isinstance(v, (int, np.integer)) for v in ids_b) else 0.0, "min") > 0.5
    idb = torch.tensor([int(v) for v in ids_b] if ints else [float(v) for v in ids_b],
                       dtype=torch.int64 if ints else torch.float64, device=dev)
    sb_d = sb.to(dev)
    lens, cols, idv = [], [], []
    for r in range(P):
        ln, cl = _gather_rows(sb_d, req[r].to(dev))
        lens.append(ln)
        cols.append(cl)
        idv.append(idb[req[r].to(dev)])
    got_len = torch.cat(comm.all_to_all_v(lens))
    got_cols = torch.cat(comm.all_to_all_v(cols))
    got_ids = torch.cat(comm.all_to_all_v(idv))
    ptr = torch.zeros(got_len.numel() + 1, dtype=torch.int64, device=dev)
    ptr[1:] = torch.cumsum(got_len.to(dev), 0)
    fetched = SparseColumn(ptr, got_cols.to(dev).to(torch.int32), torch.ones(got_cols.numel(), dtype=torch.float64,
                                                                            device=dev), sb.size)
    # fetched row i = need[i] (need is sorted by (rank, row), the answers arrive in the same order)
    nkey = need[:, 0] * (1 << 40) + need[:, 1]
    fi = torch.searchsorted(nkey, brank * (1 << 40) + brow)
    dist = _pair_jaccard(sa.to(dev), fetched, arow, fi)
    keep = dist <= threshold
    arow, fi, dist = arow[keep].cpu().tolist(), fi[keep], dist[keep].cpu()
    bid = got_ids.to(dev)[fi].cpu().tolist()
    ida = [ids_a[i] for i in arow]
    return Table({"datasetA.id": ida, "datasetB.id": bid, dist_col: dist}, num_rows=len(ida))


@rw.register_stage
class MinHashLSH(Estimator, LSHParams, HasSeed):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.lsh.MinHashLSH"

    def fit(self, *inputs):
        t = inputs[0]
        col = t.column(self.get(self.INPUT_COL))
        if isinstance(col, torch.Tensor):
            sizes = {int(col.shape[1])} if t.num_rows else set()
        elif isinstance(col, SparseColumn):
            sizes = {col.size} if t.num_rows else set()
        else:
            sizes = {v.size() for v in col}
        if get_world_distributed():
            # (min, max) vector size over the ranks; −1 / large sentinels for an empty partition
            lo = comm.all_reduce_scalar(float(min(sizes)) if sizes else float(1 << 40), "min")
            hi = comm.all_reduce_scalar(float(max(sizes)) if sizes else -1.0, "max")
            sizes = set() if hi < 0 else {int(lo), int(hi)}
        if len(sizes) > 1:
            s = sorted(sizes)
            raise RuntimeError("Vector sizes are not the same: %d %d." % (s[0], s[1]))
        if not sizes:
            raise RuntimeError("The training set is empty.")
        md = generate_model_data(self.get(self.NUM_HASH_TABLES), self.get(self.NUM_HASH_FUNCTIONS_PER_TABLE),
                                 sizes.pop(), self.get_seed())
        m = MinHashLSHModel().set_model_data(MinHashLSHModel.make_model_data_table([md]))
        rw_update(m, self)
        return m
