"""Per-batch column-major copies of a CSR partition (ops/glm.py BatchCsc, the sparse trainer's
atomic-free backward; reference SGD.java:263-268 visits batch e mod P in round e): the host
construction against a naive per-batch transpose, lazy runs of batches, and the storage sized
for a short fit growing to the whole partition."""
import torch

from flink_ml_amd.ops import glm as gk


def _naive(indptr, idx, vals, n, d, B, b):
    r0, r1 = b * B, min((b + 1) * B, n)
    ent = []
    for r in range(r0, r1):
        for j in range(int(indptr[r]), int(indptr[r + 1])):
            ent.append((int(idx[j]), r - r0, float(vals[j])))
    ent.sort(key=lambda t: (t[0], t[1]))  # by column, rows ascending
    colptr = [0] * (d + 1)
    for c, _, _ in ent:
        colptr[c + 1] += 1
    for c in range(d):
        colptr[c + 1] += colptr[c]
    return colptr, [t[1] for t in ent], [t[2] for t in ent]


def test_host_transpose_matches_naive_with_growth(monkeypatch):
    monkeypatch.setattr(gk, "CSC_RUN_MAX", 3)
    g = torch.Generator().manual_seed(3)
    n, d, B = 1_037, 57, 100
    lens = torch.randint(0, 9, (n,), generator=g)
    lens[200:300] = 0  # batch 2 is empty
    indptr = torch.zeros(n + 1, dtype=torch.int64)
    indptr[1:] = torch.cumsum(lens, 0)
    idx = torch.cat([torch.sort(torch.randperm(d, generator=g)[:int(k)]).values for k in lens]).to(torch.int32)
    vals = torch.rand(int(indptr[-1]), generator=g, dtype=torch.float64)
    csc = gk.BatchCsc.alloc(indptr, idx, vals, n, d, B, max_rounds=4)
    assert csc.cap == 0 and csc.P == 11
    csc.ensure_rounds(0, 4)
    assert csc.cap == 4 and csc.version == 0 and csc.erow.numel() == int(indptr[400])
    csc.ensure_rounds(9, 4)  # wraps: batches 9, 10, 0, 1 → the whole partition
    assert csc.cap == csc.P and csc.version == 1
    csc.ensure(range(csc.P))
    for b in range(csc.P):
        cp, er, ev = _naive(indptr, idx, vals, n, d, B, b)
        j0, j1 = int(indptr[b * B]), int(indptr[min((b + 1) * B, n)])
        assert csc.colptr[b].tolist() == cp, b
        assert csc.erow[j0:j1].tolist() == er, b
        assert csc.evals[j0:j1].tolist() == ev, b
