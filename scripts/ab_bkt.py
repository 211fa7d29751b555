"""A/B timing of the single-visit sparse bucket round (glm_sparse.hip glm_bkt_*) on the
north-star SVC shape (1M columns, 64 nnz per row, 100k-row batches): ms per round of a warmed
trainer; argv[1]: comma-separated variants ``CHUNK[:SLICE_COLS[:RB_HEADROOM]]`` (the backward's work-item
size; the number of column slices ≈ d / SLICE_COLS, rounded to a power-of-two slice width; the
forward's row-block headroom for rows of unequal length); ``--varlen``: row lengths uniform in
[nnz/2, 3·nnz/2) instead of all nnz."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer
    from flink_ml_amd.ops import glm as gk
    from flink_ml_amd.table import SparseColumn

    dev = torch.device("cuda:0")
    n, dim, nnz = 1_000_000, 1_000_000, 64
    g = torch.Generator(device=dev).manual_seed(7)
    if "--varlen" in sys.argv:
        # row lengths uniform in [nnz/2, 3·nnz/2): the forward blocks' entry counts vary
        lens = torch.randint(nnz // 2, nnz + nnz // 2, (n,), generator=g, device=dev)
        indptr = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        indptr[1:] = torch.cumsum(lens, 0)
        idx = torch.randint(0, dim, (int(indptr[-1]),), generator=g, device=dev, dtype=torch.int32)
        vals = torch.rand((int(indptr[-1]),), generator=g, device=dev, dtype=torch.float32)
    else:
        idx = torch.sort(torch.randint(0, dim, (n, nnz), generator=g, device=dev, dtype=torch.int32), dim=1).values
        indptr = torch.arange(0, (n + 1) * nnz, nnz, dtype=torch.int64, device=dev)
        vals = torch.rand((n * nnz,), generator=g, device=dev, dtype=torch.float32)
    X = SparseColumn(indptr, idx.reshape(-1), vals, dim)
    y = torch.randint(0, 2, (n,), generator=g, device=dev).to(torch.float32)
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    variants = [[float(x) for x in v.split(":")] for v in (args[0].split(",") if args else [str(gk.BucketRound.CHUNK)])]
    gk.TILE_MIN_VISITS = 10 ** 9
    for v in variants:
        gk.BucketRound.CHUNK = int(v[0])
        gk.BucketRound.SLICE_COLS = int(v[1]) if len(v) > 1 else 256
        gk.BucketRound.RB_HEADROOM = v[2] if len(v) > 2 else 1.1
        tr = DeviceGlmTrainer(SGD(max_iter=10 ** 8, learning_rate=0.1, global_batch_size=100_000, tol=0.0),
                              np.zeros(dim), X, y, None, "hinge")
        assert tr.bkt is not None
        tr.run_rounds(2 * tr.rounds_per_graph)
        torch.cuda.synchronize()
        R = 200
        t0 = time.perf_counter()
        tr.run_rounds(R)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / R
        print(json.dumps({"chunk": int(v[0]), "slice_cols": gk.BucketRound.SLICE_COLS,
                          "rb_headroom": gk.BucketRound.RB_HEADROOM, "varlen": "--varlen" in sys.argv, "ms_per_round": round(ms, 4), "csb": tr.bkt.csb, "nb": tr.bkt.nb, "rb": tr.bkt.rb,
                          "G": tr.bkt.G, "bwd_blocks": tr.bkt.bwd_blocks}), flush=True)




if __name__ == "__main__":
    main()
