#!/usr/bin/env python3
"""Diagnostics of the fused round's dynamic row schedule (csrc/glm.hip DynLds): per-row visit
counts of one round, summarised by chunk class (static / per-XCD counter range), with and without
a vmcnt(0) before claim results are read."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer  # noqa: E402
from flink_ml_amd.ops import glm as gk, native  # noqa: E402


def main():
    n, d = 157_003, 520
    g = torch.Generator(device="cpu").manual_seed(9)
    X = torch.rand((n, d), generator=g).to(torch.bfloat16).cuda()
    y = torch.randint(0, 2, (n,), generator=g).to(torch.float32).cuda()
    lib = native.kernels()
    for sync in (0, 1):
        for B in (157_003, 100_000, 31_337):
            for ch in (16,):
                gk.set_dyn(True, ch)
                tr = DeviceGlmTrainer(SGD(max_iter=100, learning_rate=0.1, global_batch_size=B, tol=0.0), np.zeros(d),
                                      X, y, None, "logistic", use_graph=False)
                dbg = torch.zeros(B, dtype=torch.int32, device="cuda")
                P = -(-n // B)
                bad_total, chunks = 0, []
                for e in range(6):
                    dbg.zero_()
                    lib.fmlx_glm_set_dyn_debug(sync, native.ptr(dbg))
                    tr._launch_round(1)
                    torch.cuda.synchronize()
                    lib.fmlx_glm_set_dyn_debug(0, None)
                    nb_rows = min(B, n - (e % P) * B)
                    c = dbg.cpu().numpy()
                    want = np.zeros(B, dtype=np.int32)
                    want[:nb_rows] = 1
                    bad = np.nonzero(c != want)[0]
                    bad_total += len(bad)
                    chunks += sorted(set((bad // ch).tolist()))
                nb = tr.nparts
                C = -(-B // ch)
                S0 = 4 * nb
                cls = {"static": 0, "dynamic": 0}
                heads = {}
                Dn = max(C - S0, 0)
                for k in chunks:
                    if k < S0:
                        cls["static"] += 1
                    else:
                        cls["dynamic"] += 1
                        h = max(hh for hh in range(8) if S0 + (Dn * hh) // 8 <= k)
                        heads[h] = heads.get(h, 0) + 1
                bad = np.zeros(bad_total)
                print(json.dumps({"sync": sync, "B": B, "ch": ch, "blocks": nb, "chunks": C, "rows_bad_6_rounds": int(len(bad)), "bad_chunks": len(chunks),
                                  "classes": cls, "heads": heads, "first_bad_chunks": chunks[:12],
                                  "head_ranges": [S0 + (Dn * hh) // 8 for hh in range(9)]}), flush=True)


if __name__ == "__main__":
    main()
