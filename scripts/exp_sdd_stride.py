#!/usr/bin/env python3
"""Config-4 SDD (x . w1 at the expert blocks, 4-wave grouped NN) with the
leading dimensions padded off powers of two: K = 4096 vs 4224 (x rows 8 KiB
vs 8.25 KiB apart) and N = 114688 vs 114816 (w1 rows 224 KiB vs 224.25 KiB
apart), same topology; us per launch and per k-block. Tests whether the
per-block time depends on the row strides (L2 set / channel conflicts)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import sputnik_amd as sp  # noqa: E402
from sputnik_amd import matrix_utils as mu  # noqa: E402


def main():
    E, T, FF = 8, 8192, 14336
    off, idx = mu.expert_block_diagonal(E, T // E // 128, FF // 128)
    nb = int(off[-1])
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    rnd = lambda *s: (torch.rand(*s, generator=g, device="cuda") * 2 - 1).to(torch.bfloat16)
    hv = torch.empty(nb, 128, 128, dtype=torch.bfloat16, device="cuda")
    fns = {}
    for tb in (False, True):
        for K in (4096, 4224):
            for N in (E * FF, E * FF + 128):
                x = rnd(T, K)
                w1 = rnd(N, K) if tb else rnd(K, N)
                Hm = sp.BlockMatrix(T, N, 128, nb * 16384, hv, torch.from_numpy(off).cuda(),
                                    torch.from_numpy(idx.astype(np.int16)).cuda())
                sp.AllocateRowIndicesBuffer(Hm)
                sp.RowIndices(Hm, Hm.row_indices)
                X = sp.Matrix(T, K, x)
                W = sp.Matrix(N, K, w1) if tb else sp.Matrix(K, N, w1)
                assert sp.sdd_kernel(X, False, W, tb, Hm) == 3
                fns[f"{'NT' if tb else 'NN'}_K{K}_N{N}"] = (
                    lambda X=X, W=W, Hm=Hm, tb=tb, keep=(x, w1): sp.Matmul(X, False, W, tb, Hm), K)
            del x, w1
    res = {k: [] for k in fns}
    for _ in range(7):
        for k, (f, K) in fns.items():
            for _ in range(2):
                f()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                f()
            e.record()
            torch.cuda.synchronize()
            res[k].append(s.elapsed_time(e) * 200.0)
    out = {k: {"us": round(sorted(v)[3], 1),
               "us_per_kblock_round": round(sorted(v)[3] / 7 / (fns[k][1] // 128), 3)}
           for k, v in res.items()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
