#!/usr/bin/env python3
"""SDD 16384^3 (dense or --density) in every transpose with the operands'
row strides padded off 32 KiB: K and / or N = 16384 vs 16512 (the extra
128 columns / k-rows unused by the topology -- K padding adds one k-block,
so times are also reported per k-block). Same process, interleaved rounds,
median. Measures what the power-of-two strides cost the 4-wave grouped SDD."""
import argparse
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--density", type=float, default=1.0)
    ap.add_argument("--trans", default="NN,NT,TT,TN")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=4)
    a = ap.parse_args()
    M = 16384
    nbr = M // 128
    nb = int(round(nbr * nbr * a.density))
    off, idx = mu.random_topology(nbr, nbr, nb, np.random.default_rng(3))
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    rnd = lambda *s: (torch.rand(*s, generator=g, device="cuda") * 2 - 1).half()  # noqa: E731
    cv = torch.empty(nb * 16384, dtype=torch.half, device="cuda")
    fns = {}
    for tr in a.trans.split(","):
        ta, tb = tr[0] == "T", tr[1] == "T"
        for K in (16384, 16512):
            for N in (16384, 16512):
                x = rnd(*((K, M) if ta else (M, K)))
                w = rnd(*((N, K) if tb else (K, N)))
                C = sp.BlockMatrix(M, N, 128, nb * 16384, cv, torch.from_numpy(off).cuda(),
                                   torch.from_numpy(idx.astype(np.int16)).cuda())
                sp.AllocateRowIndicesBuffer(C)
                sp.RowIndices(C, C.row_indices)
                X = sp.Matrix(*((K, M) if ta else (M, K)), x)
                W = sp.Matrix(*((N, K) if tb else (K, N)), w)
                kern = sp.sdd_kernel(X, ta, W, tb, C)
                fns[f"{tr}_K{K}_N{N}"] = (
                    lambda X=X, W=W, C=C, ta=ta, tb=tb, keep=(x, w): sp.Matmul(X, ta, W, tb, C),
                    K, kern)
    res = {k: [] for k in fns}
    for _ in range(a.rounds):
        for k, (f, K, _) in fns.items():
            f()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                f()
            e.record()
            torch.cuda.synchronize()
            res[k].append(s.elapsed_time(e) * 1e3 / a.iters)
    out = {k: {"us": round(float(np.median(v)), 1), "kernel": fns[k][2],
               "us_per_kblock": round(float(np.median(v)) / (fns[k][1] // 128), 2)}
           for k, v in res.items()}
    print(json.dumps({"density": a.density, "results": out}), flush=True)


if __name__ == "__main__":
    main()
