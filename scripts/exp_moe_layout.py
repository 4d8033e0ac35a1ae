#!/usr/bin/env python3
"""Config-4 SDD in both weight layouts, same process, interleaved: w1 stored
[d_model][E d_ff] (SDD NN, bench.py MoeProblem so far) against MegaBlocks'
own [E d_ff][d_model] with sdd(x, w1.t()) (SDD NT), plus the DSD h . w2 and
the whole step in each layout. Prints one JSON line (us medians)."""
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
    E, T, DM, FF = 8, 8192, 4096, 14336
    cols = E * FF
    off, idx = mu.expert_block_diagonal(E, T // E // 128, FF // 128)
    nb = int(off[-1])
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    rnd = lambda *s: (torch.rand(*s, generator=g, device="cuda") * 2 - 1).to(torch.bfloat16)
    x, w1, w2 = rnd(T, DM), rnd(DM, cols), rnd(cols, DM)
    w1t = w1.t().contiguous()                      # [E d_ff][d_model]
    hv = torch.empty(nb, 128, 128, dtype=torch.bfloat16, device="cuda")
    Hm = sp.BlockMatrix(T, cols, 128, nb * 16384, hv, torch.from_numpy(off).cuda(),
                        torch.from_numpy(idx.astype(np.int16)).cuda())
    sp.AllocateRowIndicesBuffer(Hm)
    sp.RowIndices(Hm, Hm.row_indices)
    y = torch.empty(T, DM, dtype=torch.bfloat16, device="cuda")
    X, W1, W1T = sp.Matrix(T, DM, x), sp.Matrix(DM, cols, w1), sp.Matrix(cols, DM, w1t)
    W2, Y = sp.Matrix(cols, DM, w2), sp.Matrix(T, DM, y)
    fns = {
        "sdd_nn": lambda: sp.Matmul(X, False, W1, False, Hm),
        "sdd_nt": lambda: sp.Matmul(X, False, W1T, True, Hm),
        "dsd_nn": lambda: sp.MatmulEx(Hm, False, W2, False, Y),
    }
    kern = {"sdd_nn": sp.sdd_kernel(X, False, W1, False, Hm),
            "sdd_nt": sp.sdd_kernel(X, False, W1T, True, Hm)}
    # same result both ways (bit-identical is not required: different k
    # fragment paths; within the bf16 tolerance)
    fns["sdd_nn"]()
    ref = hv.float().clone()
    fns["sdd_nt"]()
    diff = (hv.float() - ref).abs().max().item()
    res = {k: [] for k in fns}
    for _ in range(7):
        for k, f in fns.items():
            for _ in range(3):
                f()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                f()
            e.record()
            torch.cuda.synchronize()
            res[k].append(s.elapsed_time(e) * 100.0)
    med = {k: round(sorted(v)[3], 1) for k, v in res.items()}
    flops = 2.0 * nb * 16384 * DM
    print(json.dumps({"us_median": med, "sdd_kernel": kern, "max_abs_diff_nn_nt": diff,
                      "step_tflops_nn": round(2 * flops / ((med["sdd_nn"] + med["dsd_nn"]) * 1e-6) / 1e12, 1),
                      "step_tflops_nt": round(2 * flops / ((med["sdd_nt"] + med["dsd_nn"]) * 1e-6) / 1e12, 1)}),
          flush=True)


if __name__ == "__main__":
    main()
