#!/usr/bin/env python3
"""Debug helper: integer-valued DSD on tiny topologies, reports which output
rows / columns differ from the exact product (SPUTNIK_AMD_LIB selects the
library). Usage: debug_kat.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import sputnik_amd as sp  # noqa: E402
from sputnik_amd import matrix_utils as mu  # noqa: E402


def run(rows_b, cols_b, offsets, indices, n, seed=0, ones=False):
    rng = np.random.default_rng(seed)
    nb = len(indices)
    vals = (np.ones((nb, 128, 128)) if ones else
            rng.integers(-1, 2, size=(nb, 128, 128))).astype(np.float32)
    b = (np.ones((cols_b * 128, n)) if ones else
         rng.integers(-1, 2, size=(cols_b * 128, n))).astype(np.float32)
    A = sp.BlockMatrix(rows_b * 128, cols_b * 128, 128, nb * 16384,
                       torch.from_numpy(vals).half().cuda(),
                       torch.from_numpy(np.asarray(offsets, np.int32)).cuda(),
                       torch.from_numpy(np.asarray(indices, np.int16)).cuda())
    c = torch.full((rows_b * 128, n), float("nan"), dtype=torch.float16,
                   device="cuda")
    sp.Matmul(A, False, sp.Matrix(cols_b * 128, n, torch.from_numpy(b).half().cuda()),
              False, sp.Matrix(rows_b * 128, n, c))
    torch.cuda.synchronize()
    want = mu.to_dense(rows_b * 128, cols_b * 128, np.asarray(offsets),
                       np.asarray(indices), vals).astype(np.float64) @ b
    got = c.float().cpu().numpy()
    bad = got != want
    rows = np.nonzero(bad.any(axis=1))[0]
    cols = np.nonzero(bad.any(axis=0))[0]
    print(f"R={rows_b} C={cols_b} nb={nb} n={n}: {int(bad.sum())} bad; rows "
          f"{rows[:8].tolist()}..{rows[-3:].tolist() if len(rows) else []} "
          f"({len(rows)}), cols {cols[:8].tolist()} ({len(cols)})")
    if len(rows):
        r, cc = rows[0], cols[0]
        print("   first", r, cc, "got", got[r, cc], "want", want[r, cc],
              "row diff pattern", (got[r] - want[r])[:16].tolist())


torch.cuda.set_device(0)
os.environ.setdefault("SPUTNIK_AMD_PAIRS", "0")
for nblk in (1, 2, 3, 4, 5, 8):
    run(1, 8, [0, nblk], list(range(nblk)), 512)
run(1, 8, [0, 4], [0, 1, 2, 3], 512, ones=True)
run(2, 8, [0, 3, 6], [0, 2, 5, 1, 3, 7], 512)


def probe_k(n=512):
    """A = ones (one block), B = e_t rows: reports, per k = t, the output
    (row, col) entries that miss it."""
    vals = np.ones((1, 128, 128), np.float32)
    A = sp.BlockMatrix(128, 1024, 128, 16384, torch.from_numpy(vals).half().cuda(),
                       torch.tensor([0, 1], dtype=torch.int32).cuda(),
                       torch.tensor([0], dtype=torch.int16).cuda())
    miss = {}
    for t in range(128):
        b = torch.zeros((1024, n), dtype=torch.float16, device="cuda")
        b[t] = 1
        c = torch.full((128, n), float("nan"), dtype=torch.float16, device="cuda")
        sp.Matmul(A, False, sp.Matrix(1024, n, b), False, sp.Matrix(128, n, c))
        torch.cuda.synchronize()
        bad = (c.float().cpu().numpy() != 1.0)
        if bad.any():
            r = np.nonzero(bad.any(axis=1))[0]
            cc = np.nonzero(bad.any(axis=0))[0]
            miss[t] = (len(r), r.min(), r.max(), len(cc), cc[:12].tolist())
    print("k-probe: missing k:", sorted(miss))
    for t, v in sorted(miss.items())[:12]:
        print("  k", t, "rows", v[0], v[1], "-", v[2], "cols", v[3], v[4])


probe_k()
