"""SDD k-rotation (knob sdd_krot) numerics: every rotation mode against
mode 0 and against an fp32 torch product, at one shape.
python scripts/diag_krot.py TRANS DIM DENSITY"""
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
    tr, dim, dens = sys.argv[1], int(sys.argv[2]), float(sys.argv[3])
    ta, tb = tr[0] == "T", tr[1] == "T"
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    a = torch.randn(dim, dim, generator=g, device=dev).half()
    b = torch.randn(dim, dim, generator=g, device=dev).half()
    nb = int(round((dim // 128) ** 2 * dens))
    off, idx = mu.random_topology(dim // 128, dim // 128, nb, np.random.default_rng(5))
    nz = nb * 128 * 128
    cv = torch.empty(nz, dtype=torch.half, device=dev)
    C = sp.BlockMatrix(dim, dim, 128, nz, cv, torch.from_numpy(off).to(dev),
                       torch.from_numpy(idx.astype(np.int16)).to(dev))
    sp.AllocateRowIndicesBuffer(C)
    sp.RowIndices(C, C.row_indices)
    A, B = sp.Matrix(dim, dim, a), sp.Matrix(dim, dim, b)
    af = (a.t() if ta else a).float()
    bf = (b.t() if tb else b).float()
    ref = (af @ bf)
    rows = np.repeat(np.arange(dim // 128), np.diff(off))
    ref_blocks = torch.stack([ref[r * 128:(r + 1) * 128, c * 128:(c + 1) * 128]
                              for r, c in zip(rows, idx)]).reshape(-1)
    out = {}
    base = None
    for mode in range(5):
        sp.tuning("sdd_krot", mode)
        cv.zero_()
        sp.Matmul(A, ta, B, tb, C)
        torch.cuda.synchronize()
        y = cv.float()
        if base is None:
            base = y.clone()
        err = ((y - ref_blocks).abs().max() / ref_blocks.abs().max()).item()
        out[mode] = {"max_rel_err_vs_fp32": err,
                     "max_abs_diff_vs_mode0": (y - base).abs().max().item(),
                     "finite": bool(torch.isfinite(y).all().item())}
    sp.tuning("sdd_krot", 0)
    print(json.dumps({"trans": tr, "dim": dim, "density": dens, "kernel":
                      sp.sdd_kernel(A, ta, B, tb, C), "modes": out}))


if __name__ == "__main__":
    main()
