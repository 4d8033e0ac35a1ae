"""A/B of the SDD K-split (tuning knob sdd_ksplit = max chunks; 1 = the
8-wave k-split block tile) on config 3's SDD (4096^3, 205 blocks) and a few
other shapes; prints one JSON line per shape."""
import json
import sys

import numpy as np
import torch

import sputnik_amd as sp
from sputnik_amd import matrix_utils as mu

B = 128


def problem(m, k, n, nb, seed=0):
    rng = np.random.default_rng(seed)
    off, idx = mu.random_topology(m // B, n // B, nb, rng)
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    x = (torch.rand(m * k, generator=g, device="cuda") * 2 - 1).half()
    w = (torch.rand(k * n, generator=g, device="cuda") * 2 - 1).half()
    cv = torch.empty(nb * B * B, dtype=torch.float16, device="cuda")
    C = sp.BlockMatrix(m, n, B, nb * B * B, cv,
                       torch.from_numpy(off.astype(np.int32)).cuda(),
                       torch.from_numpy(idx.astype(np.int16)).cuda())
    sp.AllocateRowIndicesBuffer(C)
    sp.RowIndices(C, C.row_indices)
    return sp.Matrix(m, k, x), sp.Matrix(k, n, w), C


def timeit(fn, iters=100):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        ts.append((a, b))
    torch.cuda.synchronize()
    us = sorted(a.elapsed_time(b) * 1e3 for a, b in ts)
    return round(us[len(us) // 2], 2), round(us[0], 2)


def main():
    sp.tuning("sdd_ksplit_min_k", 512)
    shapes = [(4096, 4096, 4096, 205), (4096, 8192, 4096, 205), (2048, 4096, 4096, 60),
              (4096, 2048, 4096, 300)]
    for m, k, n, nb in shapes:
        X, W, C = problem(m, k, n, nb)
        res = {}
        for s in (1, 2, 4, 8):
            prev = sp.tuning("sdd_ksplit", s)
            try:
                plan = sp.sdd_plan(X, False, W, False, C)
                med, mn = timeit(lambda: sp.Matmul(X, False, W, False, C))
            finally:
                sp.tuning("sdd_ksplit", prev)
            res[s] = {"plan": plan, "us": med, "min": mn,
                      "tflops": round(2.0 * nb * B * B * k / (med * 1e-6) / 1e12, 1)}
        print(json.dumps({"m": m, "k": k, "n": n, "nb": nb, "ks": res,
                          "pair_errors": sp.pair_errors()}), flush=True)


if __name__ == "__main__":
    sys.exit(main())
