#!/usr/bin/env python3
"""Config-5 decomposition probe: how much of DSD M=131072 K=N=4096 2% is
the compute on the non-empty block-rows and how much the zero fill of the
empty ones, and do they overlap inside the one launch?

  full        the shipped call (one persistent CfgTall launch)
  compact     the same blocks with the empty block-rows removed (compute +
              the non-empty rows' output only)
  fill_empty  a plain zero fill of the empty rows' output bytes
  fill_all    a plain zero fill of the whole 1 GiB output
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(fn, iters=50):
    import torch
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    import torch
    import bench
    from sputnik_amd import matrix_utils as mu
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    m, k, n = 131072, 4096, 4096
    R = m // 128
    nz = mu.nonzeros_for_density(m, k, 0.02)
    rng = np.random.default_rng(0)
    off, idx = mu.random_topology(R, k // 128, nz // (128 * 128), rng)
    cnt = np.diff(off)
    keep = np.nonzero(cnt)[0]
    empty = R - len(keep)
    coff = np.concatenate([[0], np.cumsum(cnt[keep])]).astype(np.int32)
    print("block-rows %d, non-empty %d, empty %d, nb %d" %
          (R, len(keep), empty, int(off[-1])))
    full = bench.DsdProblem(m, k, off, idx, n, False, False, "f16", 0, dev)
    comp = bench.DsdProblem(len(keep) * 128, k, coff, idx, n, False, False,
                            "f16", 0, dev)
    f_full, f_comp = full.launcher(), comp.launcher()
    out = torch.empty(m * n, dtype=torch.float16, device=dev)
    ebytes = empty * 128 * n
    res = {}
    for rep in range(3):
        res.setdefault("full", []).append(timeit(f_full))
        res.setdefault("compact", []).append(timeit(f_comp))
        res.setdefault("fill_empty", []).append(
            timeit(lambda: out[:ebytes].zero_()))
        res.setdefault("fill_all", []).append(timeit(lambda: out.zero_()))
        res.setdefault("compact+fill_empty", []).append(
            timeit(lambda: (f_comp(), out[:ebytes].zero_())))
    for key, v in res.items():
        print("%-20s %8.1f us (min %.1f)" % (key, float(np.median(v)), min(v)))


if __name__ == "__main__":
    main()
