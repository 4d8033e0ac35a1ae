#!/usr/bin/env python3
"""Makespan probe: DSD 4096^3 at 50% on the random topology (bench.py's)
vs a perfectly balanced one (every block-row exactly 16 blocks, random
columns: the reference's MakeSparseMatrixPerfectUniform shape), same values,
interleaved rounds in one process. The gap bounds what better load balancing
can win."""
import ctypes
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    import sputnik_amd as sp
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    prob = bench.Problem(4096, 4096, 4096, 0.5, "f16", 0, dev)
    rng = np.random.default_rng(1)
    cols = [np.sort(rng.choice(32, 16, replace=False)) for _ in range(32)]
    off = np.arange(33, dtype=np.int32) * 16
    idx = np.concatenate(cols).astype(np.int16)
    bal = sp.BlockMatrix(4096, 4096, 128, prob.nb * 16384, prob.a_vals,
                         torch.from_numpy(off).to(dev),
                         torch.from_numpy(idx).to(dev))
    L = sp.lib()
    stream = torch.cuda.current_stream().cuda_stream
    runs = {}
    for name, A in (("random", prob.A), ("balanced", bal)):
        ca, cb, cc = A._c(), prob.B._c(), prob.C._c()
        keep = (ca, cb, cc)
        runs[name] = (keep, lambda ca=ca, cb=cb, cc=cc: L.sputnik_dsd_ex(
            ctypes.byref(ca), 0, ctypes.byref(cb), 0, ctypes.byref(cc), 0,
            stream))
    times = {n: [] for n in runs}
    for _ in range(3):
        for n, (_, fn) in runs.items():
            fn()
    torch.cuda.synchronize()
    for _ in range(7):
        for n, (_, fn) in runs.items():
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(50):
                fn()
            e.record()
            torch.cuda.synchronize()
            times[n].append(s.elapsed_time(e) / 50 * 1e3)
    for n, t in times.items():
        print(n, "us median %.2f min %.2f" % (statistics.median(t), min(t)))
    print("row lengths random: min %d max %d" %
          (np.diff(prob.offsets).min(), np.diff(prob.offsets).max()))


if __name__ == "__main__":
    main()
