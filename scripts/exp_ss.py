#!/usr/bin/env python3
"""Times SSD / SDS / DSS (NN, MatmulEx, fp16) at 4096^3 on the library named
by SPUTNIK_AMD_LIB: sparse input 50%, sparse output 20% (DSS: both inputs 50%,
NT). One JSON line. Usage: SPUTNIK_AMD_LIB=... exp_ss.py"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import sputnik_amd as sp
    from tests import helpers as H
    torch.cuda.set_device(0)
    rng = np.random.default_rng(0)
    d = 4096
    half = d * d // 2
    A = H.HostSparse(d, d, half, rng)
    B = H.HostDense(d, d, rng)
    Cs = H.HostSparse(d, d, d * d // 5 // 16384 * 16384, rng)
    sp.AllocateRowIndicesBuffer(Cs.matrix)
    sp.RowIndices(Cs.matrix, Cs.matrix.row_indices)
    A2 = H.HostSparse(d, d, half, rng)
    for m in (A.matrix, A2.matrix):
        sp.AllocateTransposeBuffers(m)
        sp.Transpose(m)
    C, _ = H.empty_dense(d, d)
    calls = {
        "ssd": lambda: sp.MatmulEx(A.matrix, False, B.matrix, False, Cs.matrix),
        "sds": lambda: sp.MatmulEx(B.matrix, False, A.matrix, False, Cs.matrix),
        "dss": lambda: sp.MatmulEx(A.matrix, False, A2.matrix, True, C),
    }
    out = {}
    for name, fn in calls.items():
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                fn()
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) / 20 * 1e3)
        out[name] = round(statistics.median(ts), 2)
    print(json.dumps({"lib": os.path.basename(os.environ.get("SPUTNIK_AMD_LIB", "libsputnik.so")),
                      "us": out}))


if __name__ == "__main__":
    main()
