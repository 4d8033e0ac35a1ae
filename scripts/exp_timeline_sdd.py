#!/usr/bin/env python3
"""Per-workgroup timeline of the SDD K-split (dsd4w.hip kKs) from a
SPUTNIK_EXP & 512 build (run with SPUTNIK_AMD_LIB=build/tlx/tl4.so): for
each shape, the launch span and per chunk the setup (entry -> k-loop start),
the k-loop, the publish (loop end -> flag raised), the wait for the other
chunks' flags and the reduce + store, in us (s_memrealtime, 100 MHz).
Usage: exp_timeline_sdd.py"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import sputnik_amd as sp  # noqa: E402
from exp_sdd_ks import problem  # noqa: E402
from exp_timeline4w import stats  # noqa: E402


def main():
    L = sp.lib()
    L.sputnik_exp_set_debug.argtypes = [ctypes.c_void_p]
    buf = torch.zeros(16 * 4096, dtype=torch.int64, device="cuda")
    for m, k, n, nb in ((4096, 4096, 4096, 205), (4096, 2048, 4096, 300)):
        X, W, C = problem(m, k, n, nb)
        fn = lambda: sp.Matmul(X, False, W, False, C)  # noqa: E731
        t_end = time.time() + 1.0
        while time.time() < t_end:
            for _ in range(50):
                fn()
            torch.cuda.synchronize()
        L.sputnik_exp_set_debug(ctypes.c_void_p(buf.data_ptr()))
        buf.zero_()
        fn()
        torch.cuda.synchronize()
        L.sputnik_exp_set_debug(ctypes.c_void_p(0))
        t = buf.view(-1, 16).cpu().numpy().astype(np.int64)
        bid = np.nonzero(t[:, 0] > 0)[0]
        t = t[bid]
        e0 = t[:, 0].min()
        us = lambda x: x / 100.0  # noqa: E731
        out = {"m": m, "k": k, "n": n, "nb": nb, "workgroups": int(len(t)),
               "chunks": int(t[:, 14].max()),
               "span_us": round(us(t[:, 4].max() - e0), 2),
               "entry_skew_us": round(us(t[:, 0].max() - e0), 2)}
        for c in range(int(t[:, 14].max())):
            s = t[t[:, 6] == c]
            out[f"chunk{c}"] = {
                "n": int(len(s)), "blocks": stats(s[:, 8]),
                "entry": stats(us(s[:, 0] - e0)),
                "setup": stats(us(s[:, 2] - s[:, 0])),
                "loop": stats(us(s[:, 3] - s[:, 2])),
                "publish": stats(us(s[:, 9] - s[:, 3])),
                "wait": stats(us(s[:, 10] - s[:, 9])),
                "reduce_store": stats(us(s[:, 4] - s[:, 10])),
                "end": stats(us(s[:, 4] - e0))}
        xcd = bid % 8
        out["by_xcd_end_max"] = {int(x): round(us(t[xcd == x, 4].max() - e0), 2)
                                 for x in range(8) if (xcd == x).any()}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
