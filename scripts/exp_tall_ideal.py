#!/usr/bin/env python3
"""Upper bound for B reuse in the tall pipeline: an idealised config-5-like
operand (M = 131072, K = N = 4096) of 640 single-block rows, 20 per k-block,
and 384 empty rows, run (a) with the rows in random order and (b) dealt so
that the workgroups of one panel (32, equal cost ranges with
tall_odd_share = 100) meet the same k-block side by side. Same blocks, same
work. Usage: exp_tall_ideal.py [random|dealt] (one variant, for PMC passes)
or no argument (both, interleaved)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import sputnik_amd as sp  # noqa: E402


def topo(order_kind):
    R, nk, per_k = 1024, 32, 20
    rng = np.random.default_rng(9)
    ks = np.repeat(np.arange(nk), per_k)  # 640 single-block rows
    if order_kind == "random":
        rows = rng.permutation(R)[:len(ks)]
        kcol = rng.permutation(ks)
    else:  # dealt: chunk c (workgroup c of a panel) holds ranks c, c + 32, ...
        srt = np.sort(ks)
        dealt = np.concatenate([srt[c::32] for c in range(32)])
        rows = np.arange(len(ks))  # non-empty rows first, empty rows last
        kcol = dealt
    cnt = np.zeros(R, np.int32)
    cnt[rows] = 1
    idx_by_row = {r: k for r, k in zip(rows, kcol)}
    off = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int32)
    idx = np.array([idx_by_row[r] for r in range(R) if cnt[r]], np.int16)
    return off, idx


def main():
    dev = torch.device("cuda", 0)
    sp.tuning("tall_odd_share", 100)
    kinds = sys.argv[1:] or ["random", "dealt"]
    probs = {k: bench.DsdProblem(131072, 4096, *topo(k), 4096, False, False, "f16", 0, dev)
             for k in kinds}
    fns = {k: p.launcher() for k, p in probs.items()}
    res = {k: [] for k in fns}
    for _ in range(7 if len(fns) > 1 else 1):
        for k, f in fns.items():
            for _ in range(20):
                f()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(100):
                f()
            e.record()
            torch.cuda.synchronize()
            res[k].append(s.elapsed_time(e) * 10.0)
    print(json.dumps({k: round(float(np.median(v)), 2) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
