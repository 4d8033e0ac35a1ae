#!/usr/bin/env python3
"""Per-workgroup timeline of the tall DSD pipeline (dsd4w.hip kEpi 7) on
BASELINE config 5 (M=131072, K=N=4096, 2%) from a SPUTNIK_EXP & 512 build
(SPUTNIK_AMD_LIB=build/tlx/tl4.so, SPUTNIK_AMD_TALL4W=1): setup (entry ->
k-loop start), compute (-> asm end: blocks + tile stores), zero fill (->
its stores done), in us."""
import ctypes
import json
import os
import sys
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import bench  # noqa: E402
import sputnik_amd as sp  # noqa: E402
from exp_timeline4w import capture, stats  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    args = types.SimpleNamespace(seed=0, k=4096, n=4096, m=4096, dtype="f16")
    prob = bench.dsd_panel(args, 1, 0, dev, 0.02, m_total=131072)
    fn = prob.launcher()
    buf = torch.zeros(16 * 4096, dtype=torch.int64, device=dev)
    capture(fn, buf)
    t = buf.view(-1, 16).cpu().numpy().astype(np.int64)
    t = t[t[:, 0] > 0]
    e0 = t[:, 0].min()
    us = lambda x: x / 100.0  # noqa: E731
    has = t[:, 2] > 0
    out = {"workgroups": int(len(t)), "with_blocks": int(has.sum()),
           "span_us": round(us(max(t[:, 4].max(), t[:, 15].max()) - e0), 2),
           "blocks": stats(t[has, 5]),
           "setup": stats(us(t[has, 2] - t[has, 0])),
           "compute": stats(us(t[has, 4] - t[has, 2])),
           "per_block": stats(us(t[has, 4] - t[has, 2]) / np.maximum(t[has, 5], 1)),
           "compute_end": stats(us(t[has, 4] - e0)),
           "flush_sum": stats(us(t[has, 9] & 0xffffffff)),
           "after_flush_2steps_sum": stats(us(t[has, 9] >> 32)),
           "zero_fill": stats(us(t[:, 15] - np.where(t[:, 4] > 0, t[:, 4], t[:, 0]))),
           "end": stats(us(t[:, 15] - e0))}
    # per XCD (workgroup b runs on XCD b % 8 under round-robin dispatch):
    # k-loop time per block and end; and the slowest workgroups' shapes
    bid = np.nonzero(buf.view(-1, 16).cpu().numpy()[:, 0] > 0)[0]
    xcd = bid % 8
    comp = us(t[:, 4] - t[:, 2])
    out["by_xcd"] = {int(x): {"compute_p50": round(float(np.median(comp[xcd == x])), 1),
                              "compute_max": round(float(comp[xcd == x].max()), 1),
                              "blocks_sum": int(t[xcd == x, 5].sum()),
                              "tiles_sum": int(t[xcd == x, 14].sum())}
                     for x in range(8)}
    order = np.argsort(-comp)[:10]
    out["slowest"] = [[round(float(comp[i]), 1), int(t[i, 5]), int(t[i, 14]), int(xcd[i]),
                       int(bid[i])] for i in order]
    out["fastest"] = [[round(float(comp[i]), 1), int(t[i, 5]), int(t[i, 14]), int(xcd[i]),
                       int(bid[i])] for i in np.argsort(comp)[:6]]
    c = np.corrcoef(comp, t[:, 14])[0, 1] if len(t) > 2 else 0.0
    out["corr_compute_tiles"] = round(float(c), 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
