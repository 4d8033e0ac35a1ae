#!/usr/bin/env python3
"""Per-workgroup phase timeline from a SPUTNIK_EXP&16 build.
Usage: exp_timeline.py lib.so [--density D]"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--density", type=float, default=0.5)
    ap.add_argument("--m", type=int, default=4096)
    ap.add_argument("--acct", action="store_true")
    ap.add_argument("--dump", default="", help="save the raw per-workgroup stamps (.npy)")
    args = ap.parse_args()
    import torch
    import bench
    torch.cuda.set_device(0)
    prob = bench.Problem(args.m, 4096, 4096, args.density, "f16", 0,
                         torch.device("cuda", 0))
    L = ctypes.CDLL(os.path.abspath(args.lib))
    L.sputnik_exp_set_debug.argtypes = [ctypes.c_void_p]
    tiles = max((args.m // 128) * 16, 4096)
    dbg = torch.zeros(tiles * 8, dtype=torch.int64, device="cuda")
    L.sputnik_exp_set_debug(ctypes.c_void_p(dbg.data_ptr()))
    ca, cb, cc = prob.A._c(), prob.B._c(), prob.C._c()
    fn = L.sputnik_dsd_ex
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                   ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    stream = torch.cuda.current_stream().cuda_stream
    for _ in range(20):
        assert fn(ctypes.byref(ca), 0, ctypes.byref(cb), 0, ctypes.byref(cc), 0, stream) == 0
    torch.cuda.synchronize()
    d = dbg.cpu().numpy().reshape(tiles, 8).astype(np.int64)
    d = d[d[:, 4] != 0]
    if args.dump:
        np.save(args.dump, d)
    tiles = len(d)
    rt0 = d[:, 0] - d[:, 0].min()
    pro = d[:, 2] - d[:, 1]
    wall_us = (d[:, 3] - d[:, 0]) / 100.0           # realtime: 100 MHz
    loop = d[:, 4] - d[:, 2]                         # loop + epilogue cycles
    epi = np.zeros_like(loop)
    tot = d[:, 4] - d[:, 1]
    steps = d[:, 7]
    cu = (d[:, 5] << 16) | (d[:, 6] & 0xFFFF)
    # realtime is 100 MHz; memtime ~ shader clock
    span_rt = (d[:, 0].max() - d[:, 0].min()) / 100.0  # us, start skew
    res = {
        "tiles": int(tiles),
        "start_skew_us": round(span_rt, 2),
        "prologue_cycles": [int(np.median(pro)), int(pro.max())],
        "loop_cycles_median": int(np.median(loop)),
        "epilogue_cycles": [int(np.median(epi)), int(epi.max())],
        "total_cycles": [int(np.median(tot)), int(tot.max()), int(tot.min())],
        "cycles_per_step": round(float(np.sum(loop) / max(1, np.sum(steps))), 1),
        "steps": [int(steps.min()), int(np.median(steps)), int(steps.max())],
        "distinct_cu": int(len(np.unique(cu))),
        "wall_us_pct": [round(float(np.percentile(wall_us, q)), 2) for q in (0, 50, 90, 100)],
        "end_rt_us_pct": [round(float(np.percentile((d[:, 3] - d[:, 0].min()) / 100.0, q)), 2) for q in (0, 50, 90, 100)],
        "clock_ghz_pct": [round(float(np.percentile((d[:, 4] - d[:, 1]) / np.maximum(d[:, 3] - d[:, 0], 1) / 10.0, q)), 3) for q in (0, 50, 100)],
        "wg_start_rt_us_pct": [round(float(np.percentile(rt0, q)) / 100.0, 2) for q in (0, 25, 50, 75, 90, 100)],
    }
    # Correlation of loop time with steps (slope = cycles/step, intercept).
    A = np.vstack([steps, np.ones_like(steps)]).T.astype(float)
    slope, icpt = np.linalg.lstsq(A, loop.astype(float), rcond=None)[0]
    res["loop_fit"] = {"cycles_per_step": round(slope, 1), "intercept": round(icpt, 1)}
    if args.acct:
        parts = {"vmcnt_wait_barrier": d[:, 0], "dma_setup": d[:, 5] & 0xFFFFFFFF,
                 "interleaved_issue": d[:, 5] >> 32, "unused": d[:, 6] & 0xFFFFFFFF,
                 "read_wait": d[:, 6] >> 32}
        st = np.maximum(steps, 1)
        res["per_step_cycles"] = {k: round(float(np.sum(v) / np.sum(st)), 1)
                                  for k, v in parts.items()}
        for k in ("start_skew_us", "wg_start_rt_us_pct", "distinct_cu"):
            res.pop(k, None)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
