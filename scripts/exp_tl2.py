#!/usr/bin/env python3
"""Per-workgroup phase breakdown from a SPUTNIK_EXP&16 build (16 stamps per
workgroup, block_gemm.h exp_stamp). Usage: exp_tl2.py lib.so [--density D]
Prints medians/max per role of: prologue, pipeline fill, loop, collect,
epilogue staging, stores; and the start/end spread in microseconds."""
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
    ap.add_argument("--dump", default="")
    args = ap.parse_args()
    import torch
    import bench
    torch.cuda.set_device(0)
    prob = bench.Problem(args.m, 4096, 4096, args.density, "f16", 0,
                         torch.device("cuda", 0))
    L = ctypes.CDLL(os.path.abspath(args.lib))
    L.sputnik_exp_set_debug.argtypes = [ctypes.c_void_p]
    tiles = max((args.m // 128) * 16, 4096)
    dbg = torch.zeros(tiles * 16, dtype=torch.int64, device="cuda")
    L.sputnik_exp_set_debug(ctypes.c_void_p(dbg.data_ptr()))
    ca, cb, cc = prob.A._c(), prob.B._c(), prob.C._c()
    fn = L.sputnik_dsd_ex
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                   ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    stream = torch.cuda.current_stream().cuda_stream
    for _ in range(30):
        assert fn(ctypes.byref(ca), 0, ctypes.byref(cb), 0, ctypes.byref(cc), 0, stream) == 0
    torch.cuda.synchronize()
    d = dbg.cpu().numpy().reshape(tiles, 16).astype(np.int64)[:2048]
    g_all = int((d[:, 4] != 0).sum())
    steps_all = d[:g_all, 7]
    d = d[d[:, 4] != 0]
    if args.dump:
        np.save(args.dump, d)
    t0 = d[:, 0].min()
    clk = (d[:, 4] - d[:, 1]) / np.maximum(d[:, 14] - d[:, 0], 1) / 100.0  # GHz
    ph = {
        "offs_staged": d[:, 15] - d[:, 1],
        "prologue": d[:, 2] - d[:, 1],
        "fill": d[:, 8] - d[:, 2],
        "loop": d[:, 10] - d[:, 8],
        "collect": np.where(d[:, 11] > 0, d[:, 11] - d[:, 10], 0),
        "staging": d[:, 13] - np.where(d[:, 11] > 0, d[:, 11], d[:, 10]),
        "stores": d[:, 4] - d[:, 13],
    }
    steps = d[:, 7]
    out = {"tiles": int(len(d)), "clock_ghz_med": round(float(np.median(clk)), 3),
           "start_us": [round(float(np.percentile((d[:, 0] - t0) / 100, q)), 2) for q in (0, 50, 100)],
           "end_us": [round(float(np.percentile((d[:, 14] - t0) / 100, q)), 2) for q in (0, 50, 90, 100)]}
    roles = d[:, 12]
    for role, name in ((0, "light"), (1, "middle"), (2, "heavy"), (3, "unpaired")):
        m = roles == role
        if not m.any():
            continue
        r = {"n": int(m.sum()), "steps": [int(steps[m].min()), int(np.median(steps[m])), int(steps[m].max())]}
        for k, v in ph.items():
            r[k] = [int(np.median(v[m])), int(v[m].max())]
        lp = ph["loop"][m]
        st = np.maximum(steps[m], 1)
        r["loop_cyc_per_step"] = round(float(np.sum(lp) / np.sum(st)), 1)
        if role == 0:
            hd = d[m, 9] - d[m, 8]
            r["head_publish"] = [int(np.median(hd)), int(hd.max())]
        r["end_us"] = [round(float(np.percentile((d[m, 14] - t0) / 100, q)), 2) for q in (0, 50, 100)]
        out[name] = r
    # SPUTNIK_EXP & 128 builds: per-segment k-loop cycle sums of waves 0
    # (leading half) and kNW/2 (lagging half), per step.
    raw = dbg.cpu().numpy().astype(np.int64)
    seg = raw[2048 * 16:2048 * 16 + g_all * 16].reshape(g_all, 16) if g_all else None
    if seg is not None and seg.any():
        names = ["vmcnt+B1", "dma_issue", "read_issue", "lagwait+B2", "mfma_issue", "read_wait"]
        st = np.maximum(steps_all, 1)[:, None]
        for half, off in (("lead", 0), ("lag", 8)):
            per = seg[:, off:off + 6] / st
            out["seg_" + half] = {n: round(float(np.median(per[:, q])), 1) for q, n in enumerate(names)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
