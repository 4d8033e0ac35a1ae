#!/usr/bin/env python3
"""Per-workgroup timeline of one block_gemm launch (SPUTNIK_EXP & 512
builds; SPUTNIK_AMD_LIB selects the library). For each workload: the launch
span and, over the workgroups, when they started and how long their setup,
pipeline, pair collect and tile write took (us, 100 MHz clock).

Usage: exp_timeline.py [workload ...]  (dsd10 dsd20 dsd50 dds20 sdd20)"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import sputnik_amd as sp  # noqa: E402
from sputnik_amd import matrix_utils as mu  # noqa: E402


def topo(density, seed=0):
    nz = mu.nonzeros_for_density(4096, 4096, density)
    rng = np.random.default_rng(seed)
    return mu.random_topology(32, 32, nz // (128 * 128), rng)


def launcher(name, device):
    L = sp.lib()
    stream = torch.cuda.current_stream().cuda_stream
    if name == "panel":  # BASELINE config 5 on one GPU: M = 131072, 2%
        nz = mu.nonzeros_for_density(131072, 4096, 0.02)
        off, idx = mu.random_topology(1024, 32, nz // (128 * 128),
                                      np.random.default_rng(5))
        prob = bench.DsdProblem(131072, 4096, off, idx, 4096, False, False,
                                "f16", 0, device)
        return prob, prob.launcher()
    if name.startswith("dsd"):
        off, idx = topo(int(name[3:]) / 100)
        prob = bench.DsdProblem(4096, 4096, off, idx, 4096, False, False,
                                "f16", 0, device)
        return prob, prob.launcher()
    prob = bench.PairProblem(4096, int(name[3:]) / 100, "f16", 0, device)
    d = prob.dim
    cx, cw, cg, co = (sp.Matrix(d, d, t)._c()
                      for t in (prob.x, prob.w, prob.g, prob.out))
    cC = prob.C._c()
    keep = (cx, cw, cg, co, cC)
    if name.startswith("sdd"):
        args = (ctypes.byref(cx), 0, ctypes.byref(cw), 0, ctypes.byref(cC), 0,
                stream)
        return (prob, keep), lambda: L.sputnik_sdd(*args)
    args = (ctypes.byref(cg), 0, ctypes.byref(cC), 0, ctypes.byref(co), 0,
            stream)
    return (prob, keep), lambda: L.sputnik_dds_ex(*args)


def summarize(buf, wgs):
    t = buf[:wgs * 16].reshape(wgs, 16).astype(np.int64)
    live = t[:, 0] > 0
    t = t[live]
    t[:, 2] = np.where(t[:, 2] == 0, t[:, 3], t[:, 2])  # no pair stamp
    t0 = t[:, 0].min()
    us = lambda x: x / 100.0  # noqa: E731  (100 MHz)
    seg = {
        "start": us(t[:, 0] - t0),
        "setup": us(t[:, 1] - t[:, 0]),
        "to_pairs": us(t[:, 11] - t[:, 0]),
        "offsets_load": us(np.where(t[:, 13] > 0, t[:, 13] - t[:, 11], 0)),
        "rank": us(np.where(t[:, 12] > 0, t[:, 12] - t[:, 13], 0)),
        "after_rank": us(np.where(t[:, 12] > 0, t[:, 1] - t[:, 12], 0)),
        "pipeline": us(t[:, 2] - t[:, 1]),
        "collect": us(t[:, 3] - t[:, 2]),
        "write": us(t[:, 4] - t[:, 3]),
        "end": us(t[:, 4] - t0),
    }
    out = {"workgroups": int(live.sum()), "span_us": float(seg["end"].max())}
    for k, v in seg.items():
        out[k] = {"p50": round(float(np.median(v)), 2),
                  "p90": round(float(np.percentile(v, 90)), 2),
                  "max": round(float(v.max()), 2)}
    steps = t[:, 7]
    role = t[:, 8]
    prod = role == 1
    cons = role == 2
    if cons.any():
        pub = {int(t[i, 10]): t[i, 5] for i in np.nonzero(prod)[0]}
        rows = []
        for i in np.nonzero(cons)[0]:
            pt = pub.get(int(t[i, 10]))
            rows.append((us(t[i, 2] - t0), us(pt - t0) if pt else -1,
                         us(t[i, 6] - t[i, 2]), us(t[i, 3] - t[i, 6])))
        rows = np.array(rows)
        out_c = {"pipeline_end": rows[:, 0], "producer_published": rows[:, 1],
                 "poll": rows[:, 2], "partial_load": rows[:, 3]}
        out_pairs = {k: {"p50": round(float(np.median(v)), 2),
                         "max": round(float(v.max()), 2)}
                     for k, v in out_c.items()}
        worst = int(np.argmax(rows[:, 0] + rows[:, 2] + rows[:, 3]))
        out_pairs["worst"] = [round(float(x), 2) for x in rows[worst]]
    else:
        out_pairs = None
    out["steps"] = {"mean": round(float(steps.mean()), 1),
                    "max": int(steps.max())}
    dur = seg["end"] - seg["start"]
    out["by_steps"] = {}
    for lo, hi in ((0, 0), (1, 4), (5, 8), (9, 10 ** 9)):
        sel = (steps >= lo) & (steps <= hi)
        if sel.any():
            out["by_steps"][f"{lo}-{hi}"] = {
                "n": int(sel.sum()),
                "dur_p50": round(float(np.median(dur[sel])), 2),
                "setup_p50": round(float(np.median(seg["setup"][sel])), 2),
                "pipe_p50": round(float(np.median(seg["pipeline"][sel])), 2),
                "write_p50": round(float(np.median(seg["write"][sel])), 2)}
    out["busy_us_total"] = round(float(dur.sum()), 1)
    # In-kernel shader clock (s_memtime / s_memrealtime x 100 MHz, entry to
    # tile written), median over workgroups (MI355X_MICROARCH.md DVFS (6)).
    dt = (t[:, 4] - t[:, 0]).astype(np.float64)
    dc = (t[:, 15] - t[:, 14]).astype(np.float64)
    ok = (dt > 0) & (dc > 0)
    if ok.any():
        out["clock_GHz"] = round(float(np.median(dc[ok] / dt[ok] * 0.1)), 3)
    # Workgroups resident over time (10 buckets of the span).
    span = float(seg["end"].max())
    edges = np.linspace(0, span, 11)
    conc = []
    for a, b in zip(edges[:-1], edges[1:]):
        mid = (a + b) / 2
        conc.append(int(((seg["start"] <= mid) & (seg["end"] > mid)).sum()))
    out["resident_over_time"] = conc
    out["roles"] = {str(r): int((role == r).sum()) for r in (0, 1, 2)}
    out["end_by_role"] = {
        str(r): {"p50": round(float(np.median(seg["end"][role == r])), 2),
                 "max": round(float(seg["end"][role == r].max()), 2)}
        for r in (0, 1, 2) if (role == r).any()}
    out["pairs"] = out_pairs
    slow = int(np.argmax(seg["end"]))
    out["last_wg"] = {k: round(float(v[slow]), 2) for k, v in seg.items()}
    out["last_wg"]["steps"] = int(steps[slow])
    out["last_wg"]["role"] = int(role[slow])
    return out


def main():
    names = sys.argv[1:] or ["dsd10", "dsd50", "dds20", "sdd20"]
    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    L = sp.lib()
    L.sputnik_exp_set_debug.argtypes = [ctypes.c_void_p]
    buf = torch.zeros(16 * 32768, dtype=torch.int64, device=device)
    L.sputnik_exp_set_debug(ctypes.c_void_p(buf.data_ptr()))
    for name in names:
        keep, fn = launcher(name, device)
        warm = float(os.environ.get("TIMELINE_WARM_S", "0"))
        t_end = time.time() + warm  # back-to-back launches so the clock settles
        for i in range(1 << 30):
            fn()
            if i >= 20 and (i % 50 == 0) and time.time() >= t_end:
                break
        torch.cuda.synchronize()
        buf.zero_()
        torch.cuda.synchronize()
        fn()
        torch.cuda.synchronize()
        host = buf.cpu().numpy()
        if os.environ.get("TIMELINE_SEG"):
            # SPUTNIK_EXP & 128 builds: per-segment shader-cycle sums of the
            # k-loop for waves 0 (leading half) and kNW/2 (lagging half) of
            # each workgroup at debug + 2048*16 + 16 b + {0, 8}.
            res = summarize(host, 2048)
            seg = host[2048 * 16:4096 * 16].reshape(2048, 2, 8)[:, :, :6]
            steps = host[:2048 * 16].reshape(2048, 16)[:, 7]
            live = steps > 0
            names_ = ["wait_b1", "dma_issue", "read_issue", "b2",
                      "mfma_issue", "read_wait"]
            res["segments_per_step"] = {
                half: {n: round(float(np.median(seg[live, h, q] /
                                                 steps[live])), 1)
                       for q, n in enumerate(names_)}
                for h, half in enumerate(("lead", "lag"))}
        else:
            res = summarize(host, 32768)
        res["workload"] = name
        print(json.dumps(res), flush=True)
        del keep
    L.sputnik_exp_set_debug(ctypes.c_void_p(0))


if __name__ == "__main__":
    main()
