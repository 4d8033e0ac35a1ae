#!/usr/bin/env python3
"""Per-workgroup timeline of the 4-wave DSD kernel (dsd4w.hip) from a
SPUTNIK_EXP & 512 build (scripts/exp_build.sh tl4:-DSPUTNIK_EXP=512; run with
SPUTNIK_AMD_LIB=build/exp/tl4.so). For the headline DSD 4096^3 at each
density: the launch span and, per role (plain / pair producer / pair
consumer), the setup (entry -> k-loop start), the k-loop, and the epilogue
(k-loop end -> stores issued, incl. a consumer's poll + partial add), in us
(s_memrealtime, 100 MHz). Usage: exp_timeline4w.py [density ...]"""
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


def stats(v):
    v = np.asarray(v, dtype=np.float64)
    if v.size == 0:
        return None
    return {"p10": round(float(np.percentile(v, 10)), 2),
            "p50": round(float(np.median(v)), 2),
            "max": round(float(v.max()), 2)}


def summarize(buf, head):
    """Per-role / per-XCD summary of one launch's timeline records."""
    t = buf.view(-1, 16).cpu().numpy().astype(np.int64)
    t = t[t[:, 0] > 0]
    e0 = t[:, 0].min()
    us = lambda x: x / 100.0  # noqa: E731
    role = t[:, 6]  # 1 producer, 2 consumer, 0 plain
    out = dict(head)
    out.update({"workgroups": int(len(t)),
           "span_us": round(us(t[:, 4].max() - e0), 2),
           "entry_skew_us": round(us(t[:, 0].max() - e0), 2),
           "first_loop_start": round(us(t[:, 2].min() - e0), 2),
           "last_loop_start": round(us(t[:, 2].max() - e0), 2),
           "last_loop_end": round(us(t[:, 3].max() - e0), 2),
           "blocks_per_wg": stats(t[:, 5])})
    for r, name in ((0, "plain"), (1, "producer"), (2, "consumer")):
        sel = role == r
        if not sel.any():
            continue
        s = t[sel]
        out[name] = {
            "n": int(sel.sum()),
            "setup": stats(us(s[:, 2] - s[:, 0])),
            "to_asm": stats(us(s[:, 1] - s[:, 0])),
            "karg": stats(us(s[:, 11] - s[:, 0])),
            "ranked": stats(us(s[:, 12] - s[:, 0])),
            "kblocks": stats(us(s[:, 13] - s[:, 0])),
            "loop": stats(us(s[:, 3] - s[:, 2])),
            "loop_per_block": stats(us(s[:, 3] - s[:, 2]) / np.maximum(s[:, 5], 1)),
            "epilogue": stats(us(s[:, 4] - s[:, 3])),
            "end": stats(us(s[:, 4] - e0)),
        }
        if r == 1 and (s[:, 9] > 0).all():  # (stamped by the late publish only)
            out[name]["publish"] = stats(us(s[:, 10] - s[:, 9]))
            out[name]["publish_at"] = stats(us(s[:, 9] - s[:, 2]))
    # per XCD (workgroups b and b + 8 share one under round-robin
    # placement; which XCD is not known, only which share): k-loop time
    # per block and end time
    bid = np.nonzero(buf.view(-1, 16).cpu().numpy()[:, 0] > 0)[0]
    xcd = bid % 8
    out["by_xcd"] = {
        str(x): {"loop_per_block_p50": round(float(np.median(
                    us(t[xcd == x, 3] - t[xcd == x, 2]) /
                    np.maximum(t[xcd == x, 5], 1))), 3),
                 "end_max": round(float(us(t[xcd == x, 4].max() - e0)), 2),
                 "loop_start_max": round(float(us(t[xcd == x, 2].max() - e0)), 2)}
        for x in range(8) if (xcd == x).any()}
    # the 12 latest-ending workgroups: end, role, blocks, first segment, XCD share
    order = np.argsort(-t[:, 4])[:12]
    out["latest"] = [[round(us(t[i, 4] - e0), 2), int(t[i, 6]), int(t[i, 5]),
                      int(t[i, 8]), int(xcd[i])] for i in order]
    return out


def capture(fn, buf):
    """fn() warm for 1 s, then one launch with the timeline buffer set."""
    L = sp.lib()
    L.sputnik_exp_set_debug.argtypes = [ctypes.c_void_p]
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


def main_dds(args, mode):
    """DDS NN of BASELINE config 3: out = g . C, C the 4096^2 block-sparse
    operand at each density (transposed metadata precomputed, MatmulEx)."""
    dev = torch.device("cuda", 0)
    sp.select_dsd_kernel(mode)
    buf = torch.zeros(16 * 4096, dtype=torch.int64, device=dev)
    for d in [float(x) for x in (args or ["0.2"])]:
        prob = bench.PairProblem(4096, d, "f16", 7, dev)
        cg = sp.Matrix(4096, 4096, prob.g)
        co = sp.Matrix(4096, 4096, prob.out)
        fn = lambda: sp.MatmulEx(cg, False, prob.C, False, co)  # noqa: E731
        capture(fn, buf)
        print(json.dumps(summarize(buf, {"op": "dds", "density": d, "mode": mode})),
              flush=True)


def main():
    # arguments: densities, and mode=N for the kernel variant
    # (sputnik_select_dsd_kernel; default 1, the shipped choice)
    mode = 1
    op = "dsd"
    args = []
    for a in sys.argv[1:]:
        if a.startswith("mode="):
            mode = int(a[5:])
        elif a.startswith("op="):
            op = a[3:]
        else:
            args.append(a)
    if op == "dds":
        return main_dds(args, mode)
    dens = [float(x) for x in (args or ["0.5", "0.1", "0.9"])]
    dev = torch.device("cuda", 0)
    L = sp.lib()
    sp.select_dsd_kernel(mode)
    L.sputnik_exp_set_debug.argtypes = [ctypes.c_void_p]
    buf = torch.zeros(16 * 4096, dtype=torch.int64, device=dev)
    for d in dens:
        nz = mu.nonzeros_for_density(4096, 4096, d)
        off, idx = mu.random_topology(32, 32, nz // 16384, np.random.default_rng(1))
        prob = bench.DsdProblem(4096, 4096, off, idx, 4096, False, False, "f16", 7, dev)
        fn = prob.launcher()
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
        out = summarize(buf, {"density": d, "mode": mode, "pair_xcd2": os.environ.get("SPUTNIK_AMD_PAIR_XCD2", "default"), "kernel": prob.kernel})
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
