"""Same-process A/B of tuning knobs on one bench workload problem:
python scripts/exp_knob_ab.py KNOB v1,v2,... [--workload panel|dsd] [--density D]
Several knobs at once: KNOB1+KNOB2 with values a1:a2,b1:b2,... (one setting
per comma, the knobs' values joined by ':').
Interleaved rounds, median per value (us)."""
import argparse
import json
import os
import sys
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import sputnik_amd as sp  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("knob")
    ap.add_argument("values")
    ap.add_argument("--workload", default="panel")
    ap.add_argument("--density", type=float, default=0.5)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    knobs = a.knob.split("+")
    vals = a.values.split(",")
    setting = {v: [int(x) for x in v.split(":")] for v in vals}
    assert all(len(x) == len(knobs) for x in setting.values()), "one value per knob"
    dev = torch.device("cuda", 0)
    args = types.SimpleNamespace(seed=0, k=4096, n=4096, m=4096, dtype="f16")
    if a.workload == "panel":
        prob = bench.dsd_panel(args, 1, 0, dev, 0.02, m_total=131072)
    elif a.workload in ("dds", "pair"):  # config 3's DDS (g . C) or the whole pair
        pp = bench.PairProblem(4096, a.density, "f16", 7, dev)
        if a.workload == "pair":
            prob = pp
        else:
            cg = sp.Matrix(4096, 4096, pp.g)
            co = sp.Matrix(4096, 4096, pp.out)
            prob = types.SimpleNamespace(
                launcher=lambda: (lambda: sp.MatmulEx(cg, False, pp.C, False, co)))
    elif a.workload in ("moe_sdd", "moe_dsd", "moe", "moe_sdd_nt"):  # config 4's products / step
        mp = bench.MoeProblem("bf16", 7, dev)
        t, dm, cols = mp.dims
        X, W1 = sp.Matrix(t, dm, mp.x), sp.Matrix(dm, cols, mp.w1)
        if a.workload == "moe_sdd_nt":  # MegaBlocks' w1 layout [E d_ff][d_model]
            w1t = mp.w1.view(dm, cols).t().contiguous()
            W1T = sp.Matrix(cols, dm, w1t)
            nt = lambda: sp.Matmul(X, False, W1T, True, mp.H)  # noqa: E731
        W2, Y = sp.Matrix(cols, dm, mp.w2), sp.Matrix(t, dm, mp.y)
        sdd = lambda: sp.Matmul(X, False, W1, False, mp.H)  # noqa: E731
        dsd = lambda: sp.MatmulEx(mp.H, False, W2, False, Y)  # noqa: E731
        f = {"moe_sdd": sdd, "moe_dsd": dsd}.get(a.workload, lambda: (sdd(), dsd()))
        if a.workload == "moe_sdd_nt":
            f = nt
        prob = types.SimpleNamespace(launcher=lambda: f)
    elif a.workload.startswith("op:"):  # op:OP:TRANS:DIM, e.g. op:sdd:NN:4096
        _, op, tr, dim = a.workload.split(":")
        oa = types.SimpleNamespace(k=int(dim), density=a.density, op=op, trans=tr,
                                   seed=0, dtype="f16", api="ex")
        prob = bench.OpProblem(oa, dev)
    else:
        prob = bench.dsd_panel(args, 1, 0, dev, a.density, m_total=4096)
    res = {v: [] for v in vals}
    prev = [sp.tuning(k) for k in knobs]
    try:
        for _ in range(a.rounds):
            for v in vals:
                for k, x in zip(knobs, setting[v]):
                    sp.tuning(k, x)
                fn = prob.launcher()
                for _ in range(5):
                    fn()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.iters):
                    fn()
                e.record()
                torch.cuda.synchronize()
                res[v].append(s.elapsed_time(e) * 1e3 / a.iters)
    finally:
        for k, x in zip(knobs, prev):
            sp.tuning(k, x)
    out = {"knob": a.knob, "workload": a.workload, "density": a.density,
           "us_median": {v: round(sorted(x)[len(x) // 2], 2) for v, x in res.items()},
           "us_min": {v: round(min(x), 2) for v, x in res.items()}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
