#!/usr/bin/env python3
"""Same-process A/B of the 4-wave grouped SDD past its row-stride gate
(tuning knob "sdd4w_max_ld", dsd4w.hip Sdd4wApplies): the MoE step (BASELINE
config 4, SDD x.w1 with w1's 224 KiB rows + DSD h.w2), its SDD alone, and
SDD NN / TN at 16384^3 50% (32 KiB rows), knob at its default (16384 B:
the 8-wave kernel there) vs 2^30 (the 4-wave kernel). Interleaved rounds,
medians. Usage: exp_sdd_gate.py [rounds]"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    import torch
    import bench
    import sputnik_amd as sp
    dev = torch.device("cuda", 0)
    L = sp.lib()
    moe = bench.MoeProblem("bf16", 0, dev)
    step = moe.launcher()
    t, dm, cols = moe.dims
    cx = sp.Matrix(t, dm, moe.x)._c()
    c1 = sp.Matrix(dm, cols, moe.w1)._c()
    cH = moe.H._c()
    stream = torch.cuda.current_stream().cuda_stream
    a1 = (ctypes.byref(cx), 0, ctypes.byref(c1), 0, ctypes.byref(cH), 1, stream)
    cases = {"moe_step": (step, moe.flops), "moe_sdd": (lambda: L.sputnik_sdd(*a1),
                                                        moe.flops / 2)}
    for tr in ("NN", "TN"):
        ns = argparse.Namespace(op="sdd", trans=tr, api="ex", k=16384, density=0.5,
                                dtype="f16", seed=0)
        prob = bench.OpProblem(ns, dev)
        cases[f"sdd_{tr}_16384"] = (prob.launcher(), prob.flops)
    arms = {"gate": 16384, "open": 1 << 30}

    def timed(fn, n):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) * 1e3 / n

    for name, (fn, flops) in cases.items():
        n = 3 if "16384" in name else 20
        res = {k: [] for k in arms}
        for k, v in arms.items():
            sp.tuning("sdd4w_max_ld", v)
            timed(fn, n)
        for _ in range(rounds):
            for k, v in arms.items():
                sp.tuning("sdd4w_max_ld", v)
                res[k].append(timed(fn, n))
        sp.tuning("sdd4w_max_ld", 16384)
        med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
        print(json.dumps({"case": name, **{k: {"us": round(m, 2),
                                                 "tflops": round(flops / m / 1e6, 1)}
                                             for k, m in med.items()}}), flush=True)


if __name__ == "__main__":
    main()
