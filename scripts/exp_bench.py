#!/usr/bin/env python3
"""Interleaved A/B timing of variant libraries (build/exp/*.so) on one
problem in one process (methodology rule: rounds interleaved, median).
Usage: exp_bench.py [--density D] [--m M] lib1.so lib2.so ..."""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--density", type=float, default=0.5)
    ap.add_argument("--m", type=int, default=4096)
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--dtype", default="f16")
    ap.add_argument("--op", default="dsd",
                    choices=["dsd", "sdd", "moe_sdd", "moe_dsd", "pair", "moe", "op"])
    # --op op: one product of bench.OpProblem (square dims = --k), MatmulEx.
    ap.add_argument("--xop", default="dsd", choices=["dsd", "dds", "sdd"])
    ap.add_argument("--trans", default="NN")
    ap.add_argument("--topo-seed", type=int, default=0)
    args = ap.parse_args()
    import torch
    import bench
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    if args.op == "op":
        import sputnik_amd as sp
        a = argparse.Namespace(op=args.xop, trans=args.trans, api="ex",
                               density=args.density, k=args.k, m=args.k,
                               n=args.k, dtype=args.dtype, seed=0)
        prob = bench.OpProblem(a, dev)
        fns = []
        for path in args.libs:
            sp._lib = None
            sp.LIB_PATH = os.path.abspath(path)
            launch = prob.launcher()
            fns.append((os.path.basename(path), lambda f=launch: f(), ()))
        args.op = f"{args.xop}_{args.trans}"
        return report(args, prob, fns)
    if args.op in ("pair", "moe"):
        # Whole BASELINE workloads (config 3 / config 4) through bench.py's
        # own launchers, one per variant library.
        import sputnik_amd as sp
        prob = (bench.PairProblem(args.k, args.density, args.dtype, 0, dev)
                if args.op == "pair" else bench.MoeProblem("bf16", 0, dev))
        fns = []
        for path in args.libs:
            sp._lib = None
            sp.LIB_PATH = os.path.abspath(path)
            launch = prob.launcher()
            fns.append((os.path.basename(path), lambda f=launch: f(), ()))
        return report(args, prob, fns)
    if args.op == "dsd":
        import numpy as np
        from sputnik_amd import matrix_utils as mu
        nz = mu.nonzeros_for_density(args.m, args.k, args.density)
        # (--topo-seed: bench.py dsd_panel's shared seed is 7919 s + seed_off,
        # 5 for config 5)
        off, idx = mu.random_topology(args.m // 128, args.k // 128,
                                      nz // (128 * 128),
                                      np.random.default_rng(args.topo_seed))
        prob = bench.DsdProblem(args.m, args.k, off, idx, args.n, False,
                                False, args.dtype, 0, dev)
        ca, cb, cc = prob.A._c(), prob.B._c(), prob.C._c()
        fname = "sputnik_dsd_ex"
    elif args.op == "sdd":
        prob = bench.PairProblem(args.k, args.density, args.dtype, 0, dev)
        import sputnik_amd as sp
        d = args.k
        ca, cb = sp.Matrix(d, d, prob.x)._c(), sp.Matrix(d, d, prob.w)._c()
        cc = prob.C._c()
        prob.flops = prob.flops / 2
        fname = "sputnik_sdd"
    else:
        prob = bench.MoeProblem("bf16", 0, dev)
        import sputnik_amd as sp
        t, dm, cols = prob.dims
        prob.flops = prob.flops / 2
        if args.op == "moe_sdd":
            ca, cb, cc = sp.Matrix(t, dm, prob.x)._c(), sp.Matrix(dm, cols, prob.w1)._c(), prob.H._c()
            fname = "sputnik_sdd"
        else:
            ca, cb, cc = prob.H._c(), sp.Matrix(cols, dm, prob.w2)._c(), sp.Matrix(t, dm, prob.y)._c()
            fname = "sputnik_dsd_ex"
    stream = torch.cuda.current_stream().cuda_stream
    fns = []
    for path in args.libs:
        L = ctypes.CDLL(os.path.abspath(path))
        fn = getattr(L, fname)
        fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                       ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                       ctypes.c_void_p]
        fn.restype = ctypes.c_int
        a = (ctypes.byref(ca), 0, ctypes.byref(cb), 0, ctypes.byref(cc),
             prob.dtype_code, stream)
        assert fn(*a) == 0, path
        fns.append((os.path.basename(path), fn, a))
    return report(args, prob, fns)


def report(args, prob, fns):
    import torch
    times = {n: [] for n, _, _ in fns}
    for _ in range(3):
        for n, fn, a in fns:
            fn(*a)
    torch.cuda.synchronize()
    for r in range(args.rounds):
        for n, fn, a in fns:
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.iters):
                fn(*a)
            e.record()
            torch.cuda.synchronize()
            times[n].append(s.elapsed_time(e) / args.iters * 1e3)
    out = {}
    for n, t in times.items():
        med = statistics.median(t)
        out[n] = {"us_median": round(med, 2), "us_min": round(min(t), 2),
                  "tflops": round(prob.flops / (med * 1e-6) / 1e12, 1)}
    print(json.dumps({"op": args.op, "density": args.density, "m": args.m, "k": args.k,
                      "n": args.n, "results": out}))


if __name__ == "__main__":
    main()
