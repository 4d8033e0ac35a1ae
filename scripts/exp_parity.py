#!/usr/bin/env python3
"""Bitwise comparison of variant libraries (build/exp/*.so) against the first
one on the products the staggered block loop serves: DSD / DDS x NN/TN/TT
(MatmulEx) at 4096^3 and densities 0.5 / 0.1 (pair launches), plus DSD at
M = 512 (split mode). Variants that only move instructions must agree bit
for bit with the base library; prints one JSON line per case.
Usage: exp_parity.py base.so variant.so ..."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    libs = sys.argv[1:]
    import torch
    import bench
    import sputnik_amd as sp
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    bad = 0
    cases = [(op, tr, d, k) for op in ("dsd", "dds") for tr in ("NN", "TN", "NT", "TT")
             for d in (0.5, 0.1) for k in (4096,)]
    for op, tr, dens, k in cases:
        a = argparse.Namespace(op=op, trans=tr, api="ex", density=dens, k=k,
                               m=k, n=k, dtype="f16", seed=1)
        prob = bench.OpProblem(a, dev)
        outs = []
        for path in libs:
            sp._lib = None
            sp.LIB_PATH = os.path.abspath(path)
            prob.out.fill_(float("nan"))
            f = prob.launcher()
            f()
            torch.cuda.synchronize()
            outs.append(prob.out.clone())
        res = {os.path.basename(p): bool(torch.equal(o.view(torch.int16), outs[0].view(torch.int16)))
               for p, o in zip(libs[1:], outs[1:])}
        finite = bool(torch.isfinite(outs[0].float()).all())
        bad += sum(not v for v in res.values()) + (not finite)
        print(json.dumps({"case": f"{op} {tr} {dens}", "finite": finite, "equal": res}), flush=True)
    # split mode (few-row panels) and persistent tall launches
    import numpy as np
    from sputnik_amd import matrix_utils as mu
    for m, dens in ((512, 0.5), (1024, 0.5), (65536, 0.02), (32768, 0.3)):
        nz = mu.nonzeros_for_density(m, 4096, dens)
        off, idx = mu.random_topology(m // 128, 32, nz // (128 * 128), np.random.default_rng(3))
        prob = bench.DsdProblem(m, 4096, off, idx, 4096, False, False, "f16", 0, dev)
        outs = []
        for path in libs:
            sp._lib = None
            sp.LIB_PATH = os.path.abspath(path)
            f = prob.launcher()
            f()
            torch.cuda.synchronize()
            outs.append(prob.c_vals.clone())
        res = {os.path.basename(p): bool(torch.equal(o, outs[0])) for p, o in zip(libs[1:], outs[1:])}
        bad += sum(not v for v in res.values())
        print(json.dumps({"case": f"dsd M={m} {dens}", "equal": res}), flush=True)
    print(json.dumps({"mismatches": bad}))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
