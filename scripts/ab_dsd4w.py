"""Same-process A/B of the DSD NN kernels: the 4-wave hand-scheduled kernel
(dsd4w.hip) vs the 8-wave block_gemm_kernel, on the headline problem
(bench.py's DsdProblem, 4096^3, random uniform topology) at each density.
Interleaved rounds of `calls` back-to-back launches; medians.

python scripts/ab_dsd4w.py [--densities 0.5,0.1,0.3,0.9] [--rounds 7]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--densities", default="0.5,0.1,0.3,0.9")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--calls", type=int, default=50)
    ap.add_argument("--dtype", default="f16")
    ap.add_argument("--dim", type=int, default=4096)
    ap.add_argument("--op", default="dsd", choices=["dsd", "dds", "sdd"],  # (--trans: OpProblem)
                    help="dds / sdd: bench.py's OpProblem DDS NN / SDD NN")
    ap.add_argument("--trans", default="NN")
    ap.add_argument("--m", type=int, default=0, help="DSD NN: rows of A (default --dim)")
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    import sputnik_amd as sp
    from sputnik_amd import matrix_utils as mu

    dev = torch.device("cuda:0")
    d = a.dim
    for dens in [float(x) for x in a.densities.split(",")]:
        rng = np.random.default_rng(1)
        nz = mu.nonzeros_for_density(d, d, dens)
        mr = a.m or d
        nz = mu.nonzeros_for_density(mr, d, dens)
        off, idx = mu.random_topology(mr // 128, d // 128, nz // 16384, rng)
        if a.op in ("dds", "sdd") or a.trans != "NN":
            ns = argparse.Namespace(op=a.op, trans=a.trans, api="ex", k=d,
                                    density=dens, dtype=a.dtype, seed=0)
            prob = bench.OpProblem(ns, dev)
        else:
            prob = bench.DsdProblem(mr, d, off, idx, d, False, False, a.dtype, 7, dev)
        fn = prob.launcher()

        def timed(four):
            sp.select_dsd_kernel(four)
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.calls):
                fn()
            e.record()
            torch.cuda.synchronize()
            return s.elapsed_time(e) * 1e3 / a.calls

        arms = ({"8wave": 0, "4wave": 5, "4wave_bar2": 6} if a.op == "sdd"
                else {"8wave": 0, "4wave_ds": 5, "4wave_bar2": 6, "4wave_il": 7})
        for mode in arms.values():
            timed(mode)
            for _ in range(100):
                fn()
        torch.cuda.synchronize()
        ts = {k: [] for k in arms}
        for _ in range(a.rounds):
            for k, mode in arms.items():
                ts[k].append(timed(mode))
        sp.select_dsd_kernel(1)
        med = lambda v: sorted(v)[len(v) // 2]
        out = {"op": a.op, "trans": a.trans, "density": dens, "dtype": a.dtype, "dim": d}
        for k, v in ts.items():
            out[k] = {"us": round(med(v), 2),
                      "tflops": round(prob.flops / med(v) / 1e6, 1),
                      "min": round(min(v), 2)}
        out["pair_errors"] = sp.pair_errors()
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
