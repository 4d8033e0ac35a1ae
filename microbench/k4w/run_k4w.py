"""Experiment driver: the 4-wave hand-scheduled DSD kernel (k4w.hip) against
the shipped kernel, same data, one process, interleaved timing.

python microbench/k4w/run_k4w.py [--build-only] [--density 0.5] [--uniform]
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
SO = os.path.join(HERE, "libk4w.so")


def build():
    subprocess.run([sys.executable, os.path.join(HERE, "gen_k4w.py"),
                    os.path.join(HERE, "k4w_loop.inc")], check=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared",
                    "--offload-arch=gfx950", "-save-temps=obj",
                    os.path.join(HERE, "k4w.hip"), "-o", SO], check=True, cwd=HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build-only", action="store_true")
    ap.add_argument("--density", type=float, default=0.5)
    ap.add_argument("--uniform", action="store_true",
                    help="every block-row holds the same number of blocks")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--calls", type=int, default=50)
    ap.add_argument("--dtype", default="f16")
    ap.add_argument("--variants", default="0")
    a = ap.parse_args()
    if a.build_only:
        build()
        return
    import numpy as np
    import torch
    import bench
    from sputnik_amd import matrix_utils as mu

    dev = torch.device("cuda:0")
    d = 4096
    R = d // 128
    rng = np.random.default_rng(1)
    if a.uniform:
        per = int(round(R * a.density))
        off = np.arange(R + 1, dtype=np.int32) * per
        idx = np.concatenate([np.sort(rng.choice(R, per, replace=False))
                              for _ in range(R)]).astype(np.int32)
    else:
        nz = mu.nonzeros_for_density(d, d, a.density)
        off, idx = mu.random_topology(R, R, nz // (128 * 128), rng)
    prob = bench.DsdProblem(d, d, off, idx, d, False, False, a.dtype, 7, dev)
    ship = prob.launcher()
    lib = ctypes.CDLL(SO)
    offs_t = torch.from_numpy(np.asarray(off, np.int32)).to(dev)
    idx_t = torch.from_numpy(np.asarray(idx).astype(np.int16)).to(dev)
    c2 = torch.empty_like(prob.c_vals)
    grid = R * (d // 512)
    dbg = torch.zeros(grid * 8, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    bf = 1 if a.dtype == "bf16" else 0

    def mine(v=0):
        return lib.k4w_dsd(ctypes.c_void_p(prob.a_vals.data_ptr()),
                           ctypes.c_void_p(offs_t.data_ptr()),
                           ctypes.c_void_p(idx_t.data_ptr()),
                           ctypes.c_void_p(prob.b_vals.data_ptr()),
                           ctypes.c_void_p(c2.data_ptr()), d, d, d, bf, v,
                           ctypes.c_void_p(stream), ctypes.c_void_p(dbg.data_ptr()))

    ship()
    rc = mine()
    torch.cuda.synchronize()
    c1 = prob.c_vals.float().view(d, d)
    cm = c2.float().view(d, d)
    diff = (c1 - cm).abs()
    res = {"rc": rc, "max_abs_diff_vs_shipped": float(diff.max()),
           "rows_differing": int((diff.amax(1) > 0).sum()),
           "nan": bool(torch.isnan(cm).any())}
    # independent check: a few block-rows against fp32 torch
    A = torch.zeros(d, d, device=dev)
    av = prob.a_vals.float().view(-1, 128, 128)
    rows = np.repeat(np.arange(R), np.diff(off))
    for b in range(len(idx)):
        r, c = int(rows[b]), int(idx[b])
        A[r * 128:(r + 1) * 128, c * 128:(c + 1) * 128] = av[b]
    ref = A @ prob.b_vals.float().view(d, d)
    err = ((cm - ref).abs() / (ref.abs() + ref.pow(2).mean().sqrt())).max()
    res["max_rel_err_vs_fp32"] = float(err)
    print(json.dumps(res), flush=True)

    def timed(fn, calls):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(calls):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) * 1e3 / calls

    for _ in range(200):
        ship()
        mine()
    torch.cuda.synchronize()
    variants = [int(v) for v in a.variants.split(",")] if a.variants else [0]
    fns = {"shipped": ship}
    for v in variants:
        fns[f"k4w_v{v}"] = (lambda v=v: mine(v))
    times = {k: [] for k in fns}
    stamps = {}
    for _ in range(a.rounds):
        for k, fn in fns.items():
            times[k].append(timed(fn, a.calls))
            if k != "shipped":
                t = dbg.view(grid, 8).cpu().numpy().astype(np.float64)
                steps = 4 * np.diff(off)[0] if a.uniform else 64
                cyc = (t[:, 1] - t[:, 0])
                clk = cyc / np.maximum(t[:, 3] - t[:, 2], 1) * 0.1  # GHz
                e0 = t[:, 4].min()
                tl = {"span_us": (t[:, 6].max() - e0) / 100,
                      "entry_skew_us": (t[:, 4].max() - e0) / 100,
                      "prologue_us": np.median(t[:, 2] - t[:, 4]) / 100,
                      "loop_us": np.median(t[:, 3] - t[:, 2]) / 100,
                      "asm_epi_us": np.median(t[:, 5] - t[:, 3]) / 100,
                      "stores_us": np.median(t[:, 6] - t[:, 5]) / 100,
                      "last_loop_end_us": (t[:, 3].max() - e0) / 100,
                      "first_loop_end_us": (t[:, 3].min() - e0) / 100}
                stamps.setdefault(k, []).append((np.median(cyc) / steps, np.median(clk), tl))
    flops = prob.flops
    out = {"density": a.density, "uniform": a.uniform, "dtype": a.dtype}
    for k, ts in times.items():
        med = sorted(ts)[len(ts) // 2]
        out[k] = {"us": round(med, 2), "tflops": round(flops / med / 1e6, 1),
                  "min": round(min(ts), 2)}
        if k in stamps:
            st = sorted(stamps[k], key=lambda x: x[0])
            out[k]["cyc_per_step"] = round(st[len(st) // 2][0], 1)
            out[k]["ghz"] = round(float(np.median([x[1] for x in st])), 3)
            out[k]["timeline"] = {kk: round(float(v), 2) for kk, v in st[len(st) // 2][2].items()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
