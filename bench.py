#!/usr/bin/env python3
"""bench.py — the BASELINE.json metric on MI355X.

Metric: effective TFLOP/s (nnz-FLOPs, 2 * nnz_elements * N per DSD call,
reference sputnik/block/dsd/dsd_benchmark.cu:113-114) of DSD, block 128,
M=K=N=4096, fp16 in / fp32 accumulate / fp16 out, at density 0.5 (the
north-star point); densities 0.1/0.3/0.5/0.9 are reported in "by_density".

One step = one sputnik_dsd_ex call (C-ABI; NN, so no metadata work) over one
synthetic BCSR matrix already resident in HBM. Protocol as the reference
benchmark (dsd_benchmark.cu:82-107): 50 ms idle, W warm-up calls, K timed
calls between events; barrier + synchronize on both sides; max over ranks.

Multi-GPU (`--gpus N`, launched by torch.distributed.run): weak scaling by
row panels — every rank owns a 4096-row panel of an (N*4096) x 4096 BCSR
matrix (its own random topology) and a replicated B; no collective on the hot
path. value = nnz-FLOPs of all ranks / max-rank time.

Extra JSON objects: "roofline" (dominant kernel vs the MFMA/HBM peak),
"cpu_baseline" (the CPU oracle, timed on a bounded sample on rank 0 at N=1).
"""

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_MFMA_TFLOPS = 2500.0  # fp16/bf16 dense, MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0      # HBM3E spec
BLOCK = 128


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=100,
                    help="untimed calls first; >= ~10 ms of work so the clock "
                         "has settled (the reference used 10 short calls)")
    ap.add_argument("--workload", default="dsd",
                    choices=["dsd", "sdd_dds", "moe", "panel"],
                    help="dsd: the headline metric (BASELINE config 2); "
                         "sdd_dds: config 3; moe: config 4; panel: config 5")
    ap.add_argument("--m", type=int, default=4096, help="rows per rank")
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--density", type=float, default=0.5)
    ap.add_argument("--sweep", default="0.1,0.3,0.5,0.9",
                    help="densities for by_density ('' to skip)")
    ap.add_argument("--dtype", default="f16", choices=["f16", "bf16"])
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_latest.json"),
                    help="HBM traffic per launch measured by rocprofv3 --pmc")
    return ap.parse_args()


class Problem:
    """One rank's DSD operands on the device (+ host copies for the CPU leg)."""

    def __init__(self, m, k, n, density, dtype, seed, device):
        import torch
        import sputnik_amd as sp
        from sputnik_amd import matrix_utils as mu

        rng = np.random.default_rng(seed)
        nz = mu.nonzeros_for_density(m, k, density)
        self.nb = nz // (BLOCK * BLOCK)
        self.m, self.k, self.n = m, k, n
        self.offsets, self.indices = mu.random_topology(
            m // BLOCK, k // BLOCK, self.nb, rng)
        td = torch.float16 if dtype == "f16" else torch.bfloat16
        # Values drawn on the device (U(-1,1)); only topology comes from host.
        gen = torch.Generator(device=device)
        gen.manual_seed(seed)
        self.a_vals = (torch.rand(self.nb * BLOCK * BLOCK, generator=gen,
                                  device=device) * 2 - 1).to(td)
        self.b_vals = (torch.rand(k * n, generator=gen, device=device) * 2 - 1
                       ).to(td)
        self.c_vals = torch.empty(m * n, dtype=td, device=device)
        self.A = sp.BlockMatrix(
            m, k, 128, nz, self.a_vals,
            torch.from_numpy(self.offsets).to(device),
            torch.from_numpy(self.indices.astype(np.int16)).to(device))
        self.B = sp.Matrix(k, n, self.b_vals)
        self.C = sp.Matrix(m, n, self.c_vals)
        self.flops = 2.0 * nz * n
        # Algorithmic HBM bytes of one call: sparse values + metadata +
        # dense B + dense C.
        self.bytes = nz * 2 + (m // BLOCK + 1) * 4 + self.nb * 2 + k * n * 2 + m * n * 2
        self.dtype_code = 0 if dtype == "f16" else 1

    def launcher(self):
        import torch
        import sputnik_amd as sp

        L = sp.lib()
        ca, cb, cc = self.A._c(), self.B._c(), self.C._c()
        stream = torch.cuda.current_stream().cuda_stream
        fn = L.sputnik_dsd_ex
        args = (ctypes.byref(ca), 0, ctypes.byref(cb), 0, ctypes.byref(cc),
                self.dtype_code, stream)
        code = fn(*args)
        if code != 0:
            raise RuntimeError(f"sputnik_dsd_ex returned {code}")
        self._keep = (ca, cb, cc)
        return lambda: fn(*args)


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def time_steps(fn, steps, warmup, world):
    import torch

    time.sleep(0.05)  # reference cool-down (dsd_benchmark.cu:89)
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    start = torch.cuda.Event(enable_timing=True)
    end = torch.cuda.Event(enable_timing=True)
    start.record()
    for _ in range(steps):
        fn()
    end.record()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    return start.elapsed_time(end)  # ms, this rank


def max_over_ranks(x, world):
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def cpu_baseline(prob: Problem, budget_s: float):
    """The CPU oracle (reference host matmul restated, zero blocks skipped)
    on a bounded sample of the same DSD: the first block-rows of A, all of N."""
    import torch
    from oracle import oracle as O
    from sputnik_amd import matrix_utils as mu

    threads = max(1, min(16, os.cpu_count() or 1))
    b = prob.b_vals.float().cpu().numpy().reshape(prob.k, prob.n)
    a_vals = prob.a_vals.float().cpu().numpy().reshape(-1, BLOCK, BLOCK)
    mask = mu.block_mask(prob.offsets, prob.indices, prob.k // BLOCK)

    def run(r0, r1):
        o0, o1 = prob.offsets[r0], prob.offsets[r1]
        sub_off = prob.offsets[r0:r1 + 1] - o0
        dense = mu.to_dense((r1 - r0) * BLOCK, prob.k, sub_off,
                            prob.indices[o0:o1], a_vals[o0:o1])
        t0 = time.perf_counter()
        O.gemm(dense, False, b, False, a_mask=mask[r0:r1], threads=threads)
        dt = time.perf_counter() - t0
        return dt, 2.0 * (o1 - o0) * BLOCK * BLOCK * prob.n

    rows = max(1, min(threads, prob.m // BLOCK))
    dt, fl = run(0, rows)
    # Scale the sample to roughly the budget (at least the probe itself).
    per_row = dt / rows
    more = int(max(0.0, budget_s - dt) / max(per_row, 1e-9))
    r1 = min(prob.m // BLOCK, rows + more)
    total_dt, total_fl = dt, fl
    if r1 > rows:
        d2, f2 = run(rows, r1)
        total_dt += d2
        total_fl += f2
    return {
        "value": total_fl / total_dt / 1e12,
        "unit": "TFLOP/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"DSD block-rows 0..{r1 - 1} of {prob.m // BLOCK} "
                   f"(x all N={prob.n}), {total_fl / 1e9:.2f} nnz-GFLOP in "
                   f"{total_dt:.1f} s, oracle/oracle.c oracle_gemm with "
                   f"OpenMP over rows, fp32 in / double acc"),
    }

class PairProblem:
    """BASELINE config 3: MegaBlocks forward/backward pair at 4096^3, 20%:
    SDD  C_bcsr = x . w (sparse output), then DDS  out = g . C_bcsr (C's
    transposed metadata precomputed, as MegaBlocks caches it per topology).
    FLOPs = 2 nnz K (SDD) + 2 nnz M (DDS)."""

    def __init__(self, dim, density, dtype, seed, device):
        import torch
        import sputnik_amd as sp
        from sputnik_amd import matrix_utils as mu
        rng = np.random.default_rng(seed)
        nz = mu.nonzeros_for_density(dim, dim, density)
        nb = nz // (BLOCK * BLOCK)
        off, idx = mu.random_topology(dim // BLOCK, dim // BLOCK, nb, rng)
        td = torch.float16 if dtype == "f16" else torch.bfloat16
        gen = torch.Generator(device=device)
        gen.manual_seed(seed)
        rnd = lambda n: (torch.rand(n, generator=gen, device=device) * 2 - 1).to(td)
        self.x, self.w, self.g = rnd(dim * dim), rnd(dim * dim), rnd(dim * dim)
        self.out = torch.empty(dim * dim, dtype=td, device=device)
        self.cv = torch.empty(nz, dtype=td, device=device)
        self.C = sp.BlockMatrix(dim, dim, 128, nz, self.cv,
                                torch.from_numpy(off).to(device),
                                torch.from_numpy(idx.astype(np.int16)).to(device))
        sp.AllocateRowIndicesBuffer(self.C)
        sp.RowIndices(self.C, self.C.row_indices)
        sp.AllocateTransposeBuffers(self.C)
        sp.Transpose(self.C)
        self.dim, self.nb = dim, nb
        self.flops = 2.0 * nz * dim * 2
        self.dtype_code = 0 if dtype == "f16" else 1
        self.desc = (f"SDD(x,w)->C then DDS(g,C) block=128 M=K=N={dim} "
                     f"density={density} {dtype} (MatmulEx metadata)")

    def launcher(self):
        import torch
        import sputnik_amd as sp
        L = sp.lib()
        d = self.dim
        cx, cw, cg, co = (sp.Matrix(d, d, t)._c() for t in (self.x, self.w, self.g, self.out))
        cC = self.C._c()
        stream = torch.cuda.current_stream().cuda_stream
        a1 = (ctypes.byref(cx), 0, ctypes.byref(cw), 0, ctypes.byref(cC), self.dtype_code, stream)
        a2 = (ctypes.byref(cg), 0, ctypes.byref(cC), 0, ctypes.byref(co), self.dtype_code, stream)
        assert L.sputnik_sdd(*a1) == 0 and L.sputnik_dds_ex(*a2) == 0
        self._keep = (cx, cw, cg, co, cC)
        return lambda: (L.sputnik_sdd(*a1), L.sputnik_dds_ex(*a2))


class MoeProblem:
    """BASELINE config 4: MegaBlocks dMoE MLP, 8 experts, 8192 tokens,
    d_model 4096, d_ff 14336, bf16. Block-diagonal-by-expert topology:
    64 block-rows x 896 block-cols, 8 x 112 blocks per expert (12.5%).
    One step = SDD h = x . w1 at the expert blocks + DSD y = h . w2."""

    def __init__(self, dtype, seed, device, experts=8, tokens=8192,
                 d_model=4096, d_ff=14336):
        import torch
        import sputnik_amd as sp
        from sputnik_amd import matrix_utils as mu
        rpe = tokens // experts // BLOCK
        cpe = d_ff // BLOCK
        off, idx = mu.expert_block_diagonal(experts, rpe, cpe)
        nb = int(off[-1])
        nz = nb * BLOCK * BLOCK
        cols = experts * d_ff
        td = torch.float16 if dtype == "f16" else torch.bfloat16
        gen = torch.Generator(device=device)
        gen.manual_seed(seed)
        rnd = lambda n: (torch.rand(n, generator=gen, device=device) * 2 - 1).to(td)
        self.x = rnd(tokens * d_model)
        self.w1 = rnd(d_model * cols)
        self.w2 = rnd(cols * d_model)
        self.y = torch.empty(tokens * d_model, dtype=td, device=device)
        self.hv = torch.empty(nz, dtype=td, device=device)
        self.H = sp.BlockMatrix(tokens, cols, 128, nz, self.hv,
                                torch.from_numpy(off).to(device),
                                torch.from_numpy(idx.astype(np.int16)).to(device))
        sp.AllocateRowIndicesBuffer(self.H)
        sp.RowIndices(self.H, self.H.row_indices)
        self.dims = (tokens, d_model, cols)
        self.flops = 2.0 * nz * d_model * 2
        self.dtype_code = 0 if dtype == "f16" else 1
        self.dtype_name = dtype
        self.desc = (f"MoE {experts} experts tokens={tokens} d_model={d_model} "
                     f"d_ff={d_ff} {dtype}: SDD(x,w1)->h + DSD(h,w2)")

    def launcher(self):
        import torch
        import sputnik_amd as sp
        L = sp.lib()
        t, dm, cols = self.dims
        cx = sp.Matrix(t, dm, self.x)._c()
        c1 = sp.Matrix(dm, cols, self.w1)._c()
        c2 = sp.Matrix(cols, dm, self.w2)._c()
        cy = sp.Matrix(t, dm, self.y)._c()
        cH = self.H._c()
        stream = torch.cuda.current_stream().cuda_stream
        a1 = (ctypes.byref(cx), 0, ctypes.byref(c1), 0, ctypes.byref(cH), self.dtype_code, stream)
        a2 = (ctypes.byref(cH), 0, ctypes.byref(c2), 0, ctypes.byref(cy), self.dtype_code, stream)
        assert L.sputnik_sdd(*a1) == 0 and L.sputnik_dsd_ex(*a2) == 0
        self._keep = (cx, c1, c2, cy, cH)
        return lambda: (L.sputnik_sdd(*a1), L.sputnik_dsd_ex(*a2))


def run_other(args, world, rank, device):
    """Non-headline BASELINE configs: one JSON line each (same contract)."""
    import torch
    if args.workload == "sdd_dds":
        prob = PairProblem(args.k, 0.2, args.dtype, args.seed * 7919 + rank, device)
        metric = "effective TFLOP/s (nnz-FLOPs) SDD+DDS pair block=128 M=K=N=4096 20%"
    elif args.workload == "moe":
        prob = MoeProblem("bf16", args.seed * 7919 + rank, device)
        metric = "effective TFLOP/s (nnz-FLOPs) MoE SDD+DSD 8 experts bf16"
    else:  # panel: config 5, M=131072 total, row panels over ranks
        m_rank = 131072 // world
        prob = Problem(m_rank, 4096, 4096, 0.02, args.dtype,
                       args.seed * 7919 + rank, device)
        prob.desc = (f"DSD block=128 M=131072 (/{world} ranks = {m_rank}) K=N=4096 "
                     f"density=0.02 {args.dtype}")
        metric = "effective TFLOP/s (nnz-FLOPs) row-panel DSD M=131072 K=N=4096 2%"
    fn = prob.launcher()
    ms = max_over_ranks(time_steps(fn, args.steps, args.warmup, world), world)
    per = ms / args.steps
    tflops = prob.flops * world / (per * 1e-3) / 1e12
    extra = {}
    if args.workload == "panel" and world > 1:
        # Optional gather of the dense result (config 5): reported beside the
        # hot path, never inside it.
        import torch.distributed as dist
        full = torch.empty(world * prob.c_vals.numel(), dtype=prob.c_vals.dtype,
                           device=device)
        dist.all_gather_into_tensor(full, prob.c_vals)
        torch.cuda.synchronize()
        barrier(world)
        t0 = time.perf_counter()
        for _ in range(5):
            dist.all_gather_into_tensor(full, prob.c_vals)
        torch.cuda.synchronize()
        ag = max_over_ranks((time.perf_counter() - t0) / 5 * 1e3, world)
        extra["allgather_ms"] = round(ag, 4)
        extra["allgather_GBps_per_rank"] = round(
            full.numel() * full.element_size() * (world - 1) / world / (ag * 1e-3) / 1e9, 1)
        del full
    if rank == 0:
        print(json.dumps({**extra,
            "metric": metric, "value": round(tflops, 2), "unit": "TFLOP/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(per, 5), "higher_is_better": True,
            "scaling": "weak" if args.workload != "panel" else "strong",
            "vs_baseline": None,
            "dtype": getattr(prob, "dtype_name", args.dtype),
            "data": "synthetic", "config": {"workload": prob.desc},
        }))


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}",
              file=sys.stderr)

    import torch
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=device)

    if args.workload != "dsd":
        run_other(args, world, rank, device)
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return

    # Headline density first, then the sweep.
    densities = [args.density] + [float(d) for d in args.sweep.split(",")
                                  if d and float(d) != args.density]
    results = {}
    head = None
    for d in densities:
        prob = Problem(args.m, args.k, args.n, d, args.dtype,
                       args.seed * 7919 + rank, device)
        fn = prob.launcher()
        ms = time_steps(fn, args.steps, args.warmup, world)
        ms = max_over_ranks(ms, world)
        per_step = ms / args.steps
        tflops = prob.flops * world / (per_step * 1e-3) / 1e12
        results[d] = {"value": round(tflops, 2), "ms_per_step": round(per_step, 5),
                      "nnz_blocks_per_rank": prob.nb}
        if head is None:
            head = (prob, per_step, tflops)
        else:
            del prob
        torch.cuda.empty_cache()

    prob, per_step, tflops = head
    # Dominant (only) kernel of a step: block_gemm DSD NN. One launch per
    # step, so the event-timed average over the K launches is its duration.
    kernel_s = per_step * 1e-3
    achieved = prob.flops / kernel_s / 1e12
    traffic = None
    if os.path.exists(args.pmc):
        try:
            with open(args.pmc) as f:
                pmc = json.load(f)
            key = f"dsd_{args.m}x{args.k}x{args.n}_{args.density}_{args.dtype}"
            traffic = pmc.get(key, {}).get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None
    roofline = {
        "bound": "mfma",
        "achieved": round(achieved, 2),
        "peak": PEAK_MFMA_TFLOPS,
        "unit": "TFLOP/s",
        "frac": round(achieved / PEAK_MFMA_TFLOPS, 4),
        "traffic": traffic,
        "kernel": "block_gemm_kernel<f16, DSD NN, CfgWide8S: 128x512 tile, staggered>",
        "algorithmic_bytes": prob.bytes,
        "algorithmic_flops": prob.flops,
    }

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(prob, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "effective TFLOP/s (nnz-FLOPs) DSD block=128 M=K=N=4096 "
                      "@ 1/2/4/8 GPU vs density",
            "value": round(tflops, 2),
            "unit": "TFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(per_step, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (RANDOM_UNIFORM block topology, U(-1,1) values)",
            "config": {
                "workload": f"DSD block=128 M={args.m}/rank K={args.k} "
                            f"N={args.n} density={args.density} "
                            f"{args.dtype} (NN, MatmulEx)",
                "block": 128, "m_per_rank": args.m, "k": args.k, "n": args.n,
                "density": args.density,
                "parallelism": f"row-panel x{world}, no collective",
            },
            "by_density": {str(k): v for k, v in results.items()},
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))

    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
