#!/usr/bin/env python3
"""bench.py — the BASELINE.json metric on MI355X.

Metric: effective TFLOP/s (nnz-FLOPs, 2 * nnz_elements * N per DSD call,
reference sputnik/block/dsd/dsd_benchmark.cu:113-114) of DSD, block 128,
M=K=N=4096, fp16 in / fp32 accumulate / fp16 out, at density 0.5 (the
north-star point); densities 0.1/0.3/0.5/0.9 are reported in "by_density",
each with its own roofline (MFMA- or HBM-bound by arithmetic intensity).

One step = one sputnik_dsd_ex call (C-ABI; NN, so no metadata work) over one
synthetic BCSR matrix already resident in HBM. Protocol as the reference
benchmark (dsd_benchmark.cu:82-107): 50 ms idle, W warm-up calls, K timed
calls between HIP events on the launch stream; barrier + synchronize on both
sides; max over ranks.

Multi-GPU (`--gpus N`, launched by torch.distributed.run): one BCSR matrix
(the same topology on every rank, from a shared seed) is split with the
library's own shard_rows_by_nnz / slice_block_rows; every rank
runs its row panel against a replicated B; no collective on the hot path.
`--scaling strong` (the default): the matrix is the metric's own M=K=N=4096,
so N ranks share its 32 block-rows (BASELINE metric "DSD M=K=N=4096 @
1/2/4/8 GPU"). `--scaling weak`: N x 4096 rows, 4096 per rank. Either way
value = nnz-FLOPs of all ranks / max-rank time.

Other workloads (`--workload`): sdd_dds (config 3), moe (config 4), panel
(config 5: M=131072 split over the ranks, strong scaling), op (one product
and transpose: --op dsd|dds|sdd --trans NN|NT|TN|TT, --api ex|matmul; with
matmul the device Transpose runs inside every DSD TN/TT and DDS NN/TN step)
and transpose (the device Transpose alone).

Extra JSON objects: "roofline" (dominant kernel vs its MFMA or HBM roof),
"dense_anchor" (torch.matmul -> hipBLASLt on a dense GEMM of the same FLOPs,
timed beside it: what this GPU's matrix cores reach under the same clocks),
"cpu_baseline" (the CPU oracle on a bounded sample, 1 thread and all
allotted threads, rank 0 at N=1), "config1" (BASELINE config 1: the host
reference matmul at 512^3, 50%), "build" (library source hash vs the tree).
"""

import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_MFMA_TFLOPS = 2500.0  # fp16/bf16 dense, MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0      # HBM3E spec, MI355X_MICROARCH.md
RIDGE = PEAK_MFMA_TFLOPS * 1e12 / (PEAK_HBM_GBS * 1e9)  # 312.5 FLOP/B
BLOCK = 128
METRIC = ("effective TFLOP/s (nnz-FLOPs) DSD block=128 M=K=N=4096 "
          "@ 1/2/4/8 GPU vs density")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default 100; sdd_dds 1000, panel 500)")
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed calls first (default as --steps). The chip's "
                         "power management settles over ~100 ms of load, not "
                         "monotonically (DESIGN 5: 20 headline steps after 5 / "
                         "50 / 200 warmups ran 57.1 / 74.0 / 61.5 us on one box), "
                         "so the short workloads default to >= 100 ms of each")
    ap.add_argument("--workload", default="dsd",
                    choices=["dsd", "sdd_dds", "moe", "panel", "op",
                             "transpose", "sweep"],
                    help="dsd: the headline metric (BASELINE config 2); "
                         "sdd_dds: config 3; moe: config 4; panel: config 5; "
                         "op: one product/transpose; transpose: metadata")
    ap.add_argument("--graph", action="store_true",
                    help="time replays of a hipGraph captured around one step "
                         "(captured launches use a pair workspace and tile "
                         "counter of their own capture: INTEGRATION §3b)")
    ap.add_argument("--sweep-ops", default="dsd,dds,sdd")
    ap.add_argument("--sweep-dims", default="512,1024,2048,4096,8192,16384")
    ap.add_argument("--sweep-densities", default="1.0,0.5,0.1,0.01")
    ap.add_argument("--sweep-trans", default="NN,NT,TN,TT")
    ap.add_argument("--op", default="dsd", choices=["dsd", "dds", "sdd"])
    ap.add_argument("--trans", default="NN", choices=["NN", "NT", "TN", "TT"])
    ap.add_argument("--api", default="ex", choices=["ex", "matmul"])
    ap.add_argument("--m", type=int, default=4096,
                    help="rows of the DSD matrix (strong) or per rank (weak)")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="strong: ranks split one M-row matrix (the metric's "
                         "4096^3); weak: N x M rows, M per rank")
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--density", type=float, default=0.5)
    ap.add_argument("--sweep", default="0.1,0.3,0.5,0.9",
                    help="densities for by_density ('' to skip)")
    ap.add_argument("--dtype", default="f16", choices=["f16", "bf16"])
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=8.0,
                    help="per CPU-baseline leg (two legs)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL) on a node; gloo only for tests that "
                         "run several ranks on one device")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_latest.json"),
                    help="HBM traffic per launch measured by rocprofv3 --pmc "
                         "(scripts/pmc.sh), keyed by shape and build hash")
    ap.add_argument("--pmc-workloads",
                    default=os.path.join(ROOT, "profiles", "pmc_workloads.json"),
                    help="per-kernel PMC of the sdd_dds / moe / panel workloads "
                         "(scripts/pmc_workload.sh), keyed by workload and build hash")
    args = ap.parse_args()
    # per-workload defaults: config 3's 64-73 us step and config 5's 200 us
    # step need more steps than the headline's for >= 100 ms of load (config
    # 3: 100 + 100 steps 72.3-73.2 us, 1000 + 1000 steps 64.9 us on one box)
    dflt = {"sdd_dds": 1000, "panel": 500}.get(args.workload, 100)
    if args.steps is None:
        args.steps = dflt
    if args.warmup is None:
        args.warmup = dflt
    return args


# ------------------------------------------------------------------ build --

def check_build():
    """The library's compiled-in source hash against the tree bench.py runs
    in; a stale library is rebuilt (hipcc is on the GPU box too)."""
    from sputnik_amd import srchash
    want = srchash.source_hash()
    import sputnik_amd as sp
    got = sp.build_hash() if os.path.exists(sp.LIB_PATH) else None
    rebuilt = False
    if got != want:
        print(f"bench: libsputnik.so built from {got}, tree is {want}: "
              "rebuilding", file=sys.stderr)
        subprocess.run(["make", "-s", "-j", "16", "-C",
                        os.path.join(ROOT, "sputnik_amd")], check=True)
        rebuilt = True
        # A fresh process loads the rebuilt library; this one reports it.
        got = subprocess.run(
            [sys.executable, "-c",
             "import sputnik_amd as s; print(s.build_hash())"],
            capture_output=True, text=True, cwd=ROOT).stdout.strip()
        if got == want:
            raise SystemExit(subprocess.call([sys.executable] + sys.argv))
    return {"hash": got, "source_hash": want, "matches_source": got == want,
            "rebuilt": rebuilt}


# -------------------------------------------------------------- roofline --

def roofline(flops, nbytes, seconds, kernel, traffic=None):
    """Algorithmic FLOPs / bytes of one launch over its measured duration,
    against the roof its arithmetic intensity selects."""
    ai = flops / nbytes
    tflops = flops / seconds / 1e12
    gbs = nbytes / seconds / 1e9
    if ai >= RIDGE:
        bound, achieved, peak, unit = "mfma", tflops, PEAK_MFMA_TFLOPS, "TFLOP/s"
    else:
        bound, achieved, peak, unit = "hbm", gbs, PEAK_HBM_GBS, "GB/s"
    return {
        "bound": bound, "achieved": round(achieved, 2), "peak": peak,
        "unit": unit, "frac": round(achieved / peak, 4), "traffic": traffic,
        "arithmetic_intensity": round(ai, 1),
        "tflops": round(tflops, 2),
        "mfma_frac": round(tflops / PEAK_MFMA_TFLOPS, 4),
        "algorithmic_GBps": round(gbs, 1),
        "hbm_frac": round(gbs / PEAK_HBM_GBS, 4),
        "algorithmic_flops": flops, "algorithmic_bytes": nbytes,
        "kernel": kernel,
    }


def pmc_traffic(path, key, build_hash):
    """HBM bytes per launch from the PMC summary, only when it was measured
    on this exact build (scripts/pmc.sh writes the build hash)."""
    if not os.path.exists(path):
        return None, "no PMC summary"
    try:
        with open(path) as f:
            entry = json.load(f).get(key)
    except (OSError, ValueError):
        return None, "unreadable PMC summary"
    if not entry:
        return None, f"no PMC entry for {key}"
    if entry.get("build_hash") != build_hash:
        return None, (f"PMC entry measured on build {entry.get('build_hash')}, "
                      f"not {build_hash}")
    return entry.get("hbm_bytes_per_launch"), "rocprofv3 --pmc, same build"


def pmc_workload_traffic(path, workload, build_hash):
    """L2<->fabric bytes of one step of a non-headline workload: the sum over
    the library's kernels of a step (dsd4w_kernel / block_gemm launches; the
    metadata kernels run before the timed region) of their per-launch bytes
    from scripts/pmc_workload.sh, only when measured on this exact build.
    -> (bytes or None, per-kernel dict, note)."""
    try:
        with open(path) as f:
            entry = json.load(f).get(workload)
    except (OSError, ValueError):
        return None, None, "no workload PMC summary"
    if not entry:
        return None, None, f"no workload PMC entry for {workload}"
    if entry.get("build_hash") != build_hash:
        return None, None, (f"PMC entry measured on build {entry.get('build_hash')}, "
                            f"not {build_hash}")
    per = {k: {"bytes": v.get("hbm_bytes_per_launch"), "us": v.get("profiled_kernel_us"),
               "mfma_busy_frac": v.get("mfma_busy_frac"), "l2_hit": v.get("l2_hit")}
           for k, v in entry.get("kernels", {}).items()
           if ("dsd4w_kernel" in k or "block_gemm" in k) and
           v.get("hbm_bytes_per_launch") is not None}
    if not per:
        return None, None, "no library kernel in the workload PMC entry"
    return (sum(v["bytes"] for v in per.values()), per,
            "rocprofv3 --pmc (scripts/pmc_workload.sh), same build, summed over the step's kernels")


PEAK_CLOCK_GHZ = 2.4  # MI355X peak engine clock (the 2.5 PF dense fp16 figure)


def pmc_clock(path, key, build_hash, achieved_tflops, peak_tflops):
    """The clock and matrix-pipe busy fraction PMC measured for this exact
    build (scripts/pmc.sh), and `achieved` against the matrix peak at that
    clock (peak x clock / 2.4 GHz): the chip does not hold its peak clock
    under this load, so `frac` alone understates how full the pipe is."""
    try:
        with open(path) as f:
            entry = json.load(f).get(key)
    except (OSError, ValueError):
        return None
    if not entry or entry.get("build_hash") != build_hash:
        return None
    ghz = entry.get("est_clock_GHz")
    if not ghz:
        return None
    peak_at = peak_tflops * ghz / PEAK_CLOCK_GHZ
    return {"clock_GHz": ghz, "mfma_busy_frac": entry.get("mfma_busy_frac"),
            "profiled_kernel_us": entry.get("profiled_kernel_us"),
            "peak_at_clock": round(peak_at, 1),
            "frac_at_clock": round(achieved_tflops / peak_at, 4),
            "source": "rocprofv3 --pmc (profiles/pmc_latest.json), same build"}


# --------------------------------------------------------------- problems --

def _values(n, td, gen, device):
    import torch
    return (torch.rand(n, generator=gen, device=device) * 2 - 1).to(td)


_SDD_KERNELS = {
    0: "block_gemm_kernel (SDD, 8-wave k-split 128x128 block tile)",
    1: "block_gemm_kernel (SDD, 8-wave grouped 128x512 tiles)",
    2: "dsd4w_kernel (SDD NN, 4-wave grouped tiles, K split over workgroups)",
    3: "dsd4w_kernel (SDD, 4-wave grouped 128x512 tiles)",
    4: "transpose16_kernel (B^T -> B) + dsd4w_kernel (SDD, 4-wave grouped 128x512 tiles)",
}
_DSD_KERNELS = {
    0: "block_gemm_kernel ({op}, 8-wave 128x512 tile)",
    1: "dsd4w_kernel ({op}, 4 waves of 128x128)",
    2: "block_gemm_kernel ({op}, tall 128x256 x2 per CU)",
    3: "block_gemm_kernel ({op}, split mode)",
    4: "dsd4w_kernel ({op}, tall pipeline, persistent)",
}


def sdd_kernel_name(sp, a, ta, b, tb, c):
    """The SDD kernel the dispatcher picks (sputnik_sdd_kernel)."""
    return _SDD_KERNELS.get(sp.sdd_kernel(a, ta, b, tb, c), "rejected")


def dsd_kernel_name(sp, op, plan):
    """The DSD / DDS kernel of a dsd_plan / dds_plan code."""
    return _DSD_KERNELS.get(plan, "rejected").format(op=op)


def _td(dtype):
    import torch
    return torch.float16 if dtype == "f16" else torch.bfloat16


class DsdProblem:
    """One rank's DSD (op(A) sparse, op(B) dense) on the device, on an
    explicit topology of op(A)'s storage: A is stored [rows, cols] blocks."""

    def __init__(self, rows, cols, offsets, indices, n, ta, tb, dtype, seed,
                 device, api="ex"):
        import torch
        import sputnik_amd as sp
        self.nb = int(offsets[-1])
        nz = self.nb * BLOCK * BLOCK
        self.rows, self.cols, self.n = rows, cols, n
        self.offsets, self.indices = offsets, indices
        m, k = (cols, rows) if ta else (rows, cols)
        self.m, self.k, self.ta, self.tb, self.api = m, k, ta, tb, api
        td = _td(dtype)
        gen = torch.Generator(device=device)
        gen.manual_seed(seed)
        self.a_vals = _values(max(nz, 1), td, gen, device)
        self.b_vals = _values(k * n, td, gen, device)
        self.c_vals = torch.empty(m * n, dtype=td, device=device)
        self.A = sp.BlockMatrix(
            rows, cols, 128, nz, self.a_vals,
            torch.from_numpy(np.asarray(offsets, np.int32)).to(device),
            torch.from_numpy(np.asarray(indices).astype(np.int16)).to(device))
        if ta:
            sp.AllocateTransposeBuffers(self.A)
            sp.Transpose(self.A)
        self.B = sp.Matrix(*((n, k) if tb else (k, n)), self.b_vals)
        self.C = sp.Matrix(m, n, self.c_vals)
        self.flops = 2.0 * nz * n
        # Algorithmic HBM bytes of one call: sparse values + metadata (+ the
        # transposed metadata read in column order) + dense B + dense C.
        meta = (rows // BLOCK + 1) * 4 + self.nb * 2
        if ta:
            meta = (cols // BLOCK + 1) * 4 + self.nb * (2 + 4)
        self.bytes = nz * 2 + meta + k * n * 2 + m * n * 2
        self.dtype_code = 0 if dtype == "f16" else 1
        plan = sp.dsd_plan(self.A, ta, self.B, tb, self.C)
        tr = f"DSD {'T' if ta else 'N'}{'T' if tb else 'N'}"
        self.kernel = {
            1: f"dsd4w_kernel<{dtype}, {tr}, 128x512 tile, 4 waves of 128x128, "
               f"hand-scheduled k-loop>",
            2: f"block_gemm_kernel<{dtype}, {tr}, tall 128x256 x2 per CU>",
            3: f"block_gemm_kernel<{dtype}, {tr}, split mode>",
            4: f"dsd4w_kernel<{dtype}, {tr}, tall pipeline: 4 waves, one workgroup "
               f"per CU, 128x512 tiles stored at their last block>",
        }.get(plan, f"block_gemm_kernel<{dtype}, {tr}, 128x512 staggered tile>")

    def launcher(self):
        import torch
        import sputnik_amd as sp
        L = sp.lib()
        ca, cb, cc = self.A._c(), self.B._c(), self.C._c()
        stream = torch.cuda.current_stream().cuda_stream
        fn = L.sputnik_dsd_ex if self.api == "ex" else L.sputnik_dsd
        args = (ctypes.byref(ca), int(self.ta), ctypes.byref(cb), int(self.tb),
                ctypes.byref(cc), self.dtype_code, stream)
        code = fn(*args)
        if code != 0:
            raise RuntimeError(f"dsd returned {code}")
        self._keep = (ca, cb, cc)
        return lambda: fn(*args)


def dsd_panel(args, world, rank, device, density, m_total=None, seed_off=0):
    """The rank's row panel of one (world x m)-row BCSR matrix (or m_total
    rows), split by nnz with the library's sharding helpers."""
    from sputnik_amd import matrix_utils as mu
    rows_total = m_total if m_total is not None else args.m * world
    nz = mu.nonzeros_for_density(rows_total, args.k, density)
    rng = np.random.default_rng(args.seed * 7919 + seed_off)  # shared seed
    off, idx = mu.random_topology(rows_total // BLOCK, args.k // BLOCK,
                                  nz // (BLOCK * BLOCK), rng)
    r0, r1 = mu.shard_rows_by_nnz(off, world)[rank]
    po, pi, _ = mu.slice_block_rows(off, idx, np.zeros(len(idx)), r0, r1)
    prob = DsdProblem((r1 - r0) * BLOCK, args.k, po, pi, args.n, False, False,
                      args.dtype, args.seed * 7919 + rank, device)
    prob.panel = (r0, r1)
    prob.all_panels = mu.shard_rows_by_nnz(off, world)
    prob.total_nb = int(off[-1])
    return prob


# ------------------------------------------------------------------ timing --

def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def graph_step(prob):
    """One step of `prob` captured into a hipGraph (torch.cuda.CUDAGraph) on
    a side stream: the launcher is built on that stream, so the library's
    launches go into the capture. The returned callable replays it on the
    current stream."""
    import torch
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn = prob.launcher()  # binds s; runs once eagerly (workspaces exist)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        codes = fn()
    torch.cuda.synchronize()
    codes = codes if isinstance(codes, tuple) else (codes,)
    if any(c != 0 for c in codes):
        raise RuntimeError(f"launch inside graph capture returned {codes}")
    prob._graph = (g, fn)  # keep the captured arguments alive
    return g.replay


def time_steps(fn, steps, warmup, world):
    import torch

    time.sleep(0.05)  # reference cool-down (dsd_benchmark.cu:89)
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    # Events on the launch stream (the library launches on torch's current
    # stream, which is what the launchers pass).
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


def _reduce(x, world, op):
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    dev = "cpu" if dist.get_backend() == "gloo" else "cuda"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=op)
    return float(t.item())


def max_over_ranks(x, world):
    import torch.distributed as dist
    return _reduce(x, world, dist.ReduceOp.MAX if world > 1 else None)


def sum_over_ranks(x, world):
    import torch.distributed as dist
    return _reduce(x, world, dist.ReduceOp.SUM if world > 1 else None)


# ------------------------------------------------------------ CPU baseline --

def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def allotted_threads():
    """Threads the box allots this process: OMP_NUM_THREADS when set (16 on
    the GPU pool), else the affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_baseline(prob, budget_s):
    """The CPU oracle (the reference's host matmul restated, zero blocks
    skipped) on a bounded sample of the same DSD — the leading block-rows of
    A against all of B — on 1 thread and on every allotted thread."""
    from oracle import oracle as O
    from sputnik_amd import matrix_utils as mu

    b = prob.b_vals.float().cpu().numpy().reshape(prob.k, prob.n)
    a_vals = prob.a_vals.float().cpu().numpy().reshape(-1, BLOCK, BLOCK)
    mask = mu.block_mask(prob.offsets, prob.indices, prob.k // BLOCK)
    rows_b = prob.m // BLOCK

    def run(r0, r1, threads):
        o0, o1 = prob.offsets[r0], prob.offsets[r1]
        sub_off = prob.offsets[r0:r1 + 1] - o0
        dense = mu.to_dense((r1 - r0) * BLOCK, prob.k, sub_off,
                            prob.indices[o0:o1], a_vals[o0:o1])
        t0 = time.perf_counter()
        O.gemm(dense, False, b, False, a_mask=mask[r0:r1], threads=threads)
        return time.perf_counter() - t0, 2.0 * (o1 - o0) * BLOCK * BLOCK * prob.n

    def leg(threads):
        probe = max(1, min(threads, rows_b))
        dt, fl = run(0, probe, threads)
        per_row = dt / probe
        more = int(max(0.0, budget_s - dt) / max(per_row, 1e-9))
        more = (more // threads) * threads if threads > 1 else more
        r1 = min(rows_b, probe + more)
        if r1 > probe:
            d2, f2 = run(probe, r1, threads)
            dt, fl = dt + d2, fl + f2
        return {"value": round(fl / dt / 1e12, 6), "unit": "TFLOP/s",
                "cores": threads, "seconds": round(dt, 2),
                "gflop": round(fl / 1e9, 2), "block_rows": r1}

    threads = allotted_threads()
    single = leg(1)
    multi = leg(threads) if threads > 1 else single
    return {
        "value": multi["value"], "unit": "TFLOP/s", "cores": threads,
        "kind": "port",
        "sample": (f"DSD block-rows 0..{multi['block_rows'] - 1} of {rows_b} "
                   f"(x all N={prob.n}) of the timed problem, "
                   f"{multi['gflop']} nnz-GFLOP in {multi['seconds']} s on "
                   f"{threads} threads; oracle/oracle.c oracle_gemm "
                   "(Matrix::operator*, matrix_utils.h:376-391, zero blocks "
                   "skipped), fp32 in / double accumulate"),
        "single_core": single,
        "all_cores": multi,
        "nproc": os.cpu_count(),
        "threads_allotted": threads,
        "cpu_model": cpu_model(),
    }


def config1_host_reference():
    """BASELINE config 1: DSD block=128 M=K=N=512, 50% density, fp32, the
    reference's host path exactly (ToMatrix dense expansion, then the naive
    Matrix::operator*: no zero-block skip), 1 thread."""
    from oracle import oracle as O
    from sputnik_amd import matrix_utils as mu
    rng = np.random.default_rng(1)
    nz = mu.nonzeros_for_density(512, 512, 0.5)
    off, idx = mu.random_topology(4, 4, nz // (BLOCK * BLOCK), rng)
    vals = mu.random_values((len(idx), BLOCK, BLOCK), rng)
    b = mu.random_values((512, 512), rng)
    t0 = time.perf_counter()
    dense = O.bcsr_to_dense(512, 512, off, idx, vals)
    O.gemm(dense, False, b, False, threads=1)
    dt = time.perf_counter() - t0
    flops = 2.0 * nz * 512
    return {"metric": "effective GFLOP/s (nnz-FLOPs) DSD block=128 "
                      "M=K=N=512 50% fp32, host reference",
            "value": round(flops / dt / 1e9, 4), "unit": "GFLOP/s",
            "ms": round(dt * 1e3, 2), "cores": 1, "kind": "port",
            "cpu_model": cpu_model()}


# --------------------------------------------------- other workloads ------

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
        td = _td(dtype)
        gen = torch.Generator(device=device)
        gen.manual_seed(seed)
        self.x, self.w, self.g = (_values(dim * dim, td, gen, device)
                                  for _ in range(3))
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
        self.anchor_shape = (dim, dim, int(round(dim * density)))
        self.bytes = 2 * (nz * 2 + 2 * dim * dim * 2) + nb * 8
        self.dtype_code = 0 if dtype == "f16" else 1
        # (what the dispatcher actually picks: sputnik_sdd_kernel /
        # sputnik_dds_plan)
        X, W, G = (sp.Matrix(dim, dim, t) for t in (self.x, self.w, self.g))
        self.kernel = (sdd_kernel_name(sp, X, False, W, False, self.C) + " + " +
                       dsd_kernel_name(sp, "DDS NN", sp.dds_plan(
                           G, False, self.C, False, sp.Matrix(dim, dim, self.out))))
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
        td = _td(dtype)
        gen = torch.Generator(device=device)
        gen.manual_seed(seed)
        self.x = _values(tokens * d_model, td, gen, device)
        self.w1 = _values(d_model * cols, td, gen, device)
        self.w2 = _values(cols * d_model, td, gen, device)
        self.y = torch.empty(tokens * d_model, dtype=td, device=device)
        self.hv = torch.empty(nz, dtype=td, device=device)
        self.H = sp.BlockMatrix(tokens, cols, 128, nz, self.hv,
                                torch.from_numpy(off).to(device),
                                torch.from_numpy(idx.astype(np.int16)).to(device))
        sp.AllocateRowIndicesBuffer(self.H)
        sp.RowIndices(self.H, self.H.row_indices)
        self.dims = (tokens, d_model, cols)
        self.flops = 2.0 * nz * d_model * 2
        # Dense anchor: one GEMM of half the step's FLOPs (tokens x d_model
        # x d_ff / experts, the per-expert width), reported per GEMM.
        self.anchor_shape = (tokens, d_model, d_ff // experts)
        self.bytes = (2 * nz * 2 + tokens * d_model * 2 * 2 +
                      2 * d_model * cols * 2)
        self.dtype_code = 0 if dtype == "f16" else 1
        self.dtype_name = dtype
        X, W1 = sp.Matrix(tokens, d_model, self.x), sp.Matrix(d_model, cols, self.w1)
        W2, Y = sp.Matrix(cols, d_model, self.w2), sp.Matrix(tokens, d_model, self.y)
        self.kernel = (sdd_kernel_name(sp, X, False, W1, False, self.H) + " + " +
                       dsd_kernel_name(sp, "DSD NN", sp.dsd_plan(self.H, False, W2, False, Y)))
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


class OpProblem:
    """One product with one transpose combination at M=K=N (4096, density
    as given): DSD / DDS through MatmulEx (metadata precomputed) or Matmul
    (the device Transpose inside every step where the sparse operand is read
    in column order: DSD TN/TT, DDS NN/TN), or SDD (no metadata)."""

    def __init__(self, args, device):
        import torch
        import sputnik_amd as sp
        from sputnik_amd import matrix_utils as mu
        d, dens, op = args.k, args.density, args.op
        ta, tb = args.trans[0] == "T", args.trans[1] == "T"
        rng = np.random.default_rng(args.seed)
        nz = mu.nonzeros_for_density(d, d, dens)
        nb = nz // (BLOCK * BLOCK)
        off, idx = mu.random_topology(d // BLOCK, d // BLOCK, nb, rng)
        td = _td(args.dtype)
        gen = torch.Generator(device=device)
        gen.manual_seed(args.seed)
        self.sv = _values(nz, td, gen, device)
        self.x = _values(d * d, td, gen, device)
        self.out = torch.empty(d * d, dtype=td, device=device)
        self.S = sp.BlockMatrix(d, d, 128, nz, self.sv,
                                torch.from_numpy(off).to(device),
                                torch.from_numpy(idx.astype(np.int16)).to(device))
        sp.AllocateTransposeBuffers(self.S)
        sp.Transpose(self.S)
        self.S.create_metadata = args.api == "matmul"
        if op == "sdd":
            self.y = _values(d * d, td, gen, device)
            sp.AllocateRowIndicesBuffer(self.S)
            sp.RowIndices(self.S, self.S.row_indices)
        self.op, self.ta, self.tb, self.api = op, ta, tb, args.api
        self.flops = 2.0 * nz * d
        self.anchor_shape = (d, d, max(8, int(round(d * dens))))
        meta_t = (op == "dsd" and ta) or (op == "dds" and not tb)
        meta = (d // BLOCK + 1) * 4 + nb * (6 if meta_t else 2)
        self.bytes = (nz * 2 + meta + d * d * 2 * (2 if op == "sdd" else 1) +
                      (0 if op == "sdd" else d * d * 2))
        self.dtype_code = 0 if args.dtype == "f16" else 1
        self.meta_t = meta_t
        self.desc = (f"{op.upper()} {args.trans} block=128 M=K=N={d} "
                     f"density={dens} {args.dtype} "
                     f"({'MatmulEx' if args.api == 'ex' else 'Matmul'}"
                     f"{', device Transpose in every step' if meta_t and args.api == 'matmul' else ''})")
        # (what the dispatcher picks for this problem)
        X, O_ = sp.Matrix(d, d, self.x), sp.Matrix(d, d, self.out)
        tr = f"{op.upper()} {args.trans}"
        if op == "dsd":
            self.kernel = dsd_kernel_name(sp, tr, sp.dsd_plan(self.S, ta, X, tb, O_))
        elif op == "dds":
            self.kernel = dsd_kernel_name(sp, tr, sp.dds_plan(X, ta, self.S, tb, O_))
        else:
            self.kernel = sdd_kernel_name(sp, X, ta, sp.Matrix(d, d, self.y), tb, self.S)

    def launcher(self):
        import torch
        import sputnik_amd as sp
        L = sp.lib()
        d = self.k = self.dim = int(self.S.rows)
        cS = self.S._c()
        cx = sp.Matrix(d, d, self.x)._c()
        co = sp.Matrix(d, d, self.out)._c()
        stream = torch.cuda.current_stream().cuda_stream
        ta, tb, code = int(self.ta), int(self.tb), self.dtype_code
        if self.op == "dsd":
            fn = L.sputnik_dsd_ex if self.api == "ex" else L.sputnik_dsd
            a = (ctypes.byref(cS), ta, ctypes.byref(cx), tb, ctypes.byref(co), code, stream)
        elif self.op == "dds":
            fn = L.sputnik_dds_ex if self.api == "ex" else L.sputnik_dds
            a = (ctypes.byref(cx), ta, ctypes.byref(cS), tb, ctypes.byref(co), code, stream)
        else:
            cy = sp.Matrix(d, d, self.y)._c()
            fn = L.sputnik_sdd
            a = (ctypes.byref(cx), ta, ctypes.byref(cy), tb, ctypes.byref(cS), code, stream)
            self._y = cy
        assert fn(*a) == 0
        self._keep = (cS, cx, co)
        return lambda: fn(*a)


class TransposeProblem:
    """The device Transpose alone on the headline topology (4096^2 blocks at
    the given density): offsets_t / indices_t / block_offsets."""

    def __init__(self, args, device):
        import torch
        import sputnik_amd as sp
        from sputnik_amd import matrix_utils as mu
        d = args.k
        rng = np.random.default_rng(args.seed)
        nz = mu.nonzeros_for_density(d, d, args.density)
        nb = nz // (BLOCK * BLOCK)
        off, idx = mu.random_topology(d // BLOCK, d // BLOCK, nb, rng)
        self.S = sp.BlockMatrix(d, d, 128, nz,
                                torch.empty(1, dtype=torch.float16, device=device),
                                torch.from_numpy(off).to(device),
                                torch.from_numpy(idx.astype(np.int16)).to(device))
        sp.AllocateTransposeBuffers(self.S)
        self.flops = 0.0
        self.bytes = (d // BLOCK + 1) * 4 * 2 + nb * (2 + 2 + 4)
        self.desc = f"Transpose block=128 {d}x{d} density={args.density} ({nb} blocks)"

    def launcher(self):
        import torch
        import sputnik_amd as sp
        L = sp.lib()
        c = self.S._c()
        stream = torch.cuda.current_stream().cuda_stream
        assert L.sputnik_transpose(ctypes.byref(c), stream) == 0
        self._keep = c
        return lambda: L.sputnik_transpose(ctypes.byref(c), stream)


def run_sweep(args, device, build):
    """The reference benchmark grid (dsd_benchmark.cu:32-46 and its dds /
    sdd siblings): dims x densities x transposes per product, MatmulEx
    (metadata precomputed), fp16, one JSON line per point with the
    hipBLASLt dense GEMM of the same FLOPs beside it (density 1.0 is the
    exact dense comparison)."""
    import argparse as _ap
    import torch
    for op in [o for o in args.sweep_ops.split(",") if o]:
        for d in [int(x) for x in args.sweep_dims.split(",") if x]:
            for dens in [float(x) for x in args.sweep_densities.split(",") if x]:
                anchor = None
                for tr in [t for t in args.sweep_trans.split(",") if t]:
                    a = _ap.Namespace(**vars(args))
                    a.op, a.trans, a.api, a.density = op, tr, "ex", dens
                    a.k = a.m = a.n = d
                    try:
                        prob = OpProblem(a, device)
                        fn = prob.launcher()
                        ms = time_steps(fn, args.steps, args.warmup, 1)
                    except (RuntimeError, AssertionError) as exc:
                        emit({"op": op, "trans": tr, "dim": d, "density": dens,
                              "error": str(exc)[:200]})
                        torch.cuda.empty_cache()
                        continue
                    per = ms / args.steps
                    tflops = prob.flops / (per * 1e-3) / 1e12
                    if anchor is None:
                        anchor = dense_anchor(*prob.anchor_shape, args.dtype,
                                              device, iters=20)
                    emit({"op": op, "trans": tr, "dim": d, "density": dens,
                          "nnz_blocks": int(prob.S.nonzeros) // (BLOCK * BLOCK),
                          "us": round(per * 1e3, 2),
                          "tflops": round(tflops, 2),
                          "dense_anchor_tflops": anchor.get("tflops"),
                          "sparse_over_dense": round(tflops / anchor["tflops"], 3)
                          if "tflops" in anchor else None,
                          "build": build.get("hash")})
                    del prob, fn
                    torch.cuda.empty_cache()


def emit(line):
    print(json.dumps(line))
    sys.stdout.flush()


def run_other(args, world, rank, device, build):
    """Non-headline workloads: one JSON line each (same contract)."""
    scaling = "weak"
    if args.workload == "sdd_dds":
        prob = PairProblem(args.k, 0.2, args.dtype, args.seed * 7919 + rank, device)
        metric = "effective TFLOP/s (nnz-FLOPs) SDD+DDS pair block=128 M=K=N=4096 20%"
    elif args.workload == "moe":
        prob = MoeProblem("bf16", args.seed * 7919 + rank, device)
        metric = "effective TFLOP/s (nnz-FLOPs) MoE SDD+DSD 8 experts bf16"
    elif args.workload == "op":
        prob = OpProblem(args, device)
        metric = (f"effective TFLOP/s (nnz-FLOPs) {args.op.upper()} {args.trans} "
                  f"block=128 M=K=N={args.k} {args.density}")
    elif args.workload == "transpose":
        prob = TransposeProblem(args, device)
        metric = "microseconds per device Transpose (BCSR metadata)"
    else:  # panel: config 5, M=131072 total, row panels over ranks
        prob = dsd_panel(args, world, rank, device, 0.02, m_total=131072,
                         seed_off=5)
        r0, r1 = prob.panel
        prob.desc = (f"DSD block=128 M=131072 K=N=4096 density=0.02 "
                     f"{args.dtype}, rank {rank} block-rows {r0}..{r1 - 1} "
                     f"of 1024 (shard_rows_by_nnz over {world})")
        metric = "effective TFLOP/s (nnz-FLOPs) row-panel DSD M=131072 K=N=4096 2%"
        scaling = "strong"
        prob.anchor_shape = (prob.m, args.n, int(round(args.k * 0.02)))
    fn = graph_step(prob) if args.graph else prob.launcher()
    ms = max_over_ranks(time_steps(fn, args.steps, args.warmup, world), world)
    per = ms / args.steps
    flops_all = sum_over_ranks(prob.flops, world)
    extra = {}
    if args.workload == "transpose":
        value, unit, hib = per * 1e3, "us", False
    else:
        value, unit, hib = flops_all / (per * 1e-3) / 1e12, "TFLOP/s", True
        traffic, per_kernel, note = (None, None, "not measured for this workload")
        if args.workload in ("sdd_dds", "moe", "panel") and world == 1:
            traffic, per_kernel, note = pmc_workload_traffic(
                args.pmc_workloads, args.workload, build.get("hash"))
        extra["roofline"] = roofline(prob.flops, prob.bytes, per * 1e-3,
                                     getattr(prob, "kernel", "block_gemm_kernel"),
                                     traffic)
        extra["roofline"]["traffic_source"] = note
        if per_kernel:
            extra["roofline"]["traffic_kernels"] = per_kernel
        shape = getattr(prob, "anchor_shape", None)
        if rank == 0 and shape is not None:
            anchor = dense_anchor(*shape, getattr(prob, "dtype_name", args.dtype),
                                  device)
            if "tflops" in anchor:
                anchor["sparse_over_dense"] = round(
                    value / world / anchor["tflops"], 3)
            extra["dense_anchor"] = anchor
    if args.workload == "panel" and world > 1:
        # Optional gather of the dense result (config 5): reported beside the
        # hot path, never inside it. The library's gather_row_panels
        # (sputnik_amd/gather.py): the nnz-balanced panels differ in rows, so
        # it runs one grouped send/recv set (RCCL over xGMI), no padding.
        import torch
        import sputnik_amd as sp
        panels = [tuple(int(x) for x in pr) for pr in prob.all_panels]
        c_panel = prob.c_vals.view(prob.C.rows, args.n)
        full = sp.gather_row_panels(c_panel, panels)
        torch.cuda.synchronize()
        barrier(world)
        t0 = time.perf_counter()
        for _ in range(5):
            sp.gather_row_panels(c_panel, panels, out=full)
        torch.cuda.synchronize()
        ag = max_over_ranks((time.perf_counter() - t0) / 5 * 1e3, world)
        extra["allgather_ms"] = round(ag, 4)
        extra["allgather_method"] = ("all_gather_into_tensor" if len(
            {p1 - p0 for p0, p1 in panels}) == 1 else "batch_isend_irecv")
        extra["allgather_GBps_per_rank"] = round(
            full.numel() * full.element_size() * (world - 1) / world / (ag * 1e-3) / 1e9, 1)
        del full
    if rank == 0:
        emit({**extra,
              "metric": metric, "value": round(value, 3), "unit": unit,
              "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
              "ms_per_step": round(per, 5), "higher_is_better": hib,
              "scaling": scaling, "vs_baseline": None,
              "dtype": getattr(prob, "dtype_name", args.dtype),
              "data": "synthetic", "config": {"workload": prob.desc},
              "graph": args.graph, "build": build})


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}",
              file=sys.stderr)
    # torch first: it loads its HIP runtime, which libsputnik.so then shares
    # (loading the library first would bring in a second runtime).
    import torch
    build = check_build() if rank == 0 else None

    # One rank per GPU; the modulo only matters for tests that put several
    # (gloo) ranks on a one-GPU box.
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")
        barrier(world)  # every rank sees local rank 0's (re)built library
    if build is None:
        import sputnik_amd as sp
        build = {"hash": sp.build_hash()}

    if args.workload == "sweep":
        run_sweep(args, device, build)
        return
    if args.workload != "dsd":
        run_other(args, world, rank, device, build)
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return

    # Headline density first, then the sweep.
    densities = [args.density] + [float(d) for d in args.sweep.split(",")
                                  if d and float(d) != args.density]
    results = {}
    head = None
    m_total = args.m if args.scaling == "strong" else args.m * world
    for d in densities:
        prob = dsd_panel(args, world, rank, device, d, m_total=m_total)
        fn = graph_step(prob) if args.graph else prob.launcher()
        ms = max_over_ranks(time_steps(fn, args.steps, args.warmup, world), world)
        per_step = ms / args.steps
        flops_all = sum_over_ranks(prob.flops, world)
        tflops = flops_all / (per_step * 1e-3) / 1e12
        # (keyed by this rank's own launch: at N > 1 a rank runs a panel of
        # prob.m rows, which the N = 1 PMC pass of m_total rows does not
        # describe, so its traffic stays null)
        key = f"dsd_{prob.m}x{args.k}x{args.n}_{d}_{args.dtype}"
        traffic, note = pmc_traffic(args.pmc, key, build.get("hash"))
        roof = roofline(prob.flops, prob.bytes, per_step * 1e-3, prob.kernel,
                        traffic)
        roof["traffic_source"] = note
        if roof.get("bound") == "mfma":
            pc = pmc_clock(args.pmc, key, build.get("hash"), tflops, roof["peak"])
            if pc is not None:
                roof["pmc_clock"] = pc
        results[d] = {"value": round(tflops, 2), "ms_per_step": round(per_step, 5),
                      "nnz_blocks_per_rank": prob.nb, "roofline": roof}
        if head is None:
            head = (prob, per_step, tflops, roof)
        else:
            del prob
        torch.cuda.empty_cache()

    # Dominant (only) kernel of a step: block_gemm DSD NN, one launch per
    # step, so the event-timed average over the K launches is its duration.
    prob, per_step, tflops, roof = head

    anchor = None
    if rank == 0:
        kd = max(BLOCK, int(round(args.k * args.density / BLOCK)) * BLOCK)
        anchor = dense_anchor(prob.m, args.n, kd, args.dtype, device)
        if "tflops" in anchor:
            anchor["sparse_over_dense"] = round(tflops / world / anchor["tflops"], 3)

    cpu = None
    config1 = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(prob, args.cpu_seconds)
        config1 = config1_host_reference()

    if rank == 0:
        r0, r1 = prob.panel
        emit({
            "metric": METRIC,
            "value": round(tflops, 2),
            "unit": "TFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(per_step, 5),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (RANDOM_UNIFORM block topology, U(-1,1) values)",
            "config": {
                "workload": f"DSD block=128 M={m_total} K={args.k} "
                            f"N={args.n} density={args.density} "
                            f"{args.dtype} (NN, MatmulEx)",
                "block": 128, "m": m_total, "k": args.k, "n": args.n,
                "density": args.density,
                "parallelism": (f"row panels of one {m_total}-row "
                                f"matrix split by nnz over {world} rank(s) "
                                f"(rank 0: block-rows {r0}..{r1 - 1}), "
                                f"no collective ({args.scaling} scaling)"),
            },
            "by_density": {str(k): v for k, v in results.items()},
            "roofline": roof,
            "dense_anchor": anchor,
            "cpu_baseline": cpu,
            "config1": config1,
            "graph": args.graph,
            "build": build,
        })

    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def dense_anchor(m, n, kd, dtype, device, iters=50):
    """The vendor dense GEMM (torch.matmul -> hipBLASLt) on the same FLOPs:
    m x n x kd (kd = K x density), random normal data, timed like the sparse
    steps. The MFMA peak is a spec number; this is what a dense GEMM reaches
    on this GPU under the same clocks and power draw."""
    import torch
    dt = torch.float16 if dtype == "f16" else torch.bfloat16
    try:
        a = torch.randn(m, kd, dtype=dt, device=device)
        b = torch.randn(kd, n, dtype=dt, device=device)
        for _ in range(10):
            torch.matmul(a, b)
        torch.cuda.synchronize()
        times = []
        for _ in range(5):
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(iters):
                torch.matmul(a, b)
            e.record()
            torch.cuda.synchronize()
            times.append(s.elapsed_time(e) / iters)
    except RuntimeError as exc:  # reported, never fatal
        return {"error": str(exc)[:200]}
    ms = sorted(times)[len(times) // 2]
    return {"op": "torch.matmul (hipBLASLt)",
            "shape": [m, n, kd], "us": round(ms * 1e3, 2),
            "tflops": round(2.0 * m * n * kd / (ms * 1e-3) / 1e12, 1)}


if __name__ == "__main__":
    main()
