"""CPU, world_size 2 (gloo): row-panel sharding of DSD.

Each rank takes a contiguous, nonzero-balanced panel of block-rows
(matrix_utils.shard_rows_by_nnz), rebases it (slice_block_rows), computes its
panel of C with the CPU oracle, and the panels are all-gathered. The result
must equal the unsharded oracle product bit for bit (the per-element
arithmetic does not depend on the split). This is the N>1 path of bench.py /
INTEGRATION.md §5 with the HIP kernel replaced by the oracle (no GPU here).
"""

import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from sputnik_amd import matrix_utils as mu  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _problem():
    rng = np.random.default_rng(42)
    R, C, N = 12, 6, 64
    off, idx = mu.random_topology(R, C, 30, rng, unordered=True)
    vals = mu.random_values((30, 128, 128), rng)
    b = mu.random_values((C * 128, N), rng)
    return R, C, N, off, idx, vals, b


def _worker(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    R, C, N, off, idx, vals, b = _problem()
    shards = mu.shard_rows_by_nnz(off, world)
    r0, r1 = shards[rank]
    p_off, p_idx, p_vals = mu.slice_block_rows(off, idx, vals, r0, r1)
    rows = (r1 - r0) * 128
    panel = np.zeros((rows, N), np.float32)
    if rows:
        dense = mu.to_dense(rows, C * 128, p_off, p_idx, p_vals)
        panel = O.gemm(dense, False, b, False,
                       a_mask=mu.block_mask(p_off, p_idx, C))
    # Variable-size panels: gather sizes, pad, all_gather, trim.
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([rows]))
    maxr = int(max(s.item() for s in sizes))
    buf = torch.zeros(maxr, N)
    buf[:rows] = torch.from_numpy(panel)
    bufs = [torch.zeros(maxr, N) for _ in range(world)]
    dist.all_gather(bufs, buf)
    if rank == 0:
        full = torch.cat([bufs[i][: int(sizes[i].item())] for i in range(world)])
        np.save(out_path, full.numpy())
    dist.destroy_process_group()


def test_shard_rows_by_nnz_balanced_and_contiguous():
    rng = np.random.default_rng(0)
    off, _ = mu.random_topology(64, 32, 900, rng)
    for parts in (1, 2, 4, 8):
        sh = mu.shard_rows_by_nnz(off, parts)
        assert sh[0][0] == 0 and sh[-1][1] == 64
        assert all(a[1] == b[0] for a, b in zip(sh, sh[1:]))
        loads = [off[r1] - off[r0] for r0, r1 in sh]
        assert max(loads) - min(loads) <= 2 * np.diff(off).max()


def test_slice_block_rows_roundtrip():
    rng = np.random.default_rng(1)
    off, idx = mu.random_topology(10, 7, 25, rng)
    vals = np.arange(25)
    parts = [mu.slice_block_rows(off, idx, vals, r0, r1)
             for r0, r1 in mu.shard_rows_by_nnz(off, 3)]
    assert np.array_equal(np.concatenate([p[1] for p in parts]), idx)
    assert np.array_equal(np.concatenate([p[2] for p in parts]), vals)
    for p in parts:
        assert p[0][0] == 0


def test_two_rank_gloo_sharded_dsd_matches_unsharded(tmp_path):
    from oracle import oracle as O
    out = str(tmp_path / "c.npy")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    R, C, N, off, idx, vals, b = _problem()
    ref = O.gemm(mu.to_dense(R * 128, C * 128, off, idx, vals), False, b, False)
    assert np.array_equal(np.load(out), ref)


# ---- DDS column panels and SDD block runs ----------------------

def _pair_problem():
    rng = np.random.default_rng(7)
    M, KB, NB = 96, 5, 9           # A: M x K dense, B: K x N sparse (5 x 9 blocks)
    off, idx = mu.random_topology(KB, NB, 20, rng, unordered=True)
    vals = mu.random_values((20, 128, 128), rng)
    a = mu.random_values((M, KB * 128), rng)
    return M, KB, NB, off, idx, vals, a


def _gather_equal(local, world):
    t = torch.from_numpy(np.ascontiguousarray(local))
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([t.shape[0]]))
    maxr = int(max(s.item() for s in sizes))
    buf = torch.zeros((maxr,) + tuple(t.shape[1:]), dtype=t.dtype)
    buf[: t.shape[0]] = t
    bufs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf)
    return [bufs[i][: int(sizes[i].item())].numpy() for i in range(world)]


def _worker_dds_sdd(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    M, KB, NB, off, idx, vals, a = _pair_problem()
    # DDS: C[:, c0:c1] = A . B[:, c0:c1]; column panels balanced by nnz.
    c0, c1 = mu.shard_cols_by_nnz(off, idx, NB, world)[rank]
    p_off, p_idx, p_vals = mu.slice_block_cols(off, idx, vals, c0, c1)
    cols = (c1 - c0) * 128
    panel = np.zeros((cols, M), np.float32)   # gathered as C^T panels
    if cols:
        bd = mu.to_dense(KB * 128, cols, p_off, p_idx, p_vals)
        panel = O.gemm(a, False, bd, False,
                       b_mask=mu.block_mask(p_off, p_idx, c1 - c0)).T
    dds = np.concatenate(_gather_equal(panel, world)).T
    # SDD: C = x . w restricted to B's topology (KB x NB blocks), x = A^T
    # (K x M), w (M x N); each rank computes the stored-block run [b0, b1).
    nb = len(idx)
    b0, b1 = mu.shard_blocks(nb, world)[rank]
    s_off, s_idx = mu.slice_blocks(off, idx, b0, b1)
    rows_of = np.repeat(np.arange(KB), np.diff(s_off))
    x = a.T
    w = mu.random_values((M, NB * 128), np.random.default_rng(11))
    blocks = np.zeros((b1 - b0, 128, 128), np.float32)
    for j in range(b1 - b0):
        r, c = int(rows_of[j]), int(s_idx[j])
        blocks[j] = O.gemm(x[r * 128:(r + 1) * 128], False,
                           w[:, c * 128:(c + 1) * 128], False)
    sdd = np.concatenate(_gather_equal(blocks, world))
    if rank == 0:
        np.savez(out_path, dds=dds, sdd=sdd)
    dist.destroy_process_group()


def test_shard_cols_and_blocks_cover_exactly_once():
    rng = np.random.default_rng(3)
    off, idx = mu.random_topology(16, 24, 150, rng, unordered=True)
    counts = np.bincount(idx, minlength=24)
    for parts in (1, 2, 3, 8):
        sh = mu.shard_cols_by_nnz(off, idx, 24, parts)
        assert sh[0][0] == 0 and sh[-1][1] == 24
        assert all(p[1] == q[0] for p, q in zip(sh, sh[1:]))
        loads = [counts[c0:c1].sum() for c0, c1 in sh]
        assert sum(loads) == 150 and max(loads) - min(loads) <= 2 * counts.max()
        vals = np.arange(150)
        got = np.concatenate([mu.slice_block_cols(off, idx, vals, c0, c1)[2]
                              for c0, c1 in sh])
        assert sorted(got.tolist()) == list(range(150))
        bl = mu.shard_blocks(150, parts)
        assert bl[0][0] == 0 and bl[-1][1] == 150
        assert max(b1 - b0 for b0, b1 in bl) - min(b1 - b0 for b0, b1 in bl) <= 1
        ri = np.repeat(np.arange(16), np.diff(off))
        for b0, b1 in bl:
            s_off, s_idx = mu.slice_blocks(off, idx, b0, b1)
            assert s_off[-1] == b1 - b0 and len(s_off) == 17
            assert np.array_equal(np.repeat(np.arange(16), np.diff(s_off)),
                                  ri[b0:b1])
            assert np.array_equal(s_idx, idx[b0:b1])


def test_slice_block_cols_matches_dense_columns():
    rng = np.random.default_rng(4)
    off, idx = mu.random_topology(4, 6, 11, rng, unordered=True)
    vals = mu.random_values((11, 128, 128), rng)
    dense = mu.to_dense(512, 768, off, idx, vals)
    p_off, p_idx, p_vals = mu.slice_block_cols(off, idx, vals, 2, 5)
    assert np.array_equal(mu.to_dense(512, 384, p_off, p_idx, p_vals),
                          dense[:, 256:640])


def test_two_rank_gloo_sharded_dds_and_sdd_match_unsharded(tmp_path):
    from oracle import oracle as O
    out = str(tmp_path / "c.npz")
    mp.spawn(_worker_dds_sdd, args=(2, _free_port(), out), nprocs=2, join=True)
    M, KB, NB, off, idx, vals, a = _pair_problem()
    got = np.load(out)
    ref = O.gemm(a, False, mu.to_dense(KB * 128, NB * 128, off, idx, vals), False)
    assert np.array_equal(got["dds"], ref)
    w = mu.random_values((M, NB * 128), np.random.default_rng(11))
    full = O.gemm(a.T, False, w, False)
    ri = np.repeat(np.arange(KB), np.diff(off))
    want = np.stack([full[r * 128:(r + 1) * 128, c * 128:(c + 1) * 128]
                     for r, c in zip(ri, idx)])
    assert np.array_equal(got["sdd"], want)


# ---- the same splits on the GPU: each rank runs the HIP kernel -------------
# World size 2 with the gloo backend; both ranks share the box's one device
# (the 8-GPU node is the driver's). Integer operand values make every split
# exact, so the gathered panels must equal the unsharded launch bit for bit.

def _int_problem(seed=21):
    rng = np.random.default_rng(seed)
    R, C, N = 24, 16, 1024
    off, idx = mu.random_topology(R, C, 190, rng, unordered=True)
    vals = rng.integers(-1, 2, size=(190, 128, 128)).astype(np.float32)
    b = rng.integers(-1, 2, size=(C * 128, N)).astype(np.float32)
    return R, C, N, off, idx, vals, b


def _hip_dsd(off, idx, vals, rows_b, cols_b, b):
    import sputnik_amd as sp
    dev = torch.device("cuda", 0)
    nb = len(idx)
    A = sp.BlockMatrix(rows_b * 128, cols_b * 128, 128, nb * 16384,
                       torch.from_numpy(vals).half().to(dev),
                       torch.from_numpy(off.astype(np.int32)).to(dev),
                       torch.from_numpy(idx.astype(np.int16)).to(dev))
    bt = torch.from_numpy(b).half().to(dev)
    c = torch.full((rows_b * 128, b.shape[1]), float("nan"),
                   dtype=torch.float16, device=dev)
    sp.Matmul(A, False, sp.Matrix(*b.shape, bt),
              False, sp.Matrix(rows_b * 128, b.shape[1], c))
    torch.cuda.synchronize()
    return c.float().cpu().numpy()


def _worker_hip(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    R, C, N, off, idx, vals, b = _int_problem()
    r0, r1 = mu.shard_rows_by_nnz(off, world)[rank]
    p_off, p_idx, p_vals = mu.slice_block_rows(off, idx, vals, r0, r1)
    panel = (_hip_dsd(p_off, p_idx, p_vals, r1 - r0, C, b) if r1 > r0
             else np.zeros((0, N), np.float32))
    # The library's gather (sputnik_amd.gather_row_panels) on the host copies
    # of the HIP panels (gloo carries CPU tensors).
    import sputnik_amd as sp
    full = sp.gather_row_panels(torch.from_numpy(panel),
                                mu.shard_rows_by_nnz(off, world)).numpy()
    if rank == 0:
        np.save(out_path, full)
    dist.destroy_process_group()


@pytest.mark.gpu
def test_two_rank_gloo_sharded_hip_dsd_matches_unsharded(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = str(tmp_path / "c.npy")
    mp.spawn(_worker_hip, args=(2, _free_port(), out), nprocs=2, join=True)
    R, C, N, off, idx, vals, b = _int_problem()
    whole = _hip_dsd(off, idx, vals, R, C, b)
    exact = mu.to_dense(R * 128, C * 128, off, idx, vals).astype(np.float64) @ b
    got = np.load(out)
    assert np.array_equal(got, whole)
    assert np.array_equal(got, exact)


@pytest.mark.gpu
@pytest.mark.parametrize("scaling", ["strong", "weak"])
def test_bench_two_ranks_shard_one_matrix(scaling):
    """bench.py's N>1 path (one matrix split by shard_rows_by_nnz, max over
    ranks, whole-job value) on two ranks sharing the device, gloo backend:
    strong scaling splits the metric's own 4096-row matrix (16 block-rows
    per rank), weak scaling gives every rank 4096 rows."""
    import json
    import subprocess
    import sys
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--sweep", "",
           "--no-cpu", "--dist-backend", "gloo", "--scaling", scaling]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=300,
                         cwd=root)
    assert res.returncode == 0, res.stderr[-2000:]
    line = json.loads([x for x in res.stdout.splitlines()
                       if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert line["scaling"] == scaling
    assert "split by nnz over 2" in line["config"]["parallelism"]
    m = 4096 if scaling == "strong" else 8192
    assert line["config"]["m"] == m
    # rank 0 holds about half of the block-rows of the one matrix
    nb0 = line["by_density"]["0.5"]["nnz_blocks_per_rank"]
    total = (m // 128) * 32 // 2
    assert abs(nb0 - total / 2) <= 32, (nb0, total)


# ---- the library's full-result gathers (sputnik_amd/gather.py) --------------

def _worker_gather(rank, world, port, out_path, method):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sputnik_amd as sp
    from oracle import oracle as O
    # DSD row panels: nonzero-balanced, so the row counts differ per rank
    R, C, N, off, idx, vals, b = _problem()
    panels = mu.shard_rows_by_nnz(off, world)
    r0, r1 = panels[rank]
    p_off, p_idx, p_vals = mu.slice_block_rows(off, idx, vals, r0, r1)
    rows = (r1 - r0) * 128
    panel = np.zeros((rows, N), np.float32)
    if rows:
        panel = O.gemm(mu.to_dense(rows, C * 128, p_off, p_idx, p_vals), False,
                       b, False, a_mask=mu.block_mask(p_off, p_idx, C))
    dsd = sp.gather_row_panels(torch.from_numpy(panel), panels, method=method)
    # DDS column panels
    M, KB, NB, off2, idx2, vals2, a = _pair_problem()
    cpan = mu.shard_cols_by_nnz(off2, idx2, NB, world)
    c0, c1 = cpan[rank]
    q_off, q_idx, q_vals = mu.slice_block_cols(off2, idx2, vals2, c0, c1)
    cols = (c1 - c0) * 128
    cp = np.zeros((M, cols), np.float32)
    if cols:
        cp = O.gemm(a, False, mu.to_dense(KB * 128, cols, q_off, q_idx, q_vals),
                    False, b_mask=mu.block_mask(q_off, q_idx, c1 - c0))
    dds = sp.gather_col_panels(torch.from_numpy(np.ascontiguousarray(cp)), cpan,
                               method=method)
    # a caller's out of the wrong shape / dtype is refused before any
    # collective (on every rank alike, so nothing hangs)
    refused = 0
    for bad in (torch.empty((M, 8)), torch.empty((M, NB * 128), dtype=torch.float64)):
        try:
            sp.gather_col_panels(torch.from_numpy(np.ascontiguousarray(cp)), cpan,
                                 out=bad, method=method)
        except ValueError:
            refused += 1
    outp = torch.empty((M, NB * 128))
    dds2 = sp.gather_col_panels(torch.from_numpy(np.ascontiguousarray(cp)), cpan,
                                out=outp, method=method)
    assert dds2 is outp and torch.equal(dds2, dds)
    # SDD block runs (values stand in for computed blocks: the gather is what
    # is under test)
    runs = mu.shard_blocks(len(idx2), world)
    b0, b1 = runs[rank]
    sdd = sp.gather_block_runs(torch.from_numpy(vals2[b0:b1].reshape(-1)), runs,
                               method=method)
    if rank == 0:
        np.savez(out_path, dsd=dsd.numpy(), dds=dds.numpy(), sdd=sdd.numpy(),
                 refused=refused)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,method", [(2, "auto"), (2, "padded"),
                                          (3, "auto"), (3, "p2p")])
def test_gather_panels_match_unsharded(tmp_path, world, method):
    from oracle import oracle as O
    out = str(tmp_path / "g.npz")
    mp.spawn(_worker_gather, args=(world, _free_port(), out, method),
             nprocs=world, join=True)
    got = np.load(out)
    R, C, N, off, idx, vals, b = _problem()
    assert np.array_equal(got["dsd"], O.gemm(
        mu.to_dense(R * 128, C * 128, off, idx, vals), False, b, False))
    M, KB, NB, off2, idx2, vals2, a = _pair_problem()
    assert np.array_equal(got["dds"], O.gemm(
        a, False, mu.to_dense(KB * 128, NB * 128, off2, idx2, vals2), False))
    assert np.array_equal(got["sdd"], vals2)
    assert int(got["refused"]) == 2


def test_gather_checks_cover():
    from sputnik_amd import gather
    with pytest.raises(ValueError):
        gather._check_cover([(0, 2), (3, 4)])
    with pytest.raises(ValueError):
        gather._check_cover([(1, 2)])
    gather._check_cover([(0, 0), (0, 5), (5, 5)])


@pytest.mark.gpu
def test_bench_two_ranks_panel_gather():
    """bench.py --workload panel at world size 2 (gloo, both ranks on the
    box's device): the rank panels of config 5 and the timed full-result
    gather (sputnik_amd.gather_row_panels) beside the hot path."""
    import json
    import subprocess
    import sys
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--no-cpu",
           "--dist-backend", "gloo", "--workload", "panel"]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=300,
                         cwd=root)
    assert res.returncode == 0, res.stderr[-2000:]
    line = json.loads([x for x in res.stdout.splitlines()
                       if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert line["allgather_ms"] > 0
    assert line["allgather_method"] in ("all_gather_into_tensor",
                                        "batch_isend_irecv")
