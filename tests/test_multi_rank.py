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
