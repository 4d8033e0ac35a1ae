"""GPU: the 4-wave hand-scheduled DSD NN kernel (sputnik_amd/csrc/dsd4w.hip)
against the 8-wave kernel (block_gemm.h) and the oracle.

Both kernels accumulate every output element over the same k-steps in the
same order with the same MFMA instruction and operand roles, split paired
rows at the same block and add the head partial the same way, so their
outputs must be bit-identical (torch.equal) on every shape -- pair-balanced
or not, partial column tiles, empty rows, both dtypes. The oracle check
(north-star tolerance) pins the 4-wave kernel independently.
"""

import numpy as np
import pytest

from oracle import oracle as O
from sputnik_amd import matrix_utils as mu
from tests import helpers as H

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

import sputnik_amd as sp  # noqa: E402


def _problem(m, k, n, density, dtype, seed, empty_rows=()):
    rng = np.random.default_rng(seed)
    R, C = m // 128, k // 128
    nz = mu.nonzeros_for_density(m, k, density) // (128 * 128)
    off, idx = mu.random_topology(R, C, nz, rng, unordered=True)
    if empty_rows:
        keep = ~np.isin(np.repeat(np.arange(R), np.diff(off)), empty_rows)
        rows = np.repeat(np.arange(R), np.diff(off))[keep]
        idx = idx[keep]
        off = np.zeros(R + 1, np.int32)
        np.cumsum(np.bincount(rows, minlength=R), out=off[1:])
    td = torch.float16 if dtype == "f16" else torch.bfloat16
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    nb = int(off[-1])
    a = (torch.rand(max(nb, 1) * 16384, generator=g, device="cuda") * 2 - 1).to(td)
    b = (torch.rand(k * n, generator=g, device="cuda") * 2 - 1).to(td)
    A = sp.BlockMatrix(m, k, 128, nb * 16384, a,
                       torch.from_numpy(np.asarray(off, np.int32)).cuda(),
                       torch.from_numpy(np.asarray(idx).astype(np.int16)).cuda())
    return A, sp.Matrix(k, n, b), off, idx, a, b


def _run(A, B, m, n, dtype, mode, tb=False):
    """mode: 0 the 8-wave kernel, 2 the 4-wave kernel (workgroup epilogue),
    3 with the per-wave epilogue, 4 per-wave + specialized last block, 5
    per-wave + double-slot S image, 6 the same with a barrier every other
    step and the interleaved epilogue, 7 double slots + the interleaved
    epilogue; 2-7 regardless of the density gate."""
    td = torch.float16 if dtype == "f16" else torch.bfloat16
    c = torch.full((m * n,), float("nan"), dtype=td, device="cuda")
    prev = sp.select_dsd_kernel(mode)
    try:
        sp.MatmulEx(A, False, B, tb, sp.Matrix(m, n, c))
        torch.cuda.synchronize()
    finally:
        sp.select_dsd_kernel(prev)
    return c.view(m, n)


CASES = [
    # m, k, n, density
    (4096, 4096, 4096, 0.5),    # headline: pairs, two panels per XCD
    (4096, 4096, 4096, 0.1),
    (4096, 4096, 4096, 0.3),
    (4096, 4096, 4096, 0.9),
    (2048, 4096, 4096, 0.5),    # 16 rows
    (4096, 2048, 1032, 0.5),    # partial column tile, 3 panels
    (4096, 1024, 264, 0.5),     # one narrow panel
    (8192, 2048, 2048, 0.3),    # 64 rows: workgroup ranking (rank_block)
    (1024, 4096, 4096, 0.05),   # few blocks per row: plain launch (no pairs)
]


@pytest.mark.parametrize("m,k,n,density", CASES)
@pytest.mark.parametrize("dtype", ["f16", "bf16"])
@pytest.mark.parametrize("mode", [2, 3, 4, 5, 6, 7])
def test_dsd4w_bit_identical_to_8wave(m, k, n, density, dtype, mode):
    A, B, off, idx, a, b = _problem(m, k, n, density, dtype, seed=m + n + int(density * 100))
    c4 = _run(A, B, m, n, dtype, mode)
    c8 = _run(A, B, m, n, dtype, 0)
    assert not torch.isnan(c4.float()).any()
    assert torch.equal(c4, c8), (
        f"max diff {float((c4.float() - c8.float()).abs().max())}")
    assert sp.pair_errors() == 0


@pytest.mark.parametrize("mode", [2, 3, 4, 5, 6, 7])
def test_dsd4w_empty_rows_and_oracle(mode):
    """Empty block-rows get zero tiles; sampled rows against the oracle."""
    m, k, n = 4096, 2048, 1024
    A, B, off, idx, a, b = _problem(m, k, n, 0.5, "f16", seed=3,
                                    empty_rows=(0, 5, 31))
    c4 = _run(A, B, m, n, "f16", mode)
    c8 = _run(A, B, m, n, "f16", 0)
    assert torch.equal(c4, c8)
    for r in (0, 5, 31):
        assert torch.count_nonzero(c4[r * 128:(r + 1) * 128]) == 0
    av = a.float().cpu().numpy().reshape(-1, 128, 128)
    bv = b.float().cpu().numpy().reshape(k, n)
    for r in (1, 17, 30):
        o0, o1 = int(off[r]), int(off[r + 1])
        row = np.zeros((128, k), np.float32)
        for e in range(o0, o1):
            row[:, idx[e] * 128:(idx[e] + 1) * 128] = av[e]
        ref = O.gemm(row, False, bv, False, threads=H.oracle_threads())
        H.assert_close(c4[r * 128:(r + 1) * 128].float().cpu().numpy(), ref,
                       "f16", f"dsd4w row-block {r}")


def test_dsd4w_selector_roundtrip():
    prev = sp.select_dsd_kernel(-1)
    assert prev in (0, 1, 2, 3, 4, 5, 6, 7)
    assert sp.select_dsd_kernel(0) == prev
    assert sp.select_dsd_kernel(-1) == 0
    assert sp.select_dsd_kernel(prev) == 0
    assert sp.select_dsd_kernel(-1) == prev


# ------------------------------------------------------------------ DDS NN --
# The same kernel with the operand images swapped (dsd4w.hip kDds): C = A . B
# with B sparse in column order (its transposed metadata), against the
# 8-wave kernel's kOutT path (same k order and MFMA operand roles, so again
# torch.equal) and the oracle.

def _dds_problem(m, k, n, density, dtype, seed, empty_cols=()):
    rng = np.random.default_rng(seed)
    R, C = k // 128, n // 128
    nz = mu.nonzeros_for_density(k, n, density) // (128 * 128)
    off, idx = mu.random_topology(R, C, nz, rng, unordered=True)
    if empty_cols:
        rows = np.repeat(np.arange(R), np.diff(off))
        keep = ~np.isin(idx, empty_cols)
        rows, idx = rows[keep], idx[keep]
        off = np.zeros(R + 1, np.int32)
        np.cumsum(np.bincount(rows, minlength=R), out=off[1:])
    td = torch.float16 if dtype == "f16" else torch.bfloat16
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    nb = int(off[-1])
    a = (torch.rand(m * k, generator=g, device="cuda") * 2 - 1).to(td)
    b = (torch.rand(max(nb, 1) * 16384, generator=g, device="cuda") * 2 - 1).to(td)
    B = sp.BlockMatrix(k, n, 128, nb * 16384, b,
                       torch.from_numpy(np.asarray(off, np.int32)).cuda(),
                       torch.from_numpy(np.asarray(idx).astype(np.int16)).cuda())
    sp.AllocateTransposeBuffers(B)
    sp.Transpose(B)
    return sp.Matrix(m, k, a), B, off, idx, a, b


def _run_dds(A, B, m, n, dtype, mode):
    td = torch.float16 if dtype == "f16" else torch.bfloat16
    c = torch.full((m * n,), float("nan"), dtype=td, device="cuda")
    prev = sp.select_dsd_kernel(mode)
    try:
        sp.MatmulEx(A, False, B, False, sp.Matrix(m, n, c))
        torch.cuda.synchronize()
    finally:
        sp.select_dsd_kernel(prev)
    return c.view(m, n)


DDS_CASES = [
    # m, k, n, density
    (4096, 4096, 4096, 0.2),    # BASELINE config 3's DDS
    (4096, 4096, 4096, 0.5),
    (4096, 4096, 4096, 0.05),
    (4096, 4096, 4096, 0.9),
    (2048, 4096, 4096, 0.3),    # 4 row panels
    (1152, 2048, 2048, 0.5),    # last tile: one wave block inside M, three past it
    (4096, 2048, 8192, 0.3),    # 64 block-columns: workgroup ranking
    (4096, 4096, 1024, 0.5),    # 8 block-columns
]


@pytest.mark.parametrize("m,k,n,density", DDS_CASES)
@pytest.mark.parametrize("dtype", ["f16", "bf16"])
@pytest.mark.parametrize("mode", [3, 5])
def test_dds4w_bit_identical_to_8wave(m, k, n, density, dtype, mode):
    """mode 3: per-step rows of A; 5: double slots of 128-B row pieces."""
    A, B, off, idx, a, b = _dds_problem(m, k, n, density, dtype,
                                        seed=m + 3 * n + int(density * 100))
    c4 = _run_dds(A, B, m, n, dtype, mode)
    c8 = _run_dds(A, B, m, n, dtype, 0)
    assert not torch.isnan(c4.float()).any()
    assert torch.equal(c4, c8), (
        f"max diff {float((c4.float() - c8.float()).abs().max())}")
    assert sp.pair_errors() == 0


@pytest.mark.parametrize("mode", [3, 5])
def test_dds4w_empty_columns_and_oracle(mode):
    m, k, n = 1536, 2048, 4096
    A, B, off, idx, a, b = _dds_problem(m, k, n, 0.5, "f16", seed=5,
                                        empty_cols=(0, 7, 31))
    c4 = _run_dds(A, B, m, n, "f16", mode)
    c8 = _run_dds(A, B, m, n, "f16", 0)
    assert torch.equal(c4, c8)
    for c in (0, 7, 31):
        assert torch.count_nonzero(c4[:, c * 128:(c + 1) * 128]) == 0
    av = a.float().cpu().numpy().reshape(m, k)
    bv = b.float().cpu().numpy().reshape(-1, 128, 128)
    for c in (1, 17, 30):
        col = np.zeros((k, 128), np.float32)
        for e in range(int(off[-1])):
            if idx[e] == c:
                r = int(np.searchsorted(off, e, side="right") - 1)
                col[r * 128:(r + 1) * 128] = bv[e]
        ref = O.gemm(av, False, col, False, threads=H.oracle_threads())
        H.assert_close(c4[:, c * 128:(c + 1) * 128].float().cpu().numpy(), ref,
                       "f16", f"dds4w block-column {c}")


# ------------------------------------------------------------ grouped SDD --
# The same kernel on the grouped SDD NN launch (dsd4w.hip kSdd: up to 4
# stored blocks of a block-row per workgroup): against the 8-wave grouped
# kernel (same k order and MFMA operand roles: torch.equal) and the oracle.

def _sdd_problem(m, k, n, density, dtype, seed, uniform=0, tb=False, ta=False):
    rng = np.random.default_rng(seed)
    R, C = m // 128, n // 128
    if uniform:
        off = np.arange(R + 1, dtype=np.int32) * uniform
        idx = np.concatenate([np.sort(rng.choice(C, uniform, replace=False))
                              for _ in range(R)]).astype(np.int16)
    else:
        nz = mu.nonzeros_for_density(m, n, density) // (128 * 128)
        off, idx = mu.random_topology(R, C, nz, rng)
    td = torch.float16 if dtype == "f16" else torch.bfloat16
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    a = (torch.rand(m * k, generator=g, device="cuda") * 2 - 1).to(td)
    b = (torch.rand(k * n, generator=g, device="cuda") * 2 - 1).to(td)
    nb = int(off[-1])
    cv = torch.full((nb * 16384,), float("nan"), dtype=td, device="cuda")
    Cm = sp.BlockMatrix(m, n, 128, nb * 16384, cv,
                        torch.from_numpy(np.asarray(off, np.int32)).cuda(),
                        torch.from_numpy(np.asarray(idx).astype(np.int16)).cuda())
    sp.AllocateRowIndicesBuffer(Cm)
    sp.RowIndices(Cm, Cm.row_indices)
    Bm = sp.Matrix(n, k, b) if tb else sp.Matrix(k, n, b)
    Am = sp.Matrix(k, m, a) if ta else sp.Matrix(m, k, a)
    return Am, Bm, Cm, cv, off, idx, a, b


def _run_sdd(A, B, Cm, cv, mode, tb=False, ta=False):
    cv.fill_(float("nan"))
    prev = sp.select_dsd_kernel(mode)
    try:
        sp.Matmul(A, ta, B, tb, Cm)
        torch.cuda.synchronize()
    finally:
        sp.select_dsd_kernel(prev)
    return cv.clone()


SDD_CASES = [
    # m, k, n, density, uniform blocks per row (0: random)
    (8192, 1024, 8192, 0.5, 0),     # 2048 blocks: grouped
    (8192, 2048, 8192, 0.4, 0),
    (8192, 512, 16384, 0.2, 0),
    (8192, 1024, 8192, 0, 27),      # uniform rows: group-major order, partial groups
]


@pytest.mark.parametrize("m,k,n,density,uniform", SDD_CASES)
@pytest.mark.parametrize("dtype", ["f16", "bf16"])
@pytest.mark.parametrize("trans", ["NN", "NT", "TN", "TT"])
@pytest.mark.parametrize("mode", [5, 6])
def test_sdd4w_bit_identical_to_8wave(m, k, n, density, uniform, dtype, trans, mode):
    """mode 5: double slots; 6: and a barrier every other step (NN / NT)."""
    ta, tb = trans[0] == "T", trans[1] == "T"
    A, B, Cm, cv, off, idx, a, b = _sdd_problem(m, k, n, density, dtype, seed=m + k + n,
                                                uniform=uniform, tb=tb, ta=ta)
    c4 = _run_sdd(A, B, Cm, cv, mode, tb, ta)
    c8 = _run_sdd(A, B, Cm, cv, 0, tb, ta)
    assert not torch.isnan(c4.float()).any()
    assert torch.equal(c4, c8), (
        f"max diff {float((c4.float() - c8.float()).abs().max())}")


@pytest.mark.parametrize("trans", ["NN", "NT", "TN", "TT"])
def test_sdd4w_oracle(trans):
    ta, tb = trans[0] == "T", trans[1] == "T"
    m, k, n = 8192, 1024, 8192
    A, B, Cm, cv, off, idx, a, b = _sdd_problem(m, k, n, 0.5, "f16", seed=11, tb=tb, ta=ta)
    c4 = _run_sdd(A, B, Cm, cv, 1, tb, ta).view(-1, 128, 128).float().cpu().numpy()
    av = a.float().cpu().numpy().reshape(k, m).T if ta else \
        a.float().cpu().numpy().reshape(m, k)
    bv = b.float().cpu().numpy().reshape(n, k).T if tb else \
        b.float().cpu().numpy().reshape(k, n)
    rows = np.repeat(np.arange(m // 128), np.diff(off))
    for e in (0, 1, 2, 3, 5, 777, int(off[-1]) - 1):
        r, c = int(rows[e]), int(idx[e])
        ref = O.gemm(av[r * 128:(r + 1) * 128], False, bv[:, c * 128:(c + 1) * 128],
                     False, threads=H.oracle_threads())
        H.assert_close(c4[e], ref, "f16", f"sdd4w block {e}")


# ----------------------------------------------------------------- DSD NT --
# B stored [n][k] (MegaBlocks' dx = dh . w1^T): both images k-contiguous in
# double slots (gen_dsd4w.py "nt" without "sdd").
NT_CASES = [c for c in CASES if c[2] % 128 == 0]


@pytest.mark.parametrize("m,k,n,density", NT_CASES)
@pytest.mark.parametrize("dtype", ["f16", "bf16"])
def test_dsd4w_nt_bit_identical_to_8wave(m, k, n, density, dtype):
    A, _, off, idx, a, _ = _problem(m, k, n, density, dtype, seed=m + 2 * n + int(density * 100))
    td = torch.float16 if dtype == "f16" else torch.bfloat16
    g = torch.Generator(device="cuda")
    g.manual_seed(m + n)
    bt = (torch.rand(n * k, generator=g, device="cuda") * 2 - 1).to(td)
    Bt = sp.Matrix(n, k, bt)
    c4 = _run(A, Bt, m, n, dtype, 5, tb=True)
    c8 = _run(A, Bt, m, n, dtype, 0, tb=True)
    assert not torch.isnan(c4.float()).any()
    assert torch.equal(c4, c8), (
        f"max diff {float((c4.float() - c8.float()).abs().max())}")
    assert sp.pair_errors() == 0
    if (m, k, n) == (2048, 4096, 4096):
        av = a.float().cpu().numpy().reshape(-1, 128, 128)
        bv = bt.float().cpu().numpy().reshape(n, k)
        for r in (0, 9):
            o0, o1 = int(off[r]), int(off[r + 1])
            row = np.zeros((128, k), np.float32)
            for e in range(o0, o1):
                row[:, idx[e] * 128:(idx[e] + 1) * 128] = av[e]
            ref = O.gemm(row, False, bv, True, threads=H.oracle_threads())
            H.assert_close(c4[r * 128:(r + 1) * 128].float().cpu().numpy(), ref,
                           "f16" if dtype == "f16" else "bf16", f"dsd4w NT row-block {r}")


# ----------------------------------------------------------------- DDS NT --
# C = A . B^T with B sparse stored [n][k] (its rows k-contiguous, storage
# order): both images in double slots (dsd4w.hip kDds + kNt).

@pytest.mark.parametrize("m,k,n,density", DDS_CASES)
@pytest.mark.parametrize("dtype", ["f16", "bf16"])
def test_dds4w_nt_bit_identical_to_8wave(m, k, n, density, dtype):
    rng = np.random.default_rng(m + n + 7)
    R, C = n // 128, k // 128
    nz = mu.nonzeros_for_density(n, k, density) // (128 * 128)
    off, idx = mu.random_topology(R, C, nz, rng, unordered=True)
    td = torch.float16 if dtype == "f16" else torch.bfloat16
    g = torch.Generator(device="cuda")
    g.manual_seed(m + k)
    nb = int(off[-1])
    a = (torch.rand(m * k, generator=g, device="cuda") * 2 - 1).to(td)
    b = (torch.rand(max(nb, 1) * 16384, generator=g, device="cuda") * 2 - 1).to(td)
    B = sp.BlockMatrix(n, k, 128, nb * 16384, b,
                       torch.from_numpy(np.asarray(off, np.int32)).cuda(),
                       torch.from_numpy(np.asarray(idx).astype(np.int16)).cuda())
    A = sp.Matrix(m, k, a)

    def run(mode):
        c = torch.full((m * n,), float("nan"), dtype=td, device="cuda")
        prev = sp.select_dsd_kernel(mode)
        try:
            sp.MatmulEx(A, False, B, True, sp.Matrix(m, n, c))
            torch.cuda.synchronize()
        finally:
            sp.select_dsd_kernel(prev)
        return c.view(m, n)

    c4, c8 = run(5), run(0)
    assert not torch.isnan(c4.float()).any()
    assert torch.equal(c4, c8), (
        f"max diff {float((c4.float() - c8.float()).abs().max())}")
    assert sp.pair_errors() == 0
    if (m, k, n) == (1152, 2048, 2048):
        av = a.float().cpu().numpy().reshape(m, k)
        bv = b.float().cpu().numpy().reshape(-1, 128, 128)
        rows = np.repeat(np.arange(R), np.diff(off))
        for r in (0, 5):  # block-row r of B = output block-column r
            blk = np.zeros((128, k), np.float32)
            for e in np.nonzero(rows == r)[0]:
                blk[:, idx[e] * 128:(idx[e] + 1) * 128] = bv[e]
            ref = O.gemm(av, False, blk, True, threads=H.oracle_threads())
            H.assert_close(c4[:, r * 128:(r + 1) * 128].float().cpu().numpy(), ref,
                           "f16" if dtype == "f16" else "bf16", f"dds4w NT col {r}")


# ----------------------------------------------------------------- DSD TN --
# C = A^T . B, A sparse [k][m] through its transposed metadata (MegaBlocks'
# dw2 = h^T . dy): the shared image is the stored block's k-row slice, read
# transposed (dsd4w.hip kTn).
TN_CASES = [
    # m (= A's columns), k (= A's rows), n, density
    (4096, 4096, 4096, 0.5),
    (4096, 4096, 4096, 0.1),
    (4096, 4096, 4096, 0.9),
    (2048, 4096, 4096, 0.3),
    (4096, 2048, 1032, 0.5),
    (8192, 2048, 2048, 0.3),
]


@pytest.mark.parametrize("m,k,n,density", TN_CASES)
@pytest.mark.parametrize("dtype", ["f16", "bf16"])
def test_dsd4w_tn_bit_identical_to_8wave(m, k, n, density, dtype):
    At, B, off, idx, a, b = _problem(k, m, n, density, dtype, seed=m + 5 * n + int(density * 10))
    # _problem built A as [k][m] (its k-dim = m here) and B as [m][n]; B must
    # be [k][n]
    td = torch.float16 if dtype == "f16" else torch.bfloat16
    g = torch.Generator(device="cuda")
    g.manual_seed(m * 3 + n)
    bb = (torch.rand(k * n, generator=g, device="cuda") * 2 - 1).to(td)
    Bm = sp.Matrix(k, n, bb)
    sp.AllocateTransposeBuffers(At)
    sp.Transpose(At)

    def run(mode):
        c = torch.full((m * n,), float("nan"), dtype=td, device="cuda")
        prev = sp.select_dsd_kernel(mode)
        try:
            sp.MatmulEx(At, True, Bm, False, sp.Matrix(m, n, c))
            torch.cuda.synchronize()
        finally:
            sp.select_dsd_kernel(prev)
        return c.view(m, n)

    c4, c8 = run(1), run(0)
    assert not torch.isnan(c4.float()).any()
    assert torch.equal(c4, c8), (
        f"max diff {float((c4.float() - c8.float()).abs().max())}")
    assert sp.pair_errors() == 0
    if (m, k, n, density) == (2048, 4096, 4096, 0.3):
        av = a.float().cpu().numpy().reshape(-1, 128, 128)
        dense_a = np.zeros((k, m), np.float32)
        rows = np.repeat(np.arange(k // 128), np.diff(off))
        for e in range(int(off[-1])):
            r, c = int(rows[e]), int(idx[e])
            dense_a[r * 128:(r + 1) * 128, c * 128:(c + 1) * 128] = av[e]
        bv = bb.float().cpu().numpy().reshape(k, n)
        ref = O.gemm(dense_a[:, :256], True, bv, False, threads=H.oracle_threads())
        H.assert_close(c4[:256].float().cpu().numpy(), ref,
                       "f16" if dtype == "f16" else "bf16", "dsd4w TN rows 0..255")


# ----------------------------------------------------------------- DDS TN --
# C = A^T . B, A stored [k][m] (MegaBlocks' dw1 = x^T . dh's shape): A's
# k-row slices per wave, read transposed (dsd4w.hip kDds + kTn).

@pytest.mark.parametrize("m,k,n,density", DDS_CASES)
@pytest.mark.parametrize("dtype", ["f16", "bf16"])
def test_dds4w_tn_bit_identical_to_8wave(m, k, n, density, dtype):
    _, B, off, idx, a, b = _dds_problem(m, k, n, density, dtype,
                                        seed=2 * m + n + int(density * 100))
    At = sp.Matrix(k, m, a)  # the same m * k values, stored [k][m]
    td = torch.float16 if dtype == "f16" else torch.bfloat16

    def run(mode):
        c = torch.full((m * n,), float("nan"), dtype=td, device="cuda")
        prev = sp.select_dsd_kernel(mode)
        try:
            sp.MatmulEx(At, True, B, False, sp.Matrix(m, n, c))
            torch.cuda.synchronize()
        finally:
            sp.select_dsd_kernel(prev)
        return c.view(m, n)

    c4, c8 = run(1), run(0)
    assert not torch.isnan(c4.float()).any()
    assert torch.equal(c4, c8), (
        f"max diff {float((c4.float() - c8.float()).abs().max())}")
    assert sp.pair_errors() == 0
    if (m, k, n) == (1152, 2048, 2048):
        av = a.float().cpu().numpy().reshape(k, m)
        bv = b.float().cpu().numpy().reshape(-1, 128, 128)
        rows = np.repeat(np.arange(k // 128), np.diff(off))
        for c in (0, 9):
            col = np.zeros((k, 128), np.float32)
            for e in np.nonzero(idx == c)[0]:
                r = int(rows[e])
                col[r * 128:(r + 1) * 128] = bv[e]
            ref = O.gemm(av, True, col, False, threads=H.oracle_threads())
            H.assert_close(c4[:, c * 128:(c + 1) * 128].float().cpu().numpy(), ref,
                           "f16" if dtype == "f16" else "bf16", f"dds4w TN col {c}")


# ----------------------------------------------------------------- DSD TT --
@pytest.mark.parametrize("m,k,n,density", [c for c in TN_CASES if c[2] % 128 == 0])
@pytest.mark.parametrize("dtype", ["f16", "bf16"])
def test_dsd4w_tt_bit_identical_to_8wave(m, k, n, density, dtype):
    At, _, off, idx, a, _ = _problem(k, m, n, density, dtype, seed=m + 7 * n + int(density * 10))
    td = torch.float16 if dtype == "f16" else torch.bfloat16
    g = torch.Generator(device="cuda")
    g.manual_seed(m * 5 + n)
    bt = (torch.rand(n * k, generator=g, device="cuda") * 2 - 1).to(td)
    Bt = sp.Matrix(n, k, bt)
    sp.AllocateTransposeBuffers(At)
    sp.Transpose(At)

    def run(mode):
        c = torch.full((m * n,), float("nan"), dtype=td, device="cuda")
        prev = sp.select_dsd_kernel(mode)
        try:
            sp.MatmulEx(At, True, Bt, True, sp.Matrix(m, n, c))
            torch.cuda.synchronize()
        finally:
            sp.select_dsd_kernel(prev)
        return c.view(m, n)

    c4, c8 = run(1), run(0)
    assert not torch.isnan(c4.float()).any()
    assert torch.equal(c4, c8), (
        f"max diff {float((c4.float() - c8.float()).abs().max())}")
    assert sp.pair_errors() == 0
    if (m, k, n, density) == (2048, 4096, 4096, 0.3):
        av = a.float().cpu().numpy().reshape(-1, 128, 128)
        dense_a = np.zeros((k, m), np.float32)
        rows = np.repeat(np.arange(k // 128), np.diff(off))
        for e in range(int(off[-1])):
            r, c = int(rows[e]), int(idx[e])
            dense_a[r * 128:(r + 1) * 128, c * 128:(c + 1) * 128] = av[e]
        bv = bt.float().cpu().numpy().reshape(n, k)
        ref = O.gemm(dense_a[:, :256], True, bv, True, threads=H.oracle_threads())
        H.assert_close(c4[:256].float().cpu().numpy(), ref,
                       "f16" if dtype == "f16" else "bf16", "dsd4w TT rows 0..255")


# ----------------------------------------------------------------- DDS TT --
@pytest.mark.parametrize("m,k,n,density", DDS_CASES)
@pytest.mark.parametrize("dtype", ["f16", "bf16"])
def test_dds4w_tt_bit_identical_to_8wave(m, k, n, density, dtype):
    rng = np.random.default_rng(m + 3 * n + 11)
    R, C = n // 128, k // 128
    nz = mu.nonzeros_for_density(n, k, density) // (128 * 128)
    off, idx = mu.random_topology(R, C, nz, rng, unordered=True)
    td = torch.float16 if dtype == "f16" else torch.bfloat16
    g = torch.Generator(device="cuda")
    g.manual_seed(m + 2 * k)
    nb = int(off[-1])
    a = (torch.rand(m * k, generator=g, device="cuda") * 2 - 1).to(td)
    b = (torch.rand(max(nb, 1) * 16384, generator=g, device="cuda") * 2 - 1).to(td)
    B = sp.BlockMatrix(n, k, 128, nb * 16384, b,
                       torch.from_numpy(np.asarray(off, np.int32)).cuda(),
                       torch.from_numpy(np.asarray(idx).astype(np.int16)).cuda())
    At = sp.Matrix(k, m, a)

    def run(mode):
        c = torch.full((m * n,), float("nan"), dtype=td, device="cuda")
        prev = sp.select_dsd_kernel(mode)
        try:
            sp.MatmulEx(At, True, B, True, sp.Matrix(m, n, c))
            torch.cuda.synchronize()
        finally:
            sp.select_dsd_kernel(prev)
        return c.view(m, n)

    c4, c8 = run(1), run(0)
    assert not torch.isnan(c4.float()).any()
    assert torch.equal(c4, c8), (
        f"max diff {float((c4.float() - c8.float()).abs().max())}")
    assert sp.pair_errors() == 0
    if (m, k, n) == (1152, 2048, 2048):
        av = a.float().cpu().numpy().reshape(k, m)
        bv = b.float().cpu().numpy().reshape(-1, 128, 128)
        rows = np.repeat(np.arange(R), np.diff(off))
        for r in (0, 5):
            blk = np.zeros((128, k), np.float32)
            for e in np.nonzero(rows == r)[0]:
                blk[:, idx[e] * 128:(idx[e] + 1) * 128] = bv[e]
            ref = O.gemm(av, True, blk, True, threads=H.oracle_threads())
            H.assert_close(c4[:, r * 128:(r + 1) * 128].float().cpu().numpy(), ref,
                           "f16" if dtype == "f16" else "bf16", f"dds4w TT col {r}")


def test_dsd4w_index_preload_odd_count_last_entry():
    """Regression: the index list is preloaded with 16-byte buffer loads
    whose range check is per dword; with an odd number of entries the last
    entry shares its dword with the end of the list. Block-rows of 3, 3,
    ..., 2, 1 blocks (93 entries): the last row holds only entry 92 and runs
    as a plain tile whose first k-block comes from the preload."""
    R = 32
    counts = [3] * 30 + [2, 1]
    off = np.zeros(R + 1, np.int32)
    np.cumsum(counts, out=off[1:])
    rng = np.random.default_rng(4)
    idx = np.concatenate([np.sort(rng.choice(np.arange(1, 32), c, replace=False))
                          for c in counts]).astype(np.int16)
    nb = int(off[-1])
    assert nb % 2 == 1 and idx[-1] != 0
    g = torch.Generator(device="cuda")
    g.manual_seed(4)
    a = (torch.rand(nb * 16384, generator=g, device="cuda") * 2 - 1).half()
    b = (torch.rand(4096 * 4096, generator=g, device="cuda") * 2 - 1).half()
    A = sp.BlockMatrix(4096, 4096, 128, nb * 16384, a,
                       torch.from_numpy(off).cuda(), torch.from_numpy(idx).cuda())
    B = sp.Matrix(4096, 4096, b)
    c4 = _run(A, B, 4096, 4096, "f16", 5)
    c8 = _run(A, B, 4096, 4096, "f16", 0)
    assert torch.equal(c4, c8)
    av = a.float().cpu().numpy().reshape(-1, 128, 128)
    bv = b.float().cpu().numpy().reshape(4096, 4096)
    e = nb - 1
    ref = O.gemm(av[e], False, bv[int(idx[e]) * 128:(int(idx[e]) + 1) * 128], False,
                 threads=H.oracle_threads())
    H.assert_close(c4[31 * 128:].float().cpu().numpy(), ref, "f16", "last block-row")
