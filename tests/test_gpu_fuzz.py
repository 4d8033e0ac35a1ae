"""GPU: seeded topology fuzz of the 4-wave kernel (dsd4w.hip) for DSD, DDS
and the grouped SDD in every transpose.

Each case builds a topology with one of the edge cases the 4-wave kernel's
setup code branches on (VERDICT r04 "what's weak" 1): odd and even block
counts, a last block-row of 0, 1 or 2 blocks (with an odd count the last
entry shares its dword of the index list), 1023 / 1024 / 1025 stored blocks
(around the 1024-entry index preload, dsd4w.hip kIdxPreload), an index list
whose pointer is 2 bytes off 16-byte alignment and a transposed block-offset
list 4 bytes off (the scalar-load fallbacks),
heavy/light/empty rows (pair hand-offs), 8 / 16 / 32 block-rows (split mode,
pairs), and pair balancing on and off (tuning knob "pairs"). Then:

  * the default dispatch and the forced 4-wave kernel are bit-identical
    (torch.equal) to the 8-wave kernel (block_gemm.h), which shares no code
    with the 4-wave setup or asm body;
  * a 256-column window of the output (DSD / DDS: across three wave blocks
    of one 512-column tile; SDD: 40 stored blocks incl. the first and the
    last block-row's) against the CPU oracle (oracle/oracle.c, the
    reference's host matmul, matrix_utils.h:376-391) at the north-star
    tolerance (tests/helpers.py: 1e-2 relative fp16, 2e-2 bf16).

Reference test strategy: /root/reference/sputnik/block/dsd/dsd_test.cu:68-194
(random topologies over shapes x transposes, device vs host matmul); this
file adds the seeds and the edge cases the reference leaves to chance.
"""

import zlib

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

sp.lib()

B = 128


def _seed(*key):
    return zlib.crc32(repr(key).encode())  # stable across processes


# ---------------------------------------------------------------- topologies --

def _counts(kind, R, C, rng):
    """Blocks per row of the row operand for edge case `kind`."""
    if kind in ("nb1023", "nb1024", "nb1025"):
        total = int(kind[2:])
        c = np.full(R, total // R)
        c[: total % R] += 1
        # a ragged profile with the same total: move blocks between row pairs
        for _ in range(4 * R):
            i, j = rng.integers(0, R, 2)
            d = int(rng.integers(0, 4))
            if c[i] - d >= 1 and c[j] + d <= C:
                c[i] -= d
                c[j] += d
        if total % 2 == 1:  # last row: 1 block, the odd entry
            extra = c[-1] - 1
            c[-1] = 1
            for r in range(R - 1):
                take = min(extra, C - c[r])
                c[r] += take
                extra -= take
        return c
    c = rng.integers(max(1, C // 4), max(2, (3 * C) // 4) + 1, R)
    if kind == "skewed":  # heavy / light / empty rows: many pair hand-offs
        c = np.where(np.arange(R) % 2 == 0, rng.integers((7 * C) // 8, C + 1, R),
                     rng.integers(0, 3, R))
        c[R // 3] = 0
    elif kind == "last0":
        c[-1] = 0
        c[0] = 0
    elif kind == "odd_last1":
        c[-1] = 1
        if c.sum() % 2 == 0:
            c[0] += 1 if c[0] < C else -1
    elif kind == "even_last2":
        c[-1] = 2
        if c.sum() % 2 == 1:
            c[0] += 1 if c[0] < C else -1
    elif kind == "odd":
        if c.sum() % 2 == 0:
            c[1] += 1 if c[1] < C else -1
    return c


def row_topology(kind, R, C, rng):
    """(offsets, indices) of the row operand (op(A) for DSD, op(B)^T for
    DDS, C for SDD): R block-rows over C block-columns, each row's columns
    in random (unsorted) order; the last row's blocks never include column
    0 (a zero read in place of the index would then be visible)."""
    c = _counts(kind, R, C, rng).astype(np.int64)
    assert c.min() >= 0 and c.max() <= C, c
    off = np.zeros(R + 1, np.int32)
    np.cumsum(c, out=off[1:])
    idx = []
    for r in range(R):
        pool = np.arange(1, C) if r == R - 1 and c[r] < C else np.arange(C)
        idx.append(rng.choice(pool, int(c[r]), replace=False))
    idx = np.concatenate(idx).astype(np.int16) if R else np.zeros(0, np.int16)
    return off, idx


def stored_from_rows(off_r, idx_r, cols_r):
    """The stored CSR of a matrix whose TRANSPOSE has the row topology
    (off_r, idx_r): its rows are the row topology's columns (oracle
    Transpose, transpose.cu:87-104)."""
    off_t, idx_t, _ = O.transpose(off_r, idx_r, cols_r)
    return off_t, idx_t


def dev_index(idx, unaligned):
    """int16 index list on the device; `unaligned`: the pointer is 2 bytes
    past a 16-byte boundary (the 4-wave kernel's preload then falls back to
    scalar loads)."""
    t = torch.from_numpy(np.concatenate([[0], idx]).astype(np.int16)
                         if unaligned else idx.astype(np.int16)).cuda()
    if unaligned:
        t = t[1:]
        assert t.data_ptr() % 16 == 2
    return t


def dev_offsets(nb):
    """int32 block-offset list (filled by Transpose) 4 bytes past a 16-byte
    boundary: the 4-wave kernel's block-offset preload falls back to scalar
    loads."""
    t = torch.empty(nb + 1, dtype=torch.int32, device="cuda")[1:]
    assert t.data_ptr() % 16 == 4
    return t


def rnd(n, g, td):
    return (torch.rand(max(n, 1), generator=g, device="cuda") * 2 - 1).to(td)


def run_modes(fn):
    """fn() under the default dispatch (1), the forced 4-wave kernel (5:
    double slots, the shipped variant) and the 8-wave kernel (0)."""
    out = {}
    for mode in (1, 5, 0):
        prev = sp.select_dsd_kernel(mode)
        try:
            out[mode] = fn()
            torch.cuda.synchronize()
        finally:
            sp.select_dsd_kernel(prev)
    return out


def check_modes(out):
    ref = out[0]
    assert not torch.isnan(ref.float()).any()
    for mode in (1, 5):
        assert torch.equal(out[mode], ref), (
            f"mode {mode} vs 8-wave: max diff "
            f"{float((out[mode].float() - ref.float()).abs().max())}")
    assert sp.pair_errors() == 0


def window(rng, n_cols):
    """256 columns across three 128-column wave blocks of one 512 tile."""
    if n_cols <= 256:
        return 0, n_cols
    panels = max(1, n_cols // 512)
    p = int(rng.integers(0, panels))
    w = int(rng.integers(0, 3))
    c0 = min(512 * p + 128 * w + 64, n_cols - 256)
    return c0, c0 + 256


class Pairs:
    def __init__(self, on):
        self.on = on

    def __enter__(self):
        self.prev = sp.tuning("pairs", 1 if self.on else 0)

    def __exit__(self, *a):
        sp.tuning("pairs", self.prev)


# ----------------------------------------------------------------------- DSD --

DSD_CASES = [
    # kind, R (block-rows of op(A)), K block-cols, N, unaligned indices
    ("odd_last1", 32, 32, 4096, False),
    ("even_last2", 32, 32, 4096, False),
    ("last0", 32, 32, 4096, False),
    ("odd", 32, 32, 4096, True),
    ("nb1023", 32, 64, 4096, False),
    ("nb1024", 32, 64, 4096, False),
    ("nb1025", 32, 64, 4096, False),
    ("nb1025", 32, 64, 4096, True),
    ("skewed", 32, 32, 4096, False),
    ("odd_last1", 16, 32, 4096, False),   # split mode (4-wave, 512-col tiles)
    ("odd_last1", 8, 32, 4096, False),    # split mode (8-wave, 256-col tiles)
    ("skewed", 8, 32, 2048, True),
]


@pytest.mark.parametrize("kind,R,KB,N,unaligned", DSD_CASES)
@pytest.mark.parametrize("trans", ["NN", "NT", "TN", "TT"])
@pytest.mark.parametrize("pairs", [True, False])
def test_fuzz_dsd(kind, R, KB, N, unaligned, trans, pairs):
    ta, tb = trans[0] == "T", trans[1] == "T"
    seed = _seed(kind, R, KB, N, unaligned, trans)
    rng = np.random.default_rng(seed)
    M, K = R * B, KB * B
    off_r, idx_r = row_topology(kind, R, KB, rng)
    # A stored [M][K] (NN) or [K][M] with op(A)'s rows its columns (TN / TT)
    off, idx = stored_from_rows(off_r, idx_r, KB) if ta else (off_r, idx_r)
    nb = int(off[-1])
    dtype = "bf16" if kind == "odd" else "f16"
    td = H.torch_dtype(dtype)
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    a = rnd(nb * B * B, g, td)
    b = rnd(K * N, g, td)
    A = sp.BlockMatrix(K if ta else M, M if ta else K, B, nb * B * B, a,
                       torch.from_numpy(off.astype(np.int32)).cuda(),
                       dev_index(idx, unaligned and not ta))
    if ta:
        sp.AllocateTransposeBuffers(A)
        if unaligned:  # A^T's index list (the one the kernel reads) off by 2
            A.indices_t = dev_index(np.zeros(nb, np.int16), True)
            A.block_offsets = dev_offsets(nb)
        sp.Transpose(A)
    Bm = sp.Matrix(N, K, b) if tb else sp.Matrix(K, N, b)

    def go():
        c = torch.full((M, N), float("nan"), dtype=td, device="cuda")
        sp.MatmulEx(A, ta, Bm, tb, sp.Matrix(M, N, c))
        return c

    with Pairs(pairs):
        out = run_modes(go)
    check_modes(out)
    c0, c1 = window(rng, N)
    av = a.float().cpu().numpy()[: max(nb, 1) * B * B].reshape(-1, B, B)[:nb]
    dense = mu.to_dense(K if ta else M, M if ta else K, off, idx, av)
    op_a = dense.T if ta else dense
    bv = b.float().cpu().numpy().reshape(N, K).T if tb else \
        b.float().cpu().numpy().reshape(K, N)
    ref = O.gemm(np.ascontiguousarray(op_a), False,
                 np.ascontiguousarray(bv[:, c0:c1]), False,
                 a_mask=mu.block_mask(off_r, idx_r, KB),
                 threads=H.oracle_threads())
    H.assert_close(out[1][:, c0:c1].float().cpu().numpy(), ref, dtype,
                   f"dsd {trans} {kind} cols {c0}:{c1}")
    empty = np.nonzero(np.diff(off_r) == 0)[0]
    for r in empty:
        assert int(torch.count_nonzero(out[1][r * B:(r + 1) * B])) == 0


# ----------------------------------------------------------------------- DDS --

DDS_CASES = [
    # kind, R (block-rows of op(B)^T = N / 128), K block-cols, M, unaligned
    ("odd_last1", 32, 32, 4096, False),
    ("last0", 32, 32, 4096, True),
    ("nb1025", 32, 64, 4096, False),
    ("nb1023", 32, 64, 2048, True),
    ("skewed", 32, 32, 4096, False),
    ("even_last2", 16, 32, 4096, False),
]


@pytest.mark.parametrize("kind,R,KB,M,unaligned", DDS_CASES)
@pytest.mark.parametrize("trans", ["NN", "NT", "TN", "TT"])
@pytest.mark.parametrize("pairs", [True, False])
def test_fuzz_dds(kind, R, KB, M, unaligned, trans, pairs):
    ta, tb = trans[0] == "T", trans[1] == "T"
    seed = _seed("dds", kind, R, KB, M, unaligned, trans)
    rng = np.random.default_rng(seed)
    N, K = R * B, KB * B
    # row operand op(B)^T: [N][K]; B stored [K][N] (NN / TN: column order,
    # the transposed metadata) or [N][K] (NT / TT: the stored rows)
    off_r, idx_r = row_topology(kind, R, KB, rng)
    off, idx = (off_r, idx_r) if tb else stored_from_rows(off_r, idx_r, KB)
    nb = int(off[-1])
    dtype = "bf16" if kind == "even_last2" else "f16"
    td = H.torch_dtype(dtype)
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    a = rnd(M * K, g, td)
    bvals = rnd(nb * B * B, g, td)
    Bs = sp.BlockMatrix(N if tb else K, K if tb else N, B, nb * B * B, bvals,
                        torch.from_numpy(off.astype(np.int32)).cuda(),
                        dev_index(idx, unaligned and tb))
    if not tb:
        sp.AllocateTransposeBuffers(Bs)
        if unaligned:
            Bs.indices_t = dev_index(np.zeros(nb, np.int16), True)
            Bs.block_offsets = dev_offsets(nb)
        sp.Transpose(Bs)
    Am = sp.Matrix(K, M, a) if ta else sp.Matrix(M, K, a)

    def go():
        c = torch.full((M, N), float("nan"), dtype=td, device="cuda")
        sp.MatmulEx(Am, ta, Bs, tb, sp.Matrix(M, N, c))
        return c

    with Pairs(pairs):
        out = run_modes(go)
    check_modes(out)
    # rows of C = the j dimension of the 4-wave tile: a 256-row window
    r0, r1 = window(rng, M)
    av = a.float().cpu().numpy().reshape(K, M).T if ta else \
        a.float().cpu().numpy().reshape(M, K)
    bv = bvals.float().cpu().numpy()[: max(nb, 1) * B * B].reshape(-1, B, B)[:nb]
    dense_b = mu.to_dense(N if tb else K, K if tb else N, off, idx, bv)
    op_b = dense_b.T if tb else dense_b
    ref = O.gemm(np.ascontiguousarray(av[r0:r1]), False, np.ascontiguousarray(op_b),
                 False, b_mask=mu.block_mask(off_r, idx_r, KB).T.copy(),
                 threads=H.oracle_threads())
    H.assert_close(out[1][r0:r1].float().cpu().numpy(), ref, dtype,
                   f"dds {trans} {kind} rows {r0}:{r1}")
    for c in np.nonzero(np.diff(off_r) == 0)[0]:
        assert int(torch.count_nonzero(out[1][:, c * B:(c + 1) * B])) == 0


# ----------------------------------------------------------------------- SDD --

SDD_CASES = [
    # kind, R (block-rows of C), NB block-cols of C, K
    ("odd_last1", 32, 96, 1024),
    ("even_last2", 32, 96, 512),
    ("last0", 32, 96, 1024),
    ("nb1025", 32, 64, 1024),
    ("skewed", 32, 96, 512),
]


@pytest.mark.parametrize("kind,R,NB,K", SDD_CASES)
@pytest.mark.parametrize("trans", ["NN", "NT", "TN", "TT"])
def test_fuzz_sdd(kind, R, NB, K, trans):
    ta, tb = trans[0] == "T", trans[1] == "T"
    seed = _seed("sdd", kind, R, NB, K, trans)
    rng = np.random.default_rng(seed)
    M, N = R * B, NB * B
    off, idx = row_topology(kind, R, NB, rng)
    nb = int(off[-1])
    dtype = "bf16" if kind == "even_last2" else "f16"
    td = H.torch_dtype(dtype)
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    a = rnd(M * K, g, td)
    b = rnd(K * N, g, td)
    cv = torch.empty(nb * B * B, dtype=td, device="cuda")
    Cm = sp.BlockMatrix(M, N, B, nb * B * B, cv,
                        torch.from_numpy(off.astype(np.int32)).cuda(),
                        torch.from_numpy(idx.astype(np.int16)).cuda())
    sp.AllocateRowIndicesBuffer(Cm)
    sp.RowIndices(Cm, Cm.row_indices)
    Am = sp.Matrix(K, M, a) if ta else sp.Matrix(M, K, a)
    Bm = sp.Matrix(N, K, b) if tb else sp.Matrix(K, N, b)
    # grouped tiles (the 4-wave SDD) from 4 blocks per CU, so these
    # 1000-1300-block problems take them
    prev = sp.tuning("grouped_min_per_cu", 4)
    try:
        assert sp.sdd_plan(Am, ta, Bm, tb, Cm) == 1

        def go():
            cv.fill_(float("nan"))
            sp.Matmul(Am, ta, Bm, tb, Cm)
            return cv.clone()

        out = run_modes(go)
    finally:
        sp.tuning("grouped_min_per_cu", prev)
    check_modes(out)
    got = out[1].view(-1, B, B).float().cpu().numpy()
    av = a.float().cpu().numpy().reshape(K, M).T if ta else \
        a.float().cpu().numpy().reshape(M, K)
    bv = b.float().cpu().numpy().reshape(N, K).T if tb else \
        b.float().cpu().numpy().reshape(K, N)
    rows = np.repeat(np.arange(R), np.diff(off))
    pick = sorted(set([0, 1, 2, 3, nb - 1, nb - 2, nb - 3]
                      + [int(x) for x in rng.choice(nb, 33, replace=False)]))
    for e in pick:
        if not 0 <= e < nb:
            continue
        r, c = int(rows[e]), int(idx[e])
        ref = O.gemm(np.ascontiguousarray(av[r * B:(r + 1) * B]), False,
                     np.ascontiguousarray(bv[:, c * B:(c + 1) * B]), False)
        H.assert_close(got[e], ref, dtype, f"sdd {trans} {kind} block {e}")


# -------------------------------------------------------------- tall DSD --

TALL_CASES = [
    # kind, R (block-rows, > 256: tall), KB, N, unaligned
    ("skewed", 320, 16, 2048, False),
    ("last0", 300, 8, 1024, True),
    ("odd_last1", 280, 32, 512, False),
]


@pytest.mark.parametrize("kind,R,KB,N,unaligned", TALL_CASES)
def test_fuzz_dsd_tall_pipe(kind, R, KB, N, unaligned):
    """Tall DSD NN on the 4-wave pipeline (plan 4, dsd4w.hip kEpi 7) against
    the 8-wave tall tile (knob tall4w = 0) and the oracle: random values,
    skewed / empty / 1-block rows, an index list off 16-byte alignment.
    The two kernels sum each 128 x 128 block's k-blocks in the same order
    (CSR order, 32-deep MFMA steps), so they agree bit for bit."""
    seed = _seed("tall", kind, R, KB, N, unaligned)
    rng = np.random.default_rng(seed)
    M, K = R * B, KB * B
    off, idx = row_topology(kind, R, KB, rng)
    nb = int(off[-1])
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    a = rnd(nb * B * B, g, torch.float16)
    b = rnd(K * N, g, torch.float16)
    A = sp.BlockMatrix(M, K, B, nb * B * B, a,
                       torch.from_numpy(off.astype(np.int32)).cuda(),
                       dev_index(idx, unaligned))
    Bm = sp.Matrix(K, N, b)

    def go(tall4w):
        prev = sp.tuning("tall4w", tall4w)
        try:
            c = torch.full((M, N), float("nan"), dtype=torch.float16, device="cuda")
            plan = sp.dsd_plan(A, False, Bm, False, sp.Matrix(M, N, c))
            sp.Matmul(A, False, Bm, False, sp.Matrix(M, N, c))
            torch.cuda.synchronize()
            return c, plan
        finally:
            sp.tuning("tall4w", prev)
    got, plan = go(1)
    ref8, plan8 = go(0)
    assert plan == 4 and plan8 == 2, (plan, plan8)
    assert not torch.isnan(got.float()).any()
    assert torch.equal(got, ref8), float((got.float() - ref8.float()).abs().max())
    av = a.float().cpu().numpy()[: max(nb, 1) * B * B].reshape(-1, B, B)[:nb]
    bv = b.float().cpu().numpy().reshape(K, N)
    counts = np.diff(off)
    rows = sorted(set([0, R - 1, int(np.argmax(counts))] +
                      [int(x) for x in rng.choice(R, 5, replace=False)]))
    for r in rows:
        o0, o1 = off[r], off[r + 1]
        a_row = mu.to_dense(128, K, np.array([0, o1 - o0], np.int32), idx[o0:o1], av[o0:o1])
        ref = O.gemm(a_row, False, bv, False, threads=H.oracle_threads())
        H.assert_close(got[r * B:(r + 1) * B].float().cpu().numpy(), ref, "f16",
                       f"tall {kind} row-block {r}")

