"""GPU parity at the BASELINE.json configurations, collected before the rest
of the GPU suite (file order) so that a -x stop or a time-out elsewhere cannot
hide them:

  config 2  DSD M=K=N=4096 fp16 at 10/30/50/90% density
  config 3  SDD then DDS (MegaBlocks forward/backward pair), 4096^3, 20%
  config 4  MegaBlocks dMoE MLP: 8 experts, 8192 tokens, d_model 4096,
            d_ff 14336, bf16 (SDD x.w1 at the expert blocks, DSD h.w2)
  config 5  DSD M=131072 K=N=4096 2%, and its row-panel split

Full-size launches. Configs 2 and 3: every output element against the CPU
oracle (oracle/). Config 4: every output block / row-block through float64
linearity checksums (row sums against the operands), plus every expert's
first and last block-row against the oracle. Config 5: every row through
the same checksum, sampled block-rows against the oracle, and
size-independent properties (exact zeros of empty rows, bit-identical
sharded results). Tolerance as
tests/helpers.py (1e-2 relative fp16, 2e-2 bf16). Config 1 is the host
reference alone (tests/test_oracle.py, bench.py's config-1 line).
"""

import numpy as np
import pytest

from oracle import oracle as O
from sputnik_amd import matrix_utils as mu
from tests import helpers as H

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected here, skipped: no device
    pytest.skip("no GPU", allow_module_level=True)

import sputnik_amd as sp  # noqa: E402

sp.lib()  # fail loudly if the native library is missing


def _sync():
    torch.cuda.synchronize()


@pytest.mark.parametrize("density", [0.1, 0.3, 0.5, 0.9])
def test_dsd_baseline_config_full(density):
    """BASELINE config 2 (M=K=N=4096) at its four densities: EVERY output
    element against the oracle (all 32 block-rows; the 16-thread oracle
    with the zero-block skip takes ~2-16 s per density), plus a row-sum
    checksum (linearity: C.1 = A.(B.1)) and the pair error count."""
    rng = np.random.default_rng(7)
    nz = mu.nonzeros_for_density(4096, 4096, density)
    A = H.HostSparse(4096, 4096, nz, rng)
    B = H.HostDense(4096, 4096, rng)
    C, c_t = H.empty_dense(4096, 4096)
    sp.Matmul(A.matrix, False, B.matrix, False, C)
    _sync()
    assert sp.pair_errors() == 0
    gpu = c_t.float().cpu().numpy()
    dense_a = A.dense()
    ref = O.gemm(dense_a, False, B.values, False, a_mask=A.mask(),
                 threads=H.oracle_threads())
    for r in range(32):
        rows = slice(r * 128, (r + 1) * 128)
        H.assert_close(gpu[rows], ref[rows], "f16", f"row-block {r}")
    ones = B.values.astype(np.float64).sum(axis=1)
    checksum = dense_a.astype(np.float64) @ ones
    got = gpu.astype(np.float64).sum(axis=1)
    scale = np.sqrt(np.mean(checksum ** 2))
    assert np.abs(got - checksum).max() <= 2e-2 * scale + 1e-2 * np.abs(checksum).max()


def test_sdd_dds_pair_config3_full():
    """BASELINE config 3 (MegaBlocks fwd/bwd pair at 4096^3, 20%): every one
    of the 205 SDD blocks and every element of the DDS output against the
    oracle (the DDS on the SDD output as produced, rounded to fp16)."""
    rng = np.random.default_rng(11)
    nz = mu.nonzeros_for_density(4096, 4096, 0.2)
    x = H.HostDense(4096, 4096, rng)
    w = H.HostDense(4096, 4096, rng)
    Cs = H.HostSparse(4096, 4096, nz, rng)
    sp.AllocateRowIndicesBuffer(Cs.matrix)
    sp.RowIndices(Cs.matrix, Cs.matrix.row_indices)
    sp.Matmul(x.matrix, False, w.matrix, False, Cs.matrix)      # SDD
    g = H.HostDense(4096, 4096, rng)
    sp.AllocateTransposeBuffers(Cs.matrix)
    out, out_t = H.empty_dense(4096, 4096)
    sp.Matmul(g.matrix, False, Cs.matrix, False, out)            # DDS
    _sync()
    assert sp.pair_errors() == 0
    blocks = Cs.dev_values.float().cpu().numpy()
    rows = np.repeat(np.arange(32), np.diff(Cs.offsets))
    ref = O.gemm(x.values, False, w.values, False, out_mask=Cs.mask(),
                 threads=H.oracle_threads())
    for b in range(len(rows)):
        r, c = rows[b], Cs.indices[b]
        H.assert_close(blocks[b], ref[r * 128:(r + 1) * 128, c * 128:(c + 1) * 128],
                       "f16", f"sdd block {b}")
    sdd_dense = mu.to_dense(4096, 4096, Cs.offsets, Cs.indices, blocks)
    ref = O.gemm(g.values, False, sdd_dense, False, b_mask=Cs.mask(),
                 threads=H.oracle_threads())
    got = out_t.float().cpu().numpy()
    for r in range(32):
        H.assert_close(got[r * 128:(r + 1) * 128], ref[r * 128:(r + 1) * 128],
                       "f16", f"dds row-block {r}")


def _moe_setup(seed):
    E, T, DM, FF = 8, 8192, 4096, 14336
    cols = E * FF
    rpe, cpe = T // E // 128, FF // 128
    off, idx = mu.expert_block_diagonal(E, rpe, cpe)
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    rnd = lambda *s: (torch.rand(*s, generator=g, device="cuda") * 2 - 1).to(torch.bfloat16)
    return E, T, DM, FF, cols, rpe, cpe, off, idx, rnd


def _f64(t):
    return t.double().cpu().numpy()


def test_moe_config4_bf16_all_blocks():
    """BASELINE config 4 at full size (8 experts, 8192 tokens, d_model 4096,
    d_ff 14336, bf16, expert block-diagonal topology): SDD h = x.w1 at the
    expert blocks, then DSD y = h.w2.
      * all 7168 SDD blocks: row sums of h_b = x_r . (w1_c . 1);
      * all 64 DSD row-blocks: y . 1 = h . (w2 . 1);
      * every expert's first and last block-row of h (all its 112 blocks)
        and of y element by element against the oracle."""
    E, T, DM, FF, cols, rpe, cpe, off, idx, rnd = _moe_setup(4)
    nb = int(off[-1])
    x, w1, w2 = rnd(T, DM), rnd(DM, cols), rnd(cols, DM)
    hv = torch.full((nb, 128, 128), float("nan"), dtype=torch.bfloat16, device="cuda")
    Hm = sp.BlockMatrix(T, cols, 128, nb * 16384, hv,
                        torch.from_numpy(off).cuda(),
                        torch.from_numpy(idx.astype(np.int16)).cuda())
    sp.AllocateRowIndicesBuffer(Hm)
    sp.RowIndices(Hm, Hm.row_indices)
    y = torch.full((T, DM), float("nan"), dtype=torch.bfloat16, device="cuda")
    sp.Matmul(sp.Matrix(T, DM, x), False, sp.Matrix(DM, cols, w1), False, Hm)
    sp.Matmul(Hm, False, sp.Matrix(cols, DM, w2), False, sp.Matrix(T, DM, y))
    _sync()
    assert sp.pair_errors() == 0
    rows = np.repeat(np.arange(len(off) - 1), np.diff(off))
    # SDD checksum over every block: x (T x DM) . s1 (DM x cols/128), s1 the
    # per-block-column sums of w1
    x64 = _f64(x)
    s1 = _f64(w1).reshape(DM, cols // 128, 128).sum(axis=2)
    xs = x64 @ s1                                          # [T][cols/128]
    h32 = hv.float().cpu().numpy()                         # [nb][128][128]
    expect = xs.reshape(T // 128, 128, cols // 128)[rows, :, idx]   # [nb][128]
    H.rowsum_check(h32, expect, 2, "moe sdd")
    # DSD checksum over every row-block: y . 1 = sum_b h_b . v_c, v = w2 . 1
    v = _f64(w2).sum(axis=1).reshape(cols // 128, 128)
    hb = np.einsum("bij,bj->bi", h32.astype(np.float64), v[idx])    # [nb][128]
    ey = np.zeros((T // 128, 128))
    np.add.at(ey, rows, hb)
    y32 = y.float().cpu().numpy()
    H.rowsum_check(y32, ey.reshape(T), 1, "moe dsd")
    # every expert's first and last block-row against the oracle
    for e in range(E):
        for r in (e * rpe, (e + 1) * rpe - 1):
            c0 = e * cpe
            ref = O.gemm(x[r * 128:(r + 1) * 128].float().cpu().numpy(), False,
                         w1[:, c0 * 128:(c0 + cpe) * 128].float().cpu().numpy(),
                         False, threads=H.oracle_threads())
            got = h32[off[r]:off[r + 1]].transpose(1, 0, 2).reshape(128, FF)
            assert (idx[off[r]:off[r + 1]] == np.arange(c0, c0 + cpe)).all()
            H.assert_close(got, ref, "bf16", f"moe sdd block-row {r}")
            ref = O.gemm(got, False, w2[e * FF:(e + 1) * FF].float().cpu().numpy(),
                         False, threads=H.oracle_threads())
            H.assert_close(y32[r * 128:(r + 1) * 128], ref, "bf16",
                           f"moe dsd row-block {r}")


def test_moe_config4_backward_bf16_all_blocks():
    """The MegaBlocks backward of config 4's second layer at full size:
      dW2 = h^T . dy   (DSD TN: h^T has 896 block-rows, the tall path, with
                        h's transposed metadata built on the device),
      dh  = dy . W2^T  at h's blocks (SDD NT).
    Every output covered: dW2 . 1 = h^T . (dy . 1) over all 896 row-blocks,
    and the row sums of all 7168 dh blocks = dy_r . (W2_c^T . 1); every
    expert's first and last dW2 row-block and dh block-row against the
    oracle."""
    E, T, DM, FF, cols, rpe, cpe, off, idx, rnd = _moe_setup(44)
    nb = int(off[-1])
    hv, dy, w2 = rnd(nb, 128, 128), rnd(T, DM), rnd(cols, DM)
    mk = lambda vals: sp.BlockMatrix(T, cols, 128, nb * 16384, vals,
                                     torch.from_numpy(off).cuda(),
                                     torch.from_numpy(idx.astype(np.int16)).cuda())
    Hm = mk(hv)
    sp.AllocateTransposeBuffers(Hm)
    dw2 = torch.full((cols, DM), float("nan"), dtype=torch.bfloat16, device="cuda")
    sp.Matmul(Hm, True, sp.Matrix(T, DM, dy), False, sp.Matrix(cols, DM, dw2))
    dhv = torch.full((nb, 128, 128), float("nan"), dtype=torch.bfloat16,
                     device="cuda")
    dHm = mk(dhv)
    sp.AllocateRowIndicesBuffer(dHm)
    sp.RowIndices(dHm, dHm.row_indices)
    sp.Matmul(sp.Matrix(T, DM, dy), False, sp.Matrix(cols, DM, w2), True, dHm)
    _sync()
    assert sp.pair_errors() == 0
    rows = np.repeat(np.arange(len(off) - 1), np.diff(off))
    h32 = hv.float().cpu().numpy()
    dy64 = _f64(dy)
    # dW2 . 1 = h^T . u, u = dy . 1: block b adds h_b^T . u_r to row-block c
    u = dy64.sum(axis=1).reshape(T // 128, 128)
    cb = np.einsum("bij,bi->bj", h32.astype(np.float64), u[rows])   # [nb][128]
    ew = np.zeros((cols // 128, 128))
    np.add.at(ew, idx, cb)
    w32 = dw2.float().cpu().numpy()
    H.rowsum_check(w32, ew.reshape(cols), 1, "moe bwd dW2")
    # dh_b row sums = dy_r . s_c, s_c = sum of W2's rows in block c
    s = _f64(w2).reshape(cols // 128, 128, DM).sum(axis=1)        # [cols/128][DM]
    ds = dy64 @ s.T                                               # [T][cols/128]
    expect = ds.reshape(T // 128, 128, cols // 128)[rows, :, idx]
    d32 = dhv.float().cpu().numpy()
    H.rowsum_check(d32, expect, 2, "moe bwd dh")
    # every expert's first and last row-block / block-row against the oracle
    for e in range(E):
        t0, t1 = e * rpe * 128, (e + 1) * rpe * 128
        for c in (e * cpe, (e + 1) * cpe - 1):
            hcol = np.concatenate([h32[b] for b in range(off[e * rpe], off[(e + 1) * rpe])
                                   if idx[b] == c])
            assert hcol.shape == (t1 - t0, 128)
            ref = O.gemm(hcol.T.copy(), False, dy[t0:t1].float().cpu().numpy(),
                         False, threads=H.oracle_threads())
            H.assert_close(w32[c * 128:(c + 1) * 128], ref, "bf16",
                           f"moe bwd dW2 row-block {c}")
        for r in (e * rpe, (e + 1) * rpe - 1):
            ref = O.gemm(dy[r * 128:(r + 1) * 128].float().cpu().numpy(), False,
                         w2[e * FF:(e + 1) * FF].float().cpu().numpy(), True,
                         threads=H.oracle_threads())
            got = d32[off[r]:off[r + 1]].transpose(1, 0, 2).reshape(128, FF)
            H.assert_close(got, ref, "bf16", f"moe bwd dh block-row {r}")


def test_tall_panel_config5_sampled():
    """BASELINE config 5 at full size on one device: DSD M=131072, K=N=4096,
    2% density (656 blocks over 1024 block-rows, most rows empty). Every
    row's sum against the float64 linearity checksum C.1 = A.(B.1); empty
    block-rows must be exact zeros; sampled non-empty rows against the
    oracle; and the per-rank row-panel split (shard_rows_by_nnz) run as
    separate calls reproduces the single-call result bit-exactly."""
    rng = np.random.default_rng(5)
    M = 131072
    nz = mu.nonzeros_for_density(M, 4096, 0.02)
    A = H.HostSparse(M, 4096, nz, rng)
    B = H.HostDense(4096, 4096, rng)
    C, c_t = H.empty_dense(M, 4096)
    sp.Matmul(A.matrix, False, B.matrix, False, C)
    _sync()
    # every row: C . 1 = A . (B . 1), float64 from the operands
    v = B.values.astype(np.float64).sum(axis=1).reshape(32, 128)
    rows_of = np.repeat(np.arange(M // 128), np.diff(A.offsets))
    contrib = np.einsum("bij,bj->bi", A.values.astype(np.float64), v[A.indices])
    expect = np.zeros((M // 128, 128))
    np.add.at(expect, rows_of, contrib)
    H.rowsum_check(c_t.float().cpu().numpy(), expect.reshape(M), 1, "panel", "f16")
    counts = np.diff(A.offsets)
    empty = np.nonzero(counts == 0)[0]
    assert len(empty) > 0
    e_rows = torch.from_numpy(empty).cuda()
    blk = c_t.view(M // 128, 128, 4096)
    assert int(torch.count_nonzero(blk[e_rows])) == 0
    nonempty = np.nonzero(counts)[0]
    for r in (nonempty[0], nonempty[len(nonempty) // 2], nonempty[-1]):
        o0, o1 = A.offsets[r], A.offsets[r + 1]
        a_row = mu.to_dense(128, 4096, np.array([0, o1 - o0], np.int32),
                            A.indices[o0:o1], A.values[o0:o1])
        ref = O.gemm(a_row, False, B.values, False, threads=H.oracle_threads())
        H.assert_close(c_t[r * 128:(r + 1) * 128].float().cpu().numpy(), ref,
                       "f16", f"panel row-block {r}")
    # Row panels as 8 ranks would run them: same bits.
    for r0, r1 in mu.shard_rows_by_nnz(A.offsets, 8):
        if r1 == r0:
            continue
        po, pi, pv = mu.slice_block_rows(A.offsets, A.indices, A.values, r0, r1)
        nbp = len(pi)
        Pm = sp.BlockMatrix((r1 - r0) * 128, 4096, 128, nbp * 16384,
                            A.dev_values[A.offsets[r0]:A.offsets[r1]]
                            if nbp else A.dev_values,
                            torch.from_numpy(po).cuda(),
                            torch.from_numpy(pi.astype(np.int16)).cuda())
        Cp, cp_t = H.empty_dense((r1 - r0) * 128, 4096)
        sp.Matmul(Pm, False, B.matrix, False, Cp)
        _sync()
        assert torch.equal(cp_t, c_t[r0 * 128:r1 * 128])
