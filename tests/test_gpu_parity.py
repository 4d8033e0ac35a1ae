"""GPU parity: the HIP kernels of libsputnik.so (called through the C-ABI via
sputnik_amd) against the CPU oracle, on the reference's own test problem
lists (sputnik/block/{dsd,dds,sdd}/*_test.cu) plus edge cases and the
BASELINE sizes.

Tolerance (tests/helpers.py): |gpu - ref| <= rtol*(|ref| + rms(ref)) with
rtol = 1e-2 (fp16) / 2e-2 (bf16) against the oracle GEMM of the rounded
inputs; additionally the reference's criterion, abs 5e-2 against the fp32
oracle of the un-rounded inputs, on the reference problem lists. Metadata
builders (Transpose, RowIndices) must be bit-exact.
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


def _problems(op):
    return [pytest.param(p, id=f"{op}-{i}-m{p['m']}k{p['k']}n{p['n']}"
                         f"-nz{p['nonzeros']//16384}-{'T' if p['ta'] else 'N'}"
                         f"{'T' if p['tb'] else 'N'}{'-u' if p['unordered'] else ''}")
            for i, p in enumerate(H.load_problems(op))]


# --------------------------------------------------------------------- DSD --

def run_dsd(p, dtype="f16", seed=0, ex=False):
    rng = np.random.default_rng(seed)
    m, k, n, ta, tb = p["m"], p["k"], p["n"], p["ta"], p["tb"]
    a_rows, a_cols = (k, m) if ta else (m, k)
    A = H.HostSparse(a_rows, a_cols, p["nonzeros"], rng, dtype,
                     unordered=p["unordered"])
    B = H.HostDense(*((n, k) if tb else (k, n)), rng, dtype)
    C, c_t = H.empty_dense(m, n, dtype)
    if ta or ex:
        sp.AllocateTransposeBuffers(A.matrix)
    if ex:
        sp.Transpose(A.matrix)
        sp.MatmulEx(A.matrix, ta, B.matrix, tb, C)
    else:
        sp.Matmul(A.matrix, ta, B.matrix, tb, C)
    _sync()
    gpu = c_t.float().cpu().numpy()
    amask = A.mask().T if ta else A.mask()
    ref = O.gemm(A.dense(), ta, B.values, tb, a_mask=amask,
                 threads=H.oracle_threads())
    return gpu, ref, A, B


@pytest.mark.parametrize("p", _problems("dsd"))
def test_dsd_reference_problems(p):
    gpu, ref, A, B = run_dsd(p)
    H.assert_close(gpu, ref, "f16", "dsd")


@pytest.mark.parametrize("p", _problems("dsd")[::5])
def test_dsd_reference_criterion_unrounded(p):
    """abs 5e-2 vs the fp32 oracle of the *un-rounded* inputs, exactly the
    reference's check (dsd_test.cu:188-193)."""
    rng = np.random.default_rng(1)
    gpu, _, A, B = run_dsd(p, seed=1)
    m, k, n, ta, tb = p["m"], p["k"], p["n"], p["ta"], p["tb"]
    # Rebuild un-rounded inputs with the same stream: draw again identically.
    rng = np.random.default_rng(1)
    a_rows, a_cols = (k, m) if ta else (m, k)
    b_ = mu.BLOCK
    nb = p["nonzeros"] // (b_ * b_)
    off, idx = mu.random_topology(a_rows // b_, a_cols // b_, nb, rng,
                                  unordered=p["unordered"])
    vals = mu.random_values((nb, b_, b_), rng)
    braw = mu.random_values((n, k) if tb else (k, n), rng)
    dense_a = mu.to_dense(a_rows, a_cols, off, idx, vals)
    ref = O.gemm(dense_a, ta, braw, tb, threads=H.oracle_threads())
    assert np.abs(gpu - ref).max() <= H.REF_ABS_TOL


@pytest.mark.parametrize("p", _problems("dsd")[24:48:3])
def test_dsd_bf16(p):
    gpu, ref, _, _ = run_dsd(p, dtype="bf16")
    H.assert_close(gpu, ref, "bf16", "dsd-bf16")


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
def test_dsd_matmul_ex(ta, tb):
    p = dict(m=512, k=768, n=384, nonzeros=10 * 16384, ta=ta, tb=tb,
             unordered=True)
    gpu, ref, _, _ = run_dsd(p, ex=True)
    H.assert_close(gpu, ref, "f16", "dsd-ex")


def test_dsd_empty_rows_and_zero_matrix():
    rng = np.random.default_rng(3)
    # Block-rows 1 and 3 empty; C must be written with exact zeros there.
    offsets = np.array([0, 2, 2, 3, 3], dtype=np.int32)
    indices = np.array([0, 2, 1], dtype=np.int32)
    A = H.HostSparse(512, 384, 3 * 16384, rng, topology=(offsets, indices))
    B = H.HostDense(384, 264, rng)
    C, c_t = H.empty_dense(512, 264)
    sp.Matmul(A.matrix, False, B.matrix, False, C)
    _sync()
    gpu = c_t.float().cpu().numpy()
    assert (gpu[128:256] == 0).all() and (gpu[384:] == 0).all()
    ref = O.gemm(A.dense(), False, B.values, False)
    H.assert_close(gpu, ref, "f16")
    # No nonzero blocks at all.
    Z = H.HostSparse(256, 256, 0, rng,
                     topology=(np.zeros(3, np.int32), np.zeros(0, np.int32)))
    C2, c2 = H.empty_dense(256, 128)
    sp.Matmul(Z.matrix, False, H.HostDense(256, 128, rng).matrix, False, C2)
    _sync()
    assert (c2.float().cpu().numpy() == 0).all()


def test_dsd_deterministic():
    p = dict(m=1024, k=1024, n=1024, nonzeros=512 * 1024, ta=False, tb=False,
             unordered=False)
    rng = np.random.default_rng(5)
    A = H.HostSparse(1024, 1024, p["nonzeros"], rng)
    B = H.HostDense(1024, 1024, rng)
    outs = []
    for _ in range(2):
        C, c_t = H.empty_dense(1024, 1024)
        sp.Matmul(A.matrix, False, B.matrix, False, C)
        _sync()
        outs.append(c_t.clone())
    assert torch.equal(outs[0], outs[1])


def _skewed_topology(rows_b, cols_b, rng):
    """Block-rows with very different lengths (0 .. cols_b blocks): the LPT
    row ranking and its snake order see every rank."""
    mask = np.zeros((rows_b, cols_b), dtype=bool)
    for r in range(rows_b):
        n = int(rng.integers(0, cols_b + 1))
        mask[r, rng.choice(cols_b, n, replace=False)] = True
    mask[0, :] = True          # one full row
    mask[rows_b - 1, :] = False  # one empty row
    return mu.mask_to_bcsr(mask)


@pytest.mark.parametrize("op", ["dsd", "dds"])
@pytest.mark.parametrize("rows_b", [2, 7, 32, 63, 100])
def test_skewed_row_lengths(op, rows_b):
    """Skewed row lengths: DSD NN and DDS NT (row-order S) and their
    column-order variants, odd row counts, empty and full rows."""
    rng = np.random.default_rng(rows_b)
    kb = 24
    for t in (False, True):
        if op == "dsd":
            # C[M x N] = op(A) B; S = op(A), whose block-rows are A's rows
            # (NN) or, read through the transposed metadata, A's columns (TN).
            top = _skewed_topology(kb, rows_b, rng) if t else \
                _skewed_topology(rows_b, kb, rng)
            nz = int(top[0][-1]) * 16384
            A = H.HostSparse(*((kb * 128, rows_b * 128) if t else
                               (rows_b * 128, kb * 128)), nz, rng,
                             topology=top)
            B = H.HostDense(kb * 128, 512, rng)
            C, c_t = H.empty_dense(rows_b * 128, 512)
            if t:
                sp.AllocateTransposeBuffers(A.matrix)
            sp.Matmul(A.matrix, t, B.matrix, False, C)
            _sync()
            amask = A.mask().T if t else A.mask()
            ref = O.gemm(A.dense(), t, B.values, False, a_mask=amask,
                         threads=H.oracle_threads())
        else:
            # C[M x N] = A op(B); S = op(B)^T: B's columns (NN, transposed
            # metadata) or B's rows (NT).
            top = _skewed_topology(rows_b, kb, rng) if t else \
                _skewed_topology(kb, rows_b, rng)
            nz = int(top[0][-1]) * 16384
            Bs = H.HostSparse(*((rows_b * 128, kb * 128) if t else
                                (kb * 128, rows_b * 128)), nz, rng,
                              topology=top)
            A = H.HostDense(384, kb * 128, rng)
            C, c_t = H.empty_dense(384, rows_b * 128)
            if not t:
                sp.AllocateTransposeBuffers(Bs.matrix)
            sp.Matmul(A.matrix, False, Bs.matrix, t, C)
            _sync()
            bmask = Bs.mask().T if t else Bs.mask()
            ref = O.gemm(A.values, False, Bs.dense(), t, b_mask=bmask,
                         threads=H.oracle_threads())
        H.assert_close(c_t.float().cpu().numpy(), ref, "f16", f"{op} t={t}")


def test_graph_replay():
    """A launch captured into a HIP graph (torch.cuda.graph on a side stream)
    replays bit-identically, every time, and matches the oracle. (Inside a
    capture the pair hand-offs are off, so the captured kernel may sum in a
    different order than an eager launch; tests/test_gpu_kat.py checks the
    captured result exactly.)"""
    rng = np.random.default_rng(9)
    off, idx = _skewed_topology(16, 16, rng)
    A = H.HostSparse(2048, 2048, int(off[-1]) * 16384, rng,
                     topology=(off, idx))
    B = H.HostDense(2048, 1024, rng)
    C, c_t = H.empty_dense(2048, 1024)
    ref = O.gemm(A.dense(), False, B.values, False, a_mask=A.mask(),
                 threads=H.oracle_threads())
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        sp.Matmul(A.matrix, False, B.matrix, False, C)
    torch.cuda.current_stream().wait_stream(s)
    _sync()
    H.assert_close(c_t.float().cpu().numpy(), ref, "f16", "eager")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        sp.Matmul(A.matrix, False, B.matrix, False, C)
    c_t.fill_(float("nan"))
    g.replay()
    _sync()
    first = c_t.clone()
    H.assert_close(first.float().cpu().numpy(), ref, "f16", "replay")
    for _ in range(4):
        c_t.fill_(float("nan"))
        g.replay()
        _sync()
        assert torch.equal(c_t, first)


# --------------------------------------------------------------------- DDS --

def run_dds(p, dtype="f16", seed=0, ex=False):
    rng = np.random.default_rng(seed)
    m, k, n, ta, tb = p["m"], p["k"], p["n"], p["ta"], p["tb"]
    A = H.HostDense(*((k, m) if ta else (m, k)), rng, dtype)
    b_rows, b_cols = (n, k) if tb else (k, n)
    B = H.HostSparse(b_rows, b_cols, p["nonzeros"], rng, dtype,
                     unordered=p["unordered"])
    C, c_t = H.empty_dense(m, n, dtype)
    if not tb or ex:
        sp.AllocateTransposeBuffers(B.matrix)
    if ex:
        sp.Transpose(B.matrix)
        sp.MatmulEx(A.matrix, ta, B.matrix, tb, C)
    else:
        sp.Matmul(A.matrix, ta, B.matrix, tb, C)
    _sync()
    gpu = c_t.float().cpu().numpy()
    bmask = B.mask().T if tb else B.mask()
    ref = O.gemm(A.values, ta, B.dense(), tb, b_mask=bmask,
                 threads=H.oracle_threads())
    return gpu, ref


@pytest.mark.parametrize("p", _problems("dds"))
def test_dds_reference_problems(p):
    gpu, ref = run_dds(p)
    H.assert_close(gpu, ref, "f16", "dds")


@pytest.mark.parametrize("p", _problems("dds")[24:48:3])
def test_dds_bf16(p):
    gpu, ref = run_dds(p, dtype="bf16")
    H.assert_close(gpu, ref, "bf16", "dds-bf16")


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
def test_dds_matmul_ex(ta, tb):
    p = dict(m=264, k=640, n=512, nonzeros=9 * 16384, ta=ta, tb=tb,
             unordered=True)
    gpu, ref = run_dds(p, ex=True)
    H.assert_close(gpu, ref, "f16", "dds-ex")


# --------------------------------------------------------------------- SDD --

def run_sdd(p, dtype="f16", seed=0):
    rng = np.random.default_rng(seed)
    m, k, n, ta, tb = p["m"], p["k"], p["n"], p["ta"], p["tb"]
    A = H.HostDense(*((k, m) if ta else (m, k)), rng, dtype)
    B = H.HostDense(*((n, k) if tb else (k, n)), rng, dtype)
    Cs = H.HostSparse(m, n, p["nonzeros"], rng, dtype,
                      unordered=p["unordered"])
    Cs.dev_values.fill_(float("nan"))
    sp.AllocateRowIndicesBuffer(Cs.matrix)
    sp.RowIndices(Cs.matrix, Cs.matrix.row_indices)
    sp.Matmul(A.matrix, ta, B.matrix, tb, Cs.matrix)
    _sync()
    gpu_blocks = Cs.dev_values.float().cpu().numpy()
    mask = Cs.mask()
    ref_dense = O.gemm(A.values, ta, B.values, tb, out_mask=mask,
                       threads=H.oracle_threads())
    # Gather the reference at C's nonzero blocks, in storage order.
    rows = np.repeat(np.arange(len(Cs.offsets) - 1), np.diff(Cs.offsets))
    b_ = mu.BLOCK
    ref_blocks = np.stack([ref_dense[r * b_:(r + 1) * b_, c * b_:(c + 1) * b_]
                           for r, c in zip(rows, Cs.indices)]) \
        if len(rows) else np.zeros((0, b_, b_), np.float32)
    return gpu_blocks, ref_blocks


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("k", [1024, 1032, 2056])
def test_sdd_long_ragged_k(ta, tb, k):
    """SDD with long, ragged K (an odd number of 64-deep steps and a partial
    last step) on every transpose, unordered indices, against the oracle."""
    p = dict(m=512, k=k, n=640, nonzeros=9 * 16384, ta=ta, tb=tb,
             unordered=True)
    gpu, ref = run_sdd(p, seed=k)
    H.assert_close(gpu, ref, "f16", "sdd long k")
    if not ta and not tb:
        gpu, ref = run_sdd(p, dtype="bf16", seed=k + 1)
        H.assert_close(gpu, ref, "bf16", "sdd long k bf16")


def test_sdd_repeat_and_graph():
    """Repeated SDD calls and a captured graph replayed several times give
    identical bits."""
    p = dict(m=384, k=2048, n=512, nonzeros=7 * 16384, ta=False, tb=False,
             unordered=False)
    rng = np.random.default_rng(3)
    A = H.HostDense(384, 2048, rng)
    B = H.HostDense(2048, 512, rng)
    Cs = H.HostSparse(384, 512, p["nonzeros"], rng)
    sp.AllocateRowIndicesBuffer(Cs.matrix)
    sp.RowIndices(Cs.matrix, Cs.matrix.row_indices)
    sp.Matmul(A.matrix, False, B.matrix, False, Cs.matrix)
    _sync()
    first = Cs.dev_values.clone()
    for _ in range(5):
        sp.Matmul(A.matrix, False, B.matrix, False, Cs.matrix)
    _sync()
    assert torch.equal(Cs.dev_values, first)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):   # eager call on s: its workspace exists
        sp.Matmul(A.matrix, False, B.matrix, False, Cs.matrix)
    torch.cuda.current_stream().wait_stream(s)
    _sync()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        sp.Matmul(A.matrix, False, B.matrix, False, Cs.matrix)
    for _ in range(4):
        Cs.dev_values.fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(Cs.dev_values, first)


@pytest.mark.parametrize("p", _problems("sdd"))
def test_sdd_reference_problems(p):
    gpu, ref = run_sdd(p)
    H.assert_close(gpu, ref, "f16", "sdd")


@pytest.mark.parametrize("p", _problems("sdd")[16:40:3])
def test_sdd_bf16(p):
    gpu, ref = run_sdd(p, dtype="bf16")
    H.assert_close(gpu, ref, "bf16", "sdd-bf16")


@pytest.mark.parametrize("k", [8, 24, 72, 200])
def test_sdd_ragged_k(k):
    """K not a multiple of the 64-deep k-step (reference sdd_test K=8)."""
    for ta in (False, True):
        for tb in (False, True):
            p = dict(m=256, k=k, n=384, nonzeros=4 * 16384, ta=ta, tb=tb,
                     unordered=False)
            gpu, ref = run_sdd(p)
            H.assert_close(gpu, ref, "f16", f"sdd k={k} {ta}{tb}")


@pytest.mark.parametrize("k", [200, 1024])
@pytest.mark.parametrize("dtype", ["f16", "bf16"])
def test_sdd_grouped_tiles(k, dtype):
    """Enough output blocks (5 x CUs + 37 > the 4 x CUs of dispatch.cpp
    UseGroupedSdd) for
    the grouped SDD tiles: up to 4 consecutive stored blocks of a block-row
    per workgroup, rows whose block counts are not multiples of 4, unordered
    columns, a K tail, all four transposes; every block against the oracle.
    (test_gpu_kat.py asserts the plan at the same threshold.)"""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    nb = 5 * cus + 37
    m, n = 4096, 128 * max(64, -(-nb * 2 // 32))  # <= half of the block slots
    for ta in (False, True):
        for tb in (False, True):
            p = dict(m=m, k=k, n=n, nonzeros=nb * 16384, ta=ta, tb=tb,
                     unordered=True)
            gpu, ref = run_sdd(p, dtype=dtype, seed=k + 2 * ta + tb)
            H.assert_close(gpu, ref, dtype, f"sdd-grouped {ta}{tb} k={k}")


@pytest.mark.parametrize("op", ["dsd", "dds"])
@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("dtype", ["f16", "bf16"])
def test_tall_sparse_operand(op, ta, tb, dtype):
    """Sparse operands with more than 256 block-rows run on the tall tile
    configuration (two 128x256 workgroups per CU, dispatch.cpp UseTall):
    every transpose of DSD and DDS, a ragged dense extent (264: a partial
    256-wide tile), unordered indices, both dtypes, full-output oracle. The
    bf16 transposed products here are the MegaBlocks backward's kernel
    instances (DSD TN: dW2 = h^T dy over a tall h^T)."""
    tall = 300 * 128
    nz = 240 * 16384
    if op == "dsd":
        p = dict(m=tall, k=256, n=264, nonzeros=nz, ta=ta, tb=tb,
                 unordered=True)
        gpu, ref, _, _ = run_dsd(p, dtype=dtype)
    else:
        p = dict(m=264, k=256, n=tall, nonzeros=nz, ta=ta, tb=tb,
                 unordered=True)
        gpu, ref = run_dds(p, dtype=dtype)
    H.assert_close(gpu, ref, dtype, f"tall {op}")


# -------------------------------------------------------------- SSD / SDS --
# The reference's problem lists (sputnik/block/ssd/ssd_test.cu:76-140 and
# sds_test.cu:76-140), restated as data: (M, K, N, sparse-input blocks,
# output blocks); each runs with all four transposes.
_SS_SMALL = [(128, 128, 128, 1, 1), (128, 256, 128, 2, 1), (256, 128, 128, 2, 2),
             (128, 128, 256, 1, 2), (128, 256, 128, 1, 1), (128, 128, 256, 1, 2),
             (128, 256, 256, 1, 1), (256, 256, 256, 2, 2)]
_SS_LARGE = [(512, 512, 1024, 16, 32), (512, 512, 1024, 8, 16),
             (1024, 1024, 1024, 64, 64), (1024, 1024, 1024, 16, 16)]


def _ss_params():
    out = []
    for m, k, n, nin, nout in _SS_SMALL + _SS_LARGE:
        for ta in (False, True):
            for tb in (False, True):
                for unordered in ((False, True) if (m, k, n) == (256, 256, 256)
                                  else (False,)):
                    out.append(pytest.param(
                        (m, k, n, nin, nout, ta, tb, unordered),
                        id=f"m{m}k{k}n{n}-{nin}-{nout}-{'T' if ta else 'N'}"
                           f"{'T' if tb else 'N'}{'-u' if unordered else ''}"))
    return out


def _blocks_at(ref_dense, Cs):
    rows = np.repeat(np.arange(len(Cs.offsets) - 1), np.diff(Cs.offsets))
    return np.stack([ref_dense[r * 128:(r + 1) * 128, c * 128:(c + 1) * 128]
                     for r, c in zip(rows, Cs.indices)])


def _run_ss(op, case, dtype="f16", ex=False):
    m, k, n, nin, nout, ta, tb, unordered = case
    rng = np.random.default_rng(m * 31 + k * 7 + n + nin * 3 + nout)
    # sparse-input capacity: A is M x K (SSD), B is K x N (SDS)
    nin = min(nin, (m if op == "ssd" else n) // 128 * (k // 128))
    Cs = H.HostSparse(m, n, nout * 16384, rng, dtype)
    Cs.dev_values.fill_(float("nan"))
    sp.AllocateRowIndicesBuffer(Cs.matrix)
    sp.RowIndices(Cs.matrix, Cs.matrix.row_indices)
    if op == "ssd":
        A = H.HostSparse(*((k, m) if ta else (m, k)), nin * 16384, rng, dtype,
                         unordered=unordered)
        B = H.HostDense(*((n, k) if tb else (k, n)), rng, dtype)
        sparse = A
        ref = O.gemm(A.dense(), ta, B.values, tb, out_mask=Cs.mask(),
                     threads=H.oracle_threads())
        args = (A.matrix, ta, B.matrix, tb, Cs.matrix)
    else:
        A = H.HostDense(*((k, m) if ta else (m, k)), rng, dtype)
        B = H.HostSparse(*((n, k) if tb else (k, n)), nin * 16384, rng, dtype,
                         unordered=unordered)
        sparse = B
        ref = O.gemm(A.values, ta, B.dense(), tb, out_mask=Cs.mask(),
                     threads=H.oracle_threads())
        args = (A.matrix, ta, B.matrix, tb, Cs.matrix)
    sp.AllocateTransposeBuffers(sparse.matrix)
    if ex:
        sp.Transpose(sparse.matrix)
        sp.MatmulEx(*args)
    else:
        sp.Matmul(*args)
    _sync()
    return Cs.dev_values.float().cpu().numpy(), _blocks_at(ref, Cs)


@pytest.mark.parametrize("case", _ss_params())
def test_ssd_reference_problems(case):
    """SSD: C_bcsr = op(A_bcsr) op(B) at C's blocks (reference ssd_test.cu),
    fp16, against the oracle of the rounded inputs."""
    gpu, ref = _run_ss("ssd", case)
    H.assert_close(gpu, ref, "f16", "ssd")


@pytest.mark.parametrize("case", _ss_params())
def test_sds_reference_problems(case):
    """SDS: C_bcsr = op(A) op(B_bcsr) at C's blocks (reference sds_test.cu)."""
    gpu, ref = _run_ss("sds", case)
    H.assert_close(gpu, ref, "f16", "sds")


@pytest.mark.parametrize("op", ["ssd", "sds"])
@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
def test_ss_bf16_and_ex(op, ta, tb):
    """bf16, and MatmulEx with precomputed transposed metadata."""
    case = (512, 512, 1024, 8, 16, ta, tb, True)
    gpu, ref = _run_ss(op, case, dtype="bf16")
    H.assert_close(gpu, ref, "bf16", f"{op} bf16")
    gpu, ref = _run_ss(op, case, ex=True)
    H.assert_close(gpu, ref, "f16", f"{op} ex")


# -------------------------------------------------------------------- DSS --
# The reference's problem list (sputnik/block/dss/dss_test.cu:78-140):
# (M, K, N, A blocks, B blocks); small shapes with all four transposes, the
# larger ones NN and NT as the reference runs them.
_DSS_SMALL = [(128, 128, 128, 1, 1), (128, 256, 128, 2, 2), (256, 128, 128, 2, 1),
              (128, 128, 256, 1, 2), (128, 256, 128, 1, 2), (128, 256, 128, 2, 1),
              (128, 256, 128, 1, 1), (256, 128, 128, 1, 1), (128, 128, 256, 1, 1),
              (256, 256, 256, 2, 2)]
_DSS_LARGE = [(512, 512, 512, 16, 16), (512, 512, 512, 8, 8), (512, 512, 512, 4, 4),
              (1024, 1024, 1024, 64, 64), (1024, 1024, 1024, 32, 32),
              (1024, 1024, 1024, 16, 16)]


def _dss_params():
    out = []
    for shape in _DSS_SMALL:
        for ta in (False, True):
            for tb in (False, True):
                out.append((shape, ta, tb, shape == (256, 256, 256, 2, 2)))
    for shape in _DSS_LARGE:
        for tb in (False, True):
            out.append((shape, False, tb, False))
    return [pytest.param(p, id=f"m{p[0][0]}k{p[0][1]}n{p[0][2]}-{p[0][3]}-{p[0][4]}"
                               f"-{'T' if p[1] else 'N'}{'T' if p[2] else 'N'}"
                               f"{'-u' if p[3] else ''}") for p in out]


def _run_dss(case, dtype="f16", ex=False):
    (m, k, n, na, nb), ta, tb, unordered = case
    rng = np.random.default_rng(m + 3 * k + 7 * n + 11 * na + 13 * nb)
    A = H.HostSparse(*((k, m) if ta else (m, k)), na * 16384, rng, dtype,
                     unordered=unordered)
    B = H.HostSparse(*((n, k) if tb else (k, n)), nb * 16384, rng, dtype,
                     unordered=unordered)
    C, c_t = H.empty_dense(m, n, dtype)
    sp.AllocateTransposeBuffers(A.matrix)
    sp.AllocateTransposeBuffers(B.matrix)
    if ex:
        sp.Transpose(A.matrix)
        sp.Transpose(B.matrix)
        sp.MatmulEx(A.matrix, ta, B.matrix, tb, C)
    else:
        sp.Matmul(A.matrix, ta, B.matrix, tb, C)
    _sync()
    ref = O.gemm(A.dense(), ta, B.dense(), tb, threads=H.oracle_threads())
    return c_t.float().cpu().numpy(), ref


@pytest.mark.parametrize("case", _dss_params())
def test_dss_reference_problems(case):
    """DSS: dense C = op(A_bcsr) op(B_bcsr) (reference dss_test.cu), the
    k-blocks of each output tile being the intersection of op(A)'s row and
    op(B)'s column, against the oracle."""
    gpu, ref = _run_dss(case)
    H.assert_close(gpu, ref, "f16", "dss")


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
def test_dss_bf16_ex_and_disjoint(ta, tb):
    """bf16; MatmulEx with precomputed metadata; and operands whose patterns
    never meet (every output tile empty: exact zeros)."""
    case = ((512, 1024, 384, 12, 9), ta, tb, True)
    gpu, ref = _run_dss(case, dtype="bf16")
    H.assert_close(gpu, ref, "bf16", "dss bf16")
    gpu, ref = _run_dss(case, ex=True)
    H.assert_close(gpu, ref, "f16", "dss ex")
    # A uses only k-blocks 0..3, B only 4..7: no intersection anywhere.
    rng = np.random.default_rng(4)
    a_off = np.array([0, 2, 4], np.int32)
    a_idx = np.array([0, 3, 1, 2], np.int32)
    b_off = np.array([0, 0, 0, 0, 0, 1, 2, 2, 3], np.int32)
    b_idx = np.array([0, 1, 0], np.int32)
    A = H.HostSparse(256, 1024, 4 * 16384, rng, topology=(a_off, a_idx))
    B = H.HostSparse(1024, 256, 3 * 16384, rng, topology=(b_off, b_idx))
    C, c_t = H.empty_dense(256, 256)
    sp.AllocateTransposeBuffers(B.matrix)
    sp.Matmul(A.matrix, False, B.matrix, False, C)
    _sync()
    assert int(torch.count_nonzero(c_t)) == 0


def test_more_than_65536_blocks():
    """Block data beyond 2 GiB (71680 stored blocks: block index x 32 KiB
    overflows int32, the reference's limit): DSD NN and TN
    (transposed metadata, block_offsets > 65535) on a fully dense 128 x 560
    block grid, sampled block-rows against the oracle."""
    rows_b, cols_b, n = 128, 560, 64
    nb = rows_b * cols_b
    g = torch.Generator(device="cuda").manual_seed(65)
    vals = (torch.rand(nb * 16384, generator=g, device="cuda") * 2 - 1).half()
    off = np.arange(rows_b + 1, dtype=np.int32) * cols_b
    idx = np.tile(np.arange(cols_b, dtype=np.int16), rows_b)
    A = sp.BlockMatrix(rows_b * 128, cols_b * 128, 128, nb * 16384, vals,
                       torch.from_numpy(off).cuda(), torch.from_numpy(idx).cuda())
    rng = np.random.default_rng(66)
    for ta in (False, True):
        k = rows_b * 128 if ta else cols_b * 128
        m = cols_b * 128 if ta else rows_b * 128
        B = H.HostDense(k, n, rng)
        C, c_t = H.empty_dense(m, n)
        if ta:
            sp.AllocateTransposeBuffers(A)
        sp.Matmul(A, ta, B.matrix, False, C)
        _sync()
        for r in (0, m // 128 - 1, (m // 128) // 2):
            if ta:   # row r of A^T = block-column r of A: blocks r, r+560, ...
                blk = vals.view(nb, 128, 128)[r::cols_b].float().cpu().numpy()
                a_rows = np.concatenate([b.T for b in blk], axis=1)  # 128 x k
            else:    # block-row r: blocks r*560 .. +559
                blk = vals.view(nb, 128, 128)[r * cols_b:(r + 1) * cols_b]
                a_rows = blk.float().cpu().numpy().transpose(1, 0, 2).reshape(128, k)
            ref = O.gemm(a_rows, False, B.values, False,
                         threads=H.oracle_threads())
            H.assert_close(c_t[r * 128:(r + 1) * 128].float().cpu().numpy(),
                           ref, "f16", f"65536+ blocks ta={ta} row-block {r}")


# ------------------------------------------------------------ metadata ----

def _device_topology(offsets, indices, rows_b, cols_b):
    nb = int(offsets[-1])
    data = torch.zeros(max(nb, 1) * 128 * 128, dtype=torch.float16,
                       device="cuda")
    return sp.BlockMatrix(rows_b * 128, cols_b * 128, 128, nb * 16384, data,
                          torch.from_numpy(offsets.astype(np.int32)).cuda(),
                          torch.from_numpy(indices.astype(np.int16)).cuda())


@pytest.mark.parametrize("shape", [(3, 4, 6), (1, 1, 1), (32, 32, 512),
                                   (64, 896, 7168), (1024, 32, 656),
                                   (5, 9, 0), (16, 300, 2000), (40, 40, 1600),
                                   # several column slices per launch
                                   (2000, 2500, 20000), (4100, 5000, 9000),
                                   (1, 3000, 1500), (3000, 1, 1000)])
@pytest.mark.parametrize("unordered", [False, True])
def test_transpose_bit_exact(shape, unordered):
    rows_b, cols_b, nb = shape
    rng = np.random.default_rng(rows_b * 1000 + cols_b)
    off, idx = mu.random_topology(rows_b, cols_b, nb, rng, unordered)
    a = _device_topology(off, idx, rows_b, cols_b)
    sp.AllocateTransposeBuffers(a)
    sp.Transpose(a)
    _sync()
    ot, it, bo = O.transpose(off, idx, cols_b)
    assert np.array_equal(a.offsets_t.cpu().numpy(), ot)
    assert np.array_equal(a.indices_t.cpu().numpy()[:nb], it)
    assert np.array_equal(a.block_offsets.cpu().numpy()[:nb], bo)


def test_transpose_survey_known_answer():
    """The vector recorded from the reference's own Transpose."""
    off = np.array([0, 2, 5, 6], np.int32)
    idx = np.array([1, 3, 2, 0, 3, 1], np.int32)
    a = _device_topology(off, idx, 3, 4)
    sp.AllocateTransposeBuffers(a)
    sp.Transpose(a)
    _sync()
    assert a.offsets_t.cpu().tolist() == [0, 1, 3, 4, 6]
    assert a.indices_t.cpu().tolist() == [1, 0, 2, 1, 0, 1]
    assert a.block_offsets.cpu().tolist() == [3, 0, 5, 2, 1, 4]


@pytest.mark.parametrize("shape", [(3, 4, 6), (32, 32, 512), (1024, 32, 656),
                                   (64, 896, 7168), (7, 3, 0), (3, 200, 300)])
@pytest.mark.parametrize("trans", [False, True])
def test_bitmask_bit_exact(shape, trans):
    """Bitmask (reference bitmask.cu:7-45) against the oracle's restatement,
    in both orientations (transposed when offsets_t is set)."""
    rows_b, cols_b, nb = shape
    rng = np.random.default_rng(nb + 2 * rows_b)
    off, idx = mu.random_topology(rows_b, cols_b, nb, rng, unordered=True)
    a = _device_topology(off, idx, rows_b, cols_b)
    if trans:
        sp.AllocateTransposeBuffers(a)
        sp.Transpose(a)
    sp.AllocateBitmaskBuffers(a)
    a.bitmask.fill_(-1)  # every bit must be written
    sp.Bitmask(a)
    _sync()
    if trans:
        ot, it, _ = O.transpose(off, idx, cols_b)
        want = O.bitmask(ot, it, rows_b)
    else:
        want = O.bitmask(off, idx, cols_b)
    got = a.bitmask.cpu().numpy().view(np.uint64)[:want.size]
    assert np.array_equal(got.reshape(want.shape), want)


@pytest.mark.parametrize("shape", [(3, 4, 6), (32, 32, 512), (1024, 32, 656),
                                   (64, 896, 7168), (7, 3, 0)])
def test_row_indices_bit_exact(shape):
    rows_b, cols_b, nb = shape
    rng = np.random.default_rng(nb + 1)
    off, idx = mu.random_topology(rows_b, cols_b, nb, rng)
    a = _device_topology(off, idx, rows_b, cols_b)
    sp.AllocateRowIndicesBuffer(a)
    sp.RowIndices(a, a.row_indices)
    _sync()
    assert np.array_equal(a.row_indices.cpu().numpy()[:nb], O.row_indices(off))


# ------------------------------------------------------------- errors -----

@pytest.mark.parametrize("shape", [(1, 1, 1), (3, 4, 6), (32, 32, 512),
                                   (64, 896, 7168), (300, 40, 700),
                                   (2, 32768, 5000)])
def test_mask_to_bcsr_bit_exact(shape):
    """Device mask -> BCSR against the row-major scan of
    matrix_utils.cu:254-289 (matrix_utils.mask_to_bcsr, itself checked
    against the oracle in test_oracle.py), with an empty and a full row."""
    rb, cb, nb = shape
    rng = np.random.default_rng(rb * 7 + cb)
    perm, mask = mu.random_perm_mask(rb, cb, nb, rng)
    mask[0, :] = 0
    if rb > 2:
        mask[rb - 1, :] = 1
    off_ref, idx_ref = mu.mask_to_bcsr(mask)
    dmask = torch.from_numpy(mask.astype(np.uint8)).cuda()
    offsets = torch.full((rb + 1,), -7, dtype=torch.int32, device="cuda")
    indices = torch.full((rb * cb,), -7, dtype=torch.int16, device="cuda")
    sp.MaskToBcsr(dmask, offsets, indices)
    _sync()
    n = int(off_ref[-1])
    assert np.array_equal(offsets.cpu().numpy(), off_ref)
    assert np.array_equal(indices[:n].cpu().numpy(), idx_ref.astype(np.int16))
    assert (indices[n:].cpu().numpy() == -7).all()   # nothing past nnz


def test_mask_to_bcsr_oracle_permutation():
    """The oracle's permutation builder (oracle.c, matrix_utils.cu:262-289)
    and the device builder agree bit-exactly on the same permutation."""
    rng = np.random.default_rng(3)
    rb, cb, nb = 48, 40, 777
    perm, mask = mu.random_perm_mask(rb, cb, nb, rng)
    off_o, idx_o = O.mask_to_bcsr(perm, rb, cb, nb)
    offsets = torch.empty(rb + 1, dtype=torch.int32, device="cuda")
    indices = torch.empty(rb * cb, dtype=torch.int16, device="cuda")
    sp.MaskToBcsr(torch.from_numpy(mask.astype(np.uint8)).cuda(), offsets,
                  indices)
    _sync()
    assert np.array_equal(offsets.cpu().numpy(), off_o)
    assert np.array_equal(indices[:nb].cpu().numpy(), idx_o.astype(np.int16))


@pytest.mark.parametrize("bins", [[256, 512, 768, 1024],
                                  [128, 128, 640, 640, 1024],
                                  [0, 384, 384, 1152]])
def test_expert_topology(bins):
    """dMoE topology on the device vs its numpy restatement; equal bins give
    the expert-diagonal topology of BASELINE config 4."""
    from sputnik_amd import ops
    bpe = 3
    rows_b = bins[-1] // 128
    t = ops.expert_topology(torch.tensor(bins, dtype=torch.int32).cuda(),
                            bpe, rows_b)
    _sync()
    b = np.array(bins)
    e = np.minimum(np.searchsorted(b, np.arange(rows_b) * 128, side="right"),
                   len(bins) - 1)
    idx_ref = (e[:, None] * bpe + np.arange(bpe)[None, :]).reshape(-1)
    assert np.array_equal(t.offsets.cpu().numpy(),
                          np.arange(rows_b + 1, dtype=np.int32) * bpe)
    assert np.array_equal(t.indices.cpu().numpy(), idx_ref.astype(np.int16))
    assert t.shape == (rows_b * 128, len(bins) * bpe * 128)
    if bins == [256, 512, 768, 1024]:
        o2, i2 = mu.expert_block_diagonal(4, 2, bpe)
        assert np.array_equal(t.indices.cpu().numpy(), i2.astype(np.int16))


def test_topology_from_mask_feeds_products():
    """A device-built topology drives SDD then DSD (no host metadata)."""
    from sputnik_amd import ops
    rng = np.random.default_rng(11)
    _, mask = mu.random_perm_mask(3, 4, 7, rng)
    topo = ops.topology_from_mask(torch.from_numpy(mask).cuda())
    x = torch.rand(384, 256, device="cuda").half() - 0.5
    w = torch.rand(256, 512, device="cuda").half() - 0.5
    h = ops.sdd(x, w, topo)
    full = (x.float() @ w.float())
    m = torch.from_numpy(np.kron(mask, np.ones((128, 128)))).cuda().float()
    H.assert_close(h.to_dense().float().cpu().numpy(),
                   (full * m).cpu().numpy(), "f16", "sdd on device topology")


def test_errors_returned_not_aborted():
    rng = np.random.default_rng(0)
    A = H.HostSparse(256, 256, 2 * 16384, rng)
    B = H.HostDense(256, 128, rng)
    C, _ = H.empty_dense(256, 128)
    # Transposed sparse operand without workspaces (reference aborts).
    with pytest.raises(sp.SputnikError) as e:
        sp.Matmul(A.matrix, True, B.matrix, False, C)
    assert e.value.code == sp.hipErrorInvalidValue
    # Block size other than 128 -> hipErrorNotSupported (dsd.cu:16).
    A.matrix.block_size = 64
    with pytest.raises(sp.SputnikError) as e:
        sp.Matmul(A.matrix, False, B.matrix, False, C)
    assert e.value.code == sp.hipErrorNotSupported
    A.matrix.block_size = 128
    # Shape mismatch (no compatible kernel in the reference).
    Cbad, _ = H.empty_dense(256, 136)
    with pytest.raises(sp.SputnikError):
        sp.Matmul(A.matrix, False, B.matrix, False, Cbad)
    # SDD without row indices.
    Cs = H.HostSparse(256, 128, 16384, rng)
    with pytest.raises(sp.SputnikError):
        sp.Matmul(H.HostDense(256, 64, rng).matrix, False,
                  H.HostDense(64, 128, rng).matrix, False, Cs.matrix)
