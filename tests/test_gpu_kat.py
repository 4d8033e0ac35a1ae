"""Exact-arithmetic known-answer tests: every product, every transpose, both
element types, compared BIT-EXACTLY with a closed-form result.

The reference ships no golden vectors, so these KATs pin the
kernels independently of the CPU oracle: all operand values are small
integers (-1, 0, 1), so every product and every partial sum of the fp32
accumulation is an exact integer whatever the summation order (|sum| <= K <
2^24), and the final fp16 / bf16 rounding is exact too (|sum| <= K <= 2048
for fp16, K <= 256 for bf16). The expected output is the float64 product of
the same integer matrices (numpy on the host), converted exactly; the test
is torch.equal on the whole output (value equality: +0 and -0 compare
equal). The shapes reach every dispatch path: pair balancing (4096^2 with
one tile per CU), tall operands, partial N/M/K tiles, the grouped SDD
(>= 4 blocks per CU, checked with sputnik_sdd_plan), transposed metadata
built by Matmul (device Transpose) and precomputed for MatmulEx.
Reference test structure: sputnik/block/dsd/dsd_test.cu:68-194,
sdd_test.cu:71-89 (same products, tolerance replaced by equality).
"""

import numpy as np
import pytest

from sputnik_amd import matrix_utils as mu

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected here, skipped: no device
    pytest.skip("no GPU", allow_module_level=True)

import sputnik_amd as sp  # noqa: E402

sp.lib()  # fail loudly if the native library is missing

B = mu.BLOCK
TD = {"f16": torch.float16, "bf16": torch.bfloat16}
TRANSPOSES = [(False, False), (False, True), (True, False), (True, True)]


def _ints(rng, shape):
    return rng.integers(-1, 2, size=shape).astype(np.float32)


class ISparse:
    """BCSR operand with integer values: host dense copy + device matrix."""

    def __init__(self, rows, cols, density, rng, dtype, unordered=True,
                 nb=None, topology=None):
        self.rows, self.cols = rows, cols
        if topology is not None:
            self.offsets, self.indices = topology
            nb = int(self.offsets[-1])
        else:
            if nb is None:
                nb = mu.nonzeros_for_density(rows, cols, density) // (B * B)
            self.offsets, self.indices = mu.random_topology(
                rows // B, cols // B, nb, rng, unordered=unordered)
        self.values = _ints(rng, (nb, B, B))
        self.dense = mu.to_dense(rows, cols, self.offsets, self.indices,
                                 self.values)
        self.dev = torch.from_numpy(self.values).to(TD[dtype]).cuda()
        self.m = sp.BlockMatrix(
            rows, cols, 128, nb * B * B, self.dev,
            torch.from_numpy(self.offsets.astype(np.int32)).cuda(),
            torch.from_numpy(self.indices.astype(np.int16)).cuda())
        sp.AllocateTransposeBuffers(self.m)

    def blocks_of(self, full):
        """The stored blocks of `full` (dense [rows, cols]) at this topology."""
        rows = np.repeat(np.arange(len(self.offsets) - 1), np.diff(self.offsets))
        return np.stack([full[r * B:(r + 1) * B, c * B:(c + 1) * B]
                         for r, c in zip(rows, self.indices)]) \
            if len(rows) else np.zeros((0, B, B))


class IDense:
    def __init__(self, rows, cols, rng, dtype):
        self.values = _ints(rng, (rows, cols))
        self.dev = torch.from_numpy(self.values).to(TD[dtype]).cuda()
        self.m = sp.Matrix(rows, cols, self.dev)


def _op(x, t):
    return x.T if t else x


def _expect(x64, dtype):
    return torch.from_numpy(np.ascontiguousarray(x64)).to(TD[dtype]).cuda()


def _equal(got, want, what):
    torch.cuda.synchronize()
    if not torch.equal(got, want):
        bad = (got != want)
        n = int(bad.sum())
        idx = bad.nonzero()[0].tolist()
        raise AssertionError(f"{what}: {n} of {got.numel()} elements differ, "
                             f"first at {idx}: got {got[tuple(idx)].item()} "
                             f"want {want[tuple(idx)].item()}")


def _nan_out(rows, cols, dtype):
    t = torch.full((rows, cols), float("nan"), dtype=TD[dtype], device="cuda")
    return sp.Matrix(rows, cols, t), t


# ------------------------------------------------------------------ DSD --

def kat_dsd(m, k, n, density, ta, tb, dtype, ex=False, seed=0,
            topology=None):
    rng = np.random.default_rng(seed)
    A = ISparse(*((k, m) if ta else (m, k)), density, rng, dtype,
                topology=topology)
    Bd = IDense(*((n, k) if tb else (k, n)), rng, dtype)
    C, c_t = _nan_out(m, n, dtype)
    if ex:
        sp.Transpose(A.m)
        sp.MatmulEx(A.m, ta, Bd.m, tb, C)
    else:
        sp.Matmul(A.m, ta, Bd.m, tb, C)
    want = _op(A.dense, ta).astype(np.float64) @ _op(Bd.values, tb)
    return c_t, _expect(want, dtype), (A, Bd, C)


@pytest.mark.parametrize("ta,tb", TRANSPOSES)
@pytest.mark.parametrize("dtype,k", [("f16", 1024), ("bf16", 256)])
def test_kat_dsd(ta, tb, dtype, k):
    got, want, _ = kat_dsd(1024, k, 1032, 0.5, ta, tb, dtype)
    _equal(got, want, f"dsd {ta}{tb} {dtype}")


@pytest.mark.parametrize("ta,tb", TRANSPOSES)
@pytest.mark.parametrize("dtype,k", [("f16", 384), ("bf16", 256)])
def test_kat_dsd_ex_tall(ta, tb, dtype, k):
    """> 256 block-rows (tall tile config), MatmulEx with precomputed
    metadata, partial N tile; bf16 with K <= 256 stays exact (the MoE
    backward's tall transposed products)."""
    got, want, _ = kat_dsd(300 * 128, k, 264, 0.3, ta, tb, dtype, ex=True)
    _equal(got, want, f"dsd tall {ta}{tb} {dtype}")


def test_kat_tall_persistent_repeated():
    """Tall DSD with many more tiles than workgroup slots runs persistent
    (tiles past the first grid fetched from a per-stream counter whose base
    the host advances per launch, dispatch.cpp UseTall): repeated launches on
    one stream, interleaved with launches on a second stream, all exact."""
    rng = np.random.default_rng(11)
    A = ISparse(65536, 256, 0.3, rng, "f16")
    Bd = IDense(256, 1000, rng, "f16")  # 4 tiles of 256 columns, the last partial
    want = _expect(A.dense.astype(np.float64) @ Bd.values, "f16")
    s2 = torch.cuda.Stream()
    for i, stream in enumerate([None, None, s2, None, s2, s2, None]):
        C, c_t = _nan_out(65536, 1000, "f16")
        if stream is None:
            sp.Matmul(A.m, False, Bd.m, False, C)
        else:
            stream.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(stream):
                sp.Matmul(A.m, False, Bd.m, False, C)
            stream.synchronize()
        _equal(c_t, want, f"tall persistent launch {i}")


# Tall DSD NN on the persistent 4-wave pipeline (dsd4w.hip kEpi 7, plan 4):
# (m, k, n, density, dtype). 300 block-rows x 4 k-blocks, two 512 panels;
# a near-empty operand whose workgroup ranges are 0-1 blocks and cross
# panel boundaries (bf16); rows of up to 16 blocks over one panel; a full
# operand of 32-block rows whose workgroup ranges pass 64 blocks (the second
# lane tables, %[vent2] / %[vtile2]).
TALL_PIPE_CASES = [
    (300 * 128, 512, 1024, 0.05, "f16"),
    (300 * 128, 256, 2048, 0.02, "bf16"),
    (300 * 128, 2048, 512, 0.02, "f16"),
    (280 * 128, 4096, 1024, 1.0, "f16"),
]


@pytest.fixture
def tall_pipe():
    prev = sp.tuning("tall4w", 1)
    yield
    sp.tuning("tall4w", prev)


@pytest.mark.parametrize("m,k,n,density,dtype", TALL_PIPE_CASES)
def test_kat_dsd_tall_pipe(m, k, n, density, dtype, tall_pipe):
    """Every tile of a tall DSD NN from the persistent 4-wave pipeline:
    stored straight from the accumulators at the tile's last block, empty
    rows zero-filled after; exact against the float64 product, run twice
    (stale output from the first launch would show on a NaN-filled C)."""
    rng = np.random.default_rng(int(density * 1000) + k)
    A = ISparse(m, k, density, rng, dtype)
    Bd = IDense(k, n, rng, dtype)
    want = _expect(A.dense.astype(np.float64) @ Bd.values, dtype)
    for rep in range(2):
        C, c_t = _nan_out(m, n, dtype)
        assert sp.dsd_plan(A.m, False, Bd.m, False, C) == 4
        sp.Matmul(A.m, False, Bd.m, False, C)
        _equal(c_t, want, f"tall pipe {m}x{k}x{n} {density} {dtype} rep {rep}")


@pytest.mark.parametrize("ta", [False, True])
def test_kat_dsd_4096_pairs(ta):
    """BASELINE config 2 shape (4096^3, 50%): one tile per CU, the
    pair-balancing hand-offs between workgroups are exercised."""
    got, want, _ = kat_dsd(4096, 4096, 4096, 0.5, ta, False, "f16", seed=3)
    _equal(got, want, f"dsd 4096 ta={ta}")
    assert sp.pair_errors() == 0


@pytest.fixture(params=[1, 3], ids=["handoff1", "handoff3"])
def pair_placement(request):
    """Smallest pair hand-off (knob min_handoff, default 2), restored after."""
    prev = sp.tuning("min_handoff", request.param)
    yield request.param
    sp.tuning("min_handoff", prev)


@pytest.mark.parametrize("density", [0.1, 0.3, 0.5, 0.9])
@pytest.mark.parametrize("op", ["dsd", "dds"])
def test_kat_4096_pair_placement(op, density, pair_placement):
    """4096^3 pair launches with 1-block hand-offs allowed, or only from 3
    blocks: every split point is still exact (integer operands), no
    hand-off times out, and a second launch agrees bit for bit."""
    seed = int(density * 100) + 17
    if op == "dsd":
        got, want, (A, Bd, C) = kat_dsd(4096, 4096, 4096, density, False, False,
                                        "f16", seed=seed)
        _equal(got, want, f"dsd 4096 {density} {pair_placement}")
        first = got.clone()
        sp.Matmul(A.m, False, Bd.m, False, C)
    else:
        got, want, (A, Bs, C) = kat_dds(4096, 4096, 4096, density, False, False,
                                        "f16", seed=seed, handles=True)
        _equal(got, want, f"dds 4096 {density} {pair_placement}")
        first = got.clone()
        sp.Matmul(A.m, False, Bs.m, False, C)
    torch.cuda.synchronize()
    assert torch.equal(first, got)
    assert sp.pair_errors() == 0


@pytest.mark.parametrize("op", ["dsd", "dds"])
@pytest.mark.parametrize("n", [4096, 2048])
def test_kat_uniform_rows_xcd_map(op, n):
    """Plain 4-wave launches over 64 rows of equal count (an expert-diagonal
    topology, as MegaBlocks' h . w2): the XCD-row tile map (knob xcd_rows,
    dsd4w.hip) gives every tile to exactly one workgroup -- exact, and bit-
    identical to the panel-major map."""
    topo = mu.expert_block_diagonal(8, 8, 8)   # 64 x 64 blocks, 8 per row / column
    outs = []
    for xr in (1, 0):
        prev = sp.tuning("xcd_rows", xr)
        try:
            if op == "dsd":
                got, want, _ = kat_dsd(8192, 8192, n, None, False, False, "f16",
                                       seed=31, topology=topo)
            else:
                got, want = kat_dds(n, 8192, 8192, None, False, False, "f16",
                                    seed=31, topology=topo)
        finally:
            sp.tuning("xcd_rows", prev)
        _equal(got, want, f"{op} uniform rows n={n} xcd_rows={xr}")
        outs.append(got.clone())
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("m", [512, 1024, 2048])
@pytest.mark.parametrize("ta,tb", [(False, False), (True, False),
                                   (False, True), (True, True)])
def test_kat_dsd_split(m, ta, tb):
    """At most half as many tiles as CUs (the row panels of a strong-scaled
    4096^2): split mode, two workgroups per tile, the first half's fp32
    partial added by the second; tiles of 128 (m=512), 256 (m=1024) or 512
    (m=2048) columns."""
    got, want, _ = kat_dsd(m, 4096, 4096, 0.5, ta, tb, "f16", seed=7)
    _equal(got, want, f"dsd split m={m} ta={ta} tb={tb}")
    assert sp.pair_errors() == 0


@pytest.mark.parametrize("m,n", [(512, 1000), (1024, 264)])
@pytest.mark.parametrize("ta", [False, True])
def test_kat_dsd_split_partial_tiles(m, n, ta):
    """Split mode on narrow tiles with a partial last tile (N % 128 != 0):
    K = 1024 at density 1 gives 8 blocks per row (split needs >= 4)."""
    got, want, _ = kat_dsd(m, 1024, n, 1.0, ta, False, "f16", seed=10)
    _equal(got, want, f"dsd split m={m} n={n} ta={ta}")
    assert sp.pair_errors() == 0


@pytest.mark.parametrize("n", [512, 2048])
@pytest.mark.parametrize("tb", [False, True])
def test_kat_dds_split(n, tb):
    got, want = kat_dds(4096, 4096, n, 0.5, False, tb, "f16", seed=8)
    _equal(got, want, f"dds split n={n} tb={tb}")
    assert sp.pair_errors() == 0


def test_split_timeout_fails_loudly():
    """Split mode with every producer silent (test knob): each consumer
    times out, its tile is NaN and counted; 1024 rows = 8 block-rows on
    256-column tiles x 16 = 128 tiles, so 128 errors. The next launch is
    exact again."""
    got, want, (A, Bd, C) = kat_dsd(1024, 4096, 4096, 0.5, False, False,
                                    "f16", seed=9)
    _equal(got, want, "split before fault")
    assert sp.pair_errors() == 0
    sp.lib().sputnik_debug_pair_fault(1)
    try:
        got.fill_(0)
        sp.MatmulEx(A.m, False, Bd.m, False, C)
        torch.cuda.synchronize()
    finally:
        sp.lib().sputnik_debug_pair_fault(0)
    assert bool(torch.isnan(got.float()).all()), "every tile has a consumer"
    assert sp.pair_errors() == 128
    got.fill_(float("nan"))
    sp.MatmulEx(A.m, False, Bd.m, False, C)
    _equal(got, want, "split after fault")
    assert sp.pair_errors() == 0


# ------------------------------------------------------------------ DDS --

def kat_dds(m, k, n, density, ta, tb, dtype, ex=False, seed=0,
            topology=None, handles=False):
    rng = np.random.default_rng(seed)
    A = IDense(*((k, m) if ta else (m, k)), rng, dtype)
    Bs = ISparse(*((n, k) if tb else (k, n)), density, rng, dtype,
                 topology=topology)
    C, c_t = _nan_out(m, n, dtype)
    if ex:
        sp.Transpose(Bs.m)
        sp.MatmulEx(A.m, ta, Bs.m, tb, C)
    else:
        sp.Matmul(A.m, ta, Bs.m, tb, C)
    want = _op(A.values, ta).astype(np.float64) @ _op(Bs.dense, tb)
    if handles:
        return c_t, _expect(want, dtype), (A, Bs, C)
    return c_t, _expect(want, dtype)


@pytest.mark.parametrize("ta,tb", TRANSPOSES)
@pytest.mark.parametrize("dtype,k", [("f16", 1024), ("bf16", 256)])
def test_kat_dds(ta, tb, dtype, k):
    got, want = kat_dds(1032, k, 1024, 0.5, ta, tb, dtype)
    _equal(got, want, f"dds {ta}{tb} {dtype}")


@pytest.mark.parametrize("ta,tb", TRANSPOSES)
@pytest.mark.parametrize("dtype,k", [("f16", 384), ("bf16", 256)])
def test_kat_dds_ex_tall(ta, tb, dtype, k):
    got, want = kat_dds(264, k, 300 * 128, 0.3, ta, tb, dtype, ex=True)
    _equal(got, want, f"dds tall {ta}{tb} {dtype}")


def test_kat_dds_4096_pairs():
    got, want = kat_dds(4096, 4096, 4096, 0.5, False, False, "f16", seed=4)
    _equal(got, want, "dds 4096")
    assert sp.pair_errors() == 0


# ------------------------------------------------------------------ SDD --

def kat_sdd(m, k, n, density, ta, tb, dtype, nb=None, seed=0):
    rng = np.random.default_rng(seed)
    A = IDense(*((k, m) if ta else (m, k)), rng, dtype)
    Bd = IDense(*((n, k) if tb else (k, n)), rng, dtype)
    Cs = ISparse(m, n, density, rng, dtype, nb=nb)
    Cs.dev.fill_(float("nan"))
    sp.AllocateRowIndicesBuffer(Cs.m)
    sp.RowIndices(Cs.m, Cs.m.row_indices)
    plan = sp.sdd_plan(A.m, ta, Bd.m, tb, Cs.m)
    sp.Matmul(A.m, ta, Bd.m, tb, Cs.m)
    full = _op(A.values, ta).astype(np.float64) @ _op(Bd.values, tb)
    return Cs.dev, _expect(Cs.blocks_of(full), dtype), plan


@pytest.mark.parametrize("ta,tb", TRANSPOSES)
@pytest.mark.parametrize("dtype,k", [("f16", 1032), ("bf16", 200)])
def test_kat_sdd(ta, tb, dtype, k):
    got, want, plan = kat_sdd(1024, k, 1024, 0.5, ta, tb, dtype)
    assert plan == 0
    _equal(got, want, f"sdd {ta}{tb} {dtype}")


@pytest.mark.parametrize("ta,tb", TRANSPOSES)
@pytest.mark.parametrize("k", [256, 200])
def test_kat_sdd_grouped(ta, tb, k):
    """6 x CUs + 37 output blocks: the grouped 128x512 SDD tiles (asserted
    through the dispatcher's plan), with the last partial group of a row,
    unordered columns and a K tail (k=200)."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    nb = 6 * cus + 37
    side = 128 * int(np.ceil(np.sqrt(nb / 0.6)))
    got, want, plan = kat_sdd(side, k, side, None, ta, tb, "f16", nb=nb,
                              seed=k + 2 * ta + tb)
    assert plan == 1, "grouped SDD tiles not selected"
    _equal(got, want, f"sdd grouped {ta}{tb} k={k}")


@pytest.mark.parametrize("ta,tb", TRANSPOSES)
@pytest.mark.parametrize("m,order", [(2048, 1), (1920, 1), (2048, 0)])
def test_kat_sdd_grouped_pow2_stride(ta, tb, m, order):
    """Grouped 4-wave SDD with 32-KiB rows (n = 16384, the power-of-two
    stride the 8-wave kernel used to keep) over a random topology, in the
    band order (sdd_order 1: bands of 8 rows group-index-major, 15 rows = a
    partial last band) and row-major (0): every stored block written once."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    prev = sp.tuning("sdd_order")
    sp.tuning("sdd_order", order)
    try:
        got, want, plan = kat_sdd(m, 256, 16384, None, ta, tb, "f16", nb=4 * cus + 37,
                                  seed=m + order + 2 * ta + tb)
    finally:
        sp.tuning("sdd_order", prev)
    assert plan == 1, "grouped SDD tiles not selected"
    _equal(got, want, f"sdd pow2 {ta}{tb} m={m} order={order}")


@pytest.fixture
def bt_small():
    """The transposed-B SDD path (dispatch.cpp UseBtTranspose) from a 1-MiB
    B on (default: 256 MiB, the MALL), so small problems take it."""
    prev = sp.tuning("sdd_bt_min_mib", 1)
    yield
    sp.tuning("sdd_bt_min_mib", prev)


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("dtype,k", [("f16", 512), ("bf16", 256)])
def test_kat_sdd_bt_transpose(ta, dtype, k, bt_small):
    """SDD NT / TT with B^T transposed into the library's buffer first
    (sputnik_sdd_kernel 4), then the grouped 4-wave NN / TN kernel: exact,
    and the same again with the buffer reused and then grown (N 4096 ->
    6144), and with the path off (knob 0: the NT / TT kernel, 3). (M =
    8192: A^T's rows 16 KiB apart, so TN stays on the 4-wave kernel.)"""
    for n, seed in ((4096, 1), (4096, 2), (6144, 3)):
        rng = np.random.default_rng(seed + 10 * ta)
        m = 8192
        A = IDense(*((k, m) if ta else (m, k)), rng, dtype)
        Bd = IDense(n, k, rng, dtype)  # B^T stored [N][K]
        Cs = ISparse(m, n, 0.6, rng, dtype)
        Cs.dev.fill_(float("nan"))
        sp.AllocateRowIndicesBuffer(Cs.m)
        sp.RowIndices(Cs.m, Cs.m.row_indices)
        assert sp.sdd_kernel(A.m, ta, Bd.m, True, Cs.m) == 4
        sp.Matmul(A.m, ta, Bd.m, True, Cs.m)
        full = _op(A.values, ta).astype(np.float64) @ Bd.values.T
        want = _expect(Cs.blocks_of(full), dtype)
        _equal(Cs.dev, want, f"sdd bt {'T' if ta else 'N'}T {dtype} n={n}")
    prev = sp.tuning("sdd_bt_min_mib", 0)
    try:
        assert sp.sdd_kernel(A.m, ta, Bd.m, True, Cs.m) == 3
        Cs.dev.fill_(float("nan"))
        sp.Matmul(A.m, ta, Bd.m, True, Cs.m)
        _equal(Cs.dev, want, "sdd bt path off")
    finally:
        sp.tuning("sdd_bt_min_mib", prev)


@pytest.mark.parametrize("ta,tb", TRANSPOSES)
@pytest.mark.parametrize("case", ["tail", "uniform"])
def test_kat_sdd_tail_split(ta, tb, case):
    """SDD tail split (block_gemm.h sdd_tail_rows, knob sdd_tail_min_k
    lowered so K = 256 takes it): 8192^2 at 50% has 2 x 256 + a few groups
    of 4 blocks, so the grouped 4-wave launch takes the rows of the full
    rounds and an 8-wave launch of a block per workgroup the rest; rows of
    equal count are never split (the 8-wave launch then exits). Every
    stored block exact, against the split off."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    rng = np.random.default_rng(41 + 2 * ta + tb)
    m = n = 8192
    k = 256
    topo = mu.expert_block_diagonal(4, 16, 16) if case == "uniform" else None
    A = IDense(*((k, m) if ta else (m, k)), rng, "f16")
    Bd = IDense(*((n, k) if tb else (k, n)), rng, "f16")
    Cs = ISparse(m, n, 0.5, rng, "f16", topology=topo)
    sp.AllocateRowIndicesBuffer(Cs.m)
    sp.RowIndices(Cs.m, Cs.m.row_indices)
    if case == "tail":
        groups = int(((np.diff(Cs.offsets) + 3) // 4).sum())
        assert 0 < groups % cus <= cus // 4, groups  # a short last round
    want = _expect(Cs.blocks_of(_op(A.values, ta).astype(np.float64) @ _op(Bd.values, tb)),
                   "f16")
    prev = sp.tuning("sdd_tail_min_k", 256)
    try:
        assert sp.sdd_kernel(A.m, ta, Bd.m, tb, Cs.m) == 3
        for _ in range(2):
            Cs.dev.fill_(float("nan"))
            sp.Matmul(A.m, ta, Bd.m, tb, Cs.m)
            _equal(Cs.dev, want, f"sdd tail {case} {ta}{tb}")
        sp.tuning("sdd_tail_min_k", 0)
        Cs.dev.fill_(float("nan"))
        sp.Matmul(A.m, ta, Bd.m, tb, Cs.m)
        _equal(Cs.dev, want, f"sdd tail off {case} {ta}{tb}")
    finally:
        sp.tuning("sdd_tail_min_k", prev)


@pytest.mark.parametrize("dtype", ["f16", "bf16"])
@pytest.mark.parametrize("ex", [False, True])
def test_kat_dsd_nt_bt_transpose(dtype, ex, bt_small):
    """DSD NT over a dense A of >= 15000 rows (dispatch.cpp
    UseBtTransposeDsd): B^T transposed into the library's buffer, then the
    NN product; exact, Matmul and MatmulEx, and with the path off."""
    got, want, (A, Bd, C) = kat_dsd(16384, 256, 2048, 1.0, False, True, dtype, ex=ex,
                                    seed=51 + ex)
    _equal(got, want, f"dsd nt bt {dtype} ex={ex}")
    prev = sp.tuning("sdd_bt_min_mib", 0)
    try:
        got.fill_(float("nan"))
        (sp.MatmulEx if ex else sp.Matmul)(A.m, False, Bd.m, True, C)
        _equal(got, want, f"dsd nt bt off {dtype}")
    finally:
        sp.tuning("sdd_bt_min_mib", prev)


def test_graph_capture_sdd_tail_split():
    """The tail split's two launches (grouped 4-wave, then one-block 8-wave)
    captured into one graph: replays exact."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    rng = np.random.default_rng(61)
    m = n = 8192
    A = IDense(m, 256, rng, "f16")
    Bd = IDense(256, n, rng, "f16")
    Cs = ISparse(m, n, 0.5, rng, "f16")
    groups = int(((np.diff(Cs.offsets) + 3) // 4).sum())
    assert 0 < groups % cus <= cus // 4, groups
    sp.AllocateRowIndicesBuffer(Cs.m)
    sp.RowIndices(Cs.m, Cs.m.row_indices)
    want = _expect(Cs.blocks_of(A.values.astype(np.float64) @ Bd.values), "f16")
    prev = sp.tuning("sdd_tail_min_k", 256)
    try:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            sp.Matmul(A.m, False, Bd.m, False, Cs.m)
        for _ in range(2):
            Cs.dev.fill_(float("nan"))
            g.replay()
            _equal(Cs.dev, want, "captured sdd tail split")
    finally:
        sp.tuning("sdd_tail_min_k", prev)


def test_sdd_bt_two_threads_one_stream(bt_small):
    """Two host threads issue SDD NT on one stream, one of them with a larger
    B (so the stream's transposed-B buffer grows while the other thread's
    launches may be queued): every result exact (dispatch.cpp g_bt_mu)."""
    import threading
    probs = []
    for n, seed in ((4096, 31), (6144, 32)):
        rng = np.random.default_rng(seed)
        A = IDense(8192, 256, rng, "f16")
        Bd = IDense(n, 256, rng, "f16")
        Cs = ISparse(8192, n, 0.6, rng, "f16")
        sp.AllocateRowIndicesBuffer(Cs.m)
        sp.RowIndices(Cs.m, Cs.m.row_indices)
        want = _expect(Cs.blocks_of(A.values.astype(np.float64) @ Bd.values.T), "f16")
        probs.append((A, Bd, Cs, want))
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    errors = []

    def work(A, Bd, Cs):
        try:
            for _ in range(4):
                sp.Matmul(A.m, False, Bd.m, True, Cs.m, stream=s.cuda_stream)
        except Exception as e:  # noqa: BLE001 (reported below)
            errors.append(e)

    ts = [threading.Thread(target=work, args=pr[:3]) for pr in probs]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    s.synchronize()
    assert not errors, errors
    for A, Bd, Cs, want in probs:
        _equal(Cs.dev, want, f"sdd bt threads n={Bd.m.rows}")


def test_graph_capture_sdd_bt_keeps_nt_kernel(bt_small):
    """A captured SDD NT that would take the transposed-B path eagerly runs
    the NT kernel inside the capture (no buffer is allocated or used by a
    graph); replays are exact."""
    rng = np.random.default_rng(21)
    m, k, n = 16384, 256, 2048
    A = IDense(m, k, rng, "f16")
    Bd = IDense(n, k, rng, "f16")
    Cs = ISparse(m, n, 0.6, rng, "f16")
    sp.AllocateRowIndicesBuffer(Cs.m)
    sp.RowIndices(Cs.m, Cs.m.row_indices)
    want = _expect(Cs.blocks_of(A.values.astype(np.float64) @ Bd.values.T), "f16")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        sp.Matmul(A.m, False, Bd.m, True, Cs.m)
    for _ in range(2):
        Cs.dev.fill_(float("nan"))
        g.replay()
        _equal(Cs.dev, want, "captured sdd nt")


@pytest.mark.parametrize("ta,tb", TRANSPOSES)
@pytest.mark.parametrize("spread", [0, 1, 2])
def test_kat_sdd_uniform_rows_spread(ta, tb, spread):
    """Grouped 4-wave SDD over rows of equal count (expert-block-diagonal:
    4 experts x 8 rows x 64 blocks, 16 groups per row) in the 8 x 4 block
    order, its 4 groups per round adjacent (sdd_spread 0) or 4 apart (1; 2,
    the default: NT only): exact on integer data, block by block."""
    rng = np.random.default_rng(11 + spread + 2 * ta + tb)
    topo = mu.expert_block_diagonal(4, 8, 64)
    m, k, n = 32 * 128, 256, 4 * 64 * 128
    A = IDense(*((k, m) if ta else (m, k)), rng, "f16")
    Bd = IDense(*((n, k) if tb else (k, n)), rng, "f16")
    Cs = ISparse(m, n, None, rng, "f16", topology=topo)
    Cs.dev.fill_(float("nan"))
    sp.AllocateRowIndicesBuffer(Cs.m)
    sp.RowIndices(Cs.m, Cs.m.row_indices)
    prev = sp.tuning("sdd_spread", spread)
    try:
        kern = sp.sdd_kernel(A.m, ta, Bd.m, tb, Cs.m)
        sp.Matmul(A.m, ta, Bd.m, tb, Cs.m)
    finally:
        sp.tuning("sdd_spread", prev)
    assert kern == 3, "4-wave grouped SDD not selected"
    a, b = _op(A.values, ta).astype(np.float64), _op(Bd.values, tb).astype(np.float64)
    rows = np.repeat(np.arange(len(topo[0]) - 1), np.diff(topo[0]))
    want = np.stack([a[r * B:(r + 1) * B] @ b[:, c * B:(c + 1) * B]
                     for r, c in zip(rows, topo[1])])
    _equal(Cs.dev, _expect(want, "f16"), f"sdd uniform spread={spread} {ta}{tb}")


@pytest.mark.parametrize("ta,tb", TRANSPOSES)
@pytest.mark.parametrize("krot", [1, 2, 3, 4])
def test_kat_sdd_grouped_krot(ta, tb, krot):
    """Grouped 4-wave SDD with the k-walk rotated (knob sdd_krot: each group
    starts at its own k-block and wraps, through the kernel's two CSR
    segments), K = 1152 (9 k-blocks, so every rotation wraps unevenly), banded
    order over 32-KiB rows: exact on integer data."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    prev = sp.tuning("sdd_krot")
    sp.tuning("sdd_krot", krot)
    try:
        got, want, plan = kat_sdd(2048, 1152, 16384, None, ta, tb, "f16", nb=4 * cus + 37,
                                  seed=krot + 2 * ta + tb)
    finally:
        sp.tuning("sdd_krot", prev)
    assert plan == 1, "grouped SDD tiles not selected"
    _equal(got, want, f"sdd krot {krot} {ta}{tb}")


# (m, k, n, stored blocks, dtype): one CU's workgroup per chunk, S picked
# in-kernel from the group count (dsd4w.hip kKs): 8 rows x 60 blocks with
# K = 2048 -> S = 8 (2 k-blocks per chunk, many partial groups); 150 blocks,
# K = 1152 (9 k-blocks: chunks of 2, 2, 2, 3) -> S = 4; 300 blocks, K = 512
# -> S = 2; config 3's shape (205 blocks of 4096^2, K = 4096) -> S = 4.
KSPLIT_CASES = [
    (1024, 2048, 4096, 60, "f16"),
    (1024, 2048, 4096, 60, "bf16"),
    (4096, 1152, 4096, 150, "f16"),
    (4096, 512, 4096, 300, "f16"),
    (4096, 4096, 4096, 205, "bf16"),
]


@pytest.fixture
def ksplit_any_k():
    """The K-split on (off by default: knob sdd_ksplit = 1) for every K >=
    512 (default gate: K >= 6144, knob sdd_ksplit_min_k), so these small
    problems take it."""
    prev_s = sp.tuning("sdd_ksplit", 8)
    prev = sp.tuning("sdd_ksplit_min_k", 512)
    yield
    sp.tuning("sdd_ksplit_min_k", prev)
    sp.tuning("sdd_ksplit", prev_s)


@pytest.mark.parametrize("m,k,n,nb,dtype", KSPLIT_CASES)
def test_kat_sdd_ksplit(m, k, n, nb, dtype, ksplit_any_k):
    """SDD NN below the grouped threshold with few groups: each group's K
    split over 2-8 workgroups whose fp32 partials are summed by the chunk
    that owns each row slice (dsd4w.hip kKs, gen_dsd4w.py ksplit_path).
    Exact integer operands: every order of the fp32 sums is exact, so the
    result equals the float64 product bit for bit; a second launch on the
    and no chunk timed out."""
    got, want, plan = kat_sdd(m, k, n, None, False, False, dtype, nb=nb,
                              seed=nb + k)
    assert plan == 2, "K-split SDD not selected"
    _equal(got, want, f"sdd ksplit {m}x{k}x{n} nb={nb} {dtype}")
    assert sp.pair_errors() == 0


def test_sdd_ksplit_deterministic_and_close(ksplit_any_k):
    """Random (non-integer) operands at config 3's shape: the K-split sum
    order is fixed (each chunk adds the others' partials in chunk order after
    its own), so two launches are bit-identical; the result is within the
    north-star tolerance of the 8-wave k-split kernel (knob sdd_ksplit = 1)
    and of the oracle on 24 blocks."""
    rng = np.random.default_rng(33)
    d, nb = 4096, 205
    off, idx = mu.random_topology(d // B, d // B, nb, rng)
    g = torch.Generator(device="cuda")
    g.manual_seed(33)
    x = (torch.rand(d * d, generator=g, device="cuda") * 2 - 1).half()
    w = (torch.rand(d * d, generator=g, device="cuda") * 2 - 1).half()
    cv = torch.empty(nb * B * B, dtype=torch.float16, device="cuda")
    Cm = sp.BlockMatrix(d, d, B, nb * B * B, cv,
                        torch.from_numpy(off.astype(np.int32)).cuda(),
                        torch.from_numpy(idx.astype(np.int16)).cuda())
    sp.AllocateRowIndicesBuffer(Cm)
    sp.RowIndices(Cm, Cm.row_indices)
    X, W = sp.Matrix(d, d, x), sp.Matrix(d, d, w)
    assert sp.sdd_plan(X, False, W, False, Cm) == 2

    def run():
        cv.fill_(float("nan"))
        sp.Matmul(X, False, W, False, Cm)
        torch.cuda.synchronize()
        return cv.clone()
    a, b = run(), run()
    assert torch.equal(a, b), "K-split SDD not deterministic"
    prev = sp.tuning("sdd_ksplit", 1)
    try:
        assert sp.sdd_plan(X, False, W, False, Cm) == 0
        ref8 = run()
    finally:
        sp.tuning("sdd_ksplit", prev)
    diff = (a.float() - ref8.float()).abs().max().item()
    assert diff <= 1e-2 * ref8.float().abs().max().item(), diff
    from oracle import oracle as O
    from tests import helpers
    xv = x.float().cpu().numpy().reshape(d, d)
    wv = w.float().cpu().numpy().reshape(d, d)
    rows = np.repeat(np.arange(d // B), np.diff(off))
    got = a.view(-1, B, B).float().cpu().numpy()
    for e in sorted(set([0, nb - 1] + [int(v) for v in rng.choice(nb, 22, replace=False)])):
        r, c = int(rows[e]), int(idx[e])
        ref = O.gemm(np.ascontiguousarray(xv[r * B:(r + 1) * B]), False,
                     np.ascontiguousarray(wv[:, c * B:(c + 1) * B]), False)
        helpers.assert_close(got[e], ref, "f16", f"sdd ksplit block {e}")
    assert sp.pair_errors() == 0


def test_sdd_ksplit_timeout_fails_loudly(ksplit_any_k):
    """With the test fault on, no chunk raises its flag: every chunk times
    out after the bounded wait, its rows become NaN, the time-outs are
    counted, and the next launch is exact again (per-launch epochs)."""
    got, want, plan = kat_sdd(1024, 2048, 4096, None, False, False, "f16", nb=60,
                              seed=3)
    assert plan == 2
    _equal(got, want, "before fault")
    rng = np.random.default_rng(3)
    A = IDense(1024, 2048, rng, "f16")
    Bd = IDense(2048, 4096, rng, "f16")
    Cs = ISparse(1024, 4096, None, rng, "f16", nb=60)
    sp.AllocateRowIndicesBuffer(Cs.m)
    sp.RowIndices(Cs.m, Cs.m.row_indices)
    want2 = _expect(Cs.blocks_of(A.values.astype(np.float64) @ Bd.values), "f16")
    sp.lib().sputnik_debug_pair_fault(1)
    try:
        Cs.dev.fill_(0)
        sp.Matmul(A.m, False, Bd.m, False, Cs.m)
        torch.cuda.synchronize()
    finally:
        sp.lib().sputnik_debug_pair_fault(0)
    assert bool(torch.isnan(Cs.dev.float()).all()), "timed-out chunks not NaN"
    assert sp.pair_errors() > 0
    Cs.dev.fill_(float("nan"))
    sp.Matmul(A.m, False, Bd.m, False, Cs.m)
    _equal(Cs.dev, want2, "after fault")
    assert sp.pair_errors() == 0


def test_graph_capture_sdd_ksplit(ksplit_any_k):
    """A K-split SDD captured into a graph: replays (back to back and with
    eager launches in between) read the device-side epoch and stay exact."""
    rng = np.random.default_rng(8)
    A = IDense(4096, 4096, rng, "f16")
    Bd = IDense(4096, 4096, rng, "f16")
    Cs = ISparse(4096, 4096, None, rng, "f16", nb=205)
    sp.AllocateRowIndicesBuffer(Cs.m)
    sp.RowIndices(Cs.m, Cs.m.row_indices)
    want = _expect(Cs.blocks_of(A.values.astype(np.float64) @ Bd.values), "f16")
    assert sp.sdd_plan(A.m, False, Bd.m, False, Cs.m) == 2
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        sp.Matmul(A.m, False, Bd.m, False, Cs.m)
    for i in range(3):
        Cs.dev.fill_(float("nan"))
        g.replay()
        _equal(Cs.dev, want, f"replay {i}")
        Cs.dev.fill_(float("nan"))
        sp.Matmul(A.m, False, Bd.m, False, Cs.m)
        _equal(Cs.dev, want, f"eager {i}")
    for _ in range(6):
        g.replay()
    _equal(Cs.dev, want, "back-to-back replays")
    assert sp.pair_errors() == 0
    del g


def test_sdd_plan_ksplit_default_gate():
    """The K-split is off by default (its all-to-all chunk wait
    needs the whole grid resident): 205 blocks of 4096^2 take the 8-wave
    k-split tile at K = 4096 and 8192. Opted in (knob sdd_ksplit = 8), the
    K = 6144 gate still keeps K = 4096 off it and takes K = 8192 (exact)."""
    for k in (4096, 8192):
        got, exp, plan = kat_sdd(4096, k, 4096, None, False, False, "f16", nb=205,
                                 seed=k)
        assert plan == 0, (k, plan)
        _equal(got, exp, f"sdd 205 blocks k={k}")
    prev = sp.tuning("sdd_ksplit", 8)
    try:
        for k, want in ((4096, 0), (8192, 2)):
            got, exp, plan = kat_sdd(4096, k, 4096, None, False, False, "f16",
                                     nb=205, seed=k)
            assert plan == want, (k, plan)
            _equal(got, exp, f"sdd 205 blocks k={k} (K-split on)")
    finally:
        sp.tuning("sdd_ksplit", prev)
    assert sp.pair_errors() == 0


def test_kernel_queries_match_config3():
    """sputnik_sdd_kernel / sputnik_dds_plan (what bench.py labels its lines
    with) at config 3's shapes: 205 SDD blocks of 4096^2 at K = 4096 take
    the 8-wave k-split block tile (0), the DDS g . C the 4-wave kernel (1);
    from 4 blocks per CU the SDD takes the 4-wave grouped tiles (3)."""
    rng = np.random.default_rng(21)
    A = IDense(4096, 4096, rng, "f16")
    Bd = IDense(4096, 4096, rng, "f16")
    Cs = ISparse(4096, 4096, None, rng, "f16", nb=205)
    sp.AllocateRowIndicesBuffer(Cs.m)
    assert sp.sdd_plan(A.m, False, Bd.m, False, Cs.m) == 0
    assert sp.sdd_kernel(A.m, False, Bd.m, False, Cs.m) == 0
    out, _ = _nan_out(4096, 4096, "f16")
    assert sp.dds_plan(A.m, False, Cs.m, False, out) == 1
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    Cg = ISparse(4096, 4096, None, rng, "f16", nb=4 * cus)
    sp.AllocateRowIndicesBuffer(Cg.m)
    assert sp.sdd_plan(A.m, False, Bd.m, False, Cg.m) == 1
    assert sp.sdd_kernel(A.m, False, Bd.m, False, Cg.m) == 3
    prev = sp.select_dsd_kernel(0)  # the 8-wave kernel everywhere
    try:
        assert sp.sdd_kernel(A.m, False, Bd.m, False, Cg.m) == 1
        assert sp.dds_plan(A.m, False, Cs.m, False, out) == 0
    finally:
        sp.select_dsd_kernel(prev)


def test_sdd_plan_threshold():
    """Just below 4 blocks per CU the k-split block tile is chosen, from 4
    the grouped one (dispatch.cpp UseGroupedSdd)."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    rng = np.random.default_rng(1)
    side = 128 * 64
    for nb, want in ((4 * cus - 1, 0), (4 * cus, 1)):
        A = IDense(side, 128, rng, "f16")
        Bd = IDense(128, side, rng, "f16")
        Cs = ISparse(side, side, None, rng, "f16", nb=nb)
        assert sp.sdd_plan(A.m, False, Bd.m, False, Cs.m) == -1  # no row_indices
        sp.AllocateRowIndicesBuffer(Cs.m)
        assert sp.sdd_plan(A.m, False, Bd.m, False, Cs.m) == want, nb


# ------------------------------------------------------------ SSD / SDS --

@pytest.mark.parametrize("ta,tb", TRANSPOSES)
@pytest.mark.parametrize("op", ["ssd", "sds"])
def test_kat_ss(op, ta, tb):
    rng = np.random.default_rng(ta * 2 + tb)
    m, k, n = 1024, 768, 1152
    dtype = "f16"
    if op == "ssd":
        X = ISparse(*((k, m) if ta else (m, k)), 0.5, rng, dtype)
        Y = IDense(*((n, k) if tb else (k, n)), rng, dtype)
        full = _op(X.dense, ta).astype(np.float64) @ _op(Y.values, tb)
    else:
        X = IDense(*((k, m) if ta else (m, k)), rng, dtype)
        Y = ISparse(*((n, k) if tb else (k, n)), 0.5, rng, dtype)
        full = _op(X.values, ta).astype(np.float64) @ _op(Y.dense, tb)
    Cs = ISparse(m, n, 0.3, rng, dtype)
    Cs.dev.fill_(float("nan"))
    sp.AllocateRowIndicesBuffer(Cs.m)
    sp.RowIndices(Cs.m, Cs.m.row_indices)
    sp.Matmul(X.m, ta, Y.m, tb, Cs.m)
    _equal(Cs.dev, _expect(Cs.blocks_of(full), dtype), f"{op} {ta}{tb}")


# ------------------------------------------------------------------ DSS --

@pytest.mark.parametrize("ta,tb", TRANSPOSES)
@pytest.mark.parametrize("dtype,k", [("f16", 1024), ("bf16", 256)])
def test_kat_dss(ta, tb, dtype, k):
    rng = np.random.default_rng(10 + ta * 2 + tb)
    m, n = 896, 1024
    X = ISparse(*((k, m) if ta else (m, k)), 0.5, rng, dtype)
    Y = ISparse(*((n, k) if tb else (k, n)), 0.5, rng, dtype)
    C, c_t = _nan_out(m, n, dtype)
    sp.Matmul(X.m, ta, Y.m, tb, C)
    want = _op(X.dense, ta).astype(np.float64) @ _op(Y.dense, tb)
    _equal(c_t, _expect(want, dtype), f"dss {ta}{tb} {dtype}")


# ------------------------------------------- pair hand-off robustness --

def _skewed_rows(rng, rows_b=32, cols_b=32):
    """Block-rows alternating 28 and 4 blocks (mean 16): every heavy row
    hands 12 blocks to its light partner under pair balancing."""
    counts = np.where(np.arange(rows_b) % 2 == 0, 28, 4)
    offsets = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    indices = np.concatenate([np.sort(rng.choice(cols_b, c, replace=False))
                              for c in counts]).astype(np.int16)
    return offsets, indices


@pytest.mark.parametrize("op,ta,tb", [("dsd", False, False),
                                      ("dsd", True, False),
                                      ("dsd", False, True),
                                      ("dds", False, False),
                                      ("dds", False, True)])
def test_pair_timeout_fails_loudly(op, ta, tb):
    """A pair producer that never publishes (test knob) makes its consumer
    time out (after the bounded wait): the consumer's tile is NaN (never a
    stale or partial sum), every such consumer is counted by
    sputnik_pair_errors(), the tiles without a hand-off are exact, and the
    next launch on the same workspace is exact and error-free again
    (per-launch epochs, no flag to reset)."""
    rng = np.random.default_rng(5)
    topo = _skewed_rows(rng)
    if op == "dsd":
        got, want, (X, Y, C) = kat_dsd(4096, 4096, 4096, None, ta, tb, "f16",
                                       seed=5, topology=topo)
    else:
        got, want, (X, Y, C) = kat_dds(4096, 4096, 4096, None, ta, tb, "f16",
                                       seed=5, topology=topo, handles=True)

    def run():
        sp.MatmulEx(X.m, ta, Y.m, tb, C)

    _equal(got, want, f"{op} before fault")
    assert sp.pair_errors() == 0
    sp.lib().sputnik_debug_pair_fault(1)
    try:
        got.fill_(0)
        run()
        torch.cuda.synchronize()
    finally:
        sp.lib().sputnik_debug_pair_fault(0)
    # DDS writes C transposed: a poisoned tile is 128 columns x 512 rows.
    bad = torch.isnan(got.float())
    poisoned = (bad.any(dim=1) if op == "dsd" else bad.any(dim=0))
    assert int(poisoned.sum()) > 0, "no consumer tile was poisoned"
    errors = sp.pair_errors()
    if (op, ta, tb) in (("dsd", False, False), ("dds", False, True)):
        # S rows are the skewed stored rows: 16 heavy rows x 8 panels, each
        # handing 12 blocks to its light partner.
        assert errors == 128
    else:
        assert errors > 0
    assert sp.pair_errors() == 0  # cleared by the previous call
    ok = ~bad
    assert torch.equal(got[ok], want[ok])  # tiles without a hand-off exact
    got.fill_(float("nan"))
    run()
    _equal(got, want, f"{op} after fault")
    assert sp.pair_errors() == 0


def test_tall_persistent_two_host_threads_one_stream():
    """Two host threads launching persistent tall DSDs on one stream (ctypes
    drops the GIL, so their host-side preparation interleaves): the tile
    counter is reset on the device by each launch's last workgroup, so every
    launch computes every tile whatever order the launches were queued in."""
    import threading
    rng = np.random.default_rng(13)
    A = ISparse(65536, 256, 0.3, rng, "f16")
    Bd = IDense(256, 512, rng, "f16")
    want = _expect(A.dense.astype(np.float64) @ Bd.values, "f16")
    outs = [_nan_out(65536, 512, "f16") for _ in range(2)]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    errors = []

    def worker(i):
        try:
            torch.cuda.set_device(0)
            with torch.cuda.stream(s):
                for _ in range(8):
                    sp.MatmulEx(A.m, False, Bd.m, False, outs[i][0])
        except Exception as exc:  # reported below
            errors.append(exc)

    threads = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    s.synchronize()
    assert not errors, errors
    for i in range(2):
        _equal(outs[i][1], want, f"thread {i}")


def test_graph_capture_with_pairs():
    """A pair-balanced DSD captured into a graph gets a workspace of its own
    capture with a device-side epoch (GemmParams::pair_sync): replays on the
    capturing stream, on another stream, interleaved with eager pair
    launches on the capturing stream (whose workspace already existed), all
    stay bit-exact, and no hand-off times out."""
    got, want, (A, Bd, C) = kat_dsd(4096, 4096, 4096, 0.5, False, False,
                                    "f16", seed=6)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        sp.MatmulEx(A.m, False, Bd.m, False, C)  # creates s's workspace
    torch.cuda.current_stream().wait_stream(s)
    _equal(got, want, "eager on s")
    before = sp.capture_workspaces()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        sp.MatmulEx(A.m, False, Bd.m, False, C)
    assert sp.capture_workspaces() == before + 1, "captured launch used pairs"
    other = torch.cuda.Stream()
    for i in range(4):
        got.fill_(float("nan"))
        if i % 2:
            other.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(other):
                g.replay()
            torch.cuda.current_stream().wait_stream(other)
        else:
            g.replay()
        _equal(got, want, "graph replay")
        got.fill_(float("nan"))
        sp.MatmulEx(A.m, False, Bd.m, False, C)
        _equal(got, want, "eager between replays")
    # Back-to-back replays: each reads the epoch the previous one advanced.
    for _ in range(8):
        g.replay()
    _equal(got, want, "back-to-back replays")
    assert sp.pair_errors() == 0


def test_graph_capture_workspace_freed_with_graph():
    """A capture's pair workspace (64 MiB) and persistent counter live as long
    as the captured graph: destroying the graph and its executable releases
    them (a user object retained by the graph, dispatch.cpp
    TieToCapturedGraph), so re-capturing per shape does not pin memory or
    fill the capture tables."""
    import time
    got, want, (A, Bd, C) = kat_dsd(4096, 4096, 4096, 0.5, False, False,
                                    "f16", seed=9)
    rng = np.random.default_rng(14)
    T = ISparse(65536, 256, 0.3, rng, "f16")
    Td = IDense(256, 512, rng, "f16")
    CT, gotT = _nan_out(65536, 512, "f16")
    torch.cuda.synchronize()
    prev = sp.tuning("tall4w", 0)  # the 8-wave persistent tall path: a counter
    try:
        _capture_release_cycle(A, Bd, C, got, want, T, Td, CT)
    finally:
        sp.tuning("tall4w", prev)


def _capture_release_cycle(A, Bd, C, got, want, T, Td, CT):
    import time
    base = sp.capture_workspaces()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    for rep in range(3):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            sp.MatmulEx(A.m, False, Bd.m, False, C)
            sp.MatmulEx(T.m, False, Td.m, False, CT)
        assert sp.capture_workspaces() == base + 2, "pairs + tall counter"
        got.fill_(float("nan"))
        g.replay()
        _equal(got, want, f"replay {rep}")
        torch.cuda.synchronize()
        g.reset()
        del g
        torch.cuda.synchronize()
        n = sp.capture_workspaces()
        for _ in range(50):  # the destructor runs on HIP's callback thread
            if n == base:
                break
            time.sleep(0.02)
            n = sp.capture_workspaces()
        assert n == base, f"capture workspaces still held: {n} vs {base}"
    assert sp.pair_errors() == 0


def test_graph_capture_reuses_released_workspace():
    """Repeated capture / replay / destroy with no eager launch and no
    sputnik_capture_workspaces() call in between: each new
    capture re-ties the released workspace of the destroyed graph instead of
    allocating another 64 MiB (device memory stays flat), replays stay
    bit-exact, and sputnik_capture_workspaces() finally frees it."""
    import time
    got, want, (A, Bd, C) = kat_dsd(4096, 4096, 4096, 0.5, False, False,
                                    "f16", seed=19)
    torch.cuda.synchronize()
    base = sp.capture_workspaces()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    free = []
    for rep in range(6):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            sp.MatmulEx(A.m, False, Bd.m, False, C)
        got.fill_(float("nan"))
        g.replay()
        _equal(got, want, f"replay {rep}")
        torch.cuda.synchronize()
        g.reset()
        del g
        torch.cuda.synchronize()
        time.sleep(0.1)  # the release runs on HIP's callback thread
        free.append(torch.cuda.mem_get_info()[0])
    drop = free[1] - free[-1]
    assert drop < 48 << 20, f"device memory fell by {drop >> 20} MiB over 4 captures"
    n = sp.capture_workspaces()
    for _ in range(50):
        if n == base:
            break
        time.sleep(0.02)
        n = sp.capture_workspaces()
    assert n == base
    assert sp.pair_errors() == 0


def test_dsd_plan_is_read_only_under_capture():
    """sputnik_dsd_plan decides without allocating: called while
    a stream is being captured it creates no capture workspace, and it
    reports the same plan as outside the capture."""
    got, want, (A, Bd, C) = kat_dsd(4096, 4096, 4096, 0.5, False, False,
                                    "f16", seed=21)
    torch.cuda.synchronize()
    base = sp.capture_workspaces()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    plan_eager = sp.dsd_plan(A.m, False, Bd.m, False, C, stream=s.cuda_stream)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        plan_cap = sp.dsd_plan(A.m, False, Bd.m, False, C, stream=s.cuda_stream)
        assert sp.capture_workspaces() == base
        sp.MatmulEx(A.m, False, Bd.m, False, C)
    assert plan_cap == plan_eager == 1
    assert sp.capture_workspaces() == base + 1
    got.fill_(float("nan"))
    g.replay()
    _equal(got, want, "replay")
    del g


def test_graph_capture_split_and_dds():
    """Split mode (a 512-row DSD panel) and a pair-balanced DDS captured in
    one graph: two launches share the capture's workspace one after the
    other; replays stay bit-exact."""
    got1, want1, (A1, B1, C1) = kat_dsd(512, 4096, 4096, 0.5, False, False,
                                        "f16", seed=7)
    got2, want2, (A2, B2, C2) = kat_dds(4096, 4096, 4096, 0.5, False, False,
                                        "f16", ex=True, seed=8, handles=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        sp.MatmulEx(A1.m, False, B1.m, False, C1)
        sp.MatmulEx(A2.m, False, B2.m, False, C2)
    for _ in range(3):
        got1.fill_(float("nan"))
        got2.fill_(float("nan"))
        g.replay()
        _equal(got1, want1, "split replay")
        _equal(got2, want2, "dds replay")
    assert sp.pair_errors() == 0


def test_graph_capture_tall_persistent():
    """A tall DSD captured into a graph on a stream whose persistent tile
    counter already exists: the captured launch gets a counter pair of its
    own capture (the kernel leaves it at zero), so replays interleaved with
    eager persistent launches on the same stream all stay exact."""
    prev = sp.tuning("tall4w", 0)  # the 8-wave persistent tall path
    try:
        _tall_persistent_capture()
    finally:
        sp.tuning("tall4w", prev)


def test_graph_capture_tall_pipe_takes_no_counter():
    """The tall DSD NN pipeline (4-wave, plan 4) needs no persistent tile
    counter: a captured tall-pipe launch ties no capture workspace (ADVICE
    r05: the tall decision is made dry before the counter is allocated),
    and its replays are exact."""
    rng = np.random.default_rng(13)
    A = ISparse(65536, 256, 0.3, rng, "f16")
    Bd = IDense(256, 512, rng, "f16")
    want = _expect(A.dense.astype(np.float64) @ Bd.values, "f16")
    C, got = _nan_out(65536, 512, "f16")
    prev = sp.tuning("tall4w", 1)
    try:
        assert sp.dsd_plan(A.m, False, Bd.m, False, C) == 4
        torch.cuda.synchronize()
        before = sp.capture_workspaces()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            sp.MatmulEx(A.m, False, Bd.m, False, C)
        assert sp.capture_workspaces() == before, "tall pipe tied a workspace"
        for _ in range(2):
            got.fill_(float("nan"))
            g.replay()
            _equal(got, want, "tall pipe replay")
        del g
    finally:
        sp.tuning("tall4w", prev)


def _tall_persistent_capture():
    rng = np.random.default_rng(12)
    A = ISparse(65536, 256, 0.3, rng, "f16")
    Bd = IDense(256, 512, rng, "f16")
    want = _expect(A.dense.astype(np.float64) @ Bd.values, "f16")
    C, got = _nan_out(65536, 512, "f16")
    assert sp.dsd_plan(A.m, False, Bd.m, False, C) == 2
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        sp.MatmulEx(A.m, False, Bd.m, False, C)  # creates s's counter
    torch.cuda.current_stream().wait_stream(s)
    _equal(got, want, "eager on s")
    before = sp.capture_workspaces()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        sp.MatmulEx(A.m, False, Bd.m, False, C)
    assert sp.capture_workspaces() == before + 1, "captured launch persistent"
    for _ in range(3):
        got.fill_(float("nan"))
        g.replay()
        _equal(got, want, "graph replay")
        got.fill_(float("nan"))
        with torch.cuda.stream(s):
            sp.MatmulEx(A.m, False, Bd.m, False, C)
        s.synchronize()
        _equal(got, want, "eager persistent between replays")
