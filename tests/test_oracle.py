"""CPU: the oracle against the reference's known answers and the committed
golden vectors, plus algebraic properties of each restated function."""

import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from sputnik_amd import matrix_utils as mu
from tests import helpers as H


def test_transpose_survey_known_answer():
    """Recorded from the reference's own host Transpose."""
    ot, it, bo = O.transpose(np.array([0, 2, 5, 6]),
                             np.array([1, 3, 2, 0, 3, 1]), 4)
    assert ot.tolist() == [0, 1, 3, 4, 6]
    assert it.tolist() == [1, 0, 2, 1, 0, 1]
    assert bo.tolist() == [3, 0, 5, 2, 1, 4]


@pytest.mark.parametrize("seed", range(6))
def test_transpose_matches_stable_argsort(seed):
    """transpose.cu:87-104 restated with numpy's stable argsort."""
    rng = np.random.default_rng(seed)
    R, C = rng.integers(1, 40, size=2)
    nb = int(rng.integers(0, R * C + 1))
    off, idx = mu.random_topology(R, C, nb, rng, unordered=bool(seed % 2))
    ot, it, bo = O.transpose(off, idx, C)
    perm = np.argsort(idx, kind="stable")
    rows = np.repeat(np.arange(R), np.diff(off))
    assert np.array_equal(bo, perm)
    assert np.array_equal(it, rows[perm])
    hist = np.bincount(idx, minlength=C)
    assert np.array_equal(ot, np.concatenate([[0], np.cumsum(hist)]))


@pytest.mark.parametrize("seed", range(4))
def test_transpose_twice_is_identity_on_topology(seed):
    rng = np.random.default_rng(100 + seed)
    R, C = 17, 23
    off, idx = mu.random_topology(R, C, 150, rng)
    ot, it, _ = O.transpose(off, idx, C)
    ott, itt, _ = O.transpose(ot, it, R)
    assert np.array_equal(ott, off) and np.array_equal(itt, idx)


def test_mask_to_bcsr_matches_generator():
    rng = np.random.default_rng(0)
    for R, C, nb in [(5, 7, 12), (32, 32, 512), (1, 9, 9), (8, 8, 0)]:
        perm, mask = mu.random_perm_mask(R, C, nb, rng)
        o1, i1 = O.mask_to_bcsr(perm, R, C, nb)
        o2, i2 = mu.mask_to_bcsr(mask)
        assert np.array_equal(o1, o2) and np.array_equal(i1, i2)
        assert o1[-1] == nb


def test_row_indices():
    off = np.array([0, 2, 2, 5, 6], np.int32)
    assert O.row_indices(off).tolist() == [0, 0, 2, 2, 2, 3]


def test_bcsr_to_dense_matches_numpy():
    rng = np.random.default_rng(2)
    off, idx = mu.random_topology(3, 5, 7, rng, unordered=True)
    vals = mu.random_values((7, 128, 128), rng)
    assert np.array_equal(O.bcsr_to_dense(384, 640, off, idx, vals),
                          mu.to_dense(384, 640, off, idx, vals))


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_gemm_against_float64(ta, tb):
    rng = np.random.default_rng(3)
    m, k, n = 136, 264, 72
    a = mu.random_values((k, m) if ta else (m, k), rng)
    b = mu.random_values((n, k) if tb else (k, n), rng)
    got = O.gemm(a, ta, b, tb)
    ref = (a.T if ta else a).astype(np.float64) @ (b.T if tb else b).astype(np.float64)
    assert np.abs(got - ref).max() < 1e-5


def test_gemm_zero_skip_is_exact():
    rng = np.random.default_rng(4)
    off, idx = mu.random_topology(4, 6, 9, rng)
    vals = mu.random_values((9, 128, 128), rng)
    a = mu.to_dense(512, 768, off, idx, vals)
    b = mu.random_values((768, 200), rng)
    full = O.gemm(a, False, b, False)
    skip = O.gemm(a, False, b, False, a_mask=mu.block_mask(off, idx, 6))
    assert np.array_equal(full, skip)


def test_round_matches_numpy_and_torch():
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(5)
    x = np.concatenate([rng.uniform(-1, 1, 10000), rng.normal(0, 1e3, 1000),
                        rng.normal(0, 1e-6, 1000), [65519.0, 65520.0, -7e4]]
                       ).astype(np.float32)
    assert np.array_equal(O.round_to(x, "f16"),
                          x.astype(np.float16).astype(np.float32))
    assert np.array_equal(O.round_to(x, "bf16"),
                          torch.from_numpy(x).bfloat16().float().numpy())


def test_nonzeros_for_density_matches_reference_rounding():
    # dsd_benchmark.cu:41 RoundUp((int)d*d*s, 128*128) at d=4096.
    got = [mu.nonzeros_for_density(4096, 4096, s) // 16384
           for s in (0.1, 0.3, 0.5, 0.9, 0.2, 0.01, 1.0)]
    assert got == [103, 308, 512, 922, 205, 11, 1024]


GOLDEN = os.path.join(H.GOLDEN, "golden_vectors.npz")


@pytest.mark.skipif(not os.path.exists(GOLDEN), reason="golden not generated")
def test_golden_vectors():
    """Committed fixtures (tests/golden/make_golden.py): metadata KATs and
    small GEMM problems with inputs and expected outputs."""
    g = np.load(GOLDEN, allow_pickle=False)
    meta = json.loads(str(g["manifest"]))
    for case in meta["metadata"]:
        p = case["name"]
        off, idx = g[p + "/offsets"], g[p + "/indices"]
        ot, it, bo = O.transpose(off, idx, case["block_cols"])
        assert np.array_equal(ot, g[p + "/offsets_t"]), p
        assert np.array_equal(it, g[p + "/indices_t"]), p
        assert np.array_equal(bo, g[p + "/block_offsets"]), p
        assert np.array_equal(O.row_indices(off), g[p + "/row_indices"]), p
    for case in meta["gemm"]:
        p = case["name"]
        a_mask = g[p + "/a_mask"] if (p + "/a_mask") in g else None
        got = O.gemm(g[p + "/a"], case["ta"], g[p + "/b"], case["tb"],
                     a_mask=a_mask)
        assert np.array_equal(got, g[p + "/c"]), p


@pytest.mark.parametrize("shape", [(3, 4, 6), (5, 130, 200), (64, 64, 1000)])
def test_bitmask_matches_numpy(shape):
    """oracle_bitmask (bitmask.cu:31-39, bit_matrix.h layout) against an
    independent numpy packing of the block mask."""
    rows, cols, nb = shape
    rng = np.random.default_rng(rows * 7 + cols)
    off, idx = mu.random_topology(rows, cols, nb, rng, unordered=True)
    got = O.bitmask(off, idx, cols)
    mask = mu.block_mask(off, idx, cols).astype(bool)
    words = (cols + 63) // 64
    want = np.zeros((rows, words), dtype=np.uint64)
    for j in range(cols):
        want[:, j // 64] |= mask[:, j].astype(np.uint64) << np.uint64(j % 64)
    assert np.array_equal(got, want)
