"""CPU check of the linearity-checksum criterion the full-size config-4 GPU
tests use (tests/helpers.py rowsum_check): it passes a correctly computed,
bf16-rounded product and fails one with a single dropped block or a single
wrong k-block, at the value ranges and reduction lengths of config 4."""

import numpy as np
import pytest

from oracle import oracle as O
from tests import helpers as H


def _bf16(a):
    return O.round_to(a.astype(np.float32), "bf16")


def _u(rng, *shape):
    return _bf16(rng.uniform(-1, 1, shape))


def test_rowsum_check_sdd_shape():
    rng = np.random.default_rng(0)
    x, w = _u(rng, 256, 4096), _u(rng, 4096, 512)
    h = _bf16(x @ w)                                   # fp32 accumulate, bf16 out
    expect = x.astype(np.float64) @ w.astype(np.float64).sum(axis=1)
    H.rowsum_check(h, expect, 1, "ok")
    # one 128 x 128 block computed from the wrong k-block
    bad = h.copy()
    # (A's k-blocks shifted by one: k-block i of A meets k-block i + 1 of B)
    bad[:128, 128:256] = _bf16(np.roll(x[:128], 128, axis=1) @ w[:, 128:256])
    with pytest.raises(AssertionError):
        H.rowsum_check(bad, expect, 1, "wrong k-block")


def test_rowsum_check_dsd_shape():
    rng = np.random.default_rng(1)
    # h values as config 4's SDD output (sums of 4096 products), 14 blocks
    # of 128 per row (the expert's 112 scaled down), a 4096-wide output row
    h = _bf16(rng.normal(0, 21.3, (256, 14 * 128)))
    w2 = _u(rng, 14 * 128, 4096)
    y = _bf16(h @ w2)
    expect = h.astype(np.float64) @ w2.astype(np.float64).sum(axis=1)
    H.rowsum_check(y, expect, 1, "ok")
    dropped = h.copy()
    dropped[:128, 5 * 128:6 * 128] = 0               # one block of h missing
    with pytest.raises(AssertionError):
        H.rowsum_check(_bf16(dropped @ w2), expect, 1, "dropped block")


def test_rowsum_check_rejects_nan():
    y = np.ones((4, 8), np.float32)
    y[1, 3] = np.nan
    with pytest.raises(AssertionError):
        H.rowsum_check(y, np.full(4, 8.0), 1, "nan")
