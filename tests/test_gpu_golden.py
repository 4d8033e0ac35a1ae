"""The committed golden fixtures (tests/golden/golden_vectors.npz, made by
tests/golden/make_golden.py) fed through the HIP path via the C-ABI.

test_oracle.py::test_golden_vectors pins the oracle to the same file on the
CPU; here the device Transpose / RowIndices (reference
sputnik/block/transpose/transpose.h:10, row_indices/row_indices.h:10) must
reproduce the metadata vectors bit-exactly -- including the survey_kat case
recorded from the reference's own host Transpose -- and
the DSD kernel (and DDS, on the transposed problem) must reproduce the
fixture outputs within the north-star fp16 tolerance.
"""

from __future__ import annotations

import json
import os

import numpy as np
import pytest

from tests import helpers as H

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected here, skipped: no device
    pytest.skip("no GPU", allow_module_level=True)

GOLDEN = os.path.join(H.GOLDEN, "golden_vectors.npz")
B = 128


def _golden():
    g = np.load(GOLDEN, allow_pickle=False)
    return g, json.loads(str(g["manifest"]))


def _meta_cases():
    if not os.path.exists(GOLDEN):
        return []
    return [c["name"] for c in _golden()[1]["metadata"]]


def _sparse_gemm_cases():
    if not os.path.exists(GOLDEN):
        return []
    g, man = _golden()
    return [c["name"] for c in man["gemm"] if (c["name"] + "/a_mask") in g]


def _block_matrix(dense: np.ndarray, mask: np.ndarray):
    """BCSR (ascending column order) of a stored dense matrix whose zero
    blocks are the zeros of the stored-orientation block mask."""
    import sputnik_amd as sp

    rows, cols = dense.shape
    off = np.zeros(mask.shape[0] + 1, np.int32)
    idx, vals = [], []
    for r in range(mask.shape[0]):
        for c in np.flatnonzero(mask[r]):
            idx.append(c)
            vals.append(dense[r * B:(r + 1) * B, c * B:(c + 1) * B])
        off[r + 1] = len(idx)
    nb = len(idx)
    values = np.stack(vals) if nb else np.zeros((0, B, B), np.float32)
    dev_vals = torch.from_numpy(values).to(torch.float16).cuda()
    m = sp.BlockMatrix(rows, cols, B, nb * B * B, dev_vals,
                       torch.from_numpy(off).cuda(),
                       torch.from_numpy(np.asarray(idx, np.int16)).cuda())
    # Matmul builds the transposed metadata on the device where the product
    # needs it (DSD TN/TT, DDS NN/TN) into caller-allocated workspaces.
    sp.AllocateTransposeBuffers(m)
    return m


@pytest.mark.gpu
@pytest.mark.parametrize("name", _meta_cases())
def test_golden_metadata_on_device(name):
    import sputnik_amd as sp

    g, man = _golden()
    case = next(c for c in man["metadata"] if c["name"] == name)
    off = g[name + "/offsets"]
    idx = g[name + "/indices"]
    rows, cols = case["block_rows"] * B, case["block_cols"] * B
    nb = len(idx)
    vals = torch.zeros(max(nb, 1), B, B, dtype=torch.float16, device="cuda")
    m = sp.BlockMatrix(rows, cols, B, nb * B * B, vals,
                       torch.from_numpy(off.astype(np.int32)).cuda(),
                       torch.from_numpy(idx.astype(np.int16)).cuda())
    sp.AllocateTransposeBuffers(m)
    sp.AllocateRowIndicesBuffer(m)
    sp.Transpose(m)
    sp.RowIndices(m, m.row_indices)
    torch.cuda.synchronize()
    assert np.array_equal(m.offsets_t.cpu().numpy(), g[name + "/offsets_t"]), name
    assert np.array_equal(m.indices_t.cpu().numpy()[:nb], g[name + "/indices_t"]), name
    assert np.array_equal(m.block_offsets.cpu().numpy()[:nb],
                          g[name + "/block_offsets"]), name
    assert np.array_equal(m.row_indices.cpu().numpy()[:nb],
                          g[name + "/row_indices"]), name


@pytest.mark.gpu
@pytest.mark.parametrize("name", _sparse_gemm_cases())
def test_golden_dsd_on_device(name):
    """C = op(A_sparse) op(B) from the fixture's stored A and block mask."""
    import sputnik_amd as sp

    g, man = _golden()
    case = next(c for c in man["gemm"] if c["name"] == name)
    m, n, ta, tb = case["m"], case["n"], case["ta"], case["tb"]
    a, b, want = g[name + "/a"], g[name + "/b"], g[name + "/c"]
    # a_mask is the block mask of op(A); the stored operand's is its transpose
    # when ta.
    mask = g[name + "/a_mask"].T if ta else g[name + "/a_mask"]
    sa = _block_matrix(a, mask)
    db = torch.from_numpy(b).to(torch.float16).cuda()
    out, t = H.empty_dense(m, n)
    sp.Matmul(sa, ta, sp.Matrix(b.shape[0], b.shape[1], db), tb, out)
    torch.cuda.synchronize()
    H.assert_close(t.float().cpu().numpy(), want, "f16", name)


@pytest.mark.gpu
@pytest.mark.parametrize("name", _sparse_gemm_cases())
def test_golden_dds_transposed_on_device(name):
    """The same fixture as DDS: C^T = op(B)^T op(A_sparse)^T, i.e. the dense
    operand with the opposite transpose flag and the sparse one likewise."""
    import sputnik_amd as sp

    g, man = _golden()
    case = next(c for c in man["gemm"] if c["name"] == name)
    m, n, ta, tb = case["m"], case["n"], case["ta"], case["tb"]
    a, b, want = g[name + "/a"], g[name + "/b"], g[name + "/c"]
    mask = g[name + "/a_mask"].T if ta else g[name + "/a_mask"]
    sa = _block_matrix(a, mask)
    db = torch.from_numpy(b).to(torch.float16).cuda()
    out, t = H.empty_dense(n, m)
    sp.Matmul(sp.Matrix(b.shape[0], b.shape[1], db), not tb, sa, not ta, out)
    torch.cuda.synchronize()
    H.assert_close(t.float().cpu().numpy(), want.T, "f16", name + " (dds)")
