"""Torch op surface over the block-sparse products, in the shape MegaBlocks
drives them: a topology object holding the BCSR
metadata once (plus the transposed metadata and row indices, built on the
device the first time a product needs them, so every later call is a
`MatmulEx`), and three differentiable ops

    sdd(a, b, topo) -> SparseMatrix   (a @ b at topo's nonzero blocks)
    dsd(a_sparse, b) -> Tensor        (op(a) @ b, a possibly a .t() view)
    dds(a, b_sparse) -> Tensor        (a @ op(b))

whose backward passes are again sdd / dsd / dds with transpose flags (the
MegaBlocks forward/backward set, BASELINE config 3). Every product runs on
libsputnik.so through the C-ABI on the current torch stream; there is no
dense or CPU fallback (a missing library raises).

The BCSR wire format is the reference's `BlockMatrix` (arguments.h:48-153):
`data` holds #blocks row-major 128x128 blocks ([nb, 128, 128] here),
`offsets` int32 [rows/128 + 1] in blocks, `indices` int16 [nb] block
columns; `offsets_t` / `indices_t` / `block_offsets` are what
`Transpose` (transpose.cu:69-125) produces and `row_indices` what
`RowIndices` (row_indices.cu:7-36) produces.
"""

from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import (BlockMatrix, Matrix, Matmul, MatmulEx, RowIndices, Transpose,
               AllocateRowIndicesBuffer, AllocateTransposeBuffers)

BLOCK = 128


class _Meta:
    """Device metadata shared by every view of one topology."""

    def __init__(self, rows, cols, offsets, indices):
        self.rows, self.cols = rows, cols
        self.offsets = offsets
        self.indices = indices
        self.offsets_t = None
        self.indices_t = None
        self.block_offsets = None
        self.row_indices = None
        self.nb = int(indices.numel())

    def descriptor(self, data) -> BlockMatrix:
        return BlockMatrix(self.rows, self.cols, BLOCK, self.nb * BLOCK * BLOCK,
                           data, self.offsets, self.indices, self.offsets_t,
                           self.indices_t, self.block_offsets, self.row_indices)

    def ensure_transposed(self, data):
        if self.offsets_t is None:
            d = self.descriptor(data)
            AllocateTransposeBuffers(d)
            Transpose(d)
            self.offsets_t, self.indices_t = d.offsets_t, d.indices_t
            self.block_offsets = d.block_offsets

    def ensure_row_indices(self, data):
        if self.row_indices is None:
            d = self.descriptor(data)
            AllocateRowIndicesBuffer(d)
            RowIndices(d, d.row_indices)
            self.row_indices = d.row_indices


class SparseMatrix:
    """A block-sparse matrix (128x128 blocks). `shape` is the logical shape;
    a `.t()` view shares data and metadata and flips the transpose flag the
    products receive, as MegaBlocks/stk's transposed views do."""

    def __init__(self, size: Tuple[int, int], data: torch.Tensor,
                 offsets: torch.Tensor, indices: torch.Tensor,
                 _meta: Optional[_Meta] = None, _transposed: bool = False):
        rows, cols = int(size[0]), int(size[1])
        if rows % BLOCK or cols % BLOCK:
            raise ValueError(f"sparse shape {size} is not a multiple of 128")
        if data.dim() != 3 or tuple(data.shape[1:]) != (BLOCK, BLOCK):
            raise ValueError("data must be [#blocks, 128, 128]")
        if data.shape[0] != indices.numel():
            raise ValueError("data and indices disagree on #blocks")
        if offsets.dtype != torch.int32 or indices.dtype != torch.int16:
            raise TypeError("offsets int32, indices int16 (arguments.h:48-153)")
        if offsets.numel() != rows // BLOCK + 1:
            raise ValueError("offsets must have rows/128 + 1 entries")
        self.data = data
        self._meta = _meta or _Meta(rows, cols, offsets.contiguous(),
                                    indices.contiguous())
        self._transposed = _transposed

    # -- views ------------------------------------------------------------
    @property
    def shape(self):
        m = self._meta
        return (m.cols, m.rows) if self._transposed else (m.rows, m.cols)

    def size(self, dim=None):
        return self.shape if dim is None else self.shape[dim]

    @property
    def dtype(self):
        return self.data.dtype

    @property
    def device(self):
        return self.data.device

    @property
    def offsets(self):
        return self._meta.offsets

    @property
    def indices(self):
        return self._meta.indices

    @property
    def nnz_blocks(self) -> int:
        return self._meta.nb

    def is_transposed(self) -> bool:
        return self._transposed

    def t(self) -> "SparseMatrix":
        return SparseMatrix((self._meta.rows, self._meta.cols), self.data,
                            self._meta.offsets, self._meta.indices,
                            _meta=self._meta, _transposed=not self._transposed)

    def with_data(self, data: torch.Tensor) -> "SparseMatrix":
        """Same topology (and view), new block values."""
        return SparseMatrix((self._meta.rows, self._meta.cols), data,
                            self._meta.offsets, self._meta.indices,
                            _meta=self._meta, _transposed=self._transposed)

    def to_dense(self) -> torch.Tensor:
        """Dense copy (block scatter with torch indexing; test/debug aid)."""
        m = self._meta
        rb, cb = m.rows // BLOCK, m.cols // BLOCK
        counts = (m.offsets[1:] - m.offsets[:-1]).long()
        rows = torch.repeat_interleave(torch.arange(rb, device=self.device),
                                       counts)
        cols = m.indices.long()
        out = torch.zeros(rb, cb, BLOCK, BLOCK, dtype=self.dtype,
                          device=self.device)
        out[rows, cols] = self.data
        dense = out.permute(0, 2, 1, 3).reshape(m.rows, m.cols)
        return dense.t() if self._transposed else dense

    def _descriptor(self) -> BlockMatrix:
        return self._meta.descriptor(self.data)


# ---- dense operand plumbing --------------------------------------------------

def _dense_operand(x: torch.Tensor) -> Tuple[Matrix, bool]:
    """(stored matrix, transpose flag) for a 2-D tensor: a transposed view of
    a contiguous tensor is passed as the stored matrix with the flag set,
    anything else is made contiguous."""
    if x.dim() != 2:
        raise ValueError("dense operands are 2-D")
    if x.is_contiguous():
        return Matrix(x.shape[0], x.shape[1], x), False
    if x.t().is_contiguous():
        s = x.t()
        return Matrix(s.shape[0], s.shape[1], s), True
    x = x.contiguous()
    return Matrix(x.shape[0], x.shape[1], x), False


def _check_dtypes(*ts):
    dt = ts[0].dtype
    if dt not in (torch.float16, torch.bfloat16):
        raise TypeError(f"unsupported dtype {dt} (fp16 or bf16)")
    for t in ts[1:]:
        if t.dtype != dt:
            raise TypeError("operands must share one dtype")


# ---- raw products (no autograd) ----------------------------------------------

def _dsd(a: SparseMatrix, b: torch.Tensor) -> torch.Tensor:
    _check_dtypes(a.data, b)
    if a.shape[1] != b.shape[0]:
        raise ValueError(f"dsd shapes {a.shape} x {tuple(b.shape)}")
    bm, tb = _dense_operand(b)
    out = torch.empty(a.shape[0], b.shape[1], dtype=b.dtype, device=b.device)
    if a.is_transposed():
        a._meta.ensure_transposed(a.data)
    MatmulEx(a._descriptor(), a.is_transposed(), bm, tb,
             Matrix(out.shape[0], out.shape[1], out))
    return out


def _dds(a: torch.Tensor, b: SparseMatrix) -> torch.Tensor:
    _check_dtypes(a, b.data)
    if a.shape[1] != b.shape[0]:
        raise ValueError(f"dds shapes {tuple(a.shape)} x {b.shape}")
    am, ta = _dense_operand(a)
    out = torch.empty(a.shape[0], b.shape[1], dtype=a.dtype, device=a.device)
    if not b.is_transposed():  # row n of op(B)^T is column n of B
        b._meta.ensure_transposed(b.data)
    MatmulEx(am, ta, b._descriptor(), b.is_transposed(),
             Matrix(out.shape[0], out.shape[1], out))
    return out


def _sdd(a: torch.Tensor, b: torch.Tensor, topo: SparseMatrix) -> torch.Tensor:
    """Block values of (a @ b) at topo's nonzero blocks, in topo's storage
    order. A transposed topo view means the product is stored transposed:
    (a @ b)^T = b^T @ a^T is computed instead."""
    _check_dtypes(a, b)
    if a.shape[1] != b.shape[0] or (a.shape[0], b.shape[1]) != topo.shape:
        raise ValueError(f"sdd shapes {tuple(a.shape)} x {tuple(b.shape)} "
                         f"-> {topo.shape}")
    if topo.is_transposed():
        a, b = b.t(), a.t()
    am, ta = _dense_operand(a)
    bm, tb = _dense_operand(b)
    data = torch.empty(topo.nnz_blocks, BLOCK, BLOCK, dtype=a.dtype,
                       device=a.device)
    topo._meta.ensure_row_indices(data)
    Matmul(am, ta, bm, tb, topo._meta.descriptor(data))
    return data


# ---- autograd ---------------------------------------------------------------

class _DSD(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a_data, b, a):
        ctx.a = a
        ctx.save_for_backward(a_data, b)
        return _dsd(a.with_data(a_data), b)

    @staticmethod
    def backward(ctx, dc):
        a_data, b = ctx.saved_tensors
        a = ctx.a.with_data(a_data)
        da = db = None
        if ctx.needs_input_grad[1]:
            db = _dsd(a.t(), dc)                       # op(A)^T dC
        if ctx.needs_input_grad[0]:
            # C = S B: dS = dC B^T;  C = S^T B: dS = B dC^T (at S's blocks)
            stored = a.t() if a.is_transposed() else a
            da = (_sdd(b, dc.t(), stored) if a.is_transposed()
                  else _sdd(dc, b.t(), stored))
        return da, db, None


class _DDS(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b_data, b):
        ctx.b = b
        ctx.save_for_backward(a, b_data)
        return _dds(a, b.with_data(b_data))

    @staticmethod
    def backward(ctx, dc):
        a, b_data = ctx.saved_tensors
        b = ctx.b.with_data(b_data)
        da = db = None
        if ctx.needs_input_grad[0]:
            da = _dds(dc, b.t())                       # dC op(B)^T
        if ctx.needs_input_grad[1]:
            # C = A S: dS = A^T dC;  C = A S^T: dS = dC^T A (at S's blocks)
            stored = b.t() if b.is_transposed() else b
            db = (_sdd(dc.t(), a, stored) if b.is_transposed()
                  else _sdd(a.t(), dc, stored))
        return da, db, None


class _SDD(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, topo):
        ctx.topo = topo
        ctx.save_for_backward(a, b)
        return _sdd(a, b, topo)

    @staticmethod
    def backward(ctx, dc_data):
        a, b = ctx.saved_tensors
        dc = ctx.topo.with_data(dc_data.contiguous())
        da = db = None
        if ctx.needs_input_grad[0]:
            da = _dsd(dc, b.t())                       # dC B^T
        if ctx.needs_input_grad[1]:
            db = _dds(a.t(), dc)                       # A^T dC
        return da, db, None


def dsd(a: SparseMatrix, b: torch.Tensor) -> torch.Tensor:
    """Dense = op(sparse) @ dense (reference dsd.h:10-22)."""
    return _DSD.apply(a.data, b, a)


def dds(a: torch.Tensor, b: SparseMatrix) -> torch.Tensor:
    """Dense = dense @ op(sparse) (reference dds.h:10-22)."""
    return _DDS.apply(a, b.data, b)


def sdd(a: torch.Tensor, b: torch.Tensor, topo: SparseMatrix) -> SparseMatrix:
    """Sparse (topo's blocks) = dense @ dense (reference sdd.h:10-15)."""
    return topo.with_data(_SDD.apply(a, b, topo))


def from_dense_mask(x: torch.Tensor, mask) -> SparseMatrix:
    """SparseMatrix holding x's blocks where the [rows/128, cols/128] block
    mask is true (row-major, sorted columns: the reference's mask -> BCSR
    order, matrix_utils.cu:254-289). Test/construction aid."""
    mask = torch.as_tensor(mask, dtype=torch.bool, device=x.device)
    rb, cb = mask.shape
    counts = mask.sum(dim=1, dtype=torch.int32)
    offsets = torch.zeros(rb + 1, dtype=torch.int32, device=x.device)
    offsets[1:] = torch.cumsum(counts, 0)
    r, c = torch.nonzero(mask, as_tuple=True)
    blocks = x.reshape(rb, BLOCK, cb, BLOCK).permute(0, 2, 1, 3)[r, c]
    return SparseMatrix(tuple(x.shape), blocks.contiguous(), offsets,
                        c.to(torch.int16))


def topology_from_mask(mask: torch.Tensor, dtype=torch.float16
                       ) -> SparseMatrix:
    """SparseMatrix (uninitialised block values) whose topology is built
    on the device from a [rows/128, cols/128] block mask."""
    from . import MaskToBcsr
    mask = mask.to(torch.uint8).contiguous()
    rb, cb = mask.shape
    offsets = torch.empty(rb + 1, dtype=torch.int32, device=mask.device)
    cap = torch.empty(max(rb * cb, 1), dtype=torch.int16, device=mask.device)
    MaskToBcsr(mask, offsets, cap)
    nb = int(offsets[-1].item())  # one host sync: the block count sizes data
    data = torch.empty(nb, BLOCK, BLOCK, dtype=dtype, device=mask.device)
    return SparseMatrix((rb * BLOCK, cb * BLOCK), data, offsets,
                        cap[:nb].clone())


def expert_topology(padded_bins: torch.Tensor, blocks_per_expert: int,
                    block_rows: int, dtype=torch.bfloat16) -> SparseMatrix:
    """The dMoE topology (MegaBlocks `topology` op) built on the device:
    block-row r belongs to the expert whose padded bin holds token 128 r and
    owns that expert's `blocks_per_expert` block-columns. No host sync."""
    from . import ExpertTopology
    bins = padded_bins.to(torch.int32).contiguous()
    e = int(bins.numel())
    dev = bins.device
    offsets = torch.empty(block_rows + 1, dtype=torch.int32, device=dev)
    indices = torch.empty(block_rows * blocks_per_expert, dtype=torch.int16,
                          device=dev)
    ExpertTopology(bins, block_rows, blocks_per_expert, offsets, indices)
    data = torch.empty(block_rows * blocks_per_expert, BLOCK, BLOCK,
                       dtype=dtype, device=dev)
    return SparseMatrix((block_rows * BLOCK, e * blocks_per_expert * BLOCK),
                        data, offsets, indices)


__all__ = ["SparseMatrix", "dds", "dsd", "expert_topology", "from_dense_mask",
           "sdd", "topology_from_mask"]
