"""sputnik_amd — MI355X-native block-sparse matmul (DSD / DDS / SDD, block 128).

Python mirror of the reference's ``sputnik::block`` API (sputnik/sputnik.h,
sputnik/block/arguments.h) over the C-ABI of ``libsputnik.so``
(include/sputnik_amd.h). Names, argument meaning and the overload set follow
the reference:

    Matmul(BlockMatrix a, ta, Matrix b, tb, Matrix c)        DSD  dsd.h:10-15
    Matmul(Matrix a, ta, BlockMatrix b, tb, Matrix c)        DDS  dds.h:10-15
    Matmul(Matrix a, ta, Matrix b, tb, BlockMatrix c)        SDD  sdd.h:10-15
    MatmulEx(...)      (DSD/DDS, precomputed transposed metadata)
    RowIndices(a, row_indices), Transpose(a)
    AllocateTransposeBuffers(a), AllocateRowIndicesBuffer(a)

Device memory is held in torch tensors (plumbing only); every computation runs
in the HIP kernels of libsputnik.so. There is no CPU fallback: if the library
is missing, importing the compute entry points raises.
"""

from __future__ import annotations

import ctypes
import enum
import os
from dataclasses import dataclass, field
from typing import Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SPUTNIK_AMD_LIB") or os.path.join(_HERE, "libsputnik.so")

hipSuccess = 0
hipErrorInvalidValue = 1
hipErrorNotSupported = 801


class SputnikError(RuntimeError):
    """A non-zero hipError_t returned by libsputnik."""

    def __init__(self, code: int, what: str):
        super().__init__(f"{what} failed with hipError_t {code}")
        self.code = code


class BlockSize(enum.IntEnum):
    """reference sputnik/block/arguments.h:13-19"""

    kNone = 0
    k16 = 16
    k32 = 32
    k64 = 64
    k128 = 128


def AsInt(b) -> int:  # noqa: N802 (reference name)
    b = int(b)
    return b if b in (16, 32, 64, 128) else 0


class _CBlockMatrix(ctypes.Structure):
    """sputnik_block_matrix_t — byte-identical to the C++ BlockMatrix (88 B)."""

    _fields_ = [
        ("rows", ctypes.c_int32),
        ("cols", ctypes.c_int32),
        ("nonzeros", ctypes.c_int32),
        ("block_size", ctypes.c_int32),
        ("data", ctypes.c_void_p),
        ("offsets", ctypes.c_void_p),
        ("indices", ctypes.c_void_p),
        ("offsets_t", ctypes.c_void_p),
        ("indices_t", ctypes.c_void_p),
        ("block_offsets", ctypes.c_void_p),
        ("row_indices", ctypes.c_void_p),
        ("bitmask", ctypes.c_void_p),
        ("create_metadata", ctypes.c_uint8),
    ]


class _CMatrix(ctypes.Structure):
    """sputnik_matrix_t (16 B)."""

    _fields_ = [
        ("rows", ctypes.c_int32),
        ("cols", ctypes.c_int32),
        ("data", ctypes.c_void_p),
    ]


_P = ctypes.c_void_p
_SIGNATURES = {
    "sputnik_dsd": [_P, ctypes.c_int, _P, ctypes.c_int, _P, ctypes.c_int, _P],
    "sputnik_dsd_ex": [_P, ctypes.c_int, _P, ctypes.c_int, _P, ctypes.c_int, _P],
    "sputnik_dds": [_P, ctypes.c_int, _P, ctypes.c_int, _P, ctypes.c_int, _P],
    "sputnik_dds_ex": [_P, ctypes.c_int, _P, ctypes.c_int, _P, ctypes.c_int, _P],
    "sputnik_sdd": [_P, ctypes.c_int, _P, ctypes.c_int, _P, ctypes.c_int, _P],
    "sputnik_ssd": [_P, ctypes.c_int, _P, ctypes.c_int, _P, ctypes.c_int, _P],
    "sputnik_ssd_ex": [_P, ctypes.c_int, _P, ctypes.c_int, _P, ctypes.c_int, _P],
    "sputnik_sds": [_P, ctypes.c_int, _P, ctypes.c_int, _P, ctypes.c_int, _P],
    "sputnik_sds_ex": [_P, ctypes.c_int, _P, ctypes.c_int, _P, ctypes.c_int, _P],
    "sputnik_dss": [_P, ctypes.c_int, _P, ctypes.c_int, _P, ctypes.c_int, _P],
    "sputnik_dss_ex": [_P, ctypes.c_int, _P, ctypes.c_int, _P, ctypes.c_int, _P],
    "sputnik_row_indices": [_P, _P, _P],
    "sputnik_transpose": [_P, _P],
    "sputnik_mask_to_bcsr": [_P, ctypes.c_int, ctypes.c_int, _P, _P, _P],
    "sputnik_expert_topology": [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                _P, _P, _P],
    "sputnik_can_implement": [ctypes.c_int, _P, ctypes.c_int, _P, ctypes.c_int, _P],
    "sputnik_abi_block_matrix_size": [],
    "sputnik_abi_block_matrix_offset": [ctypes.c_int],
    "sputnik_abi_matrix_size": [],
    "sputnik_version": [],
    "sputnik_build_hash": [],
    "sputnik_bitmask": [_P, _P],
    "sputnik_bitmask_bytes": [_P],
    "sputnik_sdd_plan": [_P, ctypes.c_int, _P, ctypes.c_int, _P],
    "sputnik_pair_errors": [],
    "sputnik_debug_pair_fault": [ctypes.c_int],
    "sputnik_capture_workspaces": [],
    "sputnik_select_dsd_kernel": [ctypes.c_int],
    "sputnik_tuning_get": [ctypes.c_char_p],
    "sputnik_tuning_set": [ctypes.c_char_p, ctypes.c_int],
    "sputnik_dsd_plan": [_P, ctypes.c_int, _P, ctypes.c_int, _P, _P],
    "sputnik_sdd_kernel": [_P, ctypes.c_int, _P, ctypes.c_int, _P],
    "sputnik_dds_plan": [_P, ctypes.c_int, _P, ctypes.c_int, _P, _P],
}
_RESTYPES = {
    "sputnik_abi_block_matrix_size": ctypes.c_size_t,
    "sputnik_abi_block_matrix_offset": ctypes.c_size_t,
    "sputnik_abi_matrix_size": ctypes.c_size_t,
    "sputnik_version": ctypes.c_char_p,
    "sputnik_build_hash": ctypes.c_char_p,
    "sputnik_bitmask_bytes": ctypes.c_size_t,
    "sputnik_debug_pair_fault": None,
}

_lib: Optional[ctypes.CDLL] = None


def lib() -> ctypes.CDLL:
    """Load libsputnik.so (built by `make -C sputnik_amd`). Raises if absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` or "
                "`make -C sputnik_amd`. There is no CPU fallback.")
        # PyTorch ships its own HIP runtime (same soname as ROCm's). Load it
        # first so the library binds to that one copy; loading libsputnik.so
        # first would pull in /opt/rocm's runtime next to torch's.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        handle = ctypes.CDLL(LIB_PATH)
        for name, args in _SIGNATURES.items():
            fn = getattr(handle, name)
            fn.argtypes = args
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        _lib = handle
    return _lib


def _ptr(t) -> Optional[int]:
    if t is None:
        return None
    return t.data_ptr()


@dataclass
class Matrix:
    """Dense row-major matrix (reference arguments.h:155-162)."""

    rows: int
    cols: int
    data: object  # torch.Tensor (fp16/bf16), rows*cols elements

    def _c(self) -> _CMatrix:
        return _CMatrix(self.rows, self.cols, _ptr(self.data))


@dataclass
class BlockMatrix:
    """BCSR matrix (reference arguments.h:48-153). rows/cols/nonzeros in
    elements; offsets int32 [rows/b+1]; indices int16 [#blocks]; data holds
    #blocks row-major b x b blocks back to back."""

    rows: int
    cols: int
    block_size: int
    nonzeros: int
    data: object
    offsets: object
    indices: object
    offsets_t: object = None
    indices_t: object = None
    block_offsets: object = None
    row_indices: object = None
    bitmask: object = None
    create_metadata: bool = True

    @property
    def num_blocks(self) -> int:
        b = AsInt(self.block_size)
        return self.nonzeros // (b * b) if b else 0

    def _c(self) -> _CBlockMatrix:
        return _CBlockMatrix(
            self.rows, self.cols, self.nonzeros, int(self.block_size),
            _ptr(self.data), _ptr(self.offsets), _ptr(self.indices),
            _ptr(self.offsets_t), _ptr(self.indices_t),
            _ptr(self.block_offsets), _ptr(self.row_indices),
            _ptr(self.bitmask), 1 if self.create_metadata else 0)


def _dtype_code(t) -> int:
    import torch

    if t.dtype == torch.float16:
        return 0
    if t.dtype == torch.bfloat16:
        return 1
    raise TypeError(f"unsupported element type {t.dtype} (fp16 or bf16)")


def _stream(stream) -> Optional[int]:
    if stream is not None:
        return int(stream)
    import torch

    return torch.cuda.current_stream().cuda_stream


def _check(code: int, what: str) -> None:
    if code != hipSuccess:
        raise SputnikError(code, what)


def _call(ex: bool, a, transpose_a: bool, b, transpose_b: bool, c, stream):
    L = lib()
    ta, tb = int(bool(transpose_a)), int(bool(transpose_b))
    if isinstance(a, BlockMatrix) and isinstance(b, Matrix) and isinstance(c, Matrix):
        ca, cb, cc = a._c(), b._c(), c._c()
        fn = L.sputnik_dsd_ex if ex else L.sputnik_dsd
        code = fn(ctypes.byref(ca), ta, ctypes.byref(cb), tb, ctypes.byref(cc),
                  _dtype_code(b.data), _stream(stream))
        _check(code, "dsd")
        return
    if isinstance(a, Matrix) and isinstance(b, BlockMatrix) and isinstance(c, Matrix):
        ca, cb, cc = a._c(), b._c(), c._c()
        fn = L.sputnik_dds_ex if ex else L.sputnik_dds
        code = fn(ctypes.byref(ca), ta, ctypes.byref(cb), tb, ctypes.byref(cc),
                  _dtype_code(a.data), _stream(stream))
        _check(code, "dds")
        return
    if (not ex and isinstance(a, Matrix) and isinstance(b, Matrix)
            and isinstance(c, BlockMatrix)):
        ca, cb, cc = a._c(), b._c(), c._c()
        code = L.sputnik_sdd(ctypes.byref(ca), ta, ctypes.byref(cb), tb,
                             ctypes.byref(cc), _dtype_code(a.data),
                             _stream(stream))
        _check(code, "sdd")
        return
    if (isinstance(a, BlockMatrix) and isinstance(b, Matrix)
            and isinstance(c, BlockMatrix)):
        ca, cb, cc = a._c(), b._c(), c._c()
        fn = L.sputnik_ssd_ex if ex else L.sputnik_ssd
        code = fn(ctypes.byref(ca), ta, ctypes.byref(cb), tb, ctypes.byref(cc),
                  _dtype_code(b.data), _stream(stream))
        _check(code, "ssd")
        return
    if (isinstance(a, Matrix) and isinstance(b, BlockMatrix)
            and isinstance(c, BlockMatrix)):
        ca, cb, cc = a._c(), b._c(), c._c()
        fn = L.sputnik_sds_ex if ex else L.sputnik_sds
        code = fn(ctypes.byref(ca), ta, ctypes.byref(cb), tb, ctypes.byref(cc),
                  _dtype_code(a.data), _stream(stream))
        _check(code, "sds")
        return
    if (isinstance(a, BlockMatrix) and isinstance(b, BlockMatrix)
            and isinstance(c, Matrix)):
        ca, cb, cc = a._c(), b._c(), c._c()
        fn = L.sputnik_dss_ex if ex else L.sputnik_dss
        code = fn(ctypes.byref(ca), ta, ctypes.byref(cb), tb, ctypes.byref(cc),
                  _dtype_code(c.data), _stream(stream))
        _check(code, "dss")
        return
    raise TypeError("no Matmul overload for these operand kinds")


def Matmul(a, transpose_a, b, transpose_b, c, stream=None):  # noqa: N802
    """DSD / DDS / SDD / SSD / SDS / DSS by operand kinds, like the C++
    overload set."""
    _call(False, a, transpose_a, b, transpose_b, c, stream)


def MatmulEx(a, transpose_a, b, transpose_b, c, stream=None):  # noqa: N802
    """DSD / DDS / SSD / SDS / DSS with the transposed metadata already
    present."""
    _call(True, a, transpose_a, b, transpose_b, c, stream)


def RowIndices(a: BlockMatrix, row_indices, stream=None):  # noqa: N802
    """reference sputnik/block/row_indices/row_indices.h:10"""
    ca = a._c()
    _check(lib().sputnik_row_indices(ctypes.byref(ca), _ptr(row_indices),
                                     _stream(stream)), "RowIndices")


def Transpose(a: BlockMatrix, stream=None):  # noqa: N802
    """reference sputnik/block/transpose/transpose.h:10 (on the device)."""
    ca = a._c()
    _check(lib().sputnik_transpose(ctypes.byref(ca), _stream(stream)),
           "Transpose")


def MaskToBcsr(mask, offsets, indices, stream=None):  # noqa: N802
    """Device block mask (uint8 [R, C]) -> BCSR offsets (int32 [R+1]) and
    ascending int16 indices (capacity >= nonzeros), the reference's
    mask -> CSR scan (matrix_utils.cu:254-289), stream-ordered."""
    rows, cols = int(mask.shape[0]), int(mask.shape[1])
    _check(lib().sputnik_mask_to_bcsr(_ptr(mask), rows, cols, _ptr(offsets),
                                      _ptr(indices), _stream(stream)),
           "MaskToBcsr")


def ExpertTopology(padded_bins, block_rows, blocks_per_expert, offsets,  # noqa: N802
                   indices, stream=None):
    """MegaBlocks dMoE topology on the device from cumulative padded bins
    (int32 [experts]); see include/sputnik_amd.h."""
    _check(lib().sputnik_expert_topology(
        _ptr(padded_bins), int(padded_bins.numel()), int(block_rows),
        int(blocks_per_expert), _ptr(offsets), _ptr(indices),
        _stream(stream)), "ExpertTopology")


def Bitmask(m: BlockMatrix, stream=None):  # noqa: N802
    """reference sputnik/block/bitmask/bitmask.h:10 (on the device): the
    BitMatrix of m's topology, over the transposed order when m.offsets_t is
    set (call AllocateBitmaskBuffers after AllocateTransposeBuffers then)."""
    cm = m._c()
    _check(lib().sputnik_bitmask(ctypes.byref(cm), _stream(stream)), "Bitmask")


def AllocateBitmaskBuffers(m: BlockMatrix):  # noqa: N802
    """reference bitmask.h:16-23 (uint64 words, torch-owned)."""
    import torch

    cm = m._c()
    words = lib().sputnik_bitmask_bytes(ctypes.byref(cm)) // 8
    m.bitmask = torch.empty(max(int(words), 1), dtype=torch.int64,
                            device=m.offsets.device)


def FreeBitmaskBuffers(m: BlockMatrix):  # noqa: N802
    m.bitmask = None


def sdd_plan(a, transpose_a, b, transpose_b, c) -> int:
    """SDD tile plan the dispatcher picks on the current device: 1 grouped
    128x512 tiles, 2 grouped tiles with each group's K split over 2-8
    workgroups, 0 one k-split block per workgroup, -1 rejected."""
    ca, cb, cc = a._c(), b._c(), c._c()
    return int(lib().sputnik_sdd_plan(ctypes.byref(ca), int(bool(transpose_a)),
                                      ctypes.byref(cb), int(bool(transpose_b)),
                                      ctypes.byref(cc)))


def sdd_kernel(a, transpose_a, b, transpose_b, c) -> int:
    """The kernel behind sdd_plan's tile plan: 0 8-wave k-split block tile,
    1 8-wave grouped, 2 4-wave K-split, 3 4-wave grouped, 4 B transposed
    into a library buffer then 4-wave grouped (NT / TT over a large B), -1
    rejected (sputnik_sdd_kernel)."""
    ca, cb, cc = a._c(), b._c(), c._c()
    return int(lib().sputnik_sdd_kernel(ctypes.byref(ca), int(bool(transpose_a)),
                                        ctypes.byref(cb), int(bool(transpose_b)),
                                        ctypes.byref(cc)))


def dds_plan(a, transpose_a, b, transpose_b, c, stream=None) -> int:
    """Kernel a DDS launch on `stream` would use: 0 8-wave tile, 1 4-wave
    kernel, 2 tall, 3 split (8-wave), -1 rejected (sputnik_dds_plan)."""
    if stream is None:
        import torch
        stream = torch.cuda.current_stream().cuda_stream
    ca, cb, cc = a._c(), b._c(), c._c()
    return int(lib().sputnik_dds_plan(ctypes.byref(ca), int(bool(transpose_a)),
                                      ctypes.byref(cb), int(bool(transpose_b)),
                                      ctypes.byref(cc), ctypes.c_void_p(stream)))


def pair_errors() -> int:
    """Pair hand-offs since the last call whose consumer timed out (its
    output tile is NaN; sputnik_pair_errors() in include/sputnik_amd.h)."""
    return int(lib().sputnik_pair_errors())


def capture_workspaces() -> int:
    """Workspaces made for graph-captured launches on the current device
    (sputnik_capture_workspaces() in include/sputnik_amd.h)."""
    return int(lib().sputnik_capture_workspaces())


def build_hash() -> str:
    return lib().sputnik_build_hash().decode()


def AllocateTransposeBuffers(a: BlockMatrix):  # noqa: N802
    """reference arguments.h:233-245 (torch-owned device workspaces)."""
    import torch

    dev = a.offsets.device
    bcols = a.cols // AsInt(a.block_size)
    a.offsets_t = torch.empty(bcols + 1, dtype=torch.int32, device=dev)
    a.indices_t = torch.empty(a.num_blocks, dtype=torch.int16, device=dev)
    a.block_offsets = torch.empty(a.num_blocks, dtype=torch.int32, device=dev)


def FreeTransposeBuffers(a: BlockMatrix):  # noqa: N802
    a.offsets_t = a.indices_t = a.block_offsets = None


def AllocateRowIndicesBuffer(a: BlockMatrix):  # noqa: N802
    """reference arguments.h:259-263"""
    import torch

    a.row_indices = torch.empty(a.num_blocks, dtype=torch.int16,
                                device=a.offsets.device)


def FreeRowIndicesBuffer(a: BlockMatrix):  # noqa: N802
    a.row_indices = None


_OPS = {"dsd": 0, "dds": 1, "sdd": 2, "ssd": 3, "sds": 4, "dss": 5}


def can_implement(op: str, a, transpose_a, b, transpose_b, c) -> bool:
    """Host-only: would the library accept this problem? (no device work)"""
    ca, cb, cc = a._c(), b._c(), c._c()
    return bool(lib().sputnik_can_implement(
        _OPS[op], ctypes.byref(ca), int(bool(transpose_a)), ctypes.byref(cb),
        int(bool(transpose_b)), ctypes.byref(cc)))


def dsd_plan(a, transpose_a, b, transpose_b, c, stream=None) -> int:
    """Kernel a DSD launch on `stream` (torch's current stream by default)
    would use: 0 8-wave tile, 1 4-wave kernel, 2 tall, 3 split, 4 tall
    pipeline (4-wave, persistent), -1 rejected
    (sputnik_dsd_plan)."""
    if stream is None:
        import torch
        stream = torch.cuda.current_stream().cuda_stream
    ca, cb, cc = a._c(), b._c(), c._c()
    return int(lib().sputnik_dsd_plan(ctypes.byref(ca), int(bool(transpose_a)),
                                      ctypes.byref(cb), int(bool(transpose_b)),
                                      ctypes.byref(cc), ctypes.c_void_p(stream)))


def select_dsd_kernel(four_wave: int = -1) -> int:
    """DSD / DDS / grouped-SDD kernel choice (sputnik_select_dsd_kernel): 1
    the 4-wave hand-scheduled kernel where it pays (default), 2-7 wherever
    it applies with a fixed variant (kEpi = mode - 2: 0 workgroup epilogue,
    1 per-wave, 2 specialized last block, 3 double slots, 4 double slots +
    barrier every other step + interleaved copy-out, 5 double slots +
    interleaved copy-out; transposed and SDD launches take the variant they
    have), 0 the 8-wave kernel, -1 query only. Returns the previous
    choice."""
    return int(lib().sputnik_select_dsd_kernel(int(four_wave)))


TUNING_UNKNOWN = -(2 ** 31)


def tuning(name: str, value: Optional[int] = None) -> int:
    """UNSUPPORTED tuning knob (sputnik_tuning_get / sputnik_tuning_set,
    include/sputnik_amd.h; tests and A/B experiments only): returns the
    knob's value, or with `value` sets it and returns the previous one.
    Raises KeyError for an unknown name or an out-of-range value."""
    L = lib()
    if value is None:
        v = int(L.sputnik_tuning_get(name.encode()))
    else:
        v = int(L.sputnik_tuning_set(name.encode(), int(value)))
    if v == TUNING_UNKNOWN:
        raise KeyError(f"tuning knob {name!r} (value {value!r})")
    return v


def version() -> str:
    return lib().sputnik_version().decode()


# Full-result gathers of a sharded product (host-side torch.distributed, off
# the hot path; sputnik_amd/gather.py).
from .gather import (allgather_concat, gather_block_runs,  # noqa: E402
                     gather_col_panels, gather_row_panels)


__all__ = [
    "AllocateBitmaskBuffers", "AllocateRowIndicesBuffer",
    "AllocateTransposeBuffers", "AsInt", "Bitmask", "FreeBitmaskBuffers",
    "build_hash", "capture_workspaces", "pair_errors", "sdd_plan", "sdd_kernel",
    "dds_plan",
    "select_dsd_kernel", "dsd_plan", "tuning",
    "BlockMatrix", "BlockSize", "ExpertTopology", "FreeRowIndicesBuffer",
    "MaskToBcsr",
    "FreeTransposeBuffers", "Matmul", "MatmulEx", "Matrix", "RowIndices",
    "SputnikError", "Transpose", "can_implement", "lib", "version",
    "allgather_concat", "gather_row_panels", "gather_col_panels",
    "gather_block_runs",
]
