"""ctypes wrapper of the C oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker or the timed CPU baseline. The
product path (sputnik_amd/) never imports this module.

Parity status: partially pinned (see oracle.c header and DESIGN.md "Oracle").
"""

from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_DIR, "liboracle.so")

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", _DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        I = ctypes.c_int
        L.oracle_mask_to_bcsr.argtypes = [I, I, I, P, P, P]
        L.oracle_mask_to_bcsr.restype = I
        L.oracle_row_indices.argtypes = [I, P, P]
        L.oracle_row_indices.restype = None
        L.oracle_transpose.argtypes = [I, I, P, P, P, P, P]
        L.oracle_transpose.restype = None
        L.oracle_bitmask.argtypes = [I, I, P, P, P]
        L.oracle_bitmask.restype = None
        L.oracle_bcsr_to_dense.argtypes = [I, I, I, P, P, P, P]
        L.oracle_bcsr_to_dense.restype = None
        L.oracle_gemm.argtypes = [I, I, I, P, I, P, I, P, P, P, P, I]
        L.oracle_gemm.restype = None
        L.oracle_round.argtypes = [P, P, ctypes.c_int64, I]
        L.oracle_round.restype = None
        L.oracle_openmp_threads.argtypes = []
        L.oracle_openmp_threads.restype = I
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def mask_to_bcsr(perm: np.ndarray, rows: int, cols: int, nnz: int):
    perm = np.ascontiguousarray(perm, dtype=np.int64)
    offsets = np.zeros(rows + 1, dtype=np.int32)
    indices = np.zeros(max(nnz, 1), dtype=np.int32)
    n = lib().oracle_mask_to_bcsr(rows, cols, nnz, _p(perm), _p(offsets),
                                  _p(indices))
    return offsets, indices[:n]


def row_indices(offsets: np.ndarray) -> np.ndarray:
    offsets = np.ascontiguousarray(offsets, dtype=np.int32)
    out = np.zeros(max(int(offsets[-1]), 1), dtype=np.int16)
    lib().oracle_row_indices(len(offsets) - 1, _p(offsets), _p(out))
    return out[: int(offsets[-1])]


def transpose(offsets: np.ndarray, indices: np.ndarray, block_cols: int):
    """-> (offsets_t int32[C+1], indices_t int16[nb], block_offsets int32[nb])"""
    offsets = np.ascontiguousarray(offsets, dtype=np.int32)
    indices = np.ascontiguousarray(indices, dtype=np.int16)
    nb = int(offsets[-1])
    offsets_t = np.zeros(block_cols + 1, dtype=np.int32)
    indices_t = np.zeros(max(nb, 1), dtype=np.int16)
    block_offsets = np.zeros(max(nb, 1), dtype=np.int32)
    lib().oracle_transpose(len(offsets) - 1, block_cols, _p(offsets),
                           _p(indices), _p(offsets_t), _p(indices_t),
                           _p(block_offsets))
    return offsets_t, indices_t[:nb], block_offsets[:nb]


def bitmask(offsets: np.ndarray, indices: np.ndarray, block_cols: int):
    """-> uint64 [block_rows, ceil(block_cols/64)] (bitmask.cu:31-39)."""
    offsets = np.ascontiguousarray(offsets, dtype=np.int32)
    indices = np.ascontiguousarray(indices, dtype=np.int16)
    rows = len(offsets) - 1
    words = (block_cols + 63) // 64
    out = np.zeros((max(rows, 1), max(words, 1)), dtype=np.uint64)
    lib().oracle_bitmask(rows, block_cols, _p(offsets), _p(indices), _p(out))
    return out[:rows, :words]


def bcsr_to_dense(rows, cols, offsets, indices, values, block=128):
    offsets = np.ascontiguousarray(offsets, dtype=np.int32)
    indices = np.ascontiguousarray(indices, dtype=np.int16)
    values = np.ascontiguousarray(values, dtype=np.float32)
    out = np.empty((rows, cols), dtype=np.float32)
    lib().oracle_bcsr_to_dense(rows, cols, block, _p(offsets), _p(indices),
                               _p(values), _p(out))
    return out


def gemm(a: np.ndarray, ta: bool, b: np.ndarray, tb: bool, *, a_mask=None,
         b_mask=None, out_mask=None, out=None, threads: int = 1):
    """The reference's host matmul (matrix_utils.h:376-391) on op(a) op(b),
    float32 in / float32 out, double accumulation; optional zero-block skips."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    m = a.shape[1] if ta else a.shape[0]
    k = a.shape[0] if ta else a.shape[1]
    n = b.shape[0] if tb else b.shape[1]
    kb = b.shape[1] if tb else b.shape[0]
    assert k == kb, (a.shape, b.shape, ta, tb)
    if out is None:
        out = np.zeros((m, n), dtype=np.float32)
    masks = [None if x is None else np.ascontiguousarray(x, dtype=np.uint8)
             for x in (a_mask, b_mask, out_mask)]
    lib().oracle_gemm(m, n, k, _p(a), int(ta), _p(b), int(tb), _p(masks[0]),
                      _p(masks[1]), _p(masks[2]), _p(out), int(threads))
    return out


def round_to(x: np.ndarray, dtype: str) -> np.ndarray:
    """float32 -> nearest fp16 ('f16') / bf16 ('bf16') value, as float32."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty_like(x)
    lib().oracle_round(_p(x), _p(out), x.size, 1 if dtype == "bf16" else 0)
    return out


def openmp_threads() -> int:
    return lib().oracle_openmp_threads()
