"""Synthetic BCSR operands, as the reference's test/benchmark harness builds them.

Restates the topology half of reference sputnik/block/matrix_utils.cu:7-95
(BlockSparseMatrix with RANDOM_UNIFORM, pad_rows_to=1) on top of
sputnik/matrix_utils.cu:254-289 (mask from a shuffled iota, row-major CSR
scan) and the benchmark's nonzero count (dsd_benchmark.cu:28-46). The random
stream is numpy's, not absl's (the reference seeds absl nondeterministically,
so no stream is canonical); given the same permutation the CSR is bit-identical
to the reference's scan (checked against the C oracle in tests/test_oracle.py).

This is input generation (host, numpy), not compute: no product is evaluated
here.
"""

from __future__ import annotations

import numpy as np

BLOCK = 128


def round_up(x: int, b: int) -> int:
    """dsd_benchmark.cu:28-30"""
    return (x + b - 1) // b * b


def nonzeros_for_density(rows: int, cols: int, density: float,
                         block: int = BLOCK) -> int:
    """Element count the reference benchmark uses: RoundUp(int(d*d*s), b*b)
    (dsd_benchmark.cu:41)."""
    return round_up(int(np.float32(rows * cols) * np.float32(density)), block * block)


def mask_to_bcsr(mask: np.ndarray):
    """Row-major scan of a block mask -> (offsets int32, indices int32).
    matrix_utils.cu:269-289 with row_padding=1."""
    mask = np.asarray(mask, dtype=bool)
    offsets = np.zeros(mask.shape[0] + 1, dtype=np.int32)
    np.cumsum(mask.sum(axis=1), out=offsets[1:])
    indices = np.nonzero(mask)[1].astype(np.int32)
    return offsets, indices


def random_perm_mask(block_rows: int, block_cols: int, nnz_blocks: int,
                     rng: np.random.Generator):
    """The reference's mask construction: shuffle iota(R*C), keep entries whose
    shuffled value is < nnz (matrix_utils.cu:262-267). Returns (perm, mask)."""
    perm = rng.permutation(block_rows * block_cols).astype(np.int64)
    mask = (perm < nnz_blocks).reshape(block_rows, block_cols)
    return perm, mask


def random_topology(block_rows: int, block_cols: int, nnz_blocks: int,
                    rng: np.random.Generator, unordered: bool = False):
    """(offsets, indices) of a RANDOM_UNIFORM block topology; with
    `unordered`, each block-row's indices are shuffled like
    block/matrix_utils.cu:86-94."""
    _, mask = random_perm_mask(block_rows, block_cols, nnz_blocks, rng)
    offsets, indices = mask_to_bcsr(mask)
    if unordered:
        for i in range(block_rows):
            seg = indices[offsets[i]:offsets[i + 1]]
            rng.shuffle(seg)
    return offsets, indices


def expert_block_diagonal(num_experts: int, rows_per_expert: int,
                          cols_per_expert: int):
    """MegaBlocks dMoE topology: expert e owns block-rows
    [e*rows_per_expert, ...) x block-cols [e*cols_per_expert, ...)."""
    rows = []
    for e in range(num_experts):
        cols = np.arange(e * cols_per_expert, (e + 1) * cols_per_expert)
        rows.extend([cols] * rows_per_expert)
    counts = np.array([len(r) for r in rows])
    offsets = np.zeros(len(rows) + 1, dtype=np.int32)
    np.cumsum(counts, out=offsets[1:])
    indices = np.concatenate(rows).astype(np.int32)
    return offsets, indices


def block_mask(offsets: np.ndarray, indices: np.ndarray, block_cols: int):
    """Dense [block_rows][block_cols] 0/1 mask of a topology."""
    block_rows = len(offsets) - 1
    m = np.zeros((block_rows, block_cols), dtype=np.uint8)
    rows = np.repeat(np.arange(block_rows), np.diff(offsets))
    m[rows, indices] = 1
    return m


def random_values(shape, rng: np.random.Generator) -> np.ndarray:
    """U(-1, 1) float32 values (matrix_utils.cu:107-108, block/matrix_utils.cu:82-84)."""
    return rng.uniform(-1.0, 1.0, size=shape).astype(np.float32)


def to_dense(rows: int, cols: int, offsets, indices, values, block=BLOCK):
    """BCSR -> dense (block/matrix_utils.h:81-112), vectorised."""
    out = np.zeros((rows, cols), dtype=values.dtype)
    blocks = values.reshape(-1, block, block)
    block_rows = len(offsets) - 1
    r_of = np.repeat(np.arange(block_rows), np.diff(offsets))
    view = out.reshape(rows // block, block, cols // block, block)
    view[r_of, :, np.asarray(indices), :] = blocks
    return out


def shard_rows_by_nnz(offsets: np.ndarray, parts: int):
    """Contiguous block-row panels with balanced nonzero counts:
    returns [(r0, r1)] for each part. Greedy on the prefix sum so every part
    gets a contiguous run; empty parts are allowed when rows < parts."""
    offsets = np.asarray(offsets, dtype=np.int64)
    block_rows = len(offsets) - 1
    total = int(offsets[-1])
    bounds = [0]
    for p in range(1, parts):
        target = total * p / parts
        r = int(np.searchsorted(offsets, target, side="left"))
        r = min(max(r, bounds[-1]), block_rows)
        bounds.append(r)
    bounds.append(block_rows)
    return [(bounds[i], bounds[i + 1]) for i in range(parts)]


def slice_block_rows(offsets, indices, values, r0: int, r1: int):
    """Rebase block-rows [r0, r1) of a BCSR matrix into a standalone panel:
    offsets[r0:r1+1] - offsets[r0], with the matching indices / block values
    (SURVEY §8e). `values` is indexed by block (shape [nb, b, b] or any array
    whose first axis is the block)."""
    offsets = np.asarray(offsets)
    o0, o1 = int(offsets[r0]), int(offsets[r1])
    return (offsets[r0:r1 + 1] - o0).astype(np.int32), indices[o0:o1], values[o0:o1]


def shard_cols_by_nnz(offsets: np.ndarray, indices: np.ndarray,
                      block_cols: int, parts: int):
    """DDS sharding: contiguous block-column panels of the sparse
    operand B with balanced nonzero counts, [(c0, c1)] per part. The column
    counts are offsets_t (transpose.cu:94-97), so this is shard_rows_by_nnz
    over B's transposed row pointer; each rank computes C[:, c0·b : c1·b]
    with A replicated."""
    counts = np.bincount(np.asarray(indices, dtype=np.int64),
                         minlength=block_cols)
    offsets_t = np.concatenate([[0], np.cumsum(counts)])
    return shard_rows_by_nnz(offsets_t, parts)


def slice_block_cols(offsets, indices, values, c0: int, c1: int):
    """Block-columns [c0, c1) of a BCSR matrix as a standalone BCSR matrix
    (all block-rows, columns rebased to c0), with the matching block values.
    Storage order is kept, so a row's blocks stay in their original order."""
    offsets = np.asarray(offsets, dtype=np.int64)
    idx = np.asarray(indices)
    keep = (idx >= c0) & (idx < c1)
    row_of = np.repeat(np.arange(len(offsets) - 1), np.diff(offsets))
    per_row = np.bincount(row_of[keep], minlength=len(offsets) - 1)
    p_off = np.concatenate([[0], np.cumsum(per_row)]).astype(np.int32)
    return p_off, (idx[keep] - c0).astype(idx.dtype), values[keep]


def shard_blocks(nb: int, parts: int):
    """SDD sharding: the output's stored-block list split into
    contiguous, equal runs [(b0, b1)] (the grid is over nb, so equal counts
    are equal work). A and B are replicated."""
    bounds = [nb * p // parts for p in range(parts + 1)]
    return [(bounds[i], bounds[i + 1]) for i in range(parts)]


def slice_blocks(offsets, indices, b0: int, b1: int):
    """Stored blocks [b0, b1) of a BCSR output as a standalone BCSR topology
    over the same block-rows (rows outside the run become empty). The rank's
    `data` is the caller's data + b0·b² and its row_indices are
    row_indices[b0:b1], so no block moves; the union over ranks writes every
    stored block exactly once."""
    offsets = np.asarray(offsets, dtype=np.int64)
    p_off = (np.clip(offsets, b0, b1) - b0).astype(np.int32)
    return p_off, np.asarray(indices)[b0:b1]
