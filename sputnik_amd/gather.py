"""Assemble a sharded product's full result across ranks.

The hot path shards with no collective: DSD by nonzero-balanced block-row
panels of A (``matrix_utils.shard_rows_by_nnz``), DDS by block-column panels
of B (``shard_cols_by_nnz``), SDD by equal runs of C's stored blocks
(``shard_blocks``). A caller that wants the whole dense C (or the whole BCSR
``data`` of an SDD output) on every rank calls one of the functions here
after the product; nothing here runs inside the product.

Transport (``torch.distributed``; the "nccl" backend is RCCL over xGMI on
MI355X, "gloo" works for CPU tensors):

* equal pieces (e.g. the same number of block-rows per rank): one
  ``all_gather_into_tensor`` straight into the output;
* unequal pieces (nonzero-balanced panels rarely hold equal row counts):
  every rank sends its piece to every peer and receives each peer's piece
  in place, as one ``batch_isend_irecv`` group (``ncclGroupStart`` /
  ``ncclGroupEnd`` on RCCL). On xGMI's point-to-point mesh each peer pair
  is one link, so every link carries exactly one piece and nothing is padded.
  ``method="padded"`` instead pads every piece to the largest, runs one
  all-gather and compacts (for backends without point-to-point).

The reference has no collective of its own; this is the
``north_star``'s "RCCL all-gather over xGMI only when the caller wants the
full dense result".
"""

from __future__ import annotations

from typing import Optional, Sequence, Tuple

BLOCK = 128


def _dist():
    import torch.distributed as dist
    return dist


def allgather_concat(local, sizes: Sequence[int], group=None, out=None,
                     method: str = "auto"):
    """Concatenate every rank's ``local`` along dim 0, in rank order.

    ``sizes[r]`` is rank r's length along dim 0 (every rank passes the same
    list; ``local.shape[0] == sizes[rank]``). The trailing dims must match on
    every rank. Returns ``out`` (allocated when None) of shape
    ``(sum(sizes),) + local.shape[1:]``.
    """
    import torch
    dist = _dist()
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    sizes = [int(s) for s in sizes]
    if len(sizes) != world:
        raise ValueError(f"sizes has {len(sizes)} entries, world is {world}")
    if local.shape[0] != sizes[rank]:
        raise ValueError(f"rank {rank}: local has {local.shape[0]} rows, "
                         f"sizes says {sizes[rank]}")
    tail = tuple(local.shape[1:])
    total = sum(sizes)
    if out is None:
        out = torch.empty((total,) + tail, dtype=local.dtype, device=local.device)
    elif tuple(out.shape) != (total,) + tail or not out.is_contiguous():
        raise ValueError(f"out must be contiguous {(total,) + tail}, "
                         f"got {tuple(out.shape)}")
    local = local.contiguous()
    if local.is_cuda and dist.get_backend(group) == "gloo":
        # gloo moves host tensors only: stage through host memory (tests and
        # CPU rehearsals; RCCL ("nccl") gathers device memory directly)
        host = allgather_concat(local.cpu(), sizes, group=group, method=method)
        out.copy_(host)
        return out
    starts = [0]
    for s in sizes:
        starts.append(starts[-1] + s)
    if method not in ("auto", "p2p", "padded"):
        raise ValueError(f"unknown method {method!r}")
    if world == 1:
        out.copy_(local)
        return out
    if all(s == sizes[0] for s in sizes) and method != "padded":
        dist.all_gather_into_tensor(out, local, group=group)
        return out
    if method == "padded":
        mx = max(sizes)
        pad = torch.zeros((mx,) + tail, dtype=local.dtype, device=local.device)
        pad[: sizes[rank]] = local
        full = torch.empty((world * mx,) + tail, dtype=local.dtype,
                           device=local.device)
        dist.all_gather_into_tensor(full, pad, group=group)
        for r in range(world):
            out[starts[r]:starts[r + 1]] = full[r * mx: r * mx + sizes[r]]
        return out
    # point-to-point: one group of sends and receives, zero-size pieces skipped
    # on both sides (every rank knows every size)
    ops = []
    for peer in range(world):
        if peer == rank:
            continue
        gpeer = dist.get_global_rank(group, peer) if group is not None else peer
        if sizes[rank] > 0:
            ops.append(dist.P2POp(dist.isend, local, gpeer, group))
        if sizes[peer] > 0:
            ops.append(dist.P2POp(dist.irecv, out[starts[peer]:starts[peer + 1]],
                                  gpeer, group))
    reqs = dist.batch_isend_irecv(ops) if ops else []
    out[starts[rank]:starts[rank + 1]] = local
    for r in reqs:
        r.wait()
    return out


def gather_row_panels(c_panel, panels: Sequence[Tuple[int, int]], group=None,
                      out=None, method: str = "auto"):
    """Full dense C [M, N] from DSD row panels.

    ``panels[r] = (r0, r1)``: rank r computed block-rows [r0, r1) of C as
    its ``c_panel`` [(r1 - r0) * 128, N] (``shard_rows_by_nnz`` output: the
    panels are contiguous and cover [0, M / 128) in rank order).
    """
    _check_cover(panels)
    sizes = [(r1 - r0) * BLOCK for r0, r1 in panels]
    return allgather_concat(c_panel, sizes, group=group, out=out, method=method)


def gather_col_panels(c_panel, panels: Sequence[Tuple[int, int]], group=None,
                      out=None, method: str = "auto"):
    """Full dense C [M, N] from DDS column panels.

    ``panels[r] = (c0, c1)``: rank r computed block-columns [c0, c1) of C as
    its ``c_panel`` [M, (c1 - c0) * 128] (``shard_cols_by_nnz``). The pieces
    travel as they are (each contiguous [M][w_r]) and land in their columns.
    A caller's ``out`` must be a contiguous [M, N] tensor of c_panel's dtype
    and device. Peak memory is twice the result: the pieces arrive in one
    flat [M * N] staging tensor before they are placed in their columns.
    """
    import torch
    _check_cover(panels)
    dist = _dist()
    world = dist.get_world_size(group)
    widths = [(c1 - c0) * BLOCK for c0, c1 in panels]
    m = c_panel.shape[0]
    n = sum(widths)
    if out is not None and (tuple(out.shape) != (m, n) or not out.is_contiguous()
                            or out.dtype != c_panel.dtype
                            or out.device != c_panel.device):
        raise ValueError(f"out must be a contiguous {(m, n)} {c_panel.dtype} tensor "
                         f"on {c_panel.device}, got {tuple(out.shape)} {out.dtype} "
                         f"on {out.device}")
    flat = allgather_concat(c_panel.contiguous().reshape(-1), [m * w for w in widths],
                            group=group, method=method)
    if out is None:
        out = torch.empty((m, n), dtype=c_panel.dtype, device=c_panel.device)
    pos = 0
    for r in range(world):
        c0 = panels[r][0] * BLOCK
        w = widths[r]
        if w:
            out[:, c0:c0 + w] = flat[pos:pos + m * w].view(m, w)
        pos += m * w
    return out


def gather_block_runs(blocks, runs: Sequence[Tuple[int, int]], group=None,
                      out=None, method: str = "auto"):
    """Whole BCSR ``data`` of an SDD output from per-rank block runs.

    ``runs[r] = (b0, b1)`` (``shard_blocks``): rank r computed stored blocks
    [b0, b1) as ``blocks`` (any shape whose dim 0 is the block, e.g.
    [b1 - b0, 128, 128], or its flat view of (b1 - b0) * 128 * 128 values).
    """
    _check_cover(runs)
    if blocks.dim() == 1:
        blocks = blocks.view(-1, BLOCK, BLOCK)
    sizes = [b1 - b0 for b0, b1 in runs]
    return allgather_concat(blocks, sizes, group=group, out=out, method=method)


def _check_cover(parts: Sequence[Tuple[int, int]]):
    if not parts or parts[0][0] != 0:
        raise ValueError("pieces must start at 0")
    for (a0, a1), (b0, _) in zip(parts, parts[1:]):
        if a1 != b0 or a1 < a0:
            raise ValueError(f"pieces must be contiguous and ordered: {parts}")
    if parts[-1][1] < parts[-1][0]:
        raise ValueError(f"empty range reversed: {parts[-1]}")


__all__ = ["allgather_concat", "gather_row_panels", "gather_col_panels",
           "gather_block_runs"]
