#!/usr/bin/env python3
"""Config 5 (DSD M = 131072, K = N = 4096, 2%, tall pipeline) on the same
blocks with the block-rows permuted: bench.py's topology as is, vs rows
sorted by the k-index of their first block (empty rows kept in place), vs
fully sorted. Same work and the same per-tile sums; only which tiles run
side by side changes. Tests whether the B re-reads (PMC: 492 MB of reads
per launch for 53 MB of operands) cost time. Same process, interleaved."""
import json
import os
import sys
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from sputnik_amd import matrix_utils as mu  # noqa: E402


def permuted(off, idx, order):
    cnt = np.diff(off)
    new_off = np.concatenate([[0], np.cumsum(cnt[order])]).astype(np.int32)
    new_idx = np.concatenate([idx[off[r]:off[r + 1]] for r in order]) if len(idx) else idx
    return new_off, new_idx.astype(idx.dtype)


def main():
    dev = torch.device("cuda", 0)
    M, K, N = 131072, 4096, 4096
    nz = mu.nonzeros_for_density(M, K, 0.02)
    off, idx = mu.random_topology(M // 128, K // 128, nz // (128 * 128),
                                  np.random.default_rng(5))
    R = M // 128
    cnt = np.diff(off)
    first = np.array([idx[off[r]] if cnt[r] else -1 for r in range(R)])
    nonempty = np.nonzero(cnt)[0]
    # (a) non-empty rows sorted by first k, empty rows in their places
    order_a = np.arange(R)
    order_a[nonempty] = nonempty[np.argsort(first[nonempty], kind="stable")]
    # (b) every row sorted (empty rows first)
    order_b = np.argsort(first, kind="stable")
    # (c) sorted non-empty rows dealt into D chunks (chunk c = sorted[c::D]),
    # chunks in sequence, empty rows last: with ~D workgroups per panel each
    # taking one chunk, the workgroups' t-th tiles have nearly the same first
    # k-block, so they read the same B slice at the same time
    srt = nonempty[np.argsort(first[nonempty], kind="stable")]
    empty = np.nonzero(cnt == 0)[0]
    dealt = {D: np.concatenate([np.concatenate([srt[c::D] for c in range(D)]), empty])
             for D in (32, 31)}
    probs = {}
    for name, order in (("as_is", np.arange(R)), ("ksorted_rows", order_a),
                        ("dealt32", dealt[32]), ("dealt31", dealt[31])):
        o, i = permuted(off, idx, order)
        probs[name] = bench.DsdProblem(M, K, o, i, N, False, False, "f16", 0, dev)
    if len(sys.argv) > 1:  # one variant only (for rocprofv3 --pmc passes)
        probs = {sys.argv[1]: probs[sys.argv[1]]}
    fns = {k: p.launcher() for k, p in probs.items()}
    res = {k: [] for k in fns}
    for _ in range(7 if len(fns) > 1 else 1):
        for k, f in fns.items():
            for _ in range(20):
                f()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(100):
                f()
            e.record()
            torch.cuda.synchronize()
            res[k].append(s.elapsed_time(e) * 10.0)
    print(json.dumps({k: round(float(np.median(v)), 2) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
