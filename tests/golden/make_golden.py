#!/usr/bin/env python3
"""Generates tests/golden/golden_vectors.npz (committed).

Provenance, honestly stated: the reference ships no golden vectors and cannot
be built in this image (DESIGN.md "Oracle"), so these fixtures are produced by
the C oracle (oracle/oracle.c) from fixed seeds. They pin the oracle against
regressions and give the GPU tests fixed inputs with expected outputs. The one
fixture that comes from the reference itself is the `survey_kat` metadata
case: the input/output recorded from the reference's own host Transpose in
SURVEY.md §8(c).

Contents (all arrays; `manifest` is a JSON string):
  metadata/<name>/{offsets,indices,offsets_t,indices_t,block_offsets,row_indices}
  gemm/<name>/{a,b,c[,a_mask]}  small op(A) op(B) problems, inputs already
                                 rounded to fp16 values, c = oracle output.
"""

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import oracle as O  # noqa: E402
from sputnik_amd import matrix_utils as mu  # noqa: E402


def main():
    arrays = {}
    manifest = {"metadata": [], "gemm": []}

    def meta_case(name, off, idx, block_cols):
        off = np.asarray(off, np.int32)
        idx = np.asarray(idx, np.int32)
        ot, it, bo = O.transpose(off, idx, block_cols)
        p = f"metadata/{name}"
        arrays[p + "/offsets"] = off
        arrays[p + "/indices"] = idx
        arrays[p + "/offsets_t"] = ot
        arrays[p + "/indices_t"] = it
        arrays[p + "/block_offsets"] = bo
        arrays[p + "/row_indices"] = O.row_indices(off)
        manifest["metadata"].append({"name": p, "block_cols": block_cols,
                                     "block_rows": len(off) - 1})

    # recorded from the reference's own Transpose.
    meta_case("survey_kat", [0, 2, 5, 6], [1, 3, 2, 0, 3, 1], 4)
    rng = np.random.default_rng(20261015)
    for R, C, nb, unordered in [(4, 4, 7, False), (8, 6, 20, True),
                                (32, 32, 512, False), (16, 40, 130, True),
                                (5, 3, 0, False), (1, 9, 9, True)]:
        off, idx = mu.random_topology(R, C, nb, rng, unordered)
        meta_case(f"r{R}c{C}n{nb}{'u' if unordered else ''}", off, idx, C)
    off, idx = mu.expert_block_diagonal(2, 2, 3)
    meta_case("moe_2x2x3", off, idx, 6)

    def gemm_case(name, m, k, n, ta, tb, nb=None):
        a_mask = None
        if nb is None:
            a = O.round_to(mu.random_values((k, m) if ta else (m, k), rng), "f16")
        else:
            rows, cols = (k, m) if ta else (m, k)
            off, idx = mu.random_topology(rows // 128, cols // 128, nb, rng)
            vals = O.round_to(mu.random_values((nb, 128, 128), rng), "f16")
            a = mu.to_dense(rows, cols, off, idx, vals)
            mask = mu.block_mask(off, idx, cols // 128)
            a_mask = mask.T.copy() if ta else mask
        b = O.round_to(mu.random_values((n, k) if tb else (k, n), rng), "f16")
        c = O.gemm(a, ta, b, tb, a_mask=a_mask)
        p = f"gemm/{name}"
        arrays[p + "/a"] = a
        arrays[p + "/b"] = b
        arrays[p + "/c"] = c
        if a_mask is not None:
            arrays[p + "/a_mask"] = a_mask
        manifest["gemm"].append({"name": p, "m": m, "k": k, "n": n,
                                 "ta": bool(ta), "tb": bool(tb)})

    gemm_case("dense_nn_16x24x8", 16, 24, 8, False, False)
    gemm_case("dense_tt_8x40x16", 8, 40, 16, True, True)
    gemm_case("dsd_nn_256x256x8_half", 256, 256, 8, False, False, nb=2)
    gemm_case("dsd_tn_256x128x16", 256, 128, 16, True, False, nb=1)

    arrays["manifest"] = np.array(json.dumps(manifest))
    out = os.path.join(HERE, "golden_vectors.npz")
    np.savez_compressed(out, **arrays)
    print("wrote", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main()
