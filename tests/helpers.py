"""Shared test helpers: operand construction on the device and the parity
criterion. The expected values always come from the CPU oracle
(oracle/oracle.py), never from the library under test."""

from __future__ import annotations

import json
import os

import numpy as np

from oracle import oracle as O
from sputnik_amd import matrix_utils as mu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")

# North-star tolerance (BASELINE.json): 1e-2 relative fp16, written as
#   |gpu - ref| <= RTOL*|ref| + RTOL*rms(ref)
# where ref is the oracle GEMM of the rounded (fp16/bf16) inputs. bf16 keeps
# 8 mantissa bits, so its RTOL is 2e-2.
RTOL = {"f16": 1e-2, "bf16": 2e-2}
# The reference's own criterion: absolute 5e-2 against the fp32 oracle of the
# un-rounded inputs (dsd_test.cu:192, NanSensitiveFloatNear(5e-2)).
REF_ABS_TOL = 5e-2


def oracle_threads() -> int:
    return max(1, min(16, os.cpu_count() or 1))


def load_problems(op: str):
    with open(os.path.join(GOLDEN, "reference_test_problems.json")) as f:
        return json.load(f)[op]


def assert_close(gpu: np.ndarray, ref: np.ndarray, dtype: str, what: str = ""):
    gpu = np.asarray(gpu, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    assert gpu.shape == ref.shape, (gpu.shape, ref.shape)
    assert np.isfinite(gpu).all(), f"{what}: non-finite output"
    rms = float(np.sqrt(np.mean(ref * ref))) if ref.size else 0.0
    tol = RTOL[dtype] * (np.abs(ref) + rms)
    bad = np.abs(gpu - ref) > tol
    if bad.any():
        idx = np.argwhere(bad)[:5]
        raise AssertionError(
            f"{what}: {int(bad.sum())}/{bad.size} elements out of tolerance; "
            f"first {idx.tolist()} gpu={gpu[tuple(idx[0])]} ref={ref[tuple(idx[0])]} "
            f"max|err|={np.abs(gpu-ref).max():.3e} rms(ref)={rms:.3e}")


def torch_dtype(dtype: str):
    import torch
    return torch.float16 if dtype == "f16" else torch.bfloat16


class HostSparse:
    """A BCSR operand: host float32 values (already rounded to the device
    type), topology, and the device BlockMatrix built from them."""

    def __init__(self, rows, cols, nonzeros, rng, dtype="f16",
                 unordered=False, device="cuda", topology=None):
        import torch
        import sputnik_amd as sp

        b = mu.BLOCK
        self.rows, self.cols, self.dtype = rows, cols, dtype
        nb = nonzeros // (b * b)
        if topology is None:
            self.offsets, self.indices = mu.random_topology(
                rows // b, cols // b, nb, rng, unordered=unordered)
        else:
            self.offsets, self.indices = topology
        self.values = O.round_to(mu.random_values((nb, b, b), rng), dtype)
        td = torch_dtype(dtype)
        self.dev_values = torch.from_numpy(self.values).to(td).to(device)
        self.matrix = sp.BlockMatrix(
            rows, cols, 128, nb * b * b, self.dev_values,
            torch.from_numpy(self.offsets.astype(np.int32)).to(device),
            torch.from_numpy(self.indices.astype(np.int16)).to(device))

    def dense(self) -> np.ndarray:
        return mu.to_dense(self.rows, self.cols, self.offsets, self.indices,
                           self.values)

    def mask(self) -> np.ndarray:
        return mu.block_mask(self.offsets, self.indices, self.cols // mu.BLOCK)


class HostDense:
    def __init__(self, rows, cols, rng, dtype="f16", device="cuda"):
        import torch
        import sputnik_amd as sp

        self.raw = mu.random_values((rows, cols), rng)
        self.values = O.round_to(self.raw, dtype)
        self.dev = torch.from_numpy(self.values).to(torch_dtype(dtype)).to(device)
        self.matrix = sp.Matrix(rows, cols, self.dev)


def empty_dense(rows, cols, dtype="f16", device="cuda", fill=float("nan")):
    import torch
    import sputnik_amd as sp
    t = torch.full((rows, cols), fill, dtype=torch_dtype(dtype), device=device)
    return sp.Matrix(rows, cols, t), t


# Linearity checksums (tests/test_gpu_configs.py config 4): row sums of a
# full-size output against exact float64 sums computed from the operands.
#
# Checksum tolerance: an output of p significant bits (bf16 8, fp16 11)
# carries a round-to-nearest error e per element with |e| <= 2^-p |y|, zero
# mean, variance <= (2^-p y)^2 / 3; a row sum of n of them is off from the
# exact sum by about 2^-p sqrt(sum y^2 / 3). The bound is 8 of those (the
# fp32 accumulation error is orders of magnitude smaller). One missing or
# wrong 128-long contribution (a dropped block, a wrong k-block) moves a row
# sum by 10-40x that bound at these shapes. The launches are deterministic,
# so the check cannot flake on a fixed seed.
_ROUND_U = {"bf16": 2.0 ** -8, "f16": 2.0 ** -11}


def rowsum_check(y, expect, axis, what, dtype="bf16"):
    """y: the output (bf16 / fp16) as float32; expect: exact float64 sums of
    y along `axis` computed from the operands."""
    assert np.isfinite(y).all(), f"{what}: non-finite output"
    got = y.sum(axis=axis, dtype=np.float64)
    sq = np.square(y, dtype=np.float64).sum(axis=axis)
    rms = float(np.sqrt(np.mean(expect * expect)))
    tol = 8 * _ROUND_U[dtype] * np.sqrt(sq / 3) + 1e-6 * rms
    err = np.abs(got - expect)
    bad = err > tol
    assert not bad.any(), (
        f"{what}: {int(bad.sum())}/{bad.size} row sums out of tolerance; "
        f"max err {err.max():.3e} (tol there {tol.flat[int(np.argmax(err))]:.3e}), "
        f"rms {rms:.3e}")
