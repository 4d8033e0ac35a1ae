"""The torch op surface (sputnik_amd.ops: sdd / dsd / dds with autograd, the
MegaBlocks forward/backward set). GPU tests run every product on
libsputnik.so and compare forward values and all gradients with a plain
PyTorch fp32 reference of the same dense-masked computation; CPU tests cover
the host-side topology logic (construction checks, views, dense round trip)
without touching the library.

Tolerance: |x - ref| <= rtol*(|ref| + rms(ref)), rtol 1e-2 fp16 / 2e-2 bf16
(the north-star form, tests/helpers.py), ref = fp32 torch on the rounded
inputs.
"""

import numpy as np
import pytest
import torch

from sputnik_amd import matrix_utils as mu
from tests import helpers as H


def _topology(rb, cb, nb, seed):
    rng = np.random.default_rng(seed)
    return mu.random_topology(rb, cb, nb, rng)


def _mask(offsets, indices, cb):
    return mu.block_mask(offsets, indices, cb)


def _close(x, ref, dtype, what):
    H.assert_close(x.detach().float().cpu().numpy(),
                   ref.detach().float().cpu().numpy(), dtype,
                   what)


# ----------------------------------------------------------------- host ----

def test_sparse_matrix_host_logic():
    from sputnik_amd import ops
    off, idx = _topology(3, 2, 4, 0)
    data = torch.randn(4, 128, 128).half()
    s = ops.SparseMatrix((384, 256), data, torch.from_numpy(off),
                         torch.from_numpy(idx.astype(np.int16)))
    assert s.shape == (384, 256) and s.t().shape == (256, 384)
    assert s.t().t().shape == s.shape and s.t().is_transposed()
    assert s.t()._meta is s._meta          # views share one metadata cache
    dense = s.to_dense()
    ref = mu.to_dense(384, 256, off, idx, data.float().numpy())
    assert np.array_equal(dense.float().numpy(), ref)
    assert torch.equal(s.t().to_dense(), dense.t())
    back = ops.from_dense_mask(dense, _mask(off, idx, 2))
    assert torch.equal(back.data, data)
    assert np.array_equal(back.offsets.numpy(), off)
    assert np.array_equal(back.indices.numpy(), idx)
    with pytest.raises(ValueError):
        ops.SparseMatrix((100, 256), data, torch.from_numpy(off),
                         torch.from_numpy(idx.astype(np.int16)))
    with pytest.raises(TypeError):
        ops.SparseMatrix((384, 256), data, torch.from_numpy(off).long(),
                         torch.from_numpy(idx.astype(np.int16)))
    with pytest.raises(ValueError):
        ops.SparseMatrix((384, 256), data[:3], torch.from_numpy(off),
                         torch.from_numpy(idx.astype(np.int16)))


# ------------------------------------------------------------------ GPU ----

gpu = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import sputnik_amd as sp
    sp.lib()  # fail loudly if the native library is missing


def _sparse(rows, cols, density, dtype, seed):
    from sputnik_amd import ops
    rb, cb = rows // 128, cols // 128
    nb = max(1, int(round(rb * cb * density)))
    off, idx = _topology(rb, cb, nb, seed)
    g = torch.Generator(device="cuda").manual_seed(seed)
    data = (torch.rand(nb, 128, 128, generator=g, device="cuda") * 2 - 1).to(
        H.torch_dtype(dtype))
    return ops.SparseMatrix((rows, cols), data,
                            torch.from_numpy(off).cuda(),
                            torch.from_numpy(idx.astype(np.int16)).cuda())


def _dense(rows, cols, dtype, seed, transposed=False):
    g = torch.Generator(device="cuda").manual_seed(1000 + seed)
    shape = (cols, rows) if transposed else (rows, cols)
    x = (torch.rand(*shape, generator=g, device="cuda") * 2 - 1).to(
        H.torch_dtype(dtype))
    return x.t() if transposed else x


def _grads_ref(fn_ref, inputs, dout):
    """fp32 autograd on dense copies: returns (out, grads)."""
    leaves = [x.detach().float().requires_grad_(True) for x in inputs]
    out = fn_ref(*leaves)
    out.backward(dout.float())
    return out.detach(), [x.grad for x in leaves]


def _block_grad(sparse, dense_grad):
    """The blocks of a dense gradient at `sparse`'s stored topology."""
    from sputnik_amd import ops
    stored = sparse.t() if sparse.is_transposed() else sparse
    g = dense_grad.t() if sparse.is_transposed() else dense_grad
    mask = _mask(stored.offsets.cpu().numpy(), stored.indices.cpu().numpy(),
                 stored._meta.cols // 128)
    return ops.from_dense_mask(g.contiguous(), mask).data


@gpu
@pytest.mark.parametrize("dtype", ["f16", "bf16"])
@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
def test_dsd_forward_backward(dtype, ta, tb):
    _need_gpu()
    from sputnik_amd import ops
    M, K, N = 384, 512, 264
    a = _sparse(K, M, 0.4, dtype, 1).t() if ta else _sparse(M, K, 0.4, dtype, 1)
    b = _dense(K, N, dtype, 2, transposed=tb).requires_grad_(True)
    a.data.requires_grad_(True)
    out = ops.dsd(a, b)
    dout = _dense(M, N, dtype, 3)
    out.backward(dout)
    ref, (ga, gb) = _grads_ref(lambda x, y: x @ y, [a.to_dense(), b], dout)
    _close(out, ref, dtype, "dsd fwd")
    _close(b.grad, gb, dtype, "dsd dB")
    _close(a.data.grad, _block_grad(a, ga), dtype, "dsd dA")


@gpu
@pytest.mark.parametrize("dtype", ["f16", "bf16"])
@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
def test_dds_forward_backward(dtype, ta, tb):
    _need_gpu()
    from sputnik_amd import ops
    M, K, N = 264, 512, 384
    a = _dense(M, K, dtype, 4, transposed=ta).requires_grad_(True)
    b = _sparse(N, K, 0.4, dtype, 5).t() if tb else _sparse(K, N, 0.4, dtype, 5)
    b.data.requires_grad_(True)
    out = ops.dds(a, b)
    dout = _dense(M, N, dtype, 6)
    out.backward(dout)
    ref, (ga, gb) = _grads_ref(lambda x, y: x @ y, [a, b.to_dense()], dout)
    _close(out, ref, dtype, "dds fwd")
    _close(a.grad, ga, dtype, "dds dA")
    _close(b.data.grad, _block_grad(b, gb), dtype, "dds dB")


@gpu
@pytest.mark.parametrize("dtype", ["f16", "bf16"])
@pytest.mark.parametrize("transposed_topo", [False, True])
def test_sdd_forward_backward(dtype, transposed_topo):
    _need_gpu()
    from sputnik_amd import ops
    M, K, N = 384, 200, 512
    topo = (_sparse(N, M, 0.3, dtype, 7).t() if transposed_topo
            else _sparse(M, N, 0.3, dtype, 7))
    a = _dense(M, K, dtype, 8).requires_grad_(True)
    b = _dense(K, N, dtype, 9, transposed=True).requires_grad_(True)
    out = ops.sdd(a, b, topo)
    assert out.shape == (M, N) and out.is_transposed() == transposed_topo
    dblocks = (torch.rand_like(out.data, dtype=torch.float32) * 2 - 1).to(
        out.data.dtype)
    out.data.backward(dblocks)
    dout_dense = topo.with_data(dblocks).to_dense()
    ref, (ga, gb) = _grads_ref(lambda x, y: x @ y, [a, b], dout_dense)
    _close(out.data, _block_grad(topo, ref), dtype, "sdd fwd")
    _close(a.grad, ga, dtype, "sdd dA")
    _close(b.grad, gb, dtype, "sdd dB")


@gpu
def test_moe_mlp_forward_backward_bf16():
    """The MegaBlocks expert MLP: h = sdd(x, w1, topo); y = dsd(gelu(h), w2)
    on the expert-diagonal topology, forward and backward, vs fp32 torch."""
    _need_gpu()
    from sputnik_amd import ops
    experts, tok, d_model, ffn = 4, 256, 256, 384
    off, idx = mu.expert_block_diagonal(experts, tok // 128, ffn // 128)
    rows, cols = experts * tok, experts * ffn
    topo = ops.SparseMatrix(
        (rows, cols),
        torch.empty(len(idx), 128, 128, dtype=torch.bfloat16, device="cuda"),
        torch.from_numpy(off.astype(np.int32)).cuda(),
        torch.from_numpy(idx.astype(np.int16)).cuda())
    x = _dense(rows, d_model, "bf16", 10).requires_grad_(True)
    w1 = _dense(d_model, cols, "bf16", 11).requires_grad_(True)
    w2 = _dense(cols, d_model, "bf16", 12).requires_grad_(True)
    h = ops.sdd(x, w1, topo)
    y = ops.dsd(h.with_data(torch.nn.functional.gelu(h.data)), w2)
    dy = _dense(rows, d_model, "bf16", 13)
    y.backward(dy)
    mask = torch.from_numpy(np.kron(
        _mask(off, idx, cols // 128), np.ones((128, 128)))).cuda().float()

    def ref_fn(x_, w1_, w2_):
        return (torch.nn.functional.gelu(x_ @ w1_) * mask) @ w2_

    ref, (gx, gw1, gw2) = _grads_ref(ref_fn, [x, w1, w2], dy)
    _close(y, ref, "bf16", "moe y")
    _close(x.grad, gx, "bf16", "moe dx")
    _close(w1.grad, gw1, "bf16", "moe dw1")
    _close(w2.grad, gw2, "bf16", "moe dw2")
