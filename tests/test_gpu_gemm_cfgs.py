"""Every GEMM tile configuration of csrc/gemm.hip, forced one at a time, against the oracle.

The automatic tile picker only reaches some configurations at some shapes; tuning changes which
one runs where.  Here each configuration runs (a) the three linear-layer GEMMs of the reference
API (mat_mul_cuda, mat_mul_backwards_cuda; mat_mul.cu:132-217) on vector-path shapes (every
contiguous extent a multiple of 4) and odd shapes (guarded scalar path), and (b) a whole MLP
forward + backward through forward_propagation_cuda / backward_propagation_cuda
(neural_network.cu:74-161), which adds the fused bias + ReLU epilogue, the ReLU′ mask of grad_x,
the split-K grad_W with its bias-gradient row sums.  Tolerance: the stated fp32 GEMM bound
(helpers.gemm_tol).
"""
import numpy as np
import pytest

import ppo_ffi
from helpers import F32, assert_gemm_close, dev, empty, nn_grads_packed, nn_set_params_packed

pytestmark = pytest.mark.gpu

SHAPES = [(4096, 376, 512), (1000, 512, 256), (257, 64, 36), (513, 130, 67), (300, 17, 256)]


@pytest.fixture(scope="module")
def ncfg(lib):
    """the exact fp32-MFMA engine's configurations (the x3 engine has its own test: test_gpu_x3.py)"""
    n = lib.ppo_gemm_tune(-1, 0)
    old = lib.ppo_gemm_f32_engine(0)
    yield n
    lib.ppo_gemm_f32_engine(old)
    lib.ppo_gemm_tune(-1, 0)


def _rand(rng, shape, lo=-1.0, hi=1.0):
    return rng.uniform(lo, hi, shape).astype(F32)


@pytest.mark.parametrize("m,n,l", SHAPES)
def test_linear_every_cfg(lib, oracle, ncfg, m, n, l):
    rng = np.random.default_rng(m + 3 * n + 7 * l)
    x, W, b, g = _rand(rng, (m, n)), _rand(rng, (l, n), -0.2, 0.2), _rand(rng, l, -0.2, 0.2), _rand(rng, (m, l))
    dx, dW, db, dg = dev(lib, x), dev(lib, W), dev(lib, b), dev(lib, g)
    dy, dgx, dgW = empty(lib, m * l), empty(lib, m * n), empty(lib, l * n)
    y_ref = oracle.mat_mul(x, W, b)
    gx_ref, gW_ref = oracle.mat_mul_backwards(g, x, W)
    try:
        for c in range(ncfg):
            lib.ppo_gemm_tune(c, 0)
            lib.mat_mul_cuda(None, dy.ptr, dx.ptr, dW.ptr, db.ptr, m, n, l)
            lib.mat_mul_backwards_cuda(None, dgx.ptr, dgW.ptr, dg.ptr, dx.ptr, dW.ptr, m, n, l)
            assert_gemm_close(dy.to_numpy(F32, m * l).reshape(m, l), y_ref, n, f"cfg {c} forward")
            assert_gemm_close(dgx.to_numpy(F32, m * n).reshape(m, n), gx_ref, l, f"cfg {c} grad_x")
            assert_gemm_close(dgW.to_numpy(F32, l * n).reshape(l, n), gW_ref, m, f"cfg {c} grad_W")
    finally:
        lib.ppo_gemm_tune(-1, 0)


@pytest.mark.parametrize("sizes,m", [([376, 512, 512, 17], 2048), ([17, 256, 256, 6], 1000), ([3, 64, 64, 1], 64)])
def test_mlp_every_cfg(lib, oracle, ncfg, sizes, m):
    rng = np.random.default_rng(len(sizes) * 1000 + m)
    relu = [1] * (len(sizes) - 2) + [0]
    acts_names = ["relu"] * (len(sizes) - 2) + ["none"]
    nn = lib.create_neural_network(ppo_ffi.c_ints(sizes), ppo_ffi.c_strings(acts_names), len(sizes))
    nparams = oracle.mlp_num_params(sizes)
    params = (rng.uniform(-1, 1, nparams) * 0.1).astype(F32)
    nn_set_params_packed(lib, nn, params)
    x = _rand(rng, (m, sizes[0]))
    gout = _rand(rng, (m, sizes[-1]))
    acts = oracle.mlp_forward(sizes, relu, params, x)
    y_ref = oracle.mlp_layer_outputs(sizes, acts, m)[-1]
    g_ref = oracle.mlp_backward(sizes, relu, params, x, acts, gout)
    dx, dgo = dev(lib, x), dev(lib, gout)
    try:
        for c in range(ncfg):
            lib.ppo_gemm_tune(c, 0)
            lib.forward_propagation_cuda(nn, dx.ptr, m)
            y = ppo_ffi.d2h(lib, nn.contents.d_output, F32, m * sizes[-1]).reshape(m, sizes[-1])
            assert_gemm_close(y, y_ref, max(sizes), f"cfg {c} MLP forward")
            lib.backward_propagation_cuda(nn, dgo.ptr, m)
            assert_gemm_close(nn_grads_packed(lib, nn), g_ref, m, f"cfg {c} MLP grads")
    finally:
        lib.ppo_gemm_tune(-1, 0)
        lib.free_neural_network(nn)


def _mlp_grads_f64(sizes, params, x, gout):
    """float64 numpy forward/backward of the packed MLP ([W0, b0, W1, b1, …], W as [out, in])."""
    Ws, bs, off = [], [], 0
    for i in range(len(sizes) - 1):
        n_in, n_out = sizes[i], sizes[i + 1]
        Ws.append(params[off:off + n_in * n_out].astype(np.float64).reshape(n_out, n_in))
        off += n_in * n_out
        bs.append(params[off:off + n_out].astype(np.float64))
        off += n_out
    hs = [x.astype(np.float64)]
    for i in range(len(Ws)):
        y = hs[-1] @ Ws[i].T + bs[i]
        hs.append(np.maximum(y, 0) if i < len(Ws) - 1 else y)
    g, grads = gout.astype(np.float64), []
    for i in range(len(Ws) - 1, -1, -1):
        grads = [(g.T @ hs[i]).ravel(), g.sum(0)] + grads
        g = (g @ Ws[i]) * (hs[i] > 0) if i > 0 else g @ Ws[i]
    return np.concatenate(grads)


@pytest.mark.parametrize("sizes,m", [([376, 512, 512, 512, 17], 16384), ([64, 1024, 1024, 8], 8192)])
def test_mlp_paired_backward(lib, ncfg, sizes, m):
    """grad_W + grad_x of a layer as one launch (gemm_pair_kernel: hidden layers, and the 17-wide
    output layer) vs two launches (flag 4):
    grad_x identical bit for bit (same tiles, same k order), grad_W up to the split-K atomics'
    order; both within the GEMM bound of a float64 reference (up to ReLU-mask flips)."""
    rng = np.random.default_rng(m + len(sizes))
    nn = lib.create_neural_network(ppo_ffi.c_ints(sizes), ppo_ffi.c_strings(["relu"] * (len(sizes) - 2) + ["none"]),
                                   len(sizes))
    nparams = sum(sizes[i] * sizes[i + 1] + sizes[i + 1] for i in range(len(sizes) - 1))
    params = (rng.uniform(-1, 1, nparams) * 0.05).astype(F32)
    nn_set_params_packed(lib, nn, params)
    x, gout = _rand(rng, (m, sizes[0])), _rand(rng, (m, sizes[-1]))
    g_ref = _mlp_grads_f64(sizes, params, x, gout)
    dx, dgo = dev(lib, x), dev(lib, gout)
    out = {}
    try:
        for flags in (0, 4):
            lib.ppo_gemm_flags(flags)
            lib.forward_propagation_cuda(nn, dx.ptr, m)
            lib.backward_propagation_cuda(nn, dgo.ptr, m)
            gx = [ppo_ffi.d2h(lib, nn.contents.layers[i].d_grad_x, F32, m * sizes[i]) for i in range(1, len(sizes) - 1)]
            out[flags] = (nn_grads_packed(lib, nn), gx)
            # a pre-activation within fp32 rounding of 0 can take the other side of the ReLU than in
            # float64 (a mask flip moves a few gradient entries by O(|g|·|h|)), so the bound must hold
            # for all but a small fraction of entries here
            err = np.abs(out[flags][0] - g_ref)
            tol = 1e-4 * np.abs(g_ref).max() * max(1.0, np.sqrt(m / 1024))
            assert (err > tol).mean() < 1e-3, f"flags {flags}: {(err > tol).sum()} entries beyond {tol:.3g}"
    finally:
        lib.ppo_gemm_flags(0)
        lib.free_neural_network(nn)
    for a, b in zip(out[0][1], out[4][1]):          # every hidden layer's grad_x, output layer's included
        np.testing.assert_array_equal(a, b)
    np.testing.assert_allclose(out[0][0], out[4][0], rtol=1e-5, atol=1e-5 * np.abs(out[4][0]).max())


@pytest.mark.parametrize("sizes,m", [([376, 512, 512, 17], 64), ([376, 512, 512, 1], 200), ([17, 256, 256, 6], 64),
                                     ([1024, 1024, 17], 33)])
def test_mlp_small_batch_auto(lib, oracle, sizes, m):
    """The reference's minibatch size (B = 64) through the automatic kernel choice: the small-M
    kernels (32×32 blocks, K split over 8 waves) for the forward with its ReLU′ bits, grad_x with the
    mask, and grad_W over the whole batch with its bias-gradient sums — whole MLP against the oracle,
    both fp32 engines' automatic routes (x3 only serves m > 1024, so both run the exact kernels)."""
    rng = np.random.default_rng(sum(sizes) + m)
    relu = [1] * (len(sizes) - 2) + [0]
    names = ["relu"] * (len(sizes) - 2) + ["none"]
    nn = lib.create_neural_network(ppo_ffi.c_ints(sizes), ppo_ffi.c_strings(names), len(sizes))
    params = (rng.uniform(-1, 1, oracle.mlp_num_params(sizes)) * 0.1).astype(F32)
    nn_set_params_packed(lib, nn, params)
    x, gout = _rand(rng, (m, sizes[0])), _rand(rng, (m, sizes[-1]))
    acts = oracle.mlp_forward(sizes, relu, params, x)
    y_ref = oracle.mlp_layer_outputs(sizes, acts, m)[-1]
    g_ref = oracle.mlp_backward(sizes, relu, params, x, acts, gout)
    dx, dgo = dev(lib, x), dev(lib, gout)
    lib.ppo_gemm_tune(-1, 0)
    try:
        lib.forward_propagation_cuda(nn, dx.ptr, m)
        y = ppo_ffi.d2h(lib, nn.contents.d_output, F32, m * sizes[-1]).reshape(m, sizes[-1])
        assert_gemm_close(y, y_ref, max(sizes), "small-batch MLP forward")
        lib.backward_propagation_cuda(nn, dgo.ptr, m)
        assert_gemm_close(nn_grads_packed(lib, nn), g_ref, m, "small-batch MLP grads")
    finally:
        lib.free_neural_network(nn)
