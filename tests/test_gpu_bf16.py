"""bf16 compute mode (BASELINE config C5: "4×1024 MLP bf16") — csrc/gemm16.hip through the C ABI.

Two references:
  * a bf16-emulated one (numpy, float64 accumulation) that rounds exactly what the kernels round:
    layer inputs and the weight shadow to bf16 on the way into the MFMA, hidden activations and
    hidden gradients stored as bf16, the network output and the heads' gradient fp32, bias
    gradients summed from the bf16-rounded gradient.  Tolerance 2e-3·max|ref| (fp32 accumulation
    order only) — this pins the kernels;
  * the oracle (fp32 restatement of the reference CPU path): bf16 agrees within 3e-2·max|ref|
    (SURVEY §8c's bf16 bound) — this pins that bf16 mode still computes the reference's layers.
Every bf16 tile configuration is forced once.
"""
import numpy as np
import pytest

import ppo_ffi
from helpers import F32, dev, nn_grads_packed, nn_set_params_packed

pytestmark = pytest.mark.gpu


def bf16(a):
    """round-to-nearest-even to bf16, returned as float32 (NaN-free inputs)"""
    u = np.ascontiguousarray(a, F32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(F32)


def unpack(sizes, params):
    out, off = [], 0
    for i in range(len(sizes) - 1):
        nw = sizes[i] * sizes[i + 1]
        W = params[off:off + nw].reshape(sizes[i + 1], sizes[i])
        off += nw
        b = params[off:off + sizes[i + 1]]
        off += sizes[i + 1]
        out.append((W, b))
    return out


def emulate(sizes, params, x, gout):
    """bf16-mode forward + backward as the kernels compute it (float64 accumulation)."""
    layers = unpack(sizes, params)
    L = len(layers)
    hs = [bf16(x)]                                  # layer inputs as the MFMA sees them
    for i, (W, b) in enumerate(layers):
        z = hs[-1].astype(np.float64) @ bf16(W).astype(np.float64).T + b
        if i < L - 1:
            hs.append(bf16(np.maximum(z, 0.0).astype(F32)))
        else:
            y = z.astype(F32)
    grads = [None] * L
    g = gout.astype(F32)                            # fp32 from the heads, rounded in the loader
    for i in range(L - 1, -1, -1):
        W, _ = layers[i]
        gb16 = bf16(g).astype(np.float64)
        gW = gb16.T @ hs[i].astype(np.float64)
        gbias = gb16.sum(axis=0)
        grads[i] = (gW.astype(F32).ravel(), gbias.astype(F32))
        if i > 0:
            gx = gb16 @ bf16(W).astype(np.float64)
            gx = np.where(hs[i] > 0, gx, 0.0)
            g = bf16(gx.astype(F32))                # hidden gradients stored bf16
    packed = np.concatenate([np.concatenate([gw, gb]) for gw, gb in grads])
    return y, packed


def close(got, ref, rel, what):
    err = float(np.abs(got - ref).max())
    tol = rel * float(np.abs(ref).max()) + 1e-6
    assert err <= tol, f"{what}: max |err| {err:.3g} > {tol:.3g}"


@pytest.fixture(scope="module")
def ncfg16(lib):
    n = lib.ppo_gemm16_tune(-1)
    yield n
    lib.ppo_gemm16_tune(-1)


@pytest.mark.parametrize("sizes,m", [([1024, 1024, 1024, 17], 1024), ([376, 512, 512, 17], 2048),
                                     ([17, 256, 256, 6], 1000), ([3, 64, 64, 1], 64)])
def test_bf16_mlp_every_cfg(lib, oracle, ncfg16, sizes, m):
    rng = np.random.default_rng(sum(sizes) + m)
    relu = [1] * (len(sizes) - 2) + [0]
    names = ["relu"] * (len(sizes) - 2) + ["none"]
    nn = lib.create_neural_network(ppo_ffi.c_ints(sizes), ppo_ffi.c_strings(names), len(sizes))
    params = (rng.uniform(-1, 1, oracle.mlp_num_params(sizes)) * (1.0 / np.sqrt(max(sizes)))).astype(F32)
    nn_set_params_packed(lib, nn, params)
    assert lib.nn_set_compute_dtype(nn, 1) == 0
    x = rng.uniform(-1, 1, (m, sizes[0])).astype(F32)
    gout = rng.uniform(-1, 1, (m, sizes[-1])).astype(F32)
    y_emu, g_emu = emulate(sizes, params, x, gout)
    acts = oracle.mlp_forward(sizes, relu, params, x)
    y_ref = oracle.mlp_layer_outputs(sizes, acts, m)[-1]
    g_ref = oracle.mlp_backward(sizes, relu, params, x, acts, gout)
    dx, dgo = dev(lib, x), dev(lib, gout)
    try:
        for c in range(ncfg16):
            lib.ppo_gemm16_tune(c)
            lib.forward_propagation_cuda(nn, dx.ptr, m)
            y = ppo_ffi.d2h(lib, nn.contents.d_output, F32, m * sizes[-1]).reshape(m, sizes[-1])
            close(y, y_emu, 2e-3, f"cfg {c} forward vs bf16 emulation")
            close(y, y_ref, 3e-2, f"cfg {c} forward vs fp32 oracle")
            lib.backward_propagation_cuda(nn, dgo.ptr, m)
            g = nn_grads_packed(lib, nn)
            close(g, g_emu, 2e-3, f"cfg {c} grads vs bf16 emulation")
            close(g, g_ref, 3e-2, f"cfg {c} grads vs fp32 oracle")
    finally:
        lib.ppo_gemm16_tune(-1)
        lib.free_neural_network(nn)


def test_bf16_update_tracks_fp32(lib):
    """A whole C5-shaped PPO update in bf16 mode from the same state as fp32: value / policy losses agree
    within bf16 tolerance and the parameters move the same way."""
    sizes, T, E, B = [1024, 1024, 1024, 17], 512, 8, 1024
    N = T * E
    out = {}
    for dtype in (0, 1):
        ppo_ffi.C.CDLL("libc.so.6").srand(77)
        ppo = lib.create_ppo(ppo_ffi.c_strings(["relu", "relu", "none"]), ppo_ffi.c_ints(sizes), 4, N, 3e-4, 3e-4,
                             0.95, 0.2, 0.0, 1.0, True)
        assert lib.ppo_set_compute_dtype(ppo, dtype) == 0
        lib.ppo_fill_synthetic(ppo, E, T, 99, 1.0 / 500)
        p0 = ppo_ffi.d2h(lib, ppo.contents.V.contents.d_params, F32, ppo.contents.V.contents.num_params)
        lib.ppo_reset_stats(ppo)
        lib.ppo_update(ppo, 0.99, B, 1, 2, 1, 5)
        stats = (ppo_ffi.C.c_double * 7)()
        lib.ppo_read_stats(ppo, stats, 7)
        p1 = ppo_ffi.d2h(lib, ppo.contents.V.contents.d_params, F32, ppo.contents.V.contents.num_params)
        out[dtype] = (np.array(stats[:4]), p1 - p0)
        lib.free_ppo(ppo)
    (s32, d32), (s16, d16) = out[0], out[1]
    assert s32[1] == s16[1] and s32[3] == s16[3]
    assert abs(s16[0] - s32[0]) <= 0.03 * abs(s32[0]) + 1e-4, (s16, s32)
    assert abs(s16[2] - s32[2]) <= 0.05 * abs(s32[2]) + 1e-3, (s16, s32)
    cos = float(d16 @ d32 / (np.linalg.norm(d16) * np.linalg.norm(d32) + 1e-30))
    assert cos > 0.9, cos


def test_bf16_out_head_matches_separate(lib, monkeypatch):
    """bf16 mode's fused value head (out_head.hip with bf16 x / gx and the bf16 weight shadow; C5's
    1024-wide value network) against the separate bf16 launches (PPO_OUT_HEAD=0) from identical state:
    one value minibatch, value output, every value gradient and the loss sums within bf16 tolerance
    (the two paths round the same fp32 values to bf16; sums differ in order only)."""
    sizes, T, E = [1024, 1024, 1024, 17], 512, 8
    N = T * E
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("PPO_OUT_HEAD", mode)
        ppo_ffi.C.CDLL("libc.so.6").srand(78)
        ppo = lib.create_ppo(ppo_ffi.c_strings(["relu", "relu", "none"]), ppo_ffi.c_ints(sizes), 4, N, 3e-4, 3e-4,
                             0.95, 0.2, 0.0, 1.0, True)
        assert lib.ppo_set_compute_dtype(ppo, 1) == 0
        lib.ppo_fill_synthetic(ppo, E, T, 98, 1.0 / 500)
        lib.ppo_reset_stats(ppo)
        lib.ppo_update(ppo, 0.99, N, 1, 1, 1, 13)
        lib.ppo_synchronize()
        st = (ppo_ffi.C.c_double * 7)()
        lib.ppo_read_stats(ppo, st, 7)
        V = ppo.contents.V
        out[mode] = (nn_grads_packed(lib, V), ppo_ffi.d2h(lib, V.contents.d_output, F32, N), np.array(st[:4]))
        lib.free_ppo(ppo)
    (g0, y0, s0), (g1, y1, s1) = out["0"], out["1"]
    close(y1, y0, 1e-4, "value output (fused vs separate)")
    close(g1, g0, 2e-3, "value grads (fused vs separate)")
    np.testing.assert_allclose(s1, s0, rtol=1e-3, atol=1e-6)


@pytest.mark.parametrize("sizes,m", [([1024, 1024, 1024, 17], 2000), ([512, 512, 256, 1], 1100)])
def test_bf16_dma_matches_register_staged(lib, sizes, m):
    """The LDS-DMA kernel (gemm_bf16_dma_kernel: source-swizzled unpadded images) runs each
    output's MFMAs in the register-staged 256×256 kernel's order: forward outputs bitwise equal with
    it on and off, gradients equal up to grad_W's atomic arrival order (cfg 9 forced; M tails; bf16
    hidden layers)."""
    rng = np.random.default_rng(sum(sizes) + m)
    names = ["relu"] * (len(sizes) - 2) + ["none"]
    nn = lib.create_neural_network(ppo_ffi.c_ints(sizes), ppo_ffi.c_strings(names), len(sizes))
    params = (rng.uniform(-1, 1, sum(a * b + b for a, b in zip(sizes[:-1], sizes[1:]))) /
              np.sqrt(max(sizes))).astype(F32)
    nn_set_params_packed(lib, nn, params)
    assert lib.nn_set_compute_dtype(nn, 1) == 0
    dx = dev(lib, rng.uniform(-1, 1, (m, sizes[0])).astype(F32))
    dgo = dev(lib, rng.uniform(-1, 1, (m, sizes[-1])).astype(F32))
    out = {}
    old = lib.ppo_gemm16_dma(-1)
    try:
        lib.ppo_gemm16_tune(9)
        for on in (0, 1):
            lib.ppo_gemm16_dma(on)
            lib.forward_propagation_cuda(nn, dx.ptr, m)
            y = ppo_ffi.d2h(lib, nn.contents.d_output, F32, m * sizes[-1])
            lib.backward_propagation_cuda(nn, dgo.ptr, m)
            out[on] = (y, nn_grads_packed(lib, nn))
    finally:
        lib.ppo_gemm16_dma(old)
        lib.ppo_gemm16_tune(-1)
        lib.free_neural_network(nn)
    np.testing.assert_array_equal(out[1][0], out[0][0])
    # grad_W accumulates split-K partials with f32 atomics (arrival order varies run to run)
    close(out[1][1], out[0][1], 1e-5, "grads, DMA vs register-staged")


@pytest.mark.parametrize("sizes,m", [([1024, 1024, 1024, 1024, 17], 4096), ([1024, 1024, 1024, 17], 1024),
                                     ([384, 384, 512, 256, 1], 2048), ([1024, 1024, 1024, 17], 16384)])
def test_bf16_dma_tn_grad_w(lib, oracle, sizes, m):
    """grad_W on the LDS-DMA TN tile (gemm_bf16_dma_tn_kernel: both operands by hardware-transposed
    reads, split partials summed by the slab reduce, bias from the g image) — the automatic choice
    for bf16 g and x with l % 256 = 0, n % 128 = 0 (256 × 128 tiles by default, 256 × 256 selectable) — against the bf16
    emulation (2e-3·max|ref|, the file's bar, up to 2048 rows) and against the register-staged kernel (DMA off): the
    same rounded products, summed in another order (1e-4·max|ref|)."""
    rng = np.random.default_rng(sum(sizes) + m)
    names = ["relu"] * (len(sizes) - 2) + ["none"]
    nn = lib.create_neural_network(ppo_ffi.c_ints(sizes), ppo_ffi.c_strings(names), len(sizes))
    params = (rng.uniform(-1, 1, oracle.mlp_num_params(sizes)) * (1.0 / np.sqrt(max(sizes)))).astype(F32)
    nn_set_params_packed(lib, nn, params)
    assert lib.nn_set_compute_dtype(nn, 1) == 0
    x = rng.uniform(-1, 1, (m, sizes[0])).astype(F32)
    gout = rng.uniform(-1, 1, (m, sizes[-1])).astype(F32)
    _, g_emu = emulate(sizes, params, x, gout)
    dx, dgo = dev(lib, x), dev(lib, gout)
    out = {}
    old = lib.ppo_gemm16_dma(-1)
    old_w = lib.ppo_gemm16_tn_width(0)
    try:
        lib.ppo_gemm16_tune(-1)
        for on, width in ((1, 128), (1, 256), (0, 128)):         # both DMA tile widths, then DMA off
            lib.ppo_gemm16_dma(on)
            lib.ppo_gemm16_tn_width(width)
            lib.forward_propagation_cuda(nn, dx.ptr, m)
            lib.backward_propagation_cuda(nn, dgo.ptr, m)
            out[(on, width)] = nn_grads_packed(lib, nn)
    finally:
        lib.ppo_gemm16_dma(old)
        lib.ppo_gemm16_tn_width(old_w)
        lib.free_neural_network(nn)
    for width in (128, 256):
        if m <= 2048:  # deeper / longer: hidden bf16 rounding flips compound against the emulation
            close(out[(1, width)], g_emu, 2e-3, f"grads (DMA TN, {width}-wide) vs bf16 emulation")
        close(out[(1, width)], out[(0, 128)], 1e-4, f"grads, DMA TN {width}-wide vs register-staged")
