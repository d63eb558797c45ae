#!/usr/bin/env python3
"""Diagnostic (GPU, not collected by pytest): element-wise accuracy of one C4-shaped value or policy
minibatch gradient, x3 engine vs exact fp32 MFMA engine vs the oracle's OpenBLAS sgemm, each against
a float64 evaluation of the same forward/backward with the GPU's ReLU′ masks.

    python tests/diag_grad_accuracy.py [B]
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.join(HERE, "..", "ppo.c_amd"), os.path.join(HERE, "..", "oracle")]
import ppo_ffi  # noqa: E402
import oracle_ffi as oracle  # noqa: E402
from helpers import F32, gpu_relu_masks, nn_grads_packed, nn_params_packed  # noqa: E402

C4 = [376, 512, 512, 512, 17]
SV = C4[:-1] + [1]
RELU = [1, 1, 1, 0]


def f64_grads(sizes, params, x, gout, masks):
    """float64 forward/backward of the MLP with fixed ReLU′ masks; packed [W0, b0, ...] gradients."""
    Ws, bs, off = [], [], 0
    for i in range(len(sizes) - 1):
        n, l = sizes[i], sizes[i + 1]
        Ws.append(params[off:off + n * l].reshape(l, n).astype(np.float64)); off += n * l
        bs.append(params[off:off + l].astype(np.float64)); off += l
    acts = [x.astype(np.float64)]
    for i in range(len(Ws)):
        y = acts[-1] @ Ws[i].T + bs[i]
        if i < len(Ws) - 1:
            y = np.where(masks[i], y, 0.0)
        acts.append(y)
    g = gout.astype(np.float64)
    out = []
    for i in reversed(range(len(Ws))):
        out.append((bs[i] * 0 + g.sum(0), g.T @ acts[i]))
        if i > 0:
            g = (g @ Ws[i]) * masks[i - 1]
    packed = []
    for gb, gW in reversed(out):
        packed += [gW.ravel(), gb]
    return np.concatenate(packed), acts[-1]


def stats(name, g, ref):
    err = np.abs(g.astype(np.float64) - ref)
    scale = np.abs(ref)
    rel = err / np.maximum(scale, 1e-30)
    big = scale > 1e-3 * scale.max()
    print(f"{name:10s} max|err|/max|g| {err.max() / scale.max():.3g}  rms err {np.sqrt((err ** 2).mean()):.3g}  "
          f"median rel {np.median(rel):.3g}  rel>1e-4: {100 * (rel > 1e-4).mean():.2f} %  "
          f"rel>1e-4 among |g|>1e-3·max: {100 * (rel[big] > 1e-4).mean():.3f} %  sign flips {int((np.sign(g) != np.sign(ref)).sum())}",
          flush=True)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    lib = ppo_ffi.load()
    lib.ppo_set_device(0)
    E, T = max(8, B // 1024), 1024                  # a buffer of at least one minibatch
    N = E * T
    res = {}
    for engine in (1, 0):
        lib.ppo_gemm_f32_engine(engine)
        oracle.srand(99)
        ppo = lib.create_ppo(ppo_ffi.c_strings(["relu"] * 3 + ["none"]), ppo_ffi.c_ints(C4), 5, N, 3e-4, 3e-4, 0.95,
                             0.2, 0.0, 0.7, True)
        lib.ppo_fill_synthetic(ppo, E, T, 5, 1.0 / 500)
        v0 = nn_params_packed(lib, ppo.contents.V)
        lib.ppo_set_step_limit(ppo, 1, 0)
        lib.ppo_update(ppo, 0.99, B, 0, 1, 1, 77)
        lib.ppo_synchronize()
        gV = nn_grads_packed(lib, ppo.contents.V)
        b = ppo.contents.buffer.contents
        rows = oracle.feistel_perm(N, oracle.splitmix64(77))[:B]
        x = ppo_ffi.d2h(lib, b.d_state_p, F32, N * 376).reshape(N, 376)[rows]
        tgt = ppo_ffi.d2h(lib, b.d_adv_target_p, F32, N)[rows]
        masks = gpu_relu_masks(lib, ppo.contents.V, x)
        res[engine] = (gV, x, tgt, masks, v0)
        lib.free_ppo(ppo)
    gx3, x, tgt, masks, v0 = res[1]
    gex, x_e, tgt_e, masks_e, v0_e = res[0]
    assert np.array_equal(x, x_e) and np.array_equal(v0, v0_e)
    # the targets come from each engine's own GAE forward (they differ by fp32 rounding)
    print(f"targets x3 vs exact: max |diff| {np.abs(tgt - tgt_e).max():.3g} (max |t| {np.abs(tgt).max():.3g})")

    def ref_for(t, mk):
        _, y64 = f64_grads(SV, v0, x, np.zeros((B, 1)), mk)
        go = 2.0 * (y64.ravel() - t.astype(np.float64)) / B
        return f64_grads(SV, v0, x, go.reshape(-1, 1), mk)[0]
    ref, ref_e = ref_for(tgt, masks), ref_for(tgt_e, masks_e)
    print(f"C4 value network, one minibatch B = {B}: gradients vs float64 (same masks, same targets)")
    stats("x3", gx3, ref)
    stats("exact", gex, ref_e)
    acts = oracle.mlp_forward(SV, RELU, v0, x)
    y = oracle.mlp_layer_outputs(SV, acts, B)[-1].ravel()
    _, g = oracle.mse(y, tgt)
    stats("oracle", oracle.mlp_backward(SV, RELU, v0, x, acts, g.reshape(-1, 1)), ref)
    for name, ly in (("layer-2 W", slice(376 * 512 + 512 + 512 * 512 + 512, 376 * 512 + 512 + 2 * (512 * 512 + 512) - 512)),):
        stats("x3 " + name, gx3[ly], ref[ly])
        stats("ex " + name, gex[ly], ref_e[ly])


if __name__ == "__main__":
    main()
