"""The value network's output layer + MSE head folded into its last hidden layer's x3 kernels
(host/neural_network.c nn_value_fold_step, csrc/gemm_x3.hip FOLD variants, kernels.hip value_head_kernel)
against the fused output-head pass it replaces (PPO_VALUE_FOLD=0: csrc/out_head.hip), from identical state.
The head (y, g, loss, output bias gradient) rides on the hidden layer's grad_W launch, or runs as its own
kernel where that launch has no LDS room for its split's g (the head_fallback case).

Reference semantics: the output layer y = h·w + b (mat_mul.cu:122-163), the MSE loss and its gradient
g = 2(y − t)/m (loss.cu:5-23), the output layer's backward gW = gᵀ·h, gb = Σ g, ∂L/∂h = g·w (mat_mul.cu:
165-217), masked by the last hidden layer's ReLU′ (activation_function.cu:24-29), then that layer's backward.
The fold never forms ∂L/∂h: the hidden layer's grad_x / grad_W take the 0/1 mask of h as their operand with
g and w as row / column scales — the same products in another fp32 order, so every value gradient and the
network output agree within the stated GEMM tolerance, the loss within reduction rounding.  Production C4 /
C3 value steps against the oracle run through the fold by default (test_gpu_production.py).
"""
import ctypes as C

import numpy as np
import pytest

import ppo_ffi
from helpers import F32, assert_gemm_close, nn_grads_packed, nn_params_packed

pytestmark = pytest.mark.gpu

LIBC = C.CDLL("libc.so.6")
CASES = {
    # name: (policy layer sizes, N, B) — the value network is sizes[:-1] + [1]
    "c4": ([376, 512, 512, 512, 17], 32768, 32768),       # 256×256 forward / grad_x tiles, grad_W split-K atomics
    "shard8": ([376, 512, 512, 512, 17], 4096, 4096),     # 64×64 tiles, grad_W slabs + reduce
    "c3": ([17, 256, 256, 6], 8192, 8192),                 # width 256: 64×64 tiles
    "ragged": ([376, 512, 512, 512, 17], 5000, 2500),     # partial row tiles
    "one_hidden": ([64, 256, 6], 2048, 2048),             # the folded layer is layer 0 (the fused gather)
    # 8192-row grad_W splits: the split's g does not fit beside the LDS ring, so value_head_kernel runs
    # first instead of the head carried by grad_W (gemm_x3.hip launch_x3)
    "head_fallback": ([376, 512, 512, 512, 17], 131072, 131072),
}


def value_step(lib, sizes, N, B, fold, monkeypatch, seed=31):
    monkeypatch.setenv("PPO_VALUE_FOLD", "1" if fold else "0")
    LIBC.srand(seed)
    acts = ["relu"] * (len(sizes) - 2) + ["none"]
    ppo = lib.create_ppo(ppo_ffi.c_strings(acts), ppo_ffi.c_ints(sizes), len(sizes), N, 3e-4, 3e-4, 0.95, 0.2, 0.0,
                         1.0, True)
    E = 16 if N % 16 == 0 else 8
    lib.ppo_fill_synthetic(ppo, E, N // E, 5, 1.0 / 200)
    lib.ppo_set_step_limit(ppo, 1, 0)
    lib.ppo_reset_stats(ppo)
    v0 = nn_params_packed(lib, ppo.contents.V)
    lib.ppo_update(ppo, 0.99, B, 0, 1, 1, 11)
    lib.ppo_synchronize()
    assert lib.ppo_last_error() in (b"", None), lib.ppo_last_error()
    st = (C.c_double * 4)()
    lib.ppo_read_stats(ppo, st, 4)
    V = ppo.contents.V.contents
    out = dict(g=nn_grads_packed(lib, ppo.contents.V), v=nn_params_packed(lib, ppo.contents.V), v0=v0,
               y=ppo_ffi.d2h(lib, V.d_output, F32, B), loss=st[0], steps=st[1])
    lib.ppo_set_step_limit(ppo, -1, -1)
    lib.free_ppo(ppo)
    return out


@pytest.mark.parametrize("case", sorted(CASES))
def test_value_fold_matches_out_head(lib, case, monkeypatch):
    sizes, N, B = CASES[case]
    a = value_step(lib, sizes, N, B, True, monkeypatch)
    b = value_step(lib, sizes, N, B, False, monkeypatch)
    assert a["steps"] == b["steps"] == 1
    np.testing.assert_array_equal(a["v0"], b["v0"])
    assert_gemm_close(a["y"], b["y"], sizes[-2], f"{case}: value output y (fold vs out_head)")
    assert_gemm_close(a["g"], b["g"], B, f"{case}: value gradients (fold vs out_head)")
    np.testing.assert_allclose(a["loss"], b["loss"], rtol=1e-5)
    # the Adam step that followed: same gradients in, element-wise within 2·lr, almost all far closer
    err = np.abs(a["v"] - b["v"])
    assert err.max() <= 2 * 3e-4 * 1.0001, err.max()
    assert (err > 1e-6).mean() < 0.01, (err > 1e-6).mean()
    print(f"{case}: fold vs out_head max |Δgrad| {np.abs(a['g'] - b['g']).max():.3g} "
          f"(max |grad| {np.abs(b['g']).max():.3g}), max |Δy| {np.abs(a['y'] - b['y']).max():.3g}")
