"""Single-workgroup update path for small networks (csrc/tiny.hip) vs the multi-launch path and the
oracle.

ppo_update takes the tiny path by itself when every layer is ≤ 128 wide, the output ≤ 32 and the
minibatch fits in LDS (configs C1/C2); PPO_NO_TINY=1 forces the multi-launch path.  From identical
state both paths must produce the same minibatch gradients (stated fp32 GEMM tolerance), the same
Adam step counts, and — over a whole update — the same losses and parameter motion; the host
rand() stream must be consumed identically (checked through a following draw).
"""
import ctypes as C
import os

import numpy as np
import pytest

import ppo_ffi
from helpers import F32, assert_gemm_close, nn_grads_packed, nn_params_packed

pytestmark = pytest.mark.gpu

LIBC = C.CDLL("libc.so.6")


def run(lib, oracle, sizes, N, B, n_pol, n_val, shuffle, tiny, seed=21):
    if tiny:
        os.environ.pop("PPO_NO_TINY", None)
    else:
        os.environ["PPO_NO_TINY"] = "1"
    try:
        LIBC.srand(seed)
        acts = ["relu"] * (len(sizes) - 2) + ["none"]
        ppo = lib.create_ppo(ppo_ffi.c_strings(acts), ppo_ffi.c_ints(sizes), len(sizes), N, 3e-4, 3e-4, 0.95, 0.2,
                             0.01, 1.0, True)
        E = max(1, N // 256)
        lib.ppo_fill_synthetic(ppo, E, N // E, 17, 1.0 / 200)
        v0 = nn_params_packed(lib, ppo.contents.V)
        mu0 = nn_params_packed(lib, ppo.contents.policy.contents.mu)
        lib.ppo_reset_stats(ppo)
        LIBC.srand(seed + 1)
        lib.ppo_update(ppo, 0.99, B, n_pol, n_val, shuffle, 9)
        stats = (C.c_double * 7)()
        lib.ppo_read_stats(ppo, stats, 7)
        pol = ppo.contents.policy.contents
        out = dict(stats=np.array(stats[:4]), next_rand=LIBC.rand(),
                   v=nn_params_packed(lib, ppo.contents.V), gv=nn_grads_packed(lib, ppo.contents.V),
                   mu=nn_params_packed(lib, pol.mu), gmu=nn_grads_packed(lib, pol.mu),
                   dv=nn_params_packed(lib, ppo.contents.V) - v0, dmu=nn_params_packed(lib, pol.mu) - mu0,
                   ls=ppo_ffi.d2h(lib, pol.d_log_std, F32, pol.action_size),
                   t=(ppo.contents.adam_V.contents.time_step, ppo.contents.adam_policy.contents.time_step,
                      ppo.contents.adam_entropy.contents.time_step))
        lib.free_ppo(ppo)
        return out
    finally:
        os.environ.pop("PPO_NO_TINY", None)


@pytest.mark.parametrize("shuffle", [0, 1])
@pytest.mark.parametrize("sizes", [[3, 64, 64, 1], [3, 128, 128, 1], [8, 32, 32, 32, 4]])
def test_tiny_single_steps_match_multilaunch(lib, oracle, sizes, shuffle):
    """one value step, then one policy step: identical gradients and Adam deltas"""
    N, B = 256, 64
    for n_pol, n_val in ((0, 1), (1, 0)):
        a = run(lib, oracle, sizes, N, B, n_pol, n_val, shuffle, tiny=True)
        b = run(lib, oracle, sizes, N, B, n_pol, n_val, shuffle, tiny=False)
        assert a["t"] == b["t"]
        assert a["next_rand"] == b["next_rand"], "host rand() stream consumed differently"
        np.testing.assert_allclose(a["stats"], b["stats"], rtol=2e-4, atol=1e-6)
        # the last step's gradients (grads buffers hold the last minibatch)
        assert_gemm_close(a["gv"], b["gv"], B, "value grads")
        assert_gemm_close(a["gmu"], b["gmu"], B, "policy grads")
        lr = 3e-4
        for k in ("v", "mu", "ls"):
            err = np.abs(a[k] - b[k])
            assert err.max() <= 2 * lr * 1.0001 + 1e-7, (k, err.max())
            assert (err > 1e-6).mean() < 0.01, (k, (err > 1e-6).mean())


@pytest.mark.parametrize("shuffle", [0, 1])
def test_tiny_full_update_c2(lib, oracle, shuffle):
    """a whole C2-shaped update (10 value + 4 policy epochs of 64-row minibatches) on both paths"""
    sizes, N, B = [3, 64, 64, 1], 4096, 64
    a = run(lib, oracle, sizes, N, B, 4, 10, shuffle, tiny=True)
    b = run(lib, oracle, sizes, N, B, 4, 10, shuffle, tiny=False)
    assert a["t"] == b["t"] == (640, 256, 256)
    assert a["next_rand"] == b["next_rand"]
    assert a["stats"][1] == b["stats"][1] == 640 and a["stats"][3] == b["stats"][3] == 256
    assert abs(a["stats"][0] - b["stats"][0]) <= 0.02 * abs(b["stats"][0])
    assert abs(a["stats"][2] - b["stats"][2]) <= 0.05 * abs(b["stats"][2]) + 1e-3
    for k in ("dv", "dmu"):
        cos = float(a[k] @ b[k] / (np.linalg.norm(a[k]) * np.linalg.norm(b[k])))
        assert cos > 0.95, (k, cos)
        assert abs(np.linalg.norm(a[k]) / np.linalg.norm(b[k]) - 1) < 0.1, k


@pytest.mark.parametrize("shuffle", [0, 1])
def test_tiny_c2_kernel_matches_generic(lib, oracle, shuffle, monkeypatch):
    """The compile-time C2 kernel (tiny_c2_kernel: padded LDS weight image, VALU output layer) against the
    generic single-workgroup kernel (PPO_TINY_GENERIC=1): one value and one policy step (the same
    gradients within the fp32 GEMM tolerance, Adam deltas within two steps' worth), then 16 + 16 steps."""
    sizes, N, B = [3, 64, 64, 1], 1024, 64
    for n_pol, n_val in ((0, 1), (1, 0), (1, 4)):
        monkeypatch.delenv("PPO_TINY_GENERIC", raising=False)
        a = run(lib, oracle, sizes, N, B, n_pol, n_val, shuffle, tiny=True)
        monkeypatch.setenv("PPO_TINY_GENERIC", "1")
        b = run(lib, oracle, sizes, N, B, n_pol, n_val, shuffle, tiny=True)
        monkeypatch.delenv("PPO_TINY_GENERIC", raising=False)
        assert a["t"] == b["t"] and a["next_rand"] == b["next_rand"]
        if n_val == 4:                                   # 64 + 16 steps: the trajectories stay together
            np.testing.assert_allclose(a["stats"], b["stats"], rtol=2e-2, atol=1e-6)
            for k in ("dv", "dmu"):
                cos = float(a[k] @ b[k] / (np.linalg.norm(a[k]) * np.linalg.norm(b[k])))
                assert cos > 0.99, (k, cos)
            continue
        np.testing.assert_allclose(a["stats"], b["stats"], rtol=2e-4, atol=1e-6)
        assert_gemm_close(a["gv"], b["gv"], B, "value grads")
        assert_gemm_close(a["gmu"], b["gmu"], B, "policy grads")
        lr = 3e-4
        for k in ("v", "mu", "ls"):
            err = np.abs(a[k] - b[k])
            assert err.max() <= 2 * lr * 1.0001 + 1e-7, (k, err.max())
