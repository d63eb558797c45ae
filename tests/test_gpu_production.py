"""Production-size parity for the bench configurations C2, C3 and C5 (C4's is in test_gpu_index.py).

Each config runs at the exact shape bench.py times, on the kernels the bench runs, against the
oracle (reference ppo.cu:391-447 per minibatch; mat_mul.cu:132-217 for every product):

* C2 (Pendulum 3 → 2×64 → 1, N = 4096, B = 64): the single-workgroup path (csrc/tiny.hip) that the
  C2 bench line runs — one value and one policy minibatch (gradients and Adam deltas vs the oracle),
  then the first 16 value and 16 policy steps element by element against the oracle's update;
* C3 (17 → 2×256 → 6, N = 4096×64 = 262,144, B = 8192): one value and one policy minibatch on the x3
  engine's production 64×64 / split-K grids and the fused output heads;
* C5 (1024 → 4×1024 → 17, bf16, N = 8192×64 = 524,288, B = 16384: the bench's per-GPU shard): one
  value and one policy minibatch — every bf16 kernel teacher-forced (each layer from the GPU's own
  stored bf16 input / gradient) against the bf16 rounding model at fp32 accumulation accuracy, the
  whole gradient against the fp32 oracle (3e-2·max|ref|, SURVEY §8c's bf16 bound), Adam on the
  gradient it read; the bf16 gathered layer-0 copy equals bf16(state[rows]) bit for bit.

GAE at every production size (round 4): the device GAE (V(state) forward over the whole buffer, the
V(next_state) reuse with its own-row forward, the scan, the Welford statistics and the normalisation)
against the oracle's GAE — the reference's two full V forwards (OpenBLAS, 16 threads) and its
recursion (ref_gae) — at C3 (N = 262,144), C4 (N = 1,048,576) and the C5 shard (N = 524,288; bf16 V:
the scan teacher-forced on the GPU's own V values, V itself within the bf16 bound).  The step tests
of C3 and C4 then take their targets and advantages from the ORACLE's GAE, so no link of the fp32
production chain compares the GPU with its own output (C5's bf16 steps are compared given the
advantages they trained on, which test_c5_bf16_gae pins).

Inputs are bench.py's own: ppo_fill_synthetic (seeded device generator) after create_ppo from srand.
"""
import hashlib
import ctypes as C

import numpy as np
import pytest

import ppo_ffi
from helpers import (F32, assert_gemm_close, assert_normalised_close, assert_rel_close, gpu_relu_masks,
                     nn_grads_packed, nn_input_rows, nn_params_packed, oracle_grads_with_masks)
from test_gpu_bf16 import bf16, unpack
from test_gpu_update import adam_first_step, assert_adam_delta, make_ppo, policy_state

pytestmark = pytest.mark.gpu

RELU = lambda sizes: [1] * (len(sizes) - 2) + [0]  # noqa: E731
LR = 3e-4


def device_buffer(lib, ppo, N, S, A):
    """The device rollout as the oracle's buffer dict (whole arrays)."""
    b = ppo.contents.buffer.contents
    return dict(state=ppo_ffi.d2h(lib, b.d_state_p, F32, N * S).reshape(N, S),
                next_state=ppo_ffi.d2h(lib, b.d_next_state_p, F32, N * S).reshape(N, S),
                action=ppo_ffi.d2h(lib, b.d_action_p, F32, N * A).reshape(N, A),
                reward=ppo_ffi.d2h(lib, b.d_reward_p, F32, N),
                logprob=ppo_ffi.d2h(lib, b.d_logprob_p, F32, N),
                terminated=ppo_ffi.d2h(lib, b.d_terminated_p, np.uint8, N),
                truncated=ppo_ffi.d2h(lib, b.d_truncated_p, np.uint8, N))


_GAE_CACHE = {}


def oracle_gae(lib, oracle, ppo, sizes, N):
    """The oracle's GAE over the device buffer with the network's CURRENT V parameters (reference
    compute_gae, ppo.cu:326-369: V over every next_state and state row, then the recursion):
    (normalised advantages, targets), cached per (buffer, V parameters)."""
    v0 = nn_params_packed(lib, ppo.contents.V)
    b = ppo.contents.buffer.contents
    key = (ctypes_addr(b.d_state_p), N, hashlib.sha1(v0.tobytes()).hexdigest())
    if key not in _GAE_CACHE:
        _GAE_CACHE.clear()
        buf = device_buffer(lib, ppo, N, sizes[0], sizes[-1])
        A = sizes[-1]
        ref = oracle.ppo_update(sizes, RELU(sizes), np.zeros(oracle.mlp_num_params(sizes), F32), np.zeros(A, F32), v0,
                                buf, batch_size=1, n_epochs_policy=0, n_epochs_value=0, max_value_steps=0,
                                max_policy_steps=0)
        _GAE_CACHE[key] = (ref["advantage"], ref["adv_target"], ref["adv_mean"], ref["adv_std"])
    return _GAE_CACHE[key]


def ctypes_addr(p):
    return C.cast(p, C.c_void_p).value


def gpu_gae(lib, ppo, N):
    """Run the device GAE alone (ppo_update capped at zero minibatch steps) and read its outputs."""
    lib.ppo_set_step_limit(ppo, 0, 0)
    lib.ppo_update(ppo, 0.99, 64, 0, 0, 1, 1)
    lib.ppo_synchronize()
    b = ppo.contents.buffer.contents
    return ppo_ffi.d2h(lib, b.d_advantage_p, F32, N), ppo_ffi.d2h(lib, b.d_adv_target_p, F32, N)


def assert_gae_pinned(lib, oracle, ppo, sizes, N, what):
    """Device GAE vs the oracle's: targets 1e-5 relative + 1e-5·max|target|, normalised advantages
    1e-4 relative + 1e-4 absolute of the exact statistics (helpers.assert_normalised_close)."""
    adv_ref, tgt_ref, mean_ref, std_ref = oracle_gae(lib, oracle, ppo, sizes, N)
    adv, tgt = gpu_gae(lib, ppo, N)
    e_t = np.abs(tgt.astype(np.float64) - tgt_ref)
    e_a = np.abs(adv.astype(np.float64) - adv_ref)
    print(f"{what}: targets max err {e_t.max():.3g} (max|t| {np.abs(tgt_ref).max():.3g}), "
          f"advantages max err {e_a.max():.3g}")
    assert_rel_close(tgt, tgt_ref, 1e-5, 1e-5 * float(np.abs(tgt_ref).max()), f"{what} adv_target")
    assert_normalised_close(adv, adv_ref, mean_ref, std_ref, f"{what} normalised advantage")


def bench_ppo(lib, oracle, sizes, E, T, seed, dtype=0):
    ppo = make_ppo(lib, oracle, sizes, E * T, seed=seed)
    assert lib.ppo_set_compute_dtype(ppo, dtype) == 0
    lib.ppo_fill_synthetic(ppo, E, T, seed, 1.0 / 500)
    lib.ppo_synchronize()
    return ppo


def ref_value_grads(oracle, sv, v0, x, tgt, masks, what):
    acts = oracle.mlp_forward(sv, RELU(sv), v0, x)
    y = oracle.mlp_layer_outputs(sv, acts, x.shape[0])[-1].ravel()
    _, g = oracle.mse(y, tgt)
    return oracle_grads_with_masks(oracle, sv, RELU(sv), v0, x, g.reshape(-1, 1), masks, what, max_flips=256)


def ref_policy_grads(oracle, sizes, mu0, ls0, x, a, adv, old, masks, what, ent_coeff=0.0):
    acts = oracle.mlp_forward(sizes, RELU(sizes), mu0, x)
    mu = oracle.mlp_layer_outputs(sizes, acts, x.shape[0])[-1]
    lp = oracle.log_prob(mu, ls0, a)
    _, glp, gent = oracle.policy_loss_and_grad(adv, lp, old, oracle.entropy(ls0), ent_coeff, 0.2)
    gmu_out, gls = oracle.log_prob_backwards(mu, ls0, a, glp)
    g, _ = oracle_grads_with_masks(oracle, sizes, RELU(sizes), mu0, x, gmu_out, masks, what, max_flips=256)
    return g, gls + gent


# ----------------------------------------------------------------------------- C2: the tiny path
C2 = [3, 64, 64, 1]


@pytest.fixture(scope="module")
def c2_state(lib, oracle):
    oracle.load(use_openblas=True)
    ppo = bench_ppo(lib, oracle, C2, 1, 4096, seed=2024)
    mu0, ls0 = policy_state(lib, ppo)
    v0 = nn_params_packed(lib, ppo.contents.V)
    buf = device_buffer(lib, ppo, 4096, 3, 1)
    lib.free_ppo(ppo)
    return mu0, ls0, v0, buf


def _c2_run(lib, oracle, n_val_steps, n_pol_steps, seed):
    """A fresh C2 PPO from the fixture's seed: GAE + the first n value / policy steps on the tiny path."""
    ppo = bench_ppo(lib, oracle, C2, 1, 4096, seed=2024)
    lib.ppo_set_step_limit(ppo, n_val_steps, n_pol_steps)
    lib.ppo_reset_stats(ppo)
    lib.ppo_update(ppo, 0.99, 64, 1, 1, 1, seed)
    lib.ppo_synchronize()
    # the tiny path leaves no multi-launch forward behind (the last bits / d_x0 are GAE's, m = N)
    assert ppo.contents.V.contents.bits_m != 64, "C2 did not take the single-workgroup path"
    return ppo


def test_c2_tiny_single_steps_vs_oracle(lib, oracle, c2_state):
    """One value and one policy minibatch (B = 64) of the C2 bench update on the tiny path vs the oracle."""
    mu0, ls0, v0, buf = c2_state
    N, B, seed = 4096, 64, 515
    ppo = _c2_run(lib, oracle, 1, 1, seed)
    pol = ppo.contents.policy.contents
    gV, v1 = nn_grads_packed(lib, ppo.contents.V), nn_params_packed(lib, ppo.contents.V)
    gmu, mu1 = nn_grads_packed(lib, pol.mu), nn_params_packed(lib, pol.mu)
    gls = ppo_ffi.d2h(lib, pol.d_log_std_grad, F32, 1)
    b = ppo.contents.buffer.contents
    tgt_all = ppo_ffi.d2h(lib, b.d_adv_target_p, F32, N)
    adv_all = ppo_ffi.d2h(lib, b.d_advantage_p, F32, N)
    st = (C.c_double * 7)()
    lib.ppo_read_stats(ppo, st, 7)
    lib.free_ppo(ppo)
    ref = oracle.ppo_update(C2, RELU(C2), mu0, ls0, v0, buf, batch_size=B, n_epochs_policy=1, n_epochs_value=1,
                            shuffle_mode=1, seed=seed, max_value_steps=1, max_policy_steps=1)
    assert st[1] == ref["n_v"] == 1 and st[3] == ref["n_p"] == 1
    assert_rel_close(tgt_all, ref["adv_target"], 2e-4, 2e-4 * np.abs(ref["adv_target"]).max(), "C2 adv_target")
    assert_rel_close(adv_all, ref["advantage"], 2e-3, 2e-3, "C2 advantage")
    key = oracle.splitmix64(seed)
    rows_v = oracle.feistel_perm(N, key)[:B]
    rows_p = oracle.feistel_perm(N, (key + 1) & (2**64 - 1))[:B]
    sv = C2[:-1] + [1]
    g_ref, _ = ref_value_grads(oracle, sv, v0, buf["state"][rows_v], ref["adv_target"][rows_v], None, "C2 value")
    assert_gemm_close(gV, g_ref, B, "C2 value grads (tiny)")
    flips = assert_adam_delta(v1, ref["v"], g_ref, LR, "C2 value params")
    assert flips <= 2
    g_ref, gls_ref = ref_policy_grads(oracle, C2, mu0, ls0, buf["state"][rows_p], buf["action"][rows_p],
                                      ref["advantage"][rows_p], buf["logprob"][rows_p], None, "C2 policy")
    assert_gemm_close(gmu, g_ref, B, "C2 policy grads (tiny)")
    assert_rel_close(gls, gls_ref, 1e-3, 1e-5 * max(1.0, float(np.abs(gls_ref).max())), "C2 log_std grad")
    flips = assert_adam_delta(mu1, ref["mu"], g_ref, LR, "C2 policy params")
    assert flips <= 2


def test_c2_tiny_first_steps_elementwise(lib, oracle, c2_state):
    """The first 16 value and 16 policy steps of the C2 bench update (tiny path) against the oracle's
    update of the same buffer, element by element (bounds of test_short_update_elementwise)."""
    mu0, ls0, v0, buf = c2_state
    B, seed, n = 64, 616, 16
    ppo = _c2_run(lib, oracle, n, n, seed)
    mu1, ls1 = policy_state(lib, ppo)
    v1 = nn_params_packed(lib, ppo.contents.V)
    st = (C.c_double * 7)()
    lib.ppo_read_stats(ppo, st, 7)
    t = (ppo.contents.adam_V.contents.time_step, ppo.contents.adam_policy.contents.time_step,
         ppo.contents.adam_entropy.contents.time_step)
    lib.free_ppo(ppo)
    ref = oracle.ppo_update(C2, RELU(C2), mu0, ls0, v0, buf, batch_size=B, n_epochs_policy=1, n_epochs_value=1,
                            shuffle_mode=1, seed=seed, max_value_steps=n, max_policy_steps=n)
    assert t == (ref["t_v"], ref["t_mu"], ref["t_ent"]) == (n, n, n)
    assert st[1] == ref["n_v"] == n and st[3] == ref["n_p"] == n
    for got, want, what in ((v1, ref["v"], "V"), (mu1, ref["mu"], "mu"), (ls1, ref["log_std"], "log_std")):
        err = np.abs(got.astype(np.float64) - want)
        q = float((err <= 0.1 * LR).mean())
        print(f"C2 {what}: max err {err.max() / LR:.4f} lr, {100 * q:.3f} % within 0.1 lr")
        assert err.max() <= 2 * LR * n, f"{what}: max err {err.max()}"
        assert q >= 0.99, f"{what}: only {q * 100:.2f} % within 0.1·lr"
    np.testing.assert_allclose(st[0], ref["sum_v_loss"], rtol=1e-3)
    np.testing.assert_allclose(st[2], ref["sum_policy_loss"], rtol=1e-3, atol=1e-5)


# ----------------------------------------------------------------------------- C3: x3 production grids
C3 = [17, 256, 256, 6]


@pytest.fixture(scope="module")
def c3(lib, oracle):
    oracle.load(use_openblas=True)
    oracle.load().ref_blas_threads(16)
    ppo = bench_ppo(lib, oracle, C3, 64, 4096, seed=3131)
    yield ppo, 64 * 4096
    lib.ppo_set_step_limit(ppo, -1, -1)
    lib.free_ppo(ppo)


def _gathered(lib, nn_ptr, B, S):
    nn = nn_ptr.contents
    assert nn.bits_m == B and nn.x0_dtype == 0
    return nn_input_rows(lib, nn_ptr, B)


def test_c3_gae_vs_oracle(lib, oracle, c3):
    """C3's device GAE (N = 262,144: x3 V forward, V(next_state) reuse, scan, statistics) vs the oracle."""
    ppo, N = c3
    assert_gae_pinned(lib, oracle, ppo, C3, N, "C3 GAE")


def test_c3_timed_policy_step(lib, oracle, c3):
    """One policy minibatch of the C3 bench update (A = 6 fused clipped-surrogate head) vs the oracle."""
    ppo, N = c3
    B, seed, A = 8192, 93, 6
    pol = ppo.contents.policy.contents
    mu0 = nn_params_packed(lib, pol.mu)
    ls0 = ppo_ffi.d2h(lib, pol.d_log_std, F32, A)
    adv_all, _, _, _ = oracle_gae(lib, oracle, ppo, C3, N)
    lib.ppo_set_step_limit(ppo, 0, 1)
    lib.ppo_update(ppo, 0.99, B, 1, 0, 1, seed)
    lib.ppo_synchronize()
    gmu, mu1 = nn_grads_packed(lib, pol.mu), nn_params_packed(lib, pol.mu)
    gls = ppo_ffi.d2h(lib, pol.d_log_std_grad, F32, A)
    b = ppo.contents.buffer.contents
    rows = oracle.feistel_perm(N, oracle.splitmix64(seed))[:B]
    x = ppo_ffi.d2h(lib, b.d_state_p, F32, N * 17).reshape(N, 17)[rows]
    np.testing.assert_array_equal(_gathered(lib, pol.mu, B, 17), x)
    a = ppo_ffi.d2h(lib, b.d_action_p, F32, N * A).reshape(N, A)[rows]
    adv = adv_all[rows]                                         # the oracle's normalised advantages
    old = ppo_ffi.d2h(lib, b.d_logprob_p, F32, N)[rows]
    g_ref, gls_ref = ref_policy_grads(oracle, C3, mu0, ls0, x, a, adv, old, gpu_relu_masks(lib, pol.mu, x),
                                      "C3 policy")
    assert_gemm_close(gmu, g_ref, B, "C3 policy grads")
    assert_rel_close(gls, gls_ref, 1e-3, 1e-4 * max(1.0, float(np.abs(gls_ref).max())), "C3 log_std grad")
    flips = assert_adam_delta(mu1, adam_first_step(mu0, g_ref, LR), g_ref, LR, "C3 policy params")
    assert flips <= mu1.size // 1000


def test_c3_timed_value_step(lib, oracle, c3):
    """One value minibatch of the C3 bench update (N = 262,144, B = 8192, x3 grids, fused head) vs the oracle."""
    ppo, N = c3
    B, seed = 8192, 71
    assert lib.ppo_gemm_f32_engine(-1) == 1
    v0 = nn_params_packed(lib, ppo.contents.V)
    _, tgt_all, _, _ = oracle_gae(lib, oracle, ppo, C3, N)
    lib.ppo_set_step_limit(ppo, 1, 0)
    lib.ppo_update(ppo, 0.99, B, 0, 1, 1, seed)
    lib.ppo_synchronize()
    gV, v1 = nn_grads_packed(lib, ppo.contents.V), nn_params_packed(lib, ppo.contents.V)
    b = ppo.contents.buffer.contents
    rows = oracle.feistel_perm(N, oracle.splitmix64(seed))[:B]
    x = ppo_ffi.d2h(lib, b.d_state_p, F32, N * 17).reshape(N, 17)[rows]
    np.testing.assert_array_equal(_gathered(lib, ppo.contents.V, B, 17), x)
    tgt = tgt_all[rows]                                         # the oracle's GAE targets
    sv = C3[:-1] + [1]
    g_ref, _ = ref_value_grads(oracle, sv, v0, x, tgt, gpu_relu_masks(lib, ppo.contents.V, x), "C3 value")
    assert_gemm_close(gV, g_ref, B, "C3 value grads")
    flips = assert_adam_delta(v1, adam_first_step(v0, g_ref, LR), g_ref, LR, "C3 value params")
    assert flips <= v1.size // 1000


# ----------------------------------------------------------------------------- C4: the headline bench update
C4 = [376, 512, 512, 512, 17]


@pytest.fixture(scope="module")
def c4(lib, oracle):
    oracle.load(use_openblas=True)
    oracle.load().ref_blas_threads(16)
    ppo = bench_ppo(lib, oracle, C4, 256, 4096, seed=4141)
    yield ppo, 256 * 4096
    lib.ppo_set_step_limit(ppo, -1, -1)
    lib.free_ppo(ppo)


def test_c4_gae_vs_oracle(lib, oracle, c4):
    """The bench's C4 GAE at N = 1,048,576 (the V(state) forward over the whole buffer, the 2,368-row
    own V(next_state) forward, 512 scan workgroups and their carries, the Welford combine) vs the
    oracle's two full V forwards and recursion."""
    ppo, N = c4
    assert_gae_pinned(lib, oracle, ppo, C4, N, "C4 GAE")
    st = (C.c_double * 8)()
    lib.ppo_read_stats(ppo, st, 8)
    assert 0 < st[7] < N // 100                    # the reuse ran: only episode ends got their own forward


def test_c4_timed_policy_step(lib, oracle, c4):
    """One policy minibatch of the C4 bench update (A = 17: the policy head fused with the output
    layer's one-pass backward, out_head.hip) vs the oracle."""
    ppo, N = c4
    B, seed, A, S = 32768, 97, 17, 376
    pol = ppo.contents.policy.contents
    mu0 = nn_params_packed(lib, pol.mu)
    ls0 = ppo_ffi.d2h(lib, pol.d_log_std, F32, A)
    adv_all, _, _, _ = oracle_gae(lib, oracle, ppo, C4, N)
    lib.ppo_set_step_limit(ppo, 0, 1)
    lib.ppo_update(ppo, 0.99, B, 1, 0, 1, seed)
    lib.ppo_synchronize()
    gmu, mu1 = nn_grads_packed(lib, pol.mu), nn_params_packed(lib, pol.mu)
    gls = ppo_ffi.d2h(lib, pol.d_log_std_grad, F32, A)
    b = ppo.contents.buffer.contents
    rows = oracle.feistel_perm(N, oracle.splitmix64(seed))[:B]
    x = _gathered(lib, pol.mu, B, S)
    a = ppo_ffi.d2h(lib, b.d_action_p, F32, N * A).reshape(N, A)[rows]
    adv = adv_all[rows]                                         # the oracle's normalised advantages
    old = ppo_ffi.d2h(lib, b.d_logprob_p, F32, N)[rows]
    g_ref, gls_ref = ref_policy_grads(oracle, C4, mu0, ls0, x, a, adv, old, gpu_relu_masks(lib, pol.mu, x),
                                      "C4 policy")
    assert_gemm_close(gmu, g_ref, B, "C4 policy grads")
    assert_rel_close(gls, gls_ref, 1e-3, 1e-4 * max(1.0, float(np.abs(gls_ref).max())), "C4 log_std grad")
    flips = assert_adam_delta(mu1, adam_first_step(mu0, g_ref, LR), g_ref, LR, "C4 policy params")
    assert flips <= mu1.size // 1000


def test_c4_timed_value_step(lib, oracle, c4):
    """One value minibatch of the C4 bench update (N = 1,048,576, B = 32768: x3 grids with slab
    split-K, the fused value head) vs the oracle."""
    ppo, N = c4
    B, seed, S = 32768, 73, 376
    assert lib.ppo_gemm_f32_engine(-1) == 1
    v0 = nn_params_packed(lib, ppo.contents.V)
    _, tgt_all, _, _ = oracle_gae(lib, oracle, ppo, C4, N)
    lib.ppo_set_step_limit(ppo, 1, 0)
    lib.ppo_update(ppo, 0.99, B, 0, 1, 1, seed)
    lib.ppo_synchronize()
    gV, v1 = nn_grads_packed(lib, ppo.contents.V), nn_params_packed(lib, ppo.contents.V)
    b = ppo.contents.buffer.contents
    rows = oracle.feistel_perm(N, oracle.splitmix64(seed))[:B]
    x = _gathered(lib, ppo.contents.V, B, S)
    np.testing.assert_array_equal(x[:64], ppo_ffi.d2h(lib, b.d_state_p, F32, N * S).reshape(N, S)[rows[:64]])
    tgt = tgt_all[rows]                                         # the oracle's GAE targets
    sv = C4[:-1] + [1]
    g_ref, _ = ref_value_grads(oracle, sv, v0, x, tgt, gpu_relu_masks(lib, ppo.contents.V, x), "C4 value")
    assert_gemm_close(gV, g_ref, B, "C4 value grads")
    flips = assert_adam_delta(v1, adam_first_step(v0, g_ref, LR), g_ref, LR, "C4 value params")
    assert flips <= v1.size // 1000


# ----------------------------------------------------------------------------- C5: bf16 at the bench shard
C5 = [1024, 1024, 1024, 1024, 1024, 17]
ULP = 2.0 ** -8          # bf16 round-to-nearest: relative error ≤ 2^-8 (8 significant bits)


def emu_forward(sizes, params, x):
    """bf16-mode forward as the kernels compute it, end to end (float64 accumulation)."""
    layers = unpack(sizes, params)
    hs = [bf16(x)]
    for i, (W, b) in enumerate(layers):
        z = hs[-1].astype(np.float64) @ bf16(W).astype(np.float64).T + b
        if i < len(layers) - 1:
            hs.append(bf16(np.maximum(z, 0.0).astype(F32)))
        else:
            y = z.astype(F32)
    return hs, y


def emu_backward(sizes, params, hs, gout):
    layers = unpack(sizes, params)
    grads = [None] * len(layers)
    g = gout.astype(F32)
    for i in range(len(layers) - 1, -1, -1):
        W, _ = layers[i]
        gb16 = bf16(g).astype(np.float64)
        grads[i] = ((gb16.T @ hs[i].astype(np.float64)).astype(F32).ravel(), gb16.sum(axis=0).astype(F32))
        if i > 0:
            gx = np.where(hs[i] > 0, gb16 @ bf16(W).astype(np.float64), 0.0)
            g = bf16(gx.astype(F32))
    return np.concatenate([np.concatenate([gw, gb]) for gw, gb in grads])


def close(got, ref, rel, what):
    err = float(np.abs(got - ref).max())
    tol = rel * float(np.abs(ref).max()) + 1e-6
    assert err <= tol, f"{what}: max |err| {err:.3g} > {tol:.3g}"


def _bf16_dev(lib, ptr, rows, width):
    u = ppo_ffi.d2h(lib, ptr, np.uint16, rows * width).reshape(rows, width)
    return (u.astype(np.uint32) << 16).view(F32)


def assert_bf16_rounding(got, want, sum_abs, what):
    """got (bf16 storage) is the bf16 rounding of an fp32 accumulation of want (float64): within half
    a bf16 ulp of want, plus the fp32 accumulation bound 2^-15·Σ|terms| (sum_abs)."""
    tol = ULP * np.abs(want) + 2.0 ** -15 * sum_abs + 1e-12
    bad = np.abs(got - want) > tol
    assert not bad.any(), f"{what}: {int(bad.sum())} elements off by more than a bf16 rounding, worst " \
                          f"{float(np.abs(got - want)[bad].max()):.3g}"


def check_bf16_layers(lib, nn_ptr, sizes, params, x, gtop, top_rounded, what):
    """Teacher-forced check of every bf16 kernel of one minibatch, at production size: each layer's
    forward from the GPU's own bf16 input activation, each layer's grad_W / bias sums / grad_x from the
    GPU's own stored bf16 gradient (layers[i+1].d_grad_x) — so a bf16 rounding-boundary flip upstream
    (inherent to bf16 storage: the flip rate compounds with depth, ≈ 7e-3 of the last hidden layer's
    elements at C5) does not propagate into the comparison, and every kernel is pinned to fp32
    accumulation accuracy.  top_rounded: the output layer's gradient enters its products rounded to
    bf16 (both the separate bf16 launches and the fused bf16 value head, out_head.hip, round it as
    they stage it)."""
    nn = nn_ptr.contents
    L, B = len(sizes) - 1, x.shape[0]
    layers = unpack(sizes, params)
    hs = [bf16(x)] + [_bf16_dev(lib, nn.layers[i].d_input, B, sizes[i]) for i in range(1, L)]
    for i in range(L - 1):                                  # hidden layers: bf16(relu(x·Wᵀ + b))
        W, b = layers[i]
        z = hs[i].astype(np.float64) @ bf16(W).astype(np.float64).T + b
        sa = np.abs(hs[i]).astype(np.float64) @ np.abs(bf16(W)).astype(np.float64).T + np.abs(b)
        assert_bf16_rounding(hs[i + 1], np.maximum(z, 0.0), sa, f"{what} forward layer {i}")
    W, b = layers[L - 1]
    y = ppo_ffi.d2h(lib, nn.d_output, F32, B * sizes[L]).reshape(B, sizes[L])
    z = hs[L - 1].astype(np.float64) @ bf16(W).astype(np.float64).T + b
    close(y, z, 1e-5, f"{what} output layer (fp32 out)")
    grads = nn_grads_packed(lib, nn_ptr)
    off = 0
    for i in range(L):
        W, b = layers[i]
        nw = W.size
        if i == L - 1:
            g = (bf16(gtop) if top_rounded else gtop).astype(np.float64)
        else:
            g = _bf16_dev(lib, nn.layers[i + 1].d_grad_x, B, sizes[i + 1]).astype(np.float64)
        gW = g.T @ hs[i].astype(np.float64)
        # fp32 sums over B = 16384 rows (split-K partials, wave-level chains, f32 atomics): bounded by
        # the fp32 summation error of those terms, c·Σ|g·h| with c = 2^-15 (≈ 256 chained additions
        # of unit roundoff 2^-24 — the chains the kernels use are shorter), not by max|gW|: the
        # MSE / surrogate gradients change sign row to row, so |Σ g·h| ≪ Σ|g·h|
        c = 2.0 ** -15
        sum_abs = np.abs(g).T @ np.abs(hs[i]).astype(np.float64)
        err = np.abs(grads[off:off + nw].reshape(W.shape) - gW)
        assert (err <= c * sum_abs + 1e-9).all(), f"{what} grad_W layer {i}: worst err / Σ|g·h| " \
            f"{float((err / np.maximum(sum_abs, 1e-30)).max()):.3g}"
        errb = np.abs(grads[off + nw:off + nw + b.size] - g.sum(axis=0))
        assert (errb <= c * np.abs(g).sum(axis=0) + 1e-9).all(), f"{what} bias grad layer {i}"
        off += nw + b.size
        if i > 0:
            gx = np.where(hs[i] > 0, g @ bf16(W).astype(np.float64), 0.0)
            sa = np.abs(g) @ np.abs(bf16(W)).astype(np.float64)
            assert_bf16_rounding(_bf16_dev(lib, nn.layers[i].d_grad_x, B, sizes[i]), gx, sa,
                                 f"{what} grad_x layer {i}")
    return grads


@pytest.fixture(scope="module")
def c5(lib, oracle):
    oracle.load(use_openblas=True)
    oracle.load().ref_blas_threads(16)
    ppo = bench_ppo(lib, oracle, C5, 64, 8192, seed=5151, dtype=1)
    N = 64 * 8192
    b = ppo.contents.buffer.contents
    state = ppo_ffi.d2h(lib, b.d_state_p, F32, N * 1024).reshape(N, 1024)
    yield ppo, N, state
    lib.ppo_set_step_limit(ppo, -1, -1)
    lib.free_ppo(ppo)


def _gathered_bf16(lib, nn_ptr, B, S):
    assert nn_ptr.contents.x0_dtype == 1
    return _bf16_dev(lib, nn_ptr.contents.d_x0, B, S)


def test_c5_bf16_gae(lib, oracle, c5):
    """The C5 shard's GAE (N = 524,288) in bf16 mode: V runs on the bf16 GEMMs, so (1) the scan,
    statistics and normalisation are pinned on the GPU's own V(state) / V(next_state) values
    (ppo_gae_state) against ref_gae at the fp32 tolerances, and (2) V itself against the oracle's fp32
    forward within the bf16 bound 3e-2·max|V|, the targets / advantages likewise."""
    ppo, N, _ = c5
    adv, tgt = gpu_gae(lib, ppo, N)
    w = np.zeros(6)
    v, vn = np.empty(N, F32), np.empty(N, F32)
    assert lib.ppo_gae_state(w.ctypes.data, v.ctypes.data, vn.ctypes.data, N) == N
    b = ppo.contents.buffer.contents
    r = ppo_ffi.d2h(lib, b.d_reward_p, F32, N)
    term = ppo_ffi.d2h(lib, b.d_terminated_p, np.uint8, N)
    trunc = ppo_ffi.d2h(lib, b.d_truncated_p, np.uint8, N)
    adv_tf, tgt_tf, mean_tf, std_tf = oracle.gae(v, vn, r, term, trunc, 0.99, 0.95)
    assert_rel_close(tgt, tgt_tf, 1e-5, 1e-5 * float(np.abs(tgt_tf).max()), "C5 targets (scan on the GPU's V)")
    assert_normalised_close(adv, adv_tf, mean_tf, std_tf, "C5 advantages (scan on the GPU's V)")
    raw = tgt_tf.astype(np.float64) - v                             # the exact statistics of the scan's A
    assert w[0] == N and abs(w[1] - raw.mean()) <= 1e-5 * raw.std()
    assert abs(np.sqrt(w[2] / w[0]) - raw.std()) <= 1e-5 * raw.std()
    sv, m = C5[:-1] + [1], 32768                                 # V on the first 32768 rows, fp32 oracle
    x = ppo_ffi.d2h(lib, b.d_state_p, F32, m * 1024).reshape(m, 1024)
    v0 = nn_params_packed(lib, ppo.contents.V)
    v_ref = oracle.mlp_layer_outputs(sv, oracle.mlp_forward(sv, RELU(sv), v0, x), m)[-1].ravel()
    print(f"C5 bf16 V vs fp32 oracle: max err {np.abs(v[:m] - v_ref).max():.3g} (max|V| {np.abs(v_ref).max():.3g})")
    close(v[:m], v_ref, 3e-2, "C5 V(state) vs fp32 oracle")
    adv_ref, tgt_ref, _, _ = oracle_gae(lib, oracle, ppo, C5, N)
    for got, ref, what in ((tgt, tgt_ref, "targets"), (adv, adv_ref, "advantages")):
        err = float(np.abs(got.astype(np.float64) - ref).max())
        print(f"C5 bf16 GAE {what} vs fp32 oracle: max err {err:.3g} (max|ref| {np.abs(ref).max():.3g})")
        close(got, ref, 3e-2, f"C5 {what} vs fp32 oracle")


def test_c5_bf16_timed_policy_step(lib, oracle, c5):
    """One bf16 policy minibatch at the bench's C5 shard (A = 17 clipped surrogate, separate launches)."""
    ppo, N, state = c5
    B, seed, A = 16384, 59, 17
    pol = ppo.contents.policy.contents
    mu0 = nn_params_packed(lib, pol.mu)
    ls0 = ppo_ffi.d2h(lib, pol.d_log_std, F32, A)
    lib.ppo_set_step_limit(ppo, 0, 1)
    lib.ppo_update(ppo, 0.99, B, 1, 0, 1, seed)
    lib.ppo_synchronize()
    mu1 = nn_params_packed(lib, pol.mu)
    gls = ppo_ffi.d2h(lib, pol.d_log_std_grad, F32, A)
    b = ppo.contents.buffer.contents
    rows = oracle.feistel_perm(N, oracle.splitmix64(seed))[:B]
    x = state[rows]
    np.testing.assert_array_equal(_gathered_bf16(lib, pol.mu, B, 1024), bf16(x))
    a = ppo_ffi.d2h(lib, b.d_action_p, F32, N * A).reshape(N, A)[rows]
    adv = ppo_ffi.d2h(lib, b.d_advantage_p, F32, N)[rows]
    old = ppo_ffi.d2h(lib, b.d_logprob_p, F32, N)[rows]
    # the head (fp32) on the GPU's own network output
    y = ppo_ffi.d2h(lib, pol.mu.contents.d_output, F32, B * A).reshape(B, A)
    lp = oracle.log_prob(y, ls0, a)
    _, glp, gent = oracle.policy_loss_and_grad(adv, lp, old, oracle.entropy(ls0), 0.0, 0.2)
    gtop, gls_head = oracle.log_prob_backwards(y, ls0, a, glp)
    assert_rel_close(gls, gls_head + gent, 1e-3, 1e-4 * max(1.0, float(np.abs(gls_head).max())), "C5 log_std grad")
    gmu = check_bf16_layers(lib, pol.mu, C5, mu0, x, gtop, True, "C5 policy")
    # the GPU's advantages: in bf16 mode the GAE's V forward is bf16 too, so the fp32 oracle's advantages
    # differ by the bf16 bound (test_c5_bf16_gae pins them: V against the fp32 oracle, the scan on the
    # GPU's own V at the fp32 tolerances) — the step is compared given the advantages it trained on
    g_ref, gls_ref = ref_policy_grads(oracle, C5, mu0, ls0, x, a, adv, old, None, "C5 policy")
    close(gmu, g_ref, 3e-2, "C5 policy grads vs fp32 oracle")
    # ∂L/∂logσ_a = Σ_rows (−1 + z²)·∂L/∂lp with z = (a − μ)/σ: a sum of 16384 terms that cancel
    # (|Σ| ≪ Σ|terms|), each moved by the bf16 network's μ (≈ 2^-8 relative) — bounded by 3e-2·max|ref|
    # plus 2^-7·Σ|terms| per action dimension (the terms from the fp32 oracle's forward)
    mu_ref = oracle.mlp_layer_outputs(C5, oracle.mlp_forward(C5, RELU(C5), mu0, x), B)[-1]
    _, glp_ref, _ = oracle.policy_loss_and_grad(adv, oracle.log_prob(mu_ref, ls0, a), old, oracle.entropy(ls0), 0.0,
                                                0.2)
    z = (a.astype(np.float64) - mu_ref) * np.exp(-ls0.astype(np.float64))
    sum_abs = (np.abs(-1.0 + z * z) * np.abs(glp_ref.astype(np.float64))[:, None]).sum(axis=0)
    err = np.abs(gls.astype(np.float64) - gls_ref)
    tol = 3e-2 * float(np.abs(gls_ref).max()) + 2.0 ** -7 * sum_abs
    print(f"C5 log_std grad vs fp32 oracle: max err {err.max():.3g}, worst err/tol {float((err / tol).max()):.3f}")
    assert (err <= tol).all(), "C5 log_std grad vs fp32 oracle"
    flips = assert_adam_delta(mu1, adam_first_step(mu0, gmu, LR), gmu, LR, "C5 policy params")
    assert flips <= mu1.size // 1000
def test_c5_bf16_timed_value_step(lib, oracle, c5):
    """One bf16 value minibatch at the bench's C5 shard (N = 524,288, B = 16384, fused bf16 value head):
    every kernel teacher-forced against the bf16 rounding model, the whole gradient against the fp32
    oracle (3e-2·max|ref|), Adam on the gradient it read."""
    ppo, N, state = c5
    B, seed = 16384, 57
    V = ppo.contents.V
    v0 = nn_params_packed(lib, V)
    lib.ppo_set_step_limit(ppo, 1, 0)
    lib.ppo_update(ppo, 0.99, B, 0, 1, 1, seed)
    lib.ppo_synchronize()
    v1 = nn_params_packed(lib, V)
    b = ppo.contents.buffer.contents
    rows = oracle.feistel_perm(N, oracle.splitmix64(seed))[:B]
    x = state[rows]
    np.testing.assert_array_equal(_gathered_bf16(lib, V, B, 1024), bf16(x))      # the gather, bit for bit
    tgt = ppo_ffi.d2h(lib, b.d_adv_target_p, F32, N)[rows]
    sv = C5[:-1] + [1]
    y = ppo_ffi.d2h(lib, V.contents.d_output, F32, B)
    gtop = (2 * (y.astype(np.float64) - tgt) / B).reshape(-1, 1)
    gV = check_bf16_layers(lib, V, sv, v0, x, gtop, True, "C5 value")
    g_ref, _ = ref_value_grads(oracle, sv, v0, x, tgt, None, "C5 value")   # targets: see the policy step
    close(gV, g_ref, 3e-2, "C5 value grads vs fp32 oracle")
    # Adam (element-wise fp32) on the gradient it read — a bf16-level gradient difference would move
    # Adam's first step lr·g/(|g| + ε) where |g| is near ε
    flips = assert_adam_delta(v1, adam_first_step(v0, gV, LR), gV, LR, "C5 value params")
    assert flips <= v1.size // 1000


