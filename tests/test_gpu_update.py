"""Update-level parity: the device-resident PPO update vs the oracle's CPU update on identical state.

Checks, from the same seeded start:
  * create_ppo's rand()-driven initialisation is bit-identical to the reference initialiser;
  * GAE advantages / targets (normalised, global statistics);
  * one value minibatch and one policy minibatch: every parameter gradient (stated GEMM
    tolerance) and the Adam parameter delta (exact where |g| is not tiny, ≤ 2·lr elsewhere);
  * both shuffles: the reference's host rand() swap shuffle and libppo's device Feistel shuffle;
  * a whole C1-shaped update (10 value + 4 policy epochs): loss sums and parameter drift.
"""
import ctypes as C

import numpy as np
import pytest

import ppo_ffi
from gpu_internal import read_host_buffer, set_host_buffer
from helpers import (F32, assert_gemm_close, assert_rel_close, gpu_relu_masks, nn_grads_packed, nn_params_packed,
                     oracle_grads_with_masks)

pytestmark = pytest.mark.gpu

RELU = lambda sizes: [1] * (len(sizes) - 2) + [0]  # noqa: E731
ACTS = lambda sizes: ["relu"] * (len(sizes) - 2) + ["none"]  # noqa: E731

CONFIGS = {
    "pendulum": dict(sizes=[3, 64, 64, 1], N=256),
    "halfcheetah": dict(sizes=[17, 256, 256, 6], N=1024),
    "humanoid": dict(sizes=[376, 512, 512, 512, 17], N=2048),
    # B = N > 1024: x3 GEMM engine at width 256, A = 6 (and the opt-in fused output layer below)
    "halfcheetah_2k": dict(sizes=[17, 256, 256, 6], N=2048),
}


def make_ppo(lib, oracle, sizes, N, seed=1234, init_std=1.0, ent_coeff=0.0):
    oracle.srand(seed)
    ppo = lib.create_ppo(ppo_ffi.c_strings(ACTS(sizes)), ppo_ffi.c_ints(sizes), len(sizes), N, 3e-4, 3e-4, 0.95,
                         0.2, ent_coeff, init_std, True)
    return ppo


def synthetic_buffer(oracle, sizes, mu_params, log_std, N, seed, n_envs=4):
    rng = np.random.default_rng(seed)
    S, A = sizes[0], sizes[-1]
    state = rng.uniform(-1, 1, (N, S)).astype(F32)
    next_state = np.roll(state, -1, axis=0).copy()
    term = (rng.uniform(size=N) < 1 / 200).astype(np.uint8)
    trunc = np.zeros(N, np.uint8)
    T = N // n_envs
    trunc[T - 1::T] = 1
    trunc &= 1 - term
    ends = (term | trunc).astype(bool)
    next_state[ends] = rng.uniform(-1, 1, (int(ends.sum()), S)).astype(F32)
    acts = oracle.mlp_forward(sizes, RELU(sizes), mu_params, state)
    mu = oracle.mlp_layer_outputs(sizes, acts, N)[-1]
    action = (mu + rng.normal(size=(N, A)).astype(F32) * np.exp(log_std)).astype(F32)
    logprob = oracle.log_prob(mu, log_std, action)
    reward = (0.1 * rng.normal(size=N)).astype(F32)
    return dict(state=state, next_state=next_state, action=action, reward=reward, logprob=logprob,
                terminated=term, truncated=trunc)


def load_buffer(lib, ppo, buf):
    b = ppo.contents.buffer
    set_host_buffer(lib, b, state=buf["state"], next_state=buf["next_state"], action=buf["action"],
                    reward=buf["reward"], logprob=buf["logprob"], term=buf["terminated"], trunc=buf["truncated"])
    b.contents.idx = 0
    b.contents.full = True
    lib.buffer_to_device(b)


def policy_state(lib, ppo):
    pol = ppo.contents.policy.contents
    mu = nn_params_packed(lib, ppo.contents.policy.contents.mu)
    ls = ppo_ffi.d2h(lib, pol.d_log_std, F32, pol.action_size)
    return mu, ls


def assert_adam_delta(got, ref, g_ref, lr, what):
    """Adam step from identical state: exact where |g| is not tiny; a sign flip (≤ 2·lr) allowed elsewhere."""
    big = np.abs(g_ref) > 1e-3 * np.abs(g_ref).max()
    err = np.abs(got - ref)
    assert (err[big] <= 1e-6 * np.abs(ref[big]) + 1e-6 * lr).all(), \
        f"{what}: Adam delta mismatch on large-|g| entries, worst {err[big].max():.3g}"
    assert (err <= 2 * lr * 1.0001 + 1e-7).all(), f"{what}: delta beyond 2·lr, worst {err.max():.3g}"
    return int((err > 1e-6 * lr + 1e-6 * np.abs(ref)).sum())


def adam_first_step(theta0, g, lr):
    """Adam's first step (adam.cu:53-74, t = 1: m̂ = g, v̂ = g²) from θ0 with gradient g, float64."""
    g = np.asarray(g, np.float64)
    m_hat = (0.1 * g) / (1 - 0.9)
    v_hat = (0.001 * g * g) / (1 - 0.999)
    return (np.asarray(theta0, np.float64) - lr * m_hat / (np.sqrt(v_hat) + 1e-8)).astype(F32)


def test_create_ppo_initialisation_bitexact(lib, oracle):
    """neural_network.cu:40-51 / policy.cu:22-24 from srand(seed): μ net, then V net."""
    sizes = [17, 256, 256, 6]
    ppo = make_ppo(lib, oracle, sizes, 64, seed=42, init_std=0.5)
    mu, ls = policy_state(lib, ppo)
    v = nn_params_packed(lib, ppo.contents.V)
    oracle.srand(42)
    mu_ref = oracle.mlp_init(sizes)
    v_ref = oracle.mlp_init(sizes[:-1] + [1])
    np.testing.assert_array_equal(mu, mu_ref)
    np.testing.assert_array_equal(v, v_ref)
    np.testing.assert_array_equal(ls, np.full(6, np.log(np.float32(0.5)), F32))
    lib.free_ppo(ppo)


@pytest.mark.parametrize("cfg", sorted(CONFIGS))
@pytest.mark.parametrize("shuffle_mode", [0, 1])
def test_single_value_step(lib, oracle, cfg, shuffle_mode):
    sizes, N = CONFIGS[cfg]["sizes"], CONFIGS[cfg]["N"]
    ppo = make_ppo(lib, oracle, sizes, N)
    mu0, ls0 = policy_state(lib, ppo)
    v0 = nn_params_packed(lib, ppo.contents.V)
    buf = synthetic_buffer(oracle, sizes, mu0, ls0, N, seed=7)
    load_buffer(lib, ppo, buf)
    oracle.srand(99)
    lib.ppo_update(ppo, 0.99, N, 0, 1, shuffle_mode, 5)          # GAE + exactly one value minibatch
    lib.ppo_synchronize()
    b = ppo.contents.buffer.contents
    adv = ppo_ffi.d2h(lib, b.d_advantage_p, F32, N)
    tgt = ppo_ffi.d2h(lib, b.d_adv_target_p, F32, N)
    gV = nn_grads_packed(lib, ppo.contents.V)
    v1 = nn_params_packed(lib, ppo.contents.V)

    oracle.srand(99)
    ref = oracle.ppo_update(sizes, RELU(sizes), mu0, ls0, v0, buf, batch_size=N, n_epochs_policy=0,
                            n_epochs_value=1, shuffle_mode=shuffle_mode, seed=5)
    assert_rel_close(tgt, ref["adv_target"], 2e-4, 2e-4 * np.abs(ref["adv_target"]).max(), "adv_target")
    assert_rel_close(adv, ref["advantage"], 2e-3, 2e-3, "advantage")
    # value gradient of the minibatch (the whole buffer in permuted order) from the oracle
    sv = sizes[:-1] + [1]
    x = buf["state"]
    acts = oracle.mlp_forward(sv, RELU(sv), v0, x)
    y = oracle.mlp_layer_outputs(sv, acts, N)[-1].ravel()
    _, g = oracle.mse(y, ref["adv_target"])
    # batch == buffer: order only permutes rows; ReLU′ masks as the GPU's forward had them (a
    # pre-activation within fp32 rounding of 0 may fall on either side: oracle_grads_with_masks)
    g_ref, nflip = oracle_grads_with_masks(oracle, sv, RELU(sv), v0, x, g.reshape(-1, 1),
                                       gpu_relu_masks(lib, ppo.contents.V, x), f"{cfg} value")
    assert_gemm_close(gV, g_ref, N, f"{cfg} value grads")
    # the Adam step of those gradients (where the forwards agree on every mask bit this is the
    # oracle's own update, ref["v"])
    flips = assert_adam_delta(v1, adam_first_step(v0, g_ref, 3e-4) if nflip else ref["v"], g_ref, 3e-4,
                              f"{cfg} value params")
    assert flips <= max(2, v1.size // 1000)
    assert ppo.contents.adam_V.contents.time_step == ref["t_v"] == 1
    lib.free_ppo(ppo)


@pytest.mark.parametrize("cfg", sorted(CONFIGS))
@pytest.mark.parametrize("shuffle_mode", [0, 1])
def test_single_policy_step(lib, oracle, cfg, shuffle_mode):
    sizes, N = CONFIGS[cfg]["sizes"], CONFIGS[cfg]["N"]
    A = sizes[-1]
    ppo = make_ppo(lib, oracle, sizes, N, init_std=0.7, ent_coeff=0.01)
    mu0, ls0 = policy_state(lib, ppo)
    v0 = nn_params_packed(lib, ppo.contents.V)
    buf = synthetic_buffer(oracle, sizes, mu0, ls0, N, seed=11)
    # perturb the behaviour log-probs so ratios leave [1−ε, 1+ε] on both sides
    buf["logprob"] = (buf["logprob"] + np.random.default_rng(3).normal(scale=0.4, size=N)).astype(F32)
    load_buffer(lib, ppo, buf)
    oracle.srand(17)
    lib.ppo_update(ppo, 0.99, N, 1, 0, shuffle_mode, 9)          # GAE + exactly one policy minibatch
    lib.ppo_synchronize()
    pol = ppo.contents.policy.contents
    gmu = nn_grads_packed(lib, ppo.contents.policy.contents.mu)
    gls = ppo_ffi.d2h(lib, pol.d_log_std_grad, F32, A)
    mu1, ls1 = policy_state(lib, ppo)
    oracle.srand(17)
    ref = oracle.ppo_update(sizes, RELU(sizes), mu0, ls0, v0, buf, batch_size=N, n_epochs_policy=1,
                            n_epochs_value=0, ent_coeff=0.01, shuffle_mode=shuffle_mode, seed=9)
    # oracle gradients on the same minibatch (the whole buffer; row order does not change sums)
    x, a = buf["state"], buf["action"]
    acts = oracle.mlp_forward(sizes, RELU(sizes), mu0, x)
    mu = oracle.mlp_layer_outputs(sizes, acts, N)[-1]
    lp = oracle.log_prob(mu, ls0, a)
    _, glp, gent = oracle.policy_loss_and_grad(ref["advantage"], lp, buf["logprob"], oracle.entropy(ls0), 0.01,
                                               0.2)
    gmu_out, gls_ref = oracle.log_prob_backwards(mu, ls0, a, glp)
    g_ref, nflip = oracle_grads_with_masks(oracle, sizes, RELU(sizes), mu0, x, gmu_out,
                                       gpu_relu_masks(lib, ppo.contents.policy.contents.mu, x), f"{cfg} policy")
    gls_ref = gls_ref + gent
    assert_gemm_close(gmu, g_ref, N, f"{cfg} policy grads")
    assert_rel_close(gls, gls_ref, 1e-3, 1e-4 * max(1.0, np.abs(gls_ref).max()), "log_std grad")
    flips = assert_adam_delta(mu1, adam_first_step(mu0, g_ref, 3e-4) if nflip else ref["mu"], g_ref, 3e-4,
                              f"{cfg} policy params")
    assert flips <= max(2, mu1.size // 1000)
    assert_adam_delta(ls1, ref["log_std"], gls_ref, 3e-4, "log_std")
    assert ppo.contents.adam_policy.contents.time_step == ppo.contents.adam_entropy.contents.time_step == 1
    lib.free_ppo(ppo)


@pytest.mark.parametrize("shuffle_mode", [0, 1])
def test_full_update_c1(lib, oracle, shuffle_mode):
    """C1: Pendulum shape, N = 2048, B = 64, 10 value + 4 policy epochs (448 minibatch steps).

    Minibatch-level parity is exact up to fp32 re-association; over 448 Adam steps ReLU/clip
    branch flips make trajectories drift, so the whole-update check is statistical: loss sums
    within 2 % and parameter movement agreeing in direction (cosine > 0.95) and size (±10 %).
    """
    sizes, N, B = [3, 64, 64, 1], 2048, 64
    ppo = make_ppo(lib, oracle, sizes, N)
    mu0, ls0 = policy_state(lib, ppo)
    v0 = nn_params_packed(lib, ppo.contents.V)
    buf = synthetic_buffer(oracle, sizes, mu0, ls0, N, seed=21, n_envs=8)
    load_buffer(lib, ppo, buf)
    lib.ppo_reset_stats(ppo)
    oracle.srand(5)
    lib.ppo_update(ppo, 0.99, B, 4, 10, shuffle_mode, 77)
    st = (C.c_double * 7)()
    lib.ppo_read_stats(ppo, st, 7)
    mu1, ls1 = policy_state(lib, ppo)
    v1 = nn_params_packed(lib, ppo.contents.V)
    oracle.srand(5)
    ref = oracle.ppo_update(sizes, RELU(sizes), mu0, ls0, v0, buf, batch_size=B, shuffle_mode=shuffle_mode,
                            seed=77)
    assert st[1] == ref["n_v"] == 320 and st[3] == ref["n_p"] == 128
    assert abs(st[0] - ref["sum_v_loss"]) <= 0.02 * abs(ref["sum_v_loss"])
    assert abs(st[2] - ref["sum_policy_loss"]) <= 0.02 * abs(ref["sum_policy_loss"]) + 0.02
    for got, start, want, what in ((v1, v0, ref["v"], "V"), (mu1, mu0, ref["mu"], "mu"),
                                   (ls1, ls0, ref["log_std"], "log_std")):
        d_got, d_ref = got - start, want - start
        cos = float(d_got @ d_ref / (np.linalg.norm(d_got) * np.linalg.norm(d_ref) + 1e-30))
        ratio = float(np.linalg.norm(d_got) / (np.linalg.norm(d_ref) + 1e-30))
        assert cos > 0.95 and 0.9 < ratio < 1.1, f"{what}: cos {cos:.4f} norm ratio {ratio:.4f}"
    lib.free_ppo(ppo)


@pytest.mark.parametrize("layout", ["rollout", "random", "mixed"])
def test_gae_next_value_reuse(lib, oracle, layout, monkeypatch):
    """V(next_state[t]) is taken from V(state[t+1]) only where the rows are bitwise equal.

    rollout: next_state = state shifted by one except at episode ends (the reuse path);
    random: no row equal (every transition gets its own forward); mixed: half the rows equal,
    including rows at episode ends.  Targets equal the oracle's (two full forwards, ppo.cu:333-336)
    and the PPO_GAE_FULL=1 path's.
    """
    sizes, N = [17, 256, 256, 6], 4096
    ppo = make_ppo(lib, oracle, sizes, N)
    mu0, ls0 = policy_state(lib, ppo)
    v0 = nn_params_packed(lib, ppo.contents.V)
    buf = synthetic_buffer(oracle, sizes, mu0, ls0, N, seed=13, n_envs=8)
    rng = np.random.default_rng(5)
    if layout != "rollout":
        fresh = rng.uniform(-1, 1, buf["next_state"].shape).astype(F32)
        pick = np.ones(N, bool) if layout == "random" else rng.uniform(size=N) < 0.5
        buf["next_state"][pick] = fresh[pick]
        if layout == "mixed":
            ends = np.nonzero(buf["terminated"] | buf["truncated"])[0]
            ends = ends[ends + 1 < N]
            buf["next_state"][ends] = buf["state"][ends + 1]
    load_buffer(lib, ppo, buf)
    b = ppo.contents.buffer.contents
    out = {}
    for mode in ("reuse", "full"):
        if mode == "full":
            monkeypatch.setenv("PPO_GAE_FULL", "1")
        lib.ppo_update(ppo, 0.99, N, 0, 0, 1, 5)                 # GAE only
        lib.ppo_synchronize()
        out[mode] = ppo_ffi.d2h(lib, b.d_adv_target_p, F32, N)
    monkeypatch.delenv("PPO_GAE_FULL")
    ref = oracle.ppo_update(sizes, RELU(sizes), mu0, ls0, v0, buf, batch_size=N, n_epochs_policy=0,
                            n_epochs_value=0, shuffle_mode=1, seed=5)
    for mode, tgt in out.items():
        assert_rel_close(tgt, ref["adv_target"], 2e-4, 2e-4 * np.abs(ref["adv_target"]).max(), f"{layout} {mode}")
    assert_rel_close(out["reuse"], out["full"], 1e-4, 1e-4 * np.abs(out["full"]).max(), f"{layout} reuse vs full")
    lib.free_ppo(ppo)


@pytest.mark.parametrize("shuffle_mode", [0, 1])
def test_concurrent_value_policy_loops(lib, oracle, shuffle_mode, monkeypatch):
    """The policy loop on the side stream beside the value loop == both loops one after the other.

    Same minibatches, Adam step counts and host rand() consumption.  grad_W runs without split-K
    here (forced), so the GEMMs are deterministic: the value network must match bit for bit; in
    the policy only the head's log σ-gradient atomics can reorder.
    """
    sizes, N, B = [17, 256, 256, 6], 4096, 512
    lib.ppo_gemm_tune(-1, 1)                                       # split-K target 1: no atomics
    out = {}
    for mode in ("serial", "concurrent"):
        if mode == "serial":
            monkeypatch.setenv("PPO_SERIAL", "1")
        else:
            monkeypatch.delenv("PPO_SERIAL", raising=False)
        ppo = make_ppo(lib, oracle, sizes, N)
        mu0, ls0 = policy_state(lib, ppo)
        buf = synthetic_buffer(oracle, sizes, mu0, ls0, N, seed=3, n_envs=8)
        load_buffer(lib, ppo, buf)
        lib.ppo_reset_stats(ppo)
        oracle.srand(41)
        lib.ppo_update(ppo, 0.99, B, 2, 3, shuffle_mode, 8)
        st = (C.c_double * 9)()
        lib.ppo_read_stats(ppo, st, 9)
        mu, ls = policy_state(lib, ppo)
        out[mode] = dict(stats=np.array(st[:4]), graph_steps=st[8], v=nn_params_packed(lib, ppo.contents.V),
                         mu=mu, ls=ls,
                         next_rand=oracle.libc().rand(),
                         t=(ppo.contents.adam_V.contents.time_step, ppo.contents.adam_policy.contents.time_step,
                            ppo.contents.adam_entropy.contents.time_step))
        lib.free_ppo(ppo)
    lib.ppo_gemm_tune(-1, 0)
    a, b = out["serial"], out["concurrent"]
    assert a["t"] == b["t"] == (24, 16, 16)
    assert a["next_rand"] == b["next_rand"]
    np.testing.assert_allclose(a["stats"], b["stats"], rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(a["v"], b["v"])                 # the value loop has no atomics left
    for k in ("mu", "ls"):        # the log σ-gradient's atomics may flip an Adam step of a tiny gradient
        err = np.abs(a[k] - b[k])  # (a 1-ulp log σ difference reaches every μ gradient: measured 0.2-1.04 %
        assert err.max() <= 2 * 3e-4, (k, err.max())           # of μ elements beyond 1e-6 run to run)
        assert (err > 1e-6).mean() < 0.02, (k, (err > 1e-6).mean())


@pytest.mark.parametrize("comm,async_", [("self", "0"), ("self", "1"), ("loopback2", "0"), ("loopback2", "1")])
def test_comm_rehearsal(lib, oracle, comm, async_, monkeypatch):
    """The data-parallel path on one GPU, in both gradient all-reduce forms, while the value and policy
    loops run concurrently, exactly as at world > 1:
      * inline (default): one all-reduce per step in each loop's own stream, a communicator per loop
        (the policy loop's split from the value loop's), Adam behind it in stream order;
      * bucketed (PPO_COMM_ASYNC=1, also the fallback when the split fails on any rank): per-layer
        buckets on comm.hip's comm stream over one communicator (issuing stream -> event -> comm
        stream -> event -> Adam).
    comm = "self": a one-rank RCCL communicator (PPO_COMM_SELF=1) — the one-rank sum is the identity;
    comm = "loopback2": two identical in-process ranks (PPO_COMM_LOOPBACK=2) — the sum is 2·g and Adam
    applies ½, exact in binary.  Either way the update must equal the update without a communicator:
    value network bit for bit (split-K forced off), policy within the log σ-gradient atomics bound; the
    per-update replica check runs (loopback: world 2) and passes."""
    sizes, N, B = [17, 256, 256, 6], 4096, 512
    lib.ppo_gemm_tune(-1, 1)
    monkeypatch.delenv("PPO_SERIAL", raising=False)
    out = {}
    for mode in ("plain", "comm"):
        if mode == "comm":
            monkeypatch.setenv("PPO_COMM_ASYNC", async_)
            if comm == "self":
                monkeypatch.setenv("PPO_COMM_SELF", "1")
            else:
                monkeypatch.setenv("PPO_COMM_LOOPBACK", "2")
            assert lib.ppo_comm_init(0, 1, None) == 0, lib.ppo_last_error()
            want = "bucketed" if async_ == "1" else "inline"
            assert want in lib.ppo_comm_mode().decode(), lib.ppo_comm_mode()
            assert lib.ppo_comm_world() == (2 if comm == "loopback2" else 1)
        ppo = make_ppo(lib, oracle, sizes, N)
        mu0, ls0 = policy_state(lib, ppo)
        buf = synthetic_buffer(oracle, sizes, mu0, ls0, N, seed=5, n_envs=8)
        load_buffer(lib, ppo, buf)
        lib.ppo_reset_stats(ppo)
        oracle.srand(43)
        lib.ppo_update(ppo, 0.99, B, 2, 3, 1, 9)
        st = (C.c_double * 7)()
        lib.ppo_read_stats(ppo, st, 7)
        mu, ls = policy_state(lib, ppo)
        out[mode] = dict(stats=np.array(st[:4]), v=nn_params_packed(lib, ppo.contents.V), mu=mu, ls=ls)
        lib.free_ppo(ppo)
        if mode == "comm":
            lib.ppo_comm_finalize()
            for k in ("PPO_COMM_SELF", "PPO_COMM_LOOPBACK", "PPO_COMM_ASYNC"):
                monkeypatch.delenv(k, raising=False)
    lib.ppo_gemm_tune(-1, 0)
    a, b = out["plain"], out["comm"]
    np.testing.assert_allclose(a["stats"], b["stats"], rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(a["v"], b["v"])
    for k in ("mu", "ls"):
        err = np.abs(a[k] - b[k])
        assert err.max() <= 2 * 3e-4, (k, err.max())
        assert (err > 1e-6).mean() < 0.01, (k, (err > 1e-6).mean())


@pytest.mark.parametrize("cap,filled,B", [(4096, 3000, 512), (4096, 4096, 1000)])
def test_partial_and_ragged_buffer(lib, oracle, cap, filled, B):
    """A partly filled buffer (idx = filled < capacity, full = false) and a batch size that does not
    divide the buffer: GAE over the filled rows only, ⌊capacity / B⌋ minibatches per epoch (D13)
    whose rows wrap modulo the filled count (trajectory_buffer.cu:168-200).  One value and one policy
    epoch (8 / 4 steps) from identical state: loss sums and parameter motion track the oracle."""
    sizes = [17, 256, 256, 6]
    ppo = make_ppo(lib, oracle, sizes, cap)
    mu0, ls0 = policy_state(lib, ppo)
    v0 = nn_params_packed(lib, ppo.contents.V)
    buf = synthetic_buffer(oracle, sizes, mu0, ls0, filled, seed=17, n_envs=4)
    pad = cap - filled
    full_buf = {k: np.concatenate([v, np.full((pad,) + v.shape[1:], 7, v.dtype)]) for k, v in buf.items()}
    b = ppo.contents.buffer
    set_host_buffer(lib, b, state=full_buf["state"], next_state=full_buf["next_state"], action=full_buf["action"],
                    reward=full_buf["reward"], logprob=full_buf["logprob"], term=full_buf["terminated"],
                    trunc=full_buf["truncated"])
    b.contents.idx = filled % cap
    b.contents.full = filled == cap
    lib.buffer_to_device(b)
    lib.ppo_reset_stats(ppo)
    oracle.srand(23)
    lib.ppo_update(ppo, 0.99, B, 1, 1, 0, 3)
    st = (C.c_double * 7)()
    lib.ppo_read_stats(ppo, st, 7)
    mu1, ls1 = policy_state(lib, ppo)
    v1 = nn_params_packed(lib, ppo.contents.V)
    tgt = ppo_ffi.d2h(lib, b.contents.d_adv_target_p, F32, filled)
    oracle.srand(23)
    ref = oracle.ppo_update(sizes, RELU(sizes), mu0, ls0, v0, buf, batch_size=B, n_epochs_policy=1,
                            n_epochs_value=1, shuffle_mode=0, seed=3, capacity=cap)
    nb = cap // B
    assert st[1] == ref["n_v"] == nb and st[3] == ref["n_p"] == nb
    assert_rel_close(tgt, ref["adv_target"], 2e-4, 2e-4 * np.abs(ref["adv_target"]).max(), "adv_target")
    assert abs(st[0] - ref["sum_v_loss"]) <= 1e-3 * abs(ref["sum_v_loss"])
    assert abs(st[2] - ref["sum_policy_loss"]) <= 1e-2 * abs(ref["sum_policy_loss"]) + 1e-4
    for got, start, want, what in ((v1, v0, ref["v"], "V"), (mu1, mu0, ref["mu"], "mu"),
                                   (ls1, ls0, ref["log_std"], "log_std")):
        d_got, d_ref = got - start, want - start
        cos = float(d_got @ d_ref / (np.linalg.norm(d_got) * np.linalg.norm(d_ref) + 1e-30))
        assert cos > 0.99, f"{what}: cos {cos:.4f}"
    lib.free_ppo(ppo)


def test_degenerate_updates(lib, oracle):
    """Edge cases the loops must survive: B larger than the buffer (⌊N/B⌋ = 0 minibatches: GAE only),
    zero epochs, and an empty buffer (D19: the update ends after GAE, no rand() consumed)."""
    sizes, N = [17, 256, 256, 6], 1024
    ppo = make_ppo(lib, oracle, sizes, N)
    mu0, ls0 = policy_state(lib, ppo)
    v0 = nn_params_packed(lib, ppo.contents.V)
    buf = synthetic_buffer(oracle, sizes, mu0, ls0, N, seed=4)
    load_buffer(lib, ppo, buf)
    st = (C.c_double * 7)()
    for B, n_pol, n_val in ((4096, 4, 10), (256, 0, 0)):
        lib.ppo_reset_stats(ppo)
        lib.ppo_update(ppo, 0.99, B, n_pol, n_val, 1, 2)
        lib.ppo_read_stats(ppo, st, 7)
        assert st[1] == 0 and st[3] == 0
        np.testing.assert_array_equal(nn_params_packed(lib, ppo.contents.V), v0)
        np.testing.assert_array_equal(policy_state(lib, ppo)[0], mu0)
    assert ppo.contents.adam_V.contents.time_step == 0
    tgt = ppo_ffi.d2h(lib, ppo.contents.buffer.contents.d_adv_target_p, F32, N)
    assert np.isfinite(tgt).all() and np.abs(tgt).max() > 0          # GAE did run
    b = ppo.contents.buffer.contents
    b.idx, b.full = 0, False
    oracle.srand(8)
    lib.ppo_reset_stats(ppo)
    lib.ppo_update(ppo, 0.99, 256, 4, 10, 0, 2)                       # host shuffle: must not consume rand()
    lib.ppo_synchronize()
    lib.ppo_read_stats(ppo, st, 7)
    assert st[1] == 0 and st[3] == 0
    r = oracle.libc().rand()
    oracle.srand(8)
    assert r == oracle.libc().rand()
    lib.free_ppo(ppo)


@pytest.mark.parametrize("net", ["c3_exact", "c4_x3", "c4_exact"])
def test_short_update_elementwise(lib, oracle, net):
    """A short whole update (GAE, 2 value epochs and 1 policy epoch of 4 minibatches: up to 12 Adam
    steps per network, device Feistel shuffle on both sides) against the oracle's update of the same
    buffer, element by element (diagnostic quantiles printed; bounds below)."""
    sizes, N, B = {"c3_exact": ([17, 256, 256, 6], 2048, 512), "c4_x3": ([376, 512, 512, 512, 17], 8192, 2048),
                   "c4_exact": ([376, 512, 512, 512, 17], 8192, 2048)}[net]
    old = lib.ppo_gemm_f32_engine(0 if net.endswith("exact") else 1)
    try:
        ppo = make_ppo(lib, oracle, sizes, N, init_std=0.7)
        mu0, ls0 = policy_state(lib, ppo)
        v0 = nn_params_packed(lib, ppo.contents.V)
        buf = synthetic_buffer(oracle, sizes, mu0, ls0, N, seed=33, n_envs=8)
        load_buffer(lib, ppo, buf)
        lib.ppo_reset_stats(ppo)
        lib.ppo_update(ppo, 0.99, B, 1, 2, 1, 4242)
        lib.ppo_synchronize()
    finally:
        lib.ppo_gemm_f32_engine(old)
    st = (C.c_double * 7)()
    lib.ppo_read_stats(ppo, st, 7)
    mu1, ls1 = policy_state(lib, ppo)
    v1 = nn_params_packed(lib, ppo.contents.V)
    ref = oracle.ppo_update(sizes, RELU(sizes), mu0, ls0, v0, buf, batch_size=B, n_epochs_policy=1,
                            n_epochs_value=2, shuffle_mode=1, seed=4242)
    steps_v, steps_p = 2 * (N // B), N // B
    assert st[1] == ref["n_v"] == steps_v and st[3] == ref["n_p"] == steps_p
    lr = 3e-4
    for got, want, start, n_steps, what in ((v1, ref["v"], v0, steps_v, "V"), (mu1, ref["mu"], mu0, steps_p, "mu"),
                                            (ls1, ref["log_std"], ls0, steps_p, "log_std")):
        err = np.abs(got.astype(np.float64) - want)
        moved = np.abs(want.astype(np.float64) - start)
        q = {f: float((err <= f * lr).mean()) for f in (1e-3, 1e-2, 1e-1)}
        print(f"{net} {what}: n={err.size} within lr x 1e-3 / 1e-2 / 1e-1: " +
              " / ".join(f"{100 * v:.3f} %" for v in q.values()) +
              f"; max err {err.max():.3g} (= {err.max() / lr:.3f} lr); median movement {np.median(moved) / lr:.2f} lr")
        assert err.max() <= 2 * lr * n_steps, f"{what}: max err {err.max()}"
        assert q[1e-1] >= 0.99, f"{what}: only {q[1e-1] * 100:.2f} % within 0.1·lr"
    np.testing.assert_allclose(st[0], ref["sum_v_loss"], rtol=1e-3)
    np.testing.assert_allclose(st[2], ref["sum_policy_loss"], rtol=1e-3, atol=1e-5)
    lib.free_ppo(ppo)


@pytest.mark.parametrize("cfg", ["humanoid", "halfcheetah_2k"])
def test_out_head_matches_separate(lib, oracle, cfg, monkeypatch):
    """The fused output layer + loss head + output-layer backward (out_head.hip; value A = 1 and,
    for halfcheetah, the A = 6 policy) against the separate launches (PPO_OUT_HEAD=0) from identical
    state: one value and one policy minibatch, every gradient within the GEMM tolerance, the log
    σ-gradient and the loss sums within reduction rounding."""
    sizes, N = CONFIGS[cfg]["sizes"], CONFIGS[cfg]["N"]
    A = sizes[-1]
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("PPO_OUT_HEAD", mode)
        ppo = make_ppo(lib, oracle, sizes, N, init_std=0.7, ent_coeff=0.01)
        mu0, ls0 = policy_state(lib, ppo)
        buf = synthetic_buffer(oracle, sizes, mu0, ls0, N, seed=21)
        buf["logprob"] = (buf["logprob"] + np.random.default_rng(5).normal(scale=0.4, size=N)).astype(F32)
        load_buffer(lib, ppo, buf)
        lib.ppo_reset_stats(ppo)
        lib.ppo_update(ppo, 0.99, N, 1, 1, 1, 13)
        lib.ppo_synchronize()
        st = (C.c_double * 7)()
        lib.ppo_read_stats(ppo, st, 7)
        pol = ppo.contents.policy.contents
        out[mode] = dict(gV=nn_grads_packed(lib, ppo.contents.V), gmu=nn_grads_packed(lib, pol.mu),
                         gls=ppo_ffi.d2h(lib, pol.d_log_std_grad, F32, A), stats=np.array(st[:4]),
                         yV=ppo_ffi.d2h(lib, ppo.contents.V.contents.d_output, F32, N))
        lib.free_ppo(ppo)
    a, b = out["0"], out["1"]
    assert_gemm_close(b["gV"], a["gV"], N, f"{cfg} value grads (fused vs separate)")
    assert_gemm_close(b["gmu"], a["gmu"], N, f"{cfg} policy grads (fused vs separate)")
    assert_gemm_close(b["yV"], a["yV"], sizes[-2], f"{cfg} value output (fused vs separate)")
    assert_rel_close(b["gls"], a["gls"], 1e-3, 1e-4 * max(1.0, np.abs(a["gls"]).max()), "log_std grad")
    np.testing.assert_allclose(b["stats"], a["stats"], rtol=1e-3, atol=1e-6)


@pytest.mark.parametrize("shuffle_mode", [0, 1])
def test_graph_replay_matches_eager(lib, oracle, shuffle_mode, monkeypatch):
    """Graph replay of minibatch steps (PPO_GRAPH=1, B = 64: steps 1 … n−2 of each phase replay captured
    16-step graphs whose gather / Adam arguments come from the device step table) against the eager
    launches from identical state: the same minibatch order (host rand() permutations and the
    device Feistel order), the same Adam step counts and sizes, so the value network agrees bit for bit
    and the policy to the rounding of the fused head's log σ f32 atomics.  Graph replay is only enabled
    for this combination (fp32, fused value and A ≤ 6 policy heads: step_graphs_ok); the A = 17 wide head
    and the unfused path run eagerly even with PPO_GRAPH=1 (checked below)."""
    sizes, N, B = [17, 256, 256, 6], 4096, 64
    # this shape at B = 64 would take the single-launch cluster phases (cluster.hip) before the graph
    # path: force the multi-launch loop so graph replay is what runs (counted below)
    monkeypatch.setenv("PPO_NO_CLUSTER", "1")
    out = {}
    for mode in ("eager", "graph"):
        if mode == "eager":
            monkeypatch.delenv("PPO_GRAPH", raising=False)
        else:
            monkeypatch.setenv("PPO_GRAPH", "1")
            monkeypatch.setenv("PPO_GRAPH_STEPS", "16")
        ppo = make_ppo(lib, oracle, sizes, N, init_std=0.7, ent_coeff=0.01)
        mu0, ls0 = policy_state(lib, ppo)
        buf = synthetic_buffer(oracle, sizes, mu0, ls0, N, seed=44, n_envs=8)
        load_buffer(lib, ppo, buf)
        lib.ppo_reset_stats(ppo)
        oracle.srand(321)
        lib.ppo_update(ppo, 0.99, B, 1, 2, shuffle_mode, 77)
        lib.ppo_synchronize()
        st = (C.c_double * 9)()
        lib.ppo_read_stats(ppo, st, 9)
        mu, ls = policy_state(lib, ppo)
        out[mode] = dict(stats=np.array(st[:4]), graph_steps=st[8], v=nn_params_packed(lib, ppo.contents.V),
                         mu=mu, ls=ls,
                         gv=nn_grads_packed(lib, ppo.contents.V), next_rand=oracle.libc().rand(),
                         t=(ppo.contents.adam_V.contents.time_step, ppo.contents.adam_policy.contents.time_step,
                            ppo.contents.adam_entropy.contents.time_step))
        lib.free_ppo(ppo)
    a, b = out["eager"], out["graph"]
    # every step but each phase's first and last replayed from graphs (no silent eager fallback)
    assert a["graph_steps"] == 0 and b["graph_steps"] == (2 * N // B - 2) + (N // B - 2), b["graph_steps"]
    assert a["t"] == b["t"] == (2 * N // B, N // B, N // B)
    assert a["next_rand"] == b["next_rand"]
    assert a["stats"][1] == b["stats"][1] and a["stats"][3] == b["stats"][3]
    np.testing.assert_allclose(b["stats"], a["stats"], rtol=1e-4, atol=1e-6)
    # the value loop: the same gather rows, GEMMs, fused head (one workgroup at B = 64: no cross-workgroup
    # atomics) and Adam arithmetic with the same host-computed step sizes — bit for bit
    np.testing.assert_array_equal(a["v"], b["v"])
    lr, n_steps = 3e-4, 2 * N // B
    for key in ("mu", "ls"):
        err = np.abs(a[key].astype(np.float64) - b[key])
        assert err.max() <= 2 * lr * n_steps, (key, err.max())
        assert (err <= 0.1 * lr).mean() >= 0.99, (key, (err <= 0.1 * lr).mean())
    # the last value minibatch ran eagerly in both: its gradients are there to read
    assert np.abs(b["gv"]).max() > 0


@pytest.mark.parametrize("case", ["wide_head", "unfused"])
def test_graph_replay_declines_untested_paths(lib, oracle, case, monkeypatch):
    """PPO_GRAPH=1 with the A = 17 wide policy head or PPO_OUT_HEAD=0 (separate head launches): no graph
    is captured (step_graphs_ok), every step runs eagerly — bit-identical to the same run without
    PPO_GRAPH (split-K off: no atomics anywhere but the log σ sums, which the policy bound covers)."""
    sizes = [376, 512, 512, 17] if case == "wide_head" else [17, 256, 256, 6]
    N, B = 2048, 64
    monkeypatch.setenv("PPO_NO_CLUSTER", "1")     # the multi-launch loop, where step_graphs_ok decides
    lib.ppo_gemm_tune(-1, 1)
    out = {}
    try:
        for mode in ("eager", "graph"):
            if case == "unfused":
                monkeypatch.setenv("PPO_OUT_HEAD", "0")
            if mode == "graph":
                monkeypatch.setenv("PPO_GRAPH", "1")
            else:
                monkeypatch.delenv("PPO_GRAPH", raising=False)
            monkeypatch.setenv("PPO_SERIAL", "1")
            ppo = make_ppo(lib, oracle, sizes, N, init_std=0.7)
            mu0, ls0 = policy_state(lib, ppo)
            buf = synthetic_buffer(oracle, sizes, mu0, ls0, N, seed=45, n_envs=4)
            load_buffer(lib, ppo, buf)
            lib.ppo_reset_stats(ppo)
            lib.ppo_update(ppo, 0.99, B, 1, 1, 1, 78)
            lib.ppo_synchronize()
            st = (C.c_double * 9)()
            lib.ppo_read_stats(ppo, st, 9)
            assert st[1] == st[3] == N // B and st[8] == 0, list(st)    # every step ran, none from a graph
            out[mode] = dict(v=nn_params_packed(lib, ppo.contents.V), mu=policy_state(lib, ppo)[0])
            lib.free_ppo(ppo)
    finally:
        lib.ppo_gemm_tune(-1, 0)
    np.testing.assert_array_equal(out["eager"]["v"], out["graph"]["v"])
    err = np.abs(out["eager"]["mu"] - out["graph"]["mu"])
    assert err.max() <= 2 * 3e-4 and (err > 1e-6).mean() < 0.02


@pytest.mark.parametrize("shape", ["humanoid", "narrow_ragged"])
@pytest.mark.parametrize("fused", ["1", "0"])
def test_wide_output_backward_matches_pair(lib, oracle, monkeypatch, fused, shape):
    """The A = 17 policy network's output layer on its one-pass paths — fused = 1 (default): forward, head
    and backward in one launch (policy_out_fused_kernel: μ by exact fp32 MFMA from h staged in LDS, the
    head, grad_x and grad_W / grad_b from the same rows); fused = 0 (PPO_POLICY_FUSED=0): the forward GEMM,
    then the head fused with the one-pass backward (out_bwd_wide_kernel<HEAD>) — against the separate head
    launch + paired GEMM launch (PPO_NO_WIDE_BWD=1) from identical state: one policy minibatch of the
    humanoid config (and a 256-wide network on a ragged 1000-row minibatch: the last 16-row block partial), μ and
    every policy gradient within the GEMM tolerance (the same products summed in another order), the log σ
    gradient and the loss sums within reduction rounding."""
    if shape == "humanoid":
        sizes, N = CONFIGS["humanoid"]["sizes"], CONFIGS["humanoid"]["N"]
    else:
        sizes, N = [17, 256, 256, 17], 1000
    out = {}
    monkeypatch.setenv("PPO_POLICY_FUSED", fused)
    for mode in ("1", "0"):
        if mode == "1":
            monkeypatch.setenv("PPO_NO_WIDE_BWD", "1")
        else:
            monkeypatch.delenv("PPO_NO_WIDE_BWD", raising=False)
        ppo = make_ppo(lib, oracle, sizes, N, init_std=0.7, ent_coeff=0.01)
        mu0, ls0 = policy_state(lib, ppo)
        buf = synthetic_buffer(oracle, sizes, mu0, ls0, N, seed=23)
        load_buffer(lib, ppo, buf)
        lib.ppo_reset_stats(ppo)
        lib.ppo_update(ppo, 0.99, N, 1, 0, 1, 17)
        lib.ppo_synchronize()
        st = (C.c_double * 7)()
        lib.ppo_read_stats(ppo, st, 7)
        pol = ppo.contents.policy.contents
        out[mode] = dict(gmu=nn_grads_packed(lib, pol.mu), stats=np.array(st[:4]),
                         gls=ppo_ffi.d2h(lib, pol.d_log_std_grad, F32, sizes[-1]),
                         mu=ppo_ffi.d2h(lib, pol.mu.contents.d_output, F32, N * sizes[-1]))
        lib.free_ppo(ppo)
    a, b = out["1"], out["0"]
    assert_gemm_close(b["mu"], a["mu"], sizes[-2], "policy output μ (one-pass vs separate forward)")
    assert_gemm_close(b["gmu"], a["gmu"], N, "policy grads (wide backward vs paired GEMM)")
    assert_rel_close(b["gls"], a["gls"], 1e-4, 1e-5 * max(1.0, np.abs(a["gls"]).max()), "log_std grad")
    np.testing.assert_allclose(b["stats"], a["stats"], rtol=1e-5, atol=1e-7)
