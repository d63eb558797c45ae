"""Batched device rollout (ppo_rollout_device, csrc/rollout.hip) through the C ABI.

Checks on what the rollout wrote into the buffer:
  * Pendulum-v1: every transition re-simulated in numpy from (observation, action) with gymnasium's
    classic_control step (restated; gymnasium is not installed) — reward and next observation;
  * log-probabilities equal the oracle's log_prob (policy.cu:67-74) of the oracle's μ forward at
    the stored observation; the standardised noise (a − μ)/σ is N(0, 1);
  * env-major segment structure (ppo.cu:70-74): row e·T + t, the next row's observation is this
    row's next observation unless the episode ended, every segment ends truncated;
  * the synthetic environment (any S, A): the same structure at the C3 / C4 shapes;
  * a rollout feeds ppo_update.
"""
import numpy as np
import pytest

import ppo_ffi
from helpers import F32, nn_params_packed

pytestmark = pytest.mark.gpu


def make(lib, sizes, N, seed=3):
    ppo_ffi.C.CDLL("libc.so.6").srand(seed)
    acts = ["relu"] * (len(sizes) - 2) + ["none"]
    return lib.create_ppo(ppo_ffi.c_strings(acts), ppo_ffi.c_ints(sizes), len(sizes), N, 3e-4, 3e-4, 0.95, 0.2, 0.0,
                          1.0, True)


def read_buffer(lib, ppo, N, S, A):
    b = ppo.contents.buffer.contents
    return dict(state=ppo_ffi.d2h(lib, b.d_state_p, F32, N * S).reshape(N, S),
                next_state=ppo_ffi.d2h(lib, b.d_next_state_p, F32, N * S).reshape(N, S),
                action=ppo_ffi.d2h(lib, b.d_action_p, F32, N * A).reshape(N, A),
                logprob=ppo_ffi.d2h(lib, b.d_logprob_p, F32, N),
                reward=ppo_ffi.d2h(lib, b.d_reward_p, F32, N),
                term=ppo_ffi.d2h(lib, b.d_terminated_p, np.uint8, N),
                trunc=ppo_ffi.d2h(lib, b.d_truncated_p, np.uint8, N))


def pendulum_step(obs, u):
    """gymnasium classic_control Pendulum-v1 step (g = 10, m = l = 1, dt = 0.05)."""
    th = np.arctan2(obs[:, 1], obs[:, 0]).astype(np.float64)
    thdot = obs[:, 2].astype(np.float64)
    u = np.clip(u.astype(np.float64), -2.0, 2.0)
    an = ((th + np.pi) % (2 * np.pi)) - np.pi
    cost = an ** 2 + 0.1 * thdot ** 2 + 0.001 * u ** 2
    nthdot = np.clip(thdot + (3 * 10.0 / 2 * np.sin(th) + 3.0 * u) * 0.05, -8, 8)
    nth = th + nthdot * 0.05
    return np.stack([np.cos(nth), np.sin(nth), nthdot], 1), -cost


def check_structure(buf, E, T):
    term, trunc = buf["term"].astype(bool), buf["trunc"].astype(bool)
    seg_end = np.zeros(E * T, bool)
    seg_end[T - 1::T] = True
    assert (trunc[seg_end] | term[seg_end]).all(), "every segment must end done"
    cont = ~(term | trunc) & ~seg_end
    idx = np.nonzero(cont)[0]
    np.testing.assert_array_equal(buf["state"][idx + 1], buf["next_state"][idx])


def check_logprob(lib, oracle, ppo, buf, sizes):
    pol = ppo.contents.policy.contents
    mu_params = nn_params_packed(lib, pol.mu)
    A = sizes[-1]
    log_std = ppo_ffi.d2h(lib, pol.d_log_std, F32, A)
    relu = [1] * (len(sizes) - 2) + [0]
    acts = oracle.mlp_forward(sizes, relu, mu_params, buf["state"])
    mu = oracle.mlp_layer_outputs(sizes, acts, len(buf["state"]))[-1]
    lp_ref = oracle.log_prob(mu, log_std, buf["action"])
    err = np.abs(buf["logprob"] - lp_ref)
    assert err.max() <= 1e-3 * (1 + np.abs(lp_ref).max()), err.max()
    z = (buf["action"] - mu) / np.exp(log_std)
    assert abs(float(z.mean())) < 0.05 and abs(float(z.std()) - 1.0) < 0.05


def test_pendulum_rollout(lib, oracle):
    sizes, E, T = [3, 64, 64, 1], 64, 512
    N = E * T
    ppo = make(lib, sizes, N)
    lib.ppo_rollout_device(ppo, E, T, 0, 11)
    lib.ppo_synchronize()
    buf = read_buffer(lib, ppo, N, 3, 1)
    check_structure(buf, E, T)
    nxt, rew = pendulum_step(buf["state"], buf["action"][:, 0])
    np.testing.assert_allclose(buf["reward"], rew, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(buf["next_state"], nxt, rtol=1e-4, atol=2e-4)
    # 200-step TimeLimit: the first truncation of env 0 at t = 199
    assert buf["trunc"][199] == 1 and buf["trunc"][:199].sum() == 0
    assert not buf["term"].any()
    check_logprob(lib, oracle, ppo, buf, sizes)
    # episodes continue across calls: the next rollout starts from the last state
    last = buf["next_state"][T - 1::T]
    lib.ppo_rollout_device(ppo, E, T, 0, 11)
    lib.ppo_synchronize()
    buf2 = read_buffer(lib, ppo, N, 3, 1)
    first = buf2["state"][0::T]
    # T = 512: TimeLimit resets at t = 199 and 399 only, so every segment end is the horizon's
    # truncation and the episode continues into the next rollout
    np.testing.assert_allclose(first, last, rtol=1e-6, atol=1e-6)
    lib.free_ppo(ppo)


@pytest.mark.parametrize("sizes,E,T", [([17, 256, 256, 6], 64, 256), ([376, 512, 512, 512, 17], 32, 128)])
def test_synthetic_rollout(lib, oracle, sizes, E, T):
    N = E * T
    S, A = sizes[0], sizes[-1]
    ppo = make(lib, sizes, N)
    lib.ppo_rollout_device(ppo, E, T, 1, 5)
    lib.ppo_synchronize()
    buf = read_buffer(lib, ppo, N, S, A)
    check_structure(buf, E, T)
    assert np.abs(buf["state"]).max() <= 1.0 and np.isfinite(buf["reward"]).all()
    # o' = clip(0.95·o + 0.05·tanh(a[j mod A]) + 0.05·ε): the implied ε is N(0, 1)-like
    done = (buf["term"] | buf["trunc"]).astype(bool)
    o, o2 = buf["state"], buf["next_state"]
    tanh_a = np.tanh(buf["action"][:, np.arange(S) % A])
    inner = (np.abs(o2) < 0.999)
    eps = (o2 - 0.95 * o - 0.05 * tanh_a) / 0.05
    assert abs(float(eps[inner].mean())) < 0.05 and abs(float(eps[inner].std()) - 1.0) < 0.05
    assert buf["term"].sum() > 0 or N < 2000
    check_logprob(lib, oracle, ppo, buf, sizes)
    # the rollout feeds an update
    lib.ppo_reset_stats(ppo)
    lib.ppo_update(ppo, 0.99, N // 4, 1, 1, 1, 3)
    stats = (ppo_ffi.C.c_double * 7)()
    lib.ppo_read_stats(ppo, stats, 7)
    assert stats[1] == 4 and stats[3] == 4 and np.isfinite(stats[0]) and np.isfinite(stats[2])
    assert not done.all()
    lib.free_ppo(ppo)
