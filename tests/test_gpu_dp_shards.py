"""libppo's data-parallel path on DIFFERENT shards (reference loops ppo.cu:491-533).

bench.py --gpus 2 gives rank r the environments [r·E/2, (r+1)·E/2) of ONE rollout (its own
ppo_fill_synthetic seed, seed·1000 + r), B/2 rows per minibatch step, identical initial weights
(srand(seed)) and the same shuffle seed.  RCCL refuses two ranks on one GPU, so the two ranks run
here one after the other in one process, each through every world > 1 branch of the update
(PPO_COMM_LOOPBACK=2) with the OTHER rank's contributions supplied (ppo_comm_loopback_peers /
_peer_grads): the all-gather delivers the other shard's Welford triple, the min over ranks sees the
other shard's limit, and rank 0's gradient all-reduce adds rank 1's gradient buffer.

Checked against the oracle run as ONE reference update over the concatenated buffer (segments never
cross environments, so its GAE is the shards' GAE with global statistics):
  * each shard's normalised advantages (global Welford combine of two different triples);
  * the all-reduced gradient ÷ 2 of the first value and policy minibatch = the oracle's gradient of the
    concatenated 2·(B/2)-row global minibatch (every layer, biases, log σ), and Adam's step of it;
  * the empty-shard agreement with a disagreeing rank (the other shard empty: this rank stops after
    GAE, no collective left waiting).
C3 and C4 network shapes at their bench sizes.
"""
import ctypes as C

import numpy as np
import pytest

import ppo_ffi
from helpers import (F32, assert_gemm_close, assert_normalised_close, assert_rel_close, gpu_relu_masks,
                     nn_grads_packed, nn_input_rows, nn_params_packed, oracle_grads_with_masks)
from test_gpu_production import RELU, device_buffer
from test_gpu_update import adam_first_step, assert_adam_delta, make_ppo, policy_state

pytestmark = pytest.mark.gpu

LR = 3e-4
CFGS = {"c3": ([17, 256, 256, 6], 64, 4096, 8192), "c4": ([376, 512, 512, 512, 17], 256, 4096, 32768)}


def _addr(p):
    return C.cast(p, C.c_void_p).value


def _gathered(lib, nn_ptr, B, S):
    nn = nn_ptr.contents
    assert nn.bits_m == B and nn.x0_dtype == 0
    return nn_input_rows(lib, nn_ptr, B)


def _mu_span(pol):
    """μ's flat gradient span including the log σ gradient behind it: the policy's top all-reduce
    bucket carries align4(A) floats there (ppo.c policy_step), so the span ends at the padded end."""
    mu = pol.mu.contents
    off = (_addr(pol.d_log_std_grad) - _addr(mu.d_grads)) // 4
    assert off >= mu.num_params
    return off + (pol.action_size + 3) // 4 * 4, off


def _read_rank(lib, ppo, Bs, S, A, rows_v, rows_p, buf):
    """What one rank's first value and policy minibatch left: gradient buffers, parameters, masks."""
    pol = ppo.contents.policy.contents
    n_mu, ls_off = _mu_span(pol)
    xv, xp = buf["state"][rows_v], buf["state"][rows_p]
    np.testing.assert_array_equal(_gathered(lib, ppo.contents.V, Bs, S), xv)
    np.testing.assert_array_equal(_gathered(lib, pol.mu, Bs, S), xp)
    # gV / gmu_span: the flat (16-B padded) gradient buffers the all-reduce runs over; gV_packed /
    # gmu_packed: the reference's packed [W0, b0, W1, b1, …] order for the comparisons
    return dict(gV=ppo_ffi.d2h(lib, ppo.contents.V.contents.d_grads, F32, ppo.contents.V.contents.num_params),
                gmu_span=ppo_ffi.d2h(lib, pol.mu.contents.d_grads, F32, n_mu), ls_off=ls_off,
                gV_packed=nn_grads_packed(lib, ppo.contents.V), gmu_packed=nn_grads_packed(lib, pol.mu),
                mV=gpu_relu_masks(lib, ppo.contents.V, xv), mmu=gpu_relu_masks(lib, pol.mu, xp),
                v1=nn_params_packed(lib, ppo.contents.V), mu1=nn_params_packed(lib, pol.mu),
                adv=ppo_ffi.d2h(lib, ppo.contents.buffer.contents.d_advantage_p, F32, buf["reward"].size))


def _cat_masks(m0, m1):
    return None if m0 is None or m1 is None else [np.concatenate([a, b]) for a, b in zip(m0, m1)]


@pytest.mark.parametrize("cfg", ["c3", "c4"])
def test_two_rank_shards_vs_global_minibatch(lib, oracle, monkeypatch, cfg):
    sizes, E, T, B = CFGS[cfg]
    S, A = sizes[0], sizes[-1]
    sv = sizes[:-1] + [1]
    G, seed = 2, 1234
    Es, Bs = E // G, B // G
    Ns = Es * T
    oracle.load(use_openblas=True)
    oracle.load().ref_blas_threads(16)

    # every rank's shard and its own (local) GAE statistics, as bench.py builds them
    ranks = []
    for r in range(G):
        ppo = make_ppo(lib, oracle, sizes, Ns, seed=seed)          # srand(seed): identical initial weights
        lib.ppo_fill_synthetic(ppo, Es, T, seed * 1000 + r, 1.0 / 500)
        lib.ppo_set_step_limit(ppo, 0, 0)
        lib.ppo_update(ppo, 0.99, Bs, 0, 0, 1, seed)             # GAE only (no epoch key consumed)
        w = np.zeros(6)
        assert lib.ppo_gae_state(w.ctypes.data, None, None, 0) == Ns
        ranks.append(dict(ppo=ppo, w=w[3:].copy(), buf=device_buffer(lib, ppo, Ns, S, A)))
    v0 = nn_params_packed(lib, ranks[0]["ppo"].contents.V)
    mu0, ls0 = policy_state(lib, ranks[0]["ppo"])
    np.testing.assert_array_equal(v0, nn_params_packed(lib, ranks[1]["ppo"].contents.V))
    assert ranks[0]["w"][1] != ranks[1]["w"][1]                 # the shards' statistics really differ

    key = oracle.splitmix64(seed)
    rows_v = oracle.feistel_perm(Ns, key)[:Bs]                    # value epoch 0 (same key on every rank)
    rows_p = oracle.feistel_perm(Ns, (key + 1) & (2**64 - 1))[:Bs]  # policy epoch 0

    monkeypatch.setenv("PPO_COMM_LOOPBACK", str(G))
    assert lib.ppo_comm_init(0, 1, None) == 0, lib.ppo_last_error()
    try:
        assert lib.ppo_comm_world() == G
        # rank 1: the other rank's triple and limit; its own all-reduce stays the identical-rank ×2 (its
        # local gradient is read back as half of it, exactly)
        assert lib.ppo_comm_loopback_peers(ranks[0]["w"].ctypes.data, ppo_ffi.c_ints([Ns]), 1) == 0
        p1 = ranks[1]["ppo"]
        lib.ppo_set_step_limit(p1, 1, 1)
        lib.ppo_update(p1, 0.99, Bs, 1, 1, 1, seed)
        lib.ppo_synchronize()
        r1 = _read_rank(lib, p1, Bs, S, A, rows_v, rows_p, ranks[1]["buf"])
        g1V, g1mu = r1["gV"] / 2, r1["gmu_span"] / 2              # ×2 and ÷2 are exact
        lib.ppo_comm_loopback_clear()

        # rank 0: rank 1's triple, limit and gradients; its all-reduce is the real two-rank sum
        p0 = ranks[0]["ppo"]
        pol0 = p0.contents.policy.contents
        assert lib.ppo_comm_loopback_peers(ranks[1]["w"].ctypes.data, ppo_ffi.c_ints([Ns]), 1) == 0
        d_gV1 = ppo_ffi.DeviceArray.from_numpy(lib, g1V)
        d_gmu1 = ppo_ffi.DeviceArray.from_numpy(lib, g1mu)
        assert lib.ppo_comm_loopback_peer_grads(_addr(p0.contents.V.contents.d_grads), d_gV1.ptr, g1V.size) == 0
        assert lib.ppo_comm_loopback_peer_grads(_addr(pol0.mu.contents.d_grads), d_gmu1.ptr, g1mu.size) == 0
        lib.ppo_set_step_limit(p0, 1, 1)
        lib.ppo_reset_stats(p0)
        lib.ppo_update(p0, 0.99, Bs, 1, 1, 1, seed)
        lib.ppo_synchronize()
        r0 = _read_rank(lib, p0, Bs, S, A, rows_v, rows_p, ranks[0]["buf"])
        w_glob = np.zeros(6)
        lib.ppo_gae_state(w_glob.ctypes.data, None, None, 0)
        st = (C.c_double * 7)()
        lib.ppo_read_stats(p0, st, 7)
        assert st[1] == 1 and st[3] == 1
        t_v = p0.contents.adam_V.contents.time_step

        # the empty-shard agreement with a disagreeing rank: the other shard is empty → this rank
        # stops after GAE (no Adam step, no collective issued that rank 1 would never join)
        lib.ppo_comm_loopback_clear()
        assert lib.ppo_comm_loopback_peers(None, ppo_ffi.c_ints([0]), 1) == 0
        lib.ppo_update(p0, 0.99, Bs, 1, 1, 1, seed)
        lib.ppo_synchronize()
        assert p0.contents.adam_V.contents.time_step == t_v
        d_gV1.free()
        d_gmu1.free()
    finally:
        lib.ppo_comm_finalize()
        monkeypatch.delenv("PPO_COMM_LOOPBACK")
        for rk in ranks:
            lib.ppo_set_step_limit(rk["ppo"], -1, -1)
            lib.free_ppo(rk["ppo"])
    assert lib.ppo_comm_world() == 1

    # the oracle: ONE reference update's GAE over the concatenated buffer (global statistics)
    union = {k: np.concatenate([ranks[0]["buf"][k], ranks[1]["buf"][k]]) for k in ranks[0]["buf"]}
    ref = oracle.ppo_update(sizes, RELU(sizes), mu0, ls0, v0, union, batch_size=1, n_epochs_policy=0,
                            n_epochs_value=0, max_value_steps=0, max_policy_steps=0)
    adv_u, tgt_u = ref["advantage"], ref["adv_target"]
    assert w_glob[0] == 2 * Ns
    # normalised with the GLOBAL statistics (the exact statistics of the union's advantages: the
    # oracle's fp32 running sums drift at N ≳ 1e5, helpers.assert_normalised_close)
    raw_u = adv_u.astype(np.float64) * (np.float64(ref["adv_std"]) + 1e-8) + ref["adv_mean"]
    adv_exact = (raw_u - raw_u.mean()) / (raw_u.std() + 1e-8)
    for r, rr in ((0, r0), (1, r1)):
        assert_rel_close(rr["adv"], adv_exact[r * Ns:(r + 1) * Ns], 1e-4, 1e-4, f"{cfg} rank {r} advantages")
    assert_normalised_close(np.concatenate([r0["adv"], r1["adv"]]), adv_u, ref["adv_mean"], ref["adv_std"],
                            f"{cfg} union advantages")

    # value: the all-reduced gradient ÷ 2 = the gradient of the concatenated global minibatch
    bufs = [ranks[0]["buf"], ranks[1]["buf"]]
    x = np.concatenate([b["state"][rows_v] for b in bufs])
    tgt = np.concatenate([tgt_u[rows_v], tgt_u[Ns + rows_v]])
    acts = oracle.mlp_forward(sv, RELU(sv), v0, x)
    y = oracle.mlp_layer_outputs(sv, acts, B)[-1].ravel()
    _, g = oracle.mse(y, tgt)
    gV_ref, _ = oracle_grads_with_masks(oracle, sv, RELU(sv), v0, x, g.reshape(-1, 1), _cat_masks(r0["mV"], r1["mV"]),
                                        f"{cfg} value", max_flips=256)
    gV = r0["gV_packed"] / 2
    assert_gemm_close(gV, gV_ref, B, f"{cfg} all-reduced value gradient")
    flips = assert_adam_delta(r0["v1"], adam_first_step(v0, gV_ref, LR), gV_ref, LR, f"{cfg} value params")
    assert flips <= v0.size // 1000

    # policy: the same for μ and log σ (advantages normalised over both shards)
    x = np.concatenate([b["state"][rows_p] for b in bufs])
    a = np.concatenate([b["action"][rows_p] for b in bufs])
    old = np.concatenate([b["logprob"][rows_p] for b in bufs])
    adv = np.concatenate([adv_u[rows_p], adv_u[Ns + rows_p]])
    acts = oracle.mlp_forward(sizes, RELU(sizes), mu0, x)
    mu = oracle.mlp_layer_outputs(sizes, acts, B)[-1]
    lp = oracle.log_prob(mu, ls0, a)
    _, glp, gent = oracle.policy_loss_and_grad(adv, lp, old, oracle.entropy(ls0), 0.0, 0.2)
    gmu_out, gls_ref = oracle.log_prob_backwards(mu, ls0, a, glp)
    gmu_ref, _ = oracle_grads_with_masks(oracle, sizes, RELU(sizes), mu0, x, gmu_out,
                                         _cat_masks(r0["mmu"], r1["mmu"]), f"{cfg} policy", max_flips=256)
    n_mu = mu0.size
    gmu = r0["gmu_packed"] / 2
    gls = r0["gmu_span"][r0["ls_off"]:r0["ls_off"] + A] / 2
    assert_gemm_close(gmu, gmu_ref, B, f"{cfg} all-reduced policy gradient")
    assert_rel_close(gls, gls_ref + gent, 1e-3, 1e-4 * max(1.0, float(np.abs(gls_ref).max())), f"{cfg} log σ grad")
    flips = assert_adam_delta(r0["mu1"], adam_first_step(mu0, gmu_ref, LR), gmu_ref, LR, f"{cfg} policy params")
    assert flips <= n_mu // 1000
    # the two ranks' local gradients really differ (the test is not self-similar)
    assert np.abs(r0["gV_packed"] - r1["gV_packed"]).max() > 1e-3 * np.abs(gV_ref).max()
