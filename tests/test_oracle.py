"""CPU: pin the oracle (oracle/ref_cpu.c, the plain-C restatement of the reference CPU path) against the
independent float64 known answers in tests/golden (see make_golden.py).  The reference ships no
fixtures of its own, so parity is "unpinned" by reference outputs; these checks pin the restatement's
arithmetic to the reference's published formulas (file:line in make_golden.py)."""
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
F32 = np.float32


def gold(name):
    return np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)


def close(got, want, rtol, atol, what):
    got, want = np.asarray(got, np.float64), np.asarray(want, np.float64)
    err = np.abs(got - want)
    assert (err <= atol + rtol * np.abs(want)).all(), f"{what}: worst {err.max():.3g}"


def test_linear_forward_backward(oracle):
    g = gold("linear")
    y = oracle.mat_mul(g["x"].astype(F32), g["W"].astype(F32), g["b"].astype(F32))
    close(y, g["y"], 1e-5, 1e-5, "y")
    gx, gW = oracle.mat_mul_backwards(g["g"].astype(F32), g["x"].astype(F32), g["W"].astype(F32))
    close(gx, g["gx"], 1e-5, 1e-5, "grad_x")
    close(gW, g["gW"], 1e-5, 1e-5, "grad_W")


def test_mlp_forward_backward_vs_autograd(oracle):
    g = gold("mlp")
    sizes, relu = [int(s) for s in g["sizes"]], [int(r) for r in g["relu"]]
    p, x = g["params"].astype(F32), g["x"].astype(F32)
    acts = oracle.mlp_forward(sizes, relu, p, x)
    close(acts, g["acts"], 1e-5, 1e-5, "activations")
    grads = oracle.mlp_backward(sizes, relu, p, x, acts, g["grad_out"].astype(F32))
    close(grads, g["grads"], 1e-5, 1e-5, "parameter grads")


def test_gaussian_policy(oracle):
    g = gold("policy")
    mu, ls, a = g["mu"].astype(F32), g["log_std"].astype(F32), g["action"].astype(F32)
    close(oracle.log_prob(mu, ls, a), g["log_prob"], 1e-5, 1e-5, "log_prob")
    gmu, gls = oracle.log_prob_backwards(mu, ls, a, g["grad_in"].astype(F32))
    close(gmu, g["grad_mu"], 1e-5, 1e-5, "grad_mu")
    close(gls, g["grad_log_std"], 1e-5, 1e-5, "grad_log_std")
    assert abs(oracle.entropy(ls) - float(g["entropy"])) < 1e-5


def test_clipped_surrogate(oracle):
    g = gold("surrogate")
    loss, glp, gent = oracle.policy_loss_and_grad(g["adv"].astype(F32), g["lp"].astype(F32),
                                                  g["old_lp"].astype(F32), float(g["entropy"]),
                                                  float(g["ent_coeff"]), float(g["epsilon"]))
    assert abs(loss - float(g["loss"])) < 1e-5
    close(glp, g["grad_lp"], 1e-5, 1e-6, "grad_logprob")
    assert gent == pytest.approx(-float(g["ent_coeff"]))


def test_gae(oracle):
    g = gold("gae")
    adv, tgt, mean, std = oracle.gae(g["v"].astype(F32), g["v_next"].astype(F32), g["reward"].astype(F32),
                                     g["terminated"], g["truncated"], float(g["gamma"]), float(g["lam"]))
    close(tgt, g["adv_target"], 1e-5, 1e-5, "adv_target")
    close(adv, g["advantage"], 1e-4, 1e-5, "normalised advantage")
    assert abs(mean - float(g["mean"])) < 1e-5 and abs(std - float(g["std"])) < 1e-5


def test_adam_vs_torch(oracle):
    g = gold("adam")
    p = g["p0"].astype(F32)
    m, v = np.zeros_like(p), np.zeros_like(p)
    t = 0
    for k in range(g["grads"].shape[0]):
        t = oracle.adam_update(p, g["grads"][k].astype(F32), m, v, t, float(g["lr"]))
        close(p, g["params"][k], 1e-6, 1e-7, f"params after step {k + 1}")
    assert t == g["grads"].shape[0]


def test_glibc_rand_and_reference_shuffle(oracle):
    """The libc rand() stream the reference consumes (srand → rand) and its swap shuffle."""
    import ctypes as C

    g = gold("rand")
    libc = C.CDLL("libc.so.6")
    for seed, seq in zip(g["seeds"], g["rand"]):
        libc.srand(C.c_uint(int(seed)))
        assert [libc.rand() for _ in range(len(seq))] == [int(s) for s in seq]
    oracle.srand(int(g["shuffle_seed"]))
    np.testing.assert_array_equal(oracle.shuffle(len(g["shuffle"])), g["shuffle"])


def test_weight_init_matches_reference_formula(oracle):
    g = gold("init")
    oracle.srand(int(g["seed"]))
    np.testing.assert_array_equal(oracle.mlp_init([int(s) for s in g["sizes"]]), g["params"])


@pytest.mark.parametrize("n", [1, 2, 3, 7, 64, 1000, 4096, 65537])
def test_feistel_permutation_is_a_bijection(oracle, n):
    for key in (0, 1, 0xDEADBEEF):
        perm = oracle.feistel_perm(n, key)
        assert np.array_equal(np.sort(perm), np.arange(n))
    if n >= 64:
        assert not np.array_equal(oracle.feistel_perm(n, 1), oracle.feistel_perm(n, 2))


def test_oracle_update_counts_and_determinism(oracle):
    """ppo.cu:387-443: ⌊N/B⌋ minibatches per epoch; seeded runs are bit-reproducible."""
    sizes = [3, 16, 16, 1]
    oracle.srand(3)
    mu = oracle.mlp_init(sizes)
    v = oracle.mlp_init(sizes)
    rng = np.random.default_rng(0)
    N = 200
    buf = dict(state=rng.uniform(-1, 1, (N, 3)).astype(F32), next_state=rng.uniform(-1, 1, (N, 3)).astype(F32),
               action=rng.normal(size=(N, 1)).astype(F32), reward=rng.normal(size=N).astype(F32),
               logprob=rng.normal(size=N).astype(F32), terminated=np.zeros(N, np.uint8),
               truncated=np.zeros(N, np.uint8))
    outs = []
    for _ in range(2):
        oracle.srand(11)
        outs.append(oracle.ppo_update(sizes, [1, 1, 0], mu, np.zeros(1, F32), v, buf, batch_size=64))
    assert outs[0]["n_v"] == 10 * 3 and outs[0]["n_p"] == 4 * 3
    for k in ("mu", "v", "log_std", "advantage"):
        np.testing.assert_array_equal(outs[0][k], outs[1][k])
