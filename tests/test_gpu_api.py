"""The reference API as main.c drives it, through libppo's C ABI (GPU tests).

Covers the host-pointer half of the reference interface:
  * sample_action (policy.cu:76-89, m = 1 as collect_trajectories calls it, and m > 1): action and
    log-prob against the oracle's μ forward + Box–Muller noise (ref_gaussian_noise) from the same
    srand, and the libc rand() stream consumed exactly as the oracle consumes it;
  * host mirrors vs HBM: a host entry point after a device update must not revert the device
    parameters (it pulls them into the mirrors); a caller's edit of a host mirror is pushed;
  * main.c:46-62's sequence: create_gym_env → create_ppo → eval_ppo → train_ppo_epoch → eval_ppo →
    compute_entropy → save_ppo → free_ppo, with eval_ppo's printed J / R / episode count recomputed
    from the buffer it leaves and the whole rand() consumption predicted;
  * save_ppo byte for byte against the oracle's restatement of the reference writer
    (ppo.cu:585-611, policy.cu:207-211, neural_network.cu:283-300, adam.cu:172-189), load_ppo round
    trips, and a loaded checkpoint trains exactly like the original;
  * the reference's unchanged main.c (bin/ppo_main, linked against libppo) runs to completion.
"""
import ctypes as C
import os
import re
import struct
import subprocess

import numpy as np
import pytest

import ppo_ffi
from gpu_internal import read_host_buffer
from helpers import F32, assert_gemm_close, assert_rel_close, nn_params_packed

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RELU = lambda sizes: [1] * (len(sizes) - 2) + [0]  # noqa: E731
ACTS = lambda sizes: ["relu"] * (len(sizes) - 2) + ["none"]  # noqa: E731


def host_params(nn_ptr):
    """Packed [W0,b0,...] read from a NeuralNetwork's HOST mirrors."""
    nn = nn_ptr.contents
    out = []
    for i in range(nn.num_layers - 1):
        ly = nn.layers[i]
        nw = ly.input_size * ly.output_size
        out.append(np.ctypeslib.as_array(ly.weights, shape=(nw,)).copy())
        out.append(np.ctypeslib.as_array(ly.biases, shape=(ly.output_size,)).copy())
    return np.concatenate(out)


def rand_after(oracle, seed, k):
    """The libc rand() value after srand(seed) and k draws (libppo and the oracle share glibc's state)."""
    libc = oracle.libc()
    oracle.srand(seed)
    for _ in range(k):
        libc.rand()
    return libc.rand()


@pytest.mark.parametrize("sizes,m", [([3, 64, 64, 1], 1), ([17, 256, 256, 6], 1), ([17, 64, 6], 5),
                                     ([376, 512, 512, 17], 3)])
def test_sample_action_parity(lib, oracle, sizes, m):
    """a = μ(s) + ε·σ with ε from Box–Muller over rand() (policy.cu:46-89), log π(a|s) per row."""
    A = sizes[-1]
    oracle.srand(3)
    pol = lib.create_gaussian_policy(ppo_ffi.c_ints(sizes), ppo_ffi.c_strings(ACTS(sizes)), len(sizes), 0.6)
    params = nn_params_packed(lib, pol.contents.mu)
    log_std = np.ctypeslib.as_array(pol.contents.log_std, shape=(A,)).copy()
    state = np.random.default_rng(m + A).uniform(-1, 1, (m, sizes[0])).astype(F32)
    action = np.zeros((m, A), F32)
    logp = np.zeros(m, F32)
    oracle.srand(77)
    lib.sample_action(pol, state.ctypes.data, action.ctypes.data, logp.ctypes.data, m)
    next_rand = oracle.libc().rand()

    oracle.srand(77)
    noise = oracle.gaussian_noise(m * A).reshape(m, A)
    assert oracle.libc().rand() == next_rand                           # same rand() consumption
    acts = oracle.mlp_forward(sizes, RELU(sizes), params, state)
    mu_ref = oracle.mlp_layer_outputs(sizes, acts, m)[-1]
    sigma = np.exp(log_std).astype(F32)
    mu_got = action - noise * sigma                                   # the μ libppo added the noise to
    assert_gemm_close(mu_got, mu_ref, sizes[-2], "μ under the sample")
    assert_gemm_close(action, (mu_ref + noise * sigma).astype(F32), sizes[-2], "action")
    lp_ref = oracle.log_prob(mu_ref, log_std, action)
    assert_rel_close(logp, lp_ref, 1e-4, 1e-4 * max(1.0, float(np.abs(lp_ref).max())), "log_prob")
    lib.free_gaussian_policy(pol)


def test_host_entry_keeps_device_update(lib, oracle):
    """ppo_update (ext, device) then sample_action: the trained HBM parameters and log σ stay, the host
    mirrors receive them (the host path used to upload its stale mirrors over them)."""
    sizes, N = [17, 64, 64, 6], 2048
    oracle.srand(5)
    ppo = lib.create_ppo(ppo_ffi.c_strings(ACTS(sizes)), ppo_ffi.c_ints(sizes), len(sizes), N, 3e-4, 3e-4, 0.95,
                         0.2, 0.0, 1.0, True)
    pol = ppo.contents.policy
    mu0 = nn_params_packed(lib, pol.contents.mu)
    lib.ppo_fill_synthetic(ppo, 8, N // 8, 11, 1 / 500)
    lib.ppo_update(ppo, 0.99, 256, 1, 1, 1, 3)
    lib.ppo_synchronize()
    mu1 = nn_params_packed(lib, pol.contents.mu)
    v1 = nn_params_packed(lib, ppo.contents.V)
    ls1 = ppo_ffi.d2h(lib, pol.contents.d_log_std, F32, 6)
    assert np.abs(mu1 - mu0).max() > 0
    s = np.zeros((1, 17), F32)
    a = np.zeros((1, 6), F32)
    lp = np.zeros(1, F32)
    lib.sample_action(pol, s.ctypes.data, a.ctypes.data, lp.ctypes.data, 1)
    lib.forward_propagation(ppo.contents.V, s.ctypes.data, 1)
    np.testing.assert_array_equal(nn_params_packed(lib, pol.contents.mu), mu1)
    np.testing.assert_array_equal(nn_params_packed(lib, ppo.contents.V), v1)
    np.testing.assert_array_equal(ppo_ffi.d2h(lib, pol.contents.d_log_std, F32, 6), ls1)
    np.testing.assert_array_equal(host_params(pol.contents.mu), mu1)   # pulled into the mirrors
    np.testing.assert_array_equal(host_params(ppo.contents.V), v1)
    np.testing.assert_array_equal(np.ctypeslib.as_array(pol.contents.log_std, shape=(6,)), ls1)
    # a caller's edit of a host mirror is pushed to HBM by the next host entry point
    ly = ppo.contents.V.contents.layers[1]
    w = np.ctypeslib.as_array(ly.weights, shape=(64 * 64,))
    w[7] += 0.5
    lib.forward_propagation(ppo.contents.V, s.ctypes.data, 1)
    np.testing.assert_array_equal(ppo_ffi.d2h(lib, ly.d_weights, F32, 64 * 64), w)
    lib.free_ppo(ppo)


def parse_eval(text):
    m = re.findall(r"J: (-?[\d.]+|nan|-nan) R: (-?[\d.]+|nan|-nan) Episodes: (\d+)", text)
    assert m, text
    return [(float(j), float(r), int(e)) for j, r, e in m]


def eval_ref(reward, term, trunc, gamma):
    """eval_ppo's J / R / episode count (ppo.cu:560-583) recomputed in float32 from the buffer."""
    steps = reward.size
    f = np.float32
    rewards = f(reward[-1])
    episode_j = f(reward[-1])
    n_ep, sum_j = 1, f(0)
    for i in range(steps - 2, -1, -1):
        rewards = f(rewards + reward[i])
        episode_j = f(reward[i] + f(gamma) * episode_j)
        if term[i] or trunc[i]:
            n_ep += 1
            sum_j = f(sum_j + episode_j)
            episode_j = f(0)
    return float(sum_j / f(n_ep)), float(rewards / f(n_ep)), n_ep


def test_main_c_sequence(lib, oracle, capfd, tmp_path):
    """main.c:13-64 at one training iteration (Pendulum-v1, 2×64 MLP, 3000-step buffer, B = 64)."""
    seed, cap, B = 1234, 3000, 64
    oracle.srand(seed)
    env = lib.create_gym_env(0, seed)
    e = env.contents
    sizes = [e.state_size, 64, 64, e.action_size]
    ppo = lib.create_ppo(ppo_ffi.c_strings(ACTS(sizes)), ppo_ffi.c_ints(sizes), 4, cap, 3e-4, 3e-4, 0.95, 0.2, 0.0,
                         1.0, True)
    init_draws = oracle.mlp_num_params(sizes) + oracle.mlp_num_params(sizes[:-1] + [1])   # one rand() per W, b
    buf = ppo.contents.buffer

    def eval_and_check():
        capfd.readouterr()
        lib.eval_ppo(ppo, env, cap)
        oracle.libc().fflush(None)                                       # printf is buffered
        j, r, n = parse_eval(capfd.readouterr().out)[-1]
        rew = read_host_buffer(buf, "h_reward_p", cap)
        term = read_host_buffer(buf, "h_terminated_p", cap, np.uint8)
        trunc = read_host_buffer(buf, "h_truncated_p", cap, np.uint8)
        jr, rr, nr = eval_ref(rew, term, trunc, e.gamma)
        assert n == nr and abs(j - jr) <= 1e-4 * max(1, abs(jr)) and abs(r - rr) <= 1e-4 * max(1, abs(rr))
        assert np.isfinite(rew).all() and (rew <= 0).all()               # Pendulum costs
        assert buf.contents.idx == 0 and not buf.contents.full          # eval resets the buffer
        return j

    eval_and_check()
    mu0, v0 = nn_params_packed(lib, ppo.contents.policy.contents.mu), nn_params_packed(lib, ppo.contents.V)
    lib.train_ppo_epoch(ppo, env, cap, B, 4, 10)
    nb = cap // B
    assert ppo.contents.adam_V.contents.time_step == 10 * nb
    assert ppo.contents.adam_policy.contents.time_step == ppo.contents.adam_entropy.contents.time_step == 4 * nb
    mu1, v1 = nn_params_packed(lib, ppo.contents.policy.contents.mu), nn_params_packed(lib, ppo.contents.V)
    assert np.abs(mu1 - mu0).max() > 0 and np.abs(v1 - v0).max() > 0
    np.testing.assert_array_equal(host_params(ppo.contents.policy.contents.mu), mu1)   # train_ppo_epoch
    np.testing.assert_array_equal(host_params(ppo.contents.V), v1)                     # hands weights back
    assert buf.contents.on_device == 0                                                 # and the buffer
    ent = lib.compute_entropy(ppo.contents.policy)
    ls = np.ctypeslib.as_array(ppo.contents.policy.contents.log_std, shape=(e.action_size,))
    assert abs(ent - oracle.entropy(ls)) <= 1e-5 * max(1.0, abs(ent))
    eval_and_check()
    path = str(tmp_path / "ppo_model.bin")
    lib.save_ppo(ppo, path.encode())
    # rand() consumed as the reference consumes it: init, 2 per env step (Box–Muller, A = 1) over
    # three rollouts of `cap` steps, one swap shuffle (cap draws) per value and policy epoch
    draws = init_draws + 3 * 2 * cap + 14 * cap
    got = oracle.libc().rand()
    assert got == rand_after(oracle, seed, draws)
    lib.free_ppo(ppo)
    assert os.path.getsize(path) > 0


def _adam_state(lib, adam_ptr, lengths):
    """(size, t, b1, b2, n, packed m, packed v) of a device Adam, read back tensor by tensor."""
    a = adam_ptr.contents
    ms, vs, off = [], [], 0
    base = a.weights[0]
    for i, n in enumerate(lengths):
        src = (C.cast(a.weights[i], C.c_void_p).value - C.cast(base, C.c_void_p).value) // 4 if a.flat else off
        ms.append(ppo_ffi.d2h(lib, C.cast(a.m, C.c_void_p).value + 4 * src, F32, n))
        vs.append(ppo_ffi.d2h(lib, C.cast(a.v, C.c_void_p).value + 4 * src, F32, n))
        off += n
    return dict(size=a.size, t=a.time_step, b1=a.beta1, b2=a.beta2, n=a.num_layers, m=np.concatenate(ms),
                v=np.concatenate(vs))


def _nn_lengths(sizes):
    out = []
    for i in range(len(sizes) - 1):
        out += [sizes[i] * sizes[i + 1], sizes[i + 1]]
    return out


def _expected_checkpoint(lib, oracle, ppo, sizes):
    p = ppo.contents
    pol = p.policy.contents
    A = sizes[-1]
    vs = sizes[:-1] + [1]
    adams = [_adam_state(lib, p.adam_policy, _nn_lengths(sizes)), _adam_state(lib, p.adam_V, _nn_lengths(vs)),
             _adam_state(lib, p.adam_entropy, [A])]
    return oracle.save_ppo_bytes((p.lambda_, p.epsilon, p.ent_coeff, p.lr_policy, p.lr_V), sizes[0], A,
                                 p.buffer.contents.capacity, ppo_ffi.d2h(lib, pol.d_log_std, F32, A), sizes,
                                 ACTS(sizes), nn_params_packed(lib, pol.mu), vs, ACTS(sizes),
                                 nn_params_packed(lib, p.V), adams)


@pytest.mark.parametrize("sizes,N,B", [([3, 64, 64, 1], 2048, 64), ([17, 256, 256, 6], 4096, 512)])
def test_checkpoint_bytes_and_round_trip(lib, oracle, tmp_path, sizes, N, B):
    """save_ppo after a short update == the reference writer's bytes; load_ppo → save_ppo reproduces the
    file; a loaded checkpoint's next update equals the original's (deterministic GEMMs: no split-K)."""
    lib.ppo_gemm_tune(-1, 1)
    try:
        oracle.srand(9)
        ppo = lib.create_ppo(ppo_ffi.c_strings(ACTS(sizes)), ppo_ffi.c_ints(sizes), len(sizes), N, 3e-4, 2e-4,
                             0.95, 0.2, 0.01, 0.8, True)
        lib.ppo_fill_synthetic(ppo, 8, N // 8, 21, 1 / 300)
        lib.ppo_update(ppo, 0.99, B, 2, 3, 1, 4)
        lib.ppo_synchronize()
        f1 = str(tmp_path / "a.bin")
        lib.save_ppo(ppo, f1.encode())
        raw = open(f1, "rb").read()
        want = _expected_checkpoint(lib, oracle, ppo, sizes)
        assert len(raw) == len(want)
        assert raw == want
        # header fields decoded by hand (ppo.cu:588-597)
        lam, eps, ent, lr_p, lr_v = struct.unpack_from("<5f", raw, 0)
        S, A, cap = struct.unpack_from("<3i", raw, 20)
        assert (S, A, cap) == (sizes[0], sizes[-1], N)
        assert np.float32(lam) == np.float32(0.95) and np.float32(lr_v) == np.float32(2e-4)
        loaded = lib.load_ppo(f1.encode(), True)
        f2 = str(tmp_path / "b.bin")
        lib.save_ppo(loaded, f2.encode())
        assert open(f2, "rb").read() == raw
        lp = loaded.contents
        assert lp.adam_V.contents.time_step == ppo.contents.adam_V.contents.time_step
        # the next update from the original and from the loaded copy (same buffer contents)
        lib.ppo_fill_synthetic(loaded, 8, N // 8, 21, 1 / 300)
        lib.ppo_fill_synthetic(ppo, 8, N // 8, 21, 1 / 300)
        out = []
        for q in (ppo, loaded):
            lib.ppo_update(q, 0.99, B, 1, 1, 1, 99)
            lib.ppo_synchronize()
            out.append((nn_params_packed(lib, q.contents.V), nn_params_packed(lib, q.contents.policy.contents.mu),
                        ppo_ffi.d2h(lib, q.contents.policy.contents.d_log_std, F32, sizes[-1])))
        for a, b in zip(*out):
            np.testing.assert_array_equal(a, b)
        lib.free_ppo(loaded)
        lib.free_ppo(ppo)
    finally:
        lib.ppo_gemm_tune(-1, 0)


def test_reference_main_binary_runs(lib, tmp_path):
    """/root/reference/src/main.c, compiled unchanged against include/ and linked to libppo
    (bin/ppo_main, built by `make -C ppo.c_amd main` in the build container): 10 epochs of
    30000 steps on Pendulum-v1 with eval and the checkpoint at the end."""
    exe = os.path.join(ROOT, "ppo.c_amd", "bin", "ppo_main")
    assert os.path.exists(exe), "bin/ppo_main not built (make -C ppo.c_amd main)"
    r = subprocess.run([exe, "64"], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    evals = parse_eval(r.stdout)
    assert len(evals) == 11 and all(n >= 15 for _, _, n in evals)
    assert len(re.findall(r"Epoch: \d+ Entropy: ", r.stdout)) == 10
    size = os.path.getsize(tmp_path / "ppo_model.bin")
    # header 32 B + log_std + μ and V (2 nets: 8 B + 3 activation records + 3 layer records) + 3 Adams
    p_mu, p_v = 3 * 64 + 64 + 64 * 64 + 64 + 64 * 1 + 1, 3 * 64 + 64 + 64 * 64 + 64 + 64 + 1
    acts = 3 * 4 + len("relu\0") * 2 + len("none\0")
    want = 32 + 4 + 2 * (8 + acts + 3 * 8) + 4 * (p_mu + p_v) + 3 * 20 + 8 * (p_mu + p_v + 1)
    assert size == want
    print(r.stdout[-600:])
