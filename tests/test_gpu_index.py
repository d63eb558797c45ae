"""Index work bit-exactly and the world > 1 code paths on one GPU.

* shuffle_buffer / shuffle_buffer_cuda (trajectory_buffer.cu:126-166) against ref_shuffle after the
  same srand — assert_array_equal on every index;
* get_batch / get_batch_cuda (trajectory_buffer.cu:168-220) against ref_get_batch, ragged and
  wrapping minibatches;
* the minibatch gather fused into the layer-0 GEMM: the rows a value / policy step actually trained
  on (the gathered copy the GEMM leaves, NeuralNetwork.d_x0) equal the buffer rows the reference's
  get_batch would pick — host rand() permutation and libppo's device Feistel permutation;
* (the bench's exact C4 configuration is pinned in test_gpu_production.py, its data-parallel shards
  in test_gpu_dp_shards.py);
* PPO_COMM_LOOPBACK=k (k identical ranks in one process): grad_scale 1/k, the Welford all-gather +
  combine, the empty-shard agreement and the comm stream reproduce the one-GPU update;
* the Welford combine on unequal triples against the numpy Chan combine.
"""
import ctypes as C

import numpy as np
import pytest

import ppo_ffi
from gpu_internal import set_host_buffer
from helpers import nn_input_rows, F32, nn_params_packed
from test_gpu_update import load_buffer, make_ppo, policy_state, synthetic_buffer

pytestmark = pytest.mark.gpu

RELU = lambda sizes: [1] * (len(sizes) - 2) + [0]  # noqa: E731
ACTS = lambda sizes: ["relu"] * (len(sizes) - 2) + ["none"]  # noqa: E731


def _filled_buffer(lib, n, S, A, seed, cap=None):
    cap = cap or n
    rng = np.random.default_rng(seed)
    buf = lib.create_trajectory_buffer(cap, S, A)
    fields = dict(state=rng.uniform(-1, 1, (cap, S)).astype(F32), action=rng.normal(size=(cap, A)).astype(F32),
                  logprob=rng.normal(size=cap).astype(F32), advantage=rng.normal(size=cap).astype(F32),
                  adv_target=rng.normal(size=cap).astype(F32))
    set_host_buffer(lib, buf, **fields)
    buf.contents.idx = n % cap
    buf.contents.full = n == cap
    return buf, fields


@pytest.mark.parametrize("n,cap", [(1000, 1000), (4096, 4096), (777, 1024)])
def test_shuffle_bitexact(lib, oracle, n, cap):
    """swap(i, rand() % limit) over limit = full ? capacity : idx (D12 reproduced, not fixed)."""
    buf, _ = _filled_buffer(lib, n, 3, 1, 0, cap)
    oracle.srand(31)
    lib.shuffle_buffer(buf)
    host_perm = np.ctypeslib.as_array(buf.contents.h_random_idx, shape=(n,)).copy()
    oracle.srand(31)
    want = oracle.shuffle(n)
    np.testing.assert_array_equal(host_perm, want)
    oracle.srand(32)
    lib.shuffle_buffer_cuda(buf)                        # the same draws, into HBM
    dev_perm = ppo_ffi.d2h(lib, buf.contents.random_idx, np.int32, n)
    oracle.srand(32)
    np.testing.assert_array_equal(dev_perm, oracle.shuffle(n))
    assert sorted(dev_perm.tolist()) == list(range(n))
    lib.free_trajectory_buffer(buf, True)


@pytest.mark.parametrize("n,S,A,B", [(1000, 17, 6, 64), (1000, 376, 17, 300), (4096, 3, 1, 4096)])
def test_get_batch_bitexact(lib, oracle, n, S, A, B):
    """Minibatch k = rows perm[(k·B + i) % limit] of every field; k past ⌊n/B⌋ wraps."""
    buf, f = _filled_buffer(lib, n, S, A, 1)
    oracle.srand(7)
    lib.shuffle_buffer(buf)
    perm = np.ctypeslib.as_array(buf.contents.h_random_idx, shape=(n,)).copy()
    outs = [np.zeros((B, S), F32), np.zeros((B, A), F32), np.zeros(B, F32), np.zeros(B, F32), np.zeros(B, F32)]
    ks = sorted({0, 1, n // B, n // B + 2})
    for k in ks:                                       # host buffer, host pointers
        lib.get_batch(buf, k, B, *[o.ctypes.data for o in outs])
        rows = perm[(k * B + np.arange(B)) % n]
        for o, name in zip(outs, ("state", "action", "logprob", "advantage", "adv_target")):
            np.testing.assert_array_equal(o.reshape(B, -1), f[name][rows].reshape(B, -1), err_msg=f"{name} k={k}")
    lib.buffer_to_device(buf)
    oracle.srand(8)
    lib.shuffle_buffer_cuda(buf)
    oracle.srand(8)
    perm = oracle.shuffle(n)
    dev = [ppo_ffi.DeviceArray(lib, o.nbytes) for o in outs]
    for k in ks:                                       # device buffer, device pointers
        lib.get_batch_cuda(buf, k, B, *[d.ptr for d in dev])
        rows = perm[(k * B + np.arange(B)) % n]
        for d, o, name in zip(dev, outs, ("state", "action", "logprob", "advantage", "adv_target")):
            got = d.to_numpy(F32, o.size).reshape(B, -1)
            np.testing.assert_array_equal(got, f[name][rows].reshape(B, -1), err_msg=f"{name} k={k} (device)")
    # the oracle's get_batch over the same permutation (ref_get_batch, trajectory_buffer.cu:202-220)
    k = ks[-1]
    ref = oracle.load()
    r_out = [np.zeros_like(o) for o in outs]
    src = [np.ascontiguousarray(f[nm]) for nm in ("state", "action", "logprob", "advantage", "adv_target")]
    ref.ref_get_batch(C.c_void_p(perm.ctypes.data), n, k, B, S, A, *[C.c_void_p(a.ctypes.data) for a in src],
                      *[C.c_void_p(o.ctypes.data) for o in r_out])
    for d, o in zip(dev, r_out):
        np.testing.assert_array_equal(d.to_numpy(F32, o.size), o.ravel())
    for d in dev:
        d.free()
    lib.free_trajectory_buffer(buf, True)


def _gathered_rows(lib, nn_ptr, B, S):
    nn = nn_ptr.contents
    assert nn.bits_m == B and nn.x0_dtype == 0
    return nn_input_rows(lib, nn_ptr, B)


@pytest.mark.parametrize("shuffle_mode", [0, 1])
@pytest.mark.parametrize("B", [512, 2048])            # small-tile fused gather / x3 engine fused gather
def test_fused_gather_rows(lib, oracle, shuffle_mode, B):
    """The rows the k-th value minibatch and the j-th policy minibatch trained on (layer 0's gathered copy)
    are exactly state[perm[(k·B + i) % limit]] for the epoch's permutation: the reference's rand() swap
    shuffle (epochs drawn value-first, ppo.cu:387-447) or libppo's Feistel bijection under the epoch key
    splitmix64(seed) + e."""
    sizes, N = [17, 256, 256, 6], 8192
    ppo = make_ppo(lib, oracle, sizes, N)
    mu0, ls0 = policy_state(lib, ppo)
    buf = synthetic_buffer(oracle, sizes, mu0, ls0, N, seed=2, n_envs=8)
    load_buffer(lib, ppo, buf)
    nb = N // B
    seed = 12345
    for phase in ("value", "policy"):
        k = nb - 2                                   # a late minibatch of the first epoch
        if phase == "value":
            lib.ppo_set_step_limit(ppo, k + 1, 0)
            n_pol, n_val = 0, 2
        else:
            lib.ppo_set_step_limit(ppo, 0, k + 1)
            n_pol, n_val = 1, 3
        oracle.srand(55)
        lib.ppo_update(ppo, 0.99, B, n_pol, n_val, shuffle_mode, seed + (phase == "policy"))
        lib.ppo_synchronize()
        if shuffle_mode == 0:
            oracle.srand(55)
            perms = [oracle.shuffle(N) for _ in range(n_val + n_pol)]
            perm = perms[0] if phase == "value" else perms[n_val]
        else:
            key0 = oracle.splitmix64(seed + (phase == "policy"))
            perm = oracle.feistel_perm(N, key0 if phase == "value" else (key0 + n_val) & (2**64 - 1))
        rows = perm[(k * B + np.arange(B)) % N]
        net = ppo.contents.V if phase == "value" else ppo.contents.policy.contents.mu
        np.testing.assert_array_equal(_gathered_rows(lib, net, B, sizes[0]), buf["state"][rows], err_msg=phase)
    lib.ppo_set_step_limit(ppo, -1, -1)
    lib.free_ppo(ppo)


# ----------------------------------------------------------------------------- world > 1 on one GPU
@pytest.mark.parametrize("k,net,det", [(2, "c3", 1), (4, "c3", 1), (2, "c4", 1), (2, "c3", 0), (2, "c4", 0)])
def test_loopback_ranks_reproduce_one_gpu(lib, oracle, monkeypatch, k, net, det):
    """PPO_COMM_LOOPBACK=k: every world > 1 branch (grad_scale = 1/k, all-gather of Welford triples +
    Chan combine, empty-shard agreement — a min over the k ranks' limits on the comm stream —, comm
    stream, per-layer gradient buckets) over k identical shards.  det = 1 (split-K off): k = 2 the
    value network and advantage statistics equal the one-GPU update bit for bit; k = 4 within the
    rounding of the 3-fold M2 sum; the policy within the log σ-gradient atomics bound.  det = 0: the
    production combination under a communicator — fused output heads, split-K atomics, the top
    bucket carrying layer L-1 and the log σ gradient, gradients cleared by Adam — element by element
    within the bounds of test_short_update_elementwise.  The C4-shaped networks (≈ 718 k parameters)
    are all-reduced in three buckets per step (top two layers, layer 1, layer 0), the C3 ones in one."""
    sizes, N, B = {"c3": ([17, 256, 256, 6], 4096, 512), "c4": ([376, 512, 512, 512, 17], 2048, 1024)}[net]
    if det:
        lib.ppo_gemm_tune(-1, 1)
    out = {}
    try:
        for mode in ("one", "loop"):
            if mode == "loop":
                monkeypatch.setenv("PPO_COMM_LOOPBACK", str(k))
                assert lib.ppo_comm_init(0, 1, None) == 0, lib.ppo_last_error()
                assert lib.ppo_comm_world() == k
            ppo = make_ppo(lib, oracle, sizes, N)
            mu0, ls0 = policy_state(lib, ppo)
            buf = synthetic_buffer(oracle, sizes, mu0, ls0, N, seed=5, n_envs=8)
            load_buffer(lib, ppo, buf)
            lib.ppo_reset_stats(ppo)
            lib.ppo_update(ppo, 0.99, B, 2, 3, 1, 9)
            st = (C.c_double * 7)()
            lib.ppo_read_stats(ppo, st, 7)
            mu, ls = policy_state(lib, ppo)
            out[mode] = dict(stats=np.array(st[:]), v=nn_params_packed(lib, ppo.contents.V), mu=mu, ls=ls,
                             t=ppo.contents.adam_V.contents.time_step)
            # an empty shard: every rank agrees to stop after GAE (no collective left waiting)
            b = ppo.contents.buffer.contents
            b.idx, b.full = 0, False
            lib.ppo_update(ppo, 0.99, B, 2, 3, 1, 9)
            lib.ppo_synchronize()
            assert ppo.contents.adam_V.contents.time_step == out[mode]["t"]
            lib.free_ppo(ppo)
            if mode == "loop":
                lib.ppo_comm_finalize()
                monkeypatch.delenv("PPO_COMM_LOOPBACK")
    finally:
        lib.ppo_gemm_tune(-1, 0)
    a, b = out["one"], out["loop"]
    assert lib.ppo_comm_world() == 1
    if not det:
        lr, n_steps = 3e-4, 3 * (N // B)
        for key in ("v", "mu", "ls"):
            err = np.abs(a[key].astype(np.float64) - b[key])
            assert err.max() <= 2 * lr * n_steps, (key, err.max())
            assert (err <= 0.1 * lr).mean() >= 0.99, (key, (err <= 0.1 * lr).mean())
        np.testing.assert_allclose(a["stats"][5:], b["stats"][5:], rtol=1e-6)
        np.testing.assert_allclose(a["stats"][:4], b["stats"][:4], rtol=1e-3, atol=1e-6)
        return
    if k == 2:
        np.testing.assert_array_equal(a["v"], b["v"])
        np.testing.assert_array_equal(a["stats"][5:], b["stats"][5:])          # advantage mean / std
    else:
        np.testing.assert_allclose(a["v"], b["v"], rtol=0, atol=2 * 3e-4)
        np.testing.assert_allclose(a["stats"][5:], b["stats"][5:], rtol=1e-6)
    np.testing.assert_allclose(a["stats"][:4], b["stats"][:4], rtol=1e-5, atol=1e-6)
    for key in ("mu", "ls"):
        err = np.abs(a[key] - b[key])
        assert err.max() <= 2 * 3e-4, (key, err.max())
        assert (err > 1e-6).mean() < 0.01, (key, (err > 1e-6).mean())


def test_welford_combine_unequal(lib):
    """(n, mean, M2) triples of very different sizes and means — including empty parts — combine to the
    statistics of the concatenated data (the numpy two-pass values), as after the all-gather."""
    rng = np.random.default_rng(0)
    parts, data = [], []
    for n, mu, sd in ((1, 3.0, 0.0), (1000, -2.0, 0.5), (0, 0.0, 0.0), (37, 10.0, 4.0), (250000, 0.1, 1.0),
                      (5, -7.0, 2.0)):
        x = (mu + sd * rng.normal(size=n)).astype(np.float64)
        data.append(x)
        m = x.mean() if n else 0.0
        parts.append((float(n), m, float(((x - m) ** 2).sum()) if n else 0.0))
    d_parts = ppo_ffi.DeviceArray.from_numpy(lib, np.array(parts, np.float64).ravel())
    d_out = ppo_ffi.DeviceArray(lib, 3 * 8)
    lib.ppo_welford_combine(d_parts.ptr, len(parts), d_out.ptr)
    n, mean, m2 = d_out.to_numpy(np.float64, 3)
    allx = np.concatenate(data)
    assert n == allx.size
    assert abs(mean - allx.mean()) <= 1e-12 * max(1.0, abs(allx.mean()))
    assert abs(m2 - ((allx - allx.mean()) ** 2).sum()) <= 1e-10 * m2
    d_parts.free()
    d_out.free()
