"""The multi-workgroup single-launch phases at the reference's B = 64 (main.c:34's minibatch) against
the multi-launch loop and the oracle (reference ppo.cu:395-443): csrc/cluster.hip for S → 256 → 256 →
O networks (config C3's) and csrc/cluster_deep.hip for S → 512 → 512 → 512 → O (config C4's).

ppo_update takes it by itself for these shapes at B = 64 on one GPU; PPO_NO_CLUSTER=1 forces the
multi-launch loop.  From identical state both must give the same minibatch gradients (stated fp32 GEMM
tolerance), the same Adam step counts and host rand() consumption, and over many steps the same
parameter motion; against the oracle, single steps element by element and the first 16 + 16 steps of
an update (the bounds of test_short_update_elementwise); over long runs, within the oracle's own
chaos floor (its self-drift under a re-association of every product, measured live).
"""
import ctypes as C
import os

import numpy as np
import pytest

import ppo_ffi
from helpers import F32, assert_gemm_close, assert_rel_close, nn_grads_packed, nn_params_packed

pytestmark = pytest.mark.gpu

LIBC = C.CDLL("libc.so.6")
C3 = [17, 256, 256, 6]
C4 = [376, 512, 512, 512, 17]
NETS = pytest.mark.parametrize("sizes", [C3, C4], ids=["c3", "c4"])
RELU = lambda sizes: [1] * (len(sizes) - 2) + [0]  # noqa: E731
LR = 3e-4


def run(lib, sizes, N, B, n_pol, n_val, shuffle, cluster, seed=21, limit=None, ent=0.01):
    if cluster:
        os.environ.pop("PPO_NO_CLUSTER", None)
    else:
        os.environ["PPO_NO_CLUSTER"] = "1"
    try:
        LIBC.srand(seed)
        acts = ["relu"] * (len(sizes) - 2) + ["none"]
        ppo = lib.create_ppo(ppo_ffi.c_strings(acts), ppo_ffi.c_ints(sizes), len(sizes), N, 3e-4, 3e-4, 0.95, 0.2,
                             ent, 1.0, True)
        E = max(1, N // 256)
        lib.ppo_fill_synthetic(ppo, E, N // E, 17, 1.0 / 200)
        pol = ppo.contents.policy.contents
        v0 = nn_params_packed(lib, ppo.contents.V)
        mu0 = nn_params_packed(lib, pol.mu)
        ls0 = ppo_ffi.d2h(lib, pol.d_log_std, F32, pol.action_size)
        b = ppo.contents.buffer.contents
        buf = dict(state=ppo_ffi.d2h(lib, b.d_state_p, F32, N * sizes[0]).reshape(N, sizes[0]),
                   next_state=ppo_ffi.d2h(lib, b.d_next_state_p, F32, N * sizes[0]).reshape(N, sizes[0]),
                   action=ppo_ffi.d2h(lib, b.d_action_p, F32, N * sizes[-1]).reshape(N, sizes[-1]),
                   reward=ppo_ffi.d2h(lib, b.d_reward_p, F32, N), logprob=ppo_ffi.d2h(lib, b.d_logprob_p, F32, N),
                   terminated=ppo_ffi.d2h(lib, b.d_terminated_p, np.uint8, N),
                   truncated=ppo_ffi.d2h(lib, b.d_truncated_p, np.uint8, N))
        if limit:
            lib.ppo_set_step_limit(ppo, limit[0], limit[1])
        lib.ppo_reset_stats(ppo)
        LIBC.srand(seed + 1)
        lib.ppo_update(ppo, 0.99, B, n_pol, n_val, shuffle, 9)
        lib.ppo_synchronize()
        assert lib.ppo_last_error() in (b"", None), lib.ppo_last_error()
        stats = (C.c_double * 7)()
        lib.ppo_read_stats(ppo, stats, 7)
        out = dict(stats=np.array(stats[:4]), next_rand=LIBC.rand(), v0=v0, mu0=mu0, ls0=ls0, buf=buf,
                   v=nn_params_packed(lib, ppo.contents.V), gv=nn_grads_packed(lib, ppo.contents.V),
                   mu=nn_params_packed(lib, pol.mu), gmu=nn_grads_packed(lib, pol.mu),
                   ls=ppo_ffi.d2h(lib, pol.d_log_std, F32, pol.action_size),
                   gls=ppo_ffi.d2h(lib, pol.d_log_std_grad, F32, pol.action_size),
                   multi=ppo.contents.V.contents.bits_m == B or pol.mu.contents.bits_m == B,
                   t=(ppo.contents.adam_V.contents.time_step, ppo.contents.adam_policy.contents.time_step,
                      ppo.contents.adam_entropy.contents.time_step))
        lib.ppo_set_step_limit(ppo, -1, -1)
        lib.free_ppo(ppo)
        return out
    finally:
        os.environ.pop("PPO_NO_CLUSTER", None)


@NETS
@pytest.mark.parametrize("shuffle", [0, 1])
def test_cluster_single_steps_match_multilaunch(lib, oracle, shuffle, sizes):
    """one value step, then one policy step (B = 64): the same gradients and Adam deltas"""
    N, B = 4096, 64
    for n_pol, n_val in ((0, 1), (1, 0)):                  # one epoch each, capped at one step
        a = run(lib, sizes, N, B, n_pol, n_val, shuffle, cluster=True, limit=(n_val, n_pol))
        b = run(lib, sizes, N, B, n_pol, n_val, shuffle, cluster=False, limit=(n_val, n_pol))
        assert not a["multi"] and b["multi"], "the cluster path did not run (or the fallback did not)"
        assert a["t"] == b["t"] == (n_val, n_pol, n_pol)
        assert a["next_rand"] == b["next_rand"], "host rand() stream consumed differently"
        np.testing.assert_allclose(a["stats"], b["stats"], rtol=2e-4, atol=1e-6)
        assert_gemm_close(a["gv"], b["gv"], B, "value grads")
        assert_gemm_close(a["gmu"], b["gmu"], B, "policy grads")
        if n_pol:
            assert_rel_close(a["gls"], b["gls"], 1e-4, 1e-6, "log σ grad")
        for k in ("v", "mu", "ls"):
            err = np.abs(a[k] - b[k])
            assert err.max() <= 2 * LR * 1.0001 + 1e-7, (k, err.max())
            assert (err > 1e-6).mean() < 0.01, (k, (err > 1e-6).mean())


@NETS
def test_cluster_first_steps_vs_oracle(lib, oracle, sizes):
    """the first 16 value and 16 policy steps of an update at B = 64 on the cluster path against the
    oracle's update of the same buffer, element by element (≥ 99 % within 0.1·lr)"""
    oracle.load(use_openblas=True)
    N, B, n = 16384, 64, 16
    a = run(lib, sizes, N, B, 1, 1, 1, cluster=True, limit=(n, n), ent=0.0)
    assert not a["multi"]
    ref = oracle.ppo_update(sizes, RELU(sizes), a["mu0"], a["ls0"], a["v0"], a["buf"], batch_size=B, n_epochs_policy=1,
                            n_epochs_value=1, shuffle_mode=1, seed=9, max_value_steps=n, max_policy_steps=n)
    assert a["t"] == (ref["t_v"], ref["t_mu"], ref["t_ent"]) == (n, n, n)
    for got, want, what in ((a["v"], ref["v"], "V"), (a["mu"], ref["mu"], "mu"), (a["ls"], ref["log_std"], "log_std")):
        err = np.abs(got.astype(np.float64) - want)
        q = float((err <= 0.1 * LR).mean())
        print(f"cluster {sizes} {what}: max err {err.max() / LR:.4f} lr, {100 * q:.3f} % within 0.1 lr")
        assert err.max() <= 2 * LR * n, f"{what}: max err {err.max()}"
        assert q >= 0.99, f"{what}: only {q * 100:.2f} % within 0.1·lr"
    np.testing.assert_allclose(a["stats"][0], ref["sum_v_loss"], rtol=1e-3)
    np.testing.assert_allclose(a["stats"][2], ref["sum_policy_loss"], rtol=1e-3, atol=1e-5)


def oracle_motion(oracle, a, sizes, lim, n_pol, n_val, mode, ent=0.0):
    """The oracle's update of run()'s buffer from run()'s initial state (Feistel order, seed 9), its
    products re-associated per `mode` (oracle_ffi.blas_mode: 0 proper, 1 split-K halves, 2 double
    products rounded once) — returns (value motion, policy motion).  16 OpenBLAS threads: measured
    bit-identical to one thread (profiles/r05_oracle_chaos_floor.txt), only faster."""
    lib = oracle.load(use_openblas=True)
    oracle.blas_mode(mode)
    lib.ref_blas_threads(16)
    try:
        ref = oracle.ppo_update(sizes, RELU(sizes), a["mu0"], a["ls0"], a["v0"], a["buf"], batch_size=64,
                                n_epochs_policy=n_pol, n_epochs_value=n_val, shuffle_mode=1, seed=9,
                                max_value_steps=lim[0], max_policy_steps=lim[1], ent_coeff=ent)
    finally:
        oracle.blas_mode(0)
        lib.ref_blas_threads(1)
    return ref["v"] - a["v0"], ref["mu"] - a["mu0"]


def cos_ratio(d, dr):
    d, dr = d.astype(np.float64), dr.astype(np.float64)
    return float(d @ dr / (np.linalg.norm(d) * np.linalg.norm(dr))), float(np.linalg.norm(d) / np.linalg.norm(dr))


# Long runs are chaotic: a ReLU mask or clip branch that flips at z ≈ 0 changes a gradient outright and
# Adam normalises every element, so two valid fp32 evaluations of the same update decorrelate as they
# go, at a rate that varies with the buffer and the perturbation (tools/chaos_floor.py: C4, 512 policy
# steps, oracle self-drift cos 0.62 – 1.00 across seeds).  The bound is therefore relative to that floor,
# measured live on the same buffer and initial state: the oracle against itself with every product
# re-associated (split-K halves) and in double-precision products (profiles/r05_oracle_chaos_floor.txt,
# r05_gpu_drift_vs_chaos_floor.txt — on this test's buffer at 512 policy steps: oracle self-drift cos
# 0.62 / 0.63, multi-launch 0.60, cluster 0.78; at 64 steps 0.989 / 0.991 vs 0.989 / 0.9999).  A GPU path
# may decorrelate from the oracle at most CHAOS_FACTOR times as much as the oracle does from itself,
# plus CHAOS_SLACK (one sample of a chaotic process against two):
# 1 − cos_gpu ≤ CHAOS_FACTOR · (1 − min cos_floor) + CHAOS_SLACK.  A defect outruns it already at 64 steps.
# Round 6: CHAOS_FACTOR 2.0 → 1.25 — the measured GPU drift is 1.05× (512 policy steps, multi-launch) and
# 1.16× (the whole update's μ) the oracle's own; every check prints its margin (1 − cos_gpu) / (1 − floor)
# (profiles/r06_chaos_margins.txt).  And an absolute floor where the oracle's is low: at 512 steps a GPU
# path must keep cos ≥ CHAOS_ABS_MIN against the oracle whatever the floor.
# The whole C4 update (3584 steps, 7× the longest step test) keeps more slack: its multi-launch μ margin
# measured 1.16 (round 5) and 1.22 (round 6, profiles/r06_chaos_margins.txt) — run-to-run spread of a
# chaotic process whose split-K atomics reorder sums differently on every run.
CHAOS_FACTOR, CHAOS_SLACK, CHAOS_SLACK_WHOLE, CHAOS_ABS_MIN = 1.25, 0.02, 0.05, 0.5


def assert_within_chaos_floor(cos_gpu, floor_cos, what, slack=CHAOS_SLACK):
    bound = 1 - (CHAOS_FACTOR * (1 - min(floor_cos)) + slack)
    margin = (1 - cos_gpu) / max(1e-12, 1 - min(floor_cos))
    print(f"CHAOS_MARGIN {what}: 1-cos {1 - cos_gpu:.5f} floor 1-cos {1 - min(floor_cos):.5f} margin {margin:.3f} "
          f"(allowed {CHAOS_FACTOR} + slack {slack})")
    assert cos_gpu >= bound, f"{what}: cos {cos_gpu:.5f} < {bound:.5f} (oracle self-drift floor {floor_cos})"
    assert cos_gpu >= CHAOS_ABS_MIN, f"{what}: cos {cos_gpu:.5f} < absolute minimum {CHAOS_ABS_MIN}"


@NETS
@pytest.mark.parametrize("shuffle", [0, 1])
def test_cluster_full_update_matches_multilaunch(lib, oracle, shuffle, sizes):
    """a whole update (10 value + 4 policy epochs of 64-row minibatches over 16,384 transitions:
    2560 + 1024 steps) on both paths: step counts, rand() use, losses and parameter motion.  C4: each
    path's motion against the oracle's update, bounded by the oracle's own chaos floor over the same
    update (Feistel order; CHAOS_FACTOR, CHAOS_SLACK above)."""
    N, B = 16384, 64
    a = run(lib, sizes, N, B, 4, 10, shuffle, cluster=True)
    b = run(lib, sizes, N, B, 4, 10, shuffle, cluster=False)
    assert not a["multi"] and b["multi"]
    assert a["t"] == b["t"] == (2560, 1024, 1024)
    assert a["next_rand"] == b["next_rand"]
    assert abs(a["stats"][0] - b["stats"][0]) <= 0.02 * abs(b["stats"][0])
    assert abs(a["stats"][2] - b["stats"][2]) <= 0.05 * abs(b["stats"][2]) + 1e-3
    if sizes == C3:           # C3 stays near-deterministic (oracle self-drift cos ≥ 0.9995 at 512 steps)
        for k, k0 in (("v", "v0"), ("mu", "mu0")):
            cos, ratio = cos_ratio(a[k] - a[k0], b[k] - b[k0])
            assert cos > 0.95, (k, cos)
            assert abs(ratio - 1) < 0.1, k
        return
    if shuffle != 1:          # the oracle floor is measured in the device (Feistel) minibatch order
        return
    ref = [oracle_motion(oracle, a, sizes, (-1, -1), 4, 10, mode, ent=0.01) for mode in (0, 1, 2)]
    for idx, k, k0 in ((0, "v", "v0"), (1, "mu", "mu0")):
        floor = [cos_ratio(ref[1][idx], ref[0][idx]), cos_ratio(ref[2][idx], ref[0][idx])]
        spread = max(abs(r - 1) for _, r in floor)
        for name, x in (("cluster", a), ("multi-launch", b)):
            cos, ratio = cos_ratio(x[k] - x[k0], ref[0][idx])
            print(f"C4 full update {k}: {name} vs oracle cos {cos:.5f} ratio {ratio:.4f} | oracle self-drift "
                  f"split-K {floor[0][0]:.5f} ({floor[0][1]:.4f}) double {floor[1][0]:.5f} ({floor[1][1]:.4f})")
            assert_within_chaos_floor(cos, [c for c, _ in floor], f"C4 full update {k} {name}", CHAOS_SLACK_WHOLE)
            assert abs(ratio - 1) <= spread + 0.1, (k, name, ratio, floor)


TIMEOUT_CHILD = r"""
import ctypes as C, sys
sys.path[:0] = [sys.argv[1]]
import ppo_ffi
lib = ppo_ffi.load()
assert lib.ppo_set_device(0) == 0
sizes = [int(s) for s in sys.argv[2].split(",")]
acts = ["relu"] * (len(sizes) - 2) + ["none"]
ppo = lib.create_ppo(ppo_ffi.c_strings(acts), ppo_ffi.c_ints(sizes), len(sizes), 4096, 3e-4, 3e-4, 0.95, 0.2,
                     0.0, 1.0, True)
lib.ppo_fill_synthetic(ppo, 16, 256, 17, 1.0 / 200)
lib.ppo_update(ppo, 0.99, 64, 1, 1, 1, 9)
print("UPDATE RETURNED", flush=True)
"""


@NETS
def test_cluster_barrier_timeout_fails_loudly(lib, sizes, tmp_path):
    """A grid-barrier timeout ends the update that launched the phases — not the next update, never
    silently (the timed-out phase leaves its parameters and Adam state half-written).  The test hook
    PPO_CLUSTER_TEST_TIMEOUT=1 bounds every barrier wait at 0 ticks: the first workgroup to wait at a
    barrier that is not complete times out, sets the error word, and every other workgroup leaves at its
    next wait.  Run in a child process (the update exits it with status 1)."""
    import subprocess
    import sys

    env = dict(os.environ, PPO_CLUSTER_TEST_TIMEOUT="1")
    env.pop("PPO_NO_CLUSTER", None)
    pkg = os.path.dirname(ppo_ffi.__file__)
    r = subprocess.run([sys.executable, "-c", TIMEOUT_CHILD, pkg, ",".join(map(str, sizes))], env=env,
                       capture_output=True, text=True, timeout=120, cwd=tmp_path)
    assert r.returncode == 1, (r.returncode, r.stdout[-500:], r.stderr[-1500:])
    assert "timed out at a grid barrier" in r.stderr, r.stderr[-1500:]
    assert "UPDATE RETURNED" not in r.stdout


@pytest.mark.parametrize("steps", [64, 128, 512])
@pytest.mark.parametrize("phase", ["value", "policy"])
def test_long_run_drift_within_oracle_chaos_floor(lib, oracle, phase, steps):
    """C4 networks, 64, 128 and 512 value or policy steps (two epochs, the epoch boundary included): both GPU
    B = 64 paths (the cluster phase and the multi-launch loop) against the oracle, bounded by the
    oracle's own self-drift on the same buffer — the oracle with every product split-K re-associated,
    and in double-precision products rounded once (CHAOS_FACTOR, CHAOS_SLACK above); motion norms
    within the floor's norm spread + 0.1.  A defect would outrun the floor already at 64 steps."""
    N, B = 16384, 64
    lim, k, idx = ((steps, 0), "v", 0) if phase == "value" else ((0, steps), "mu", 1)
    a = run(lib, C4, N, B, 4, 10, 1, cluster=True, limit=lim, ent=0.0)
    b = run(lib, C4, N, B, 4, 10, 1, cluster=False, limit=lim, ent=0.0)
    assert not a["multi"] and b["multi"]
    ref = [oracle_motion(oracle, a, C4, lim, 4, 10, mode)[idx] for mode in (0, 1, 2)]
    floor = [cos_ratio(ref[1], ref[0]), cos_ratio(ref[2], ref[0])]
    fcos = [c for c, _ in floor]
    spread = max(abs(r - 1) for _, r in floor)
    for name, x in (("cluster", a), ("multi-launch", b)):
        cos, ratio = cos_ratio(x[k] - x[k + "0"], ref[0])
        print(f"C4 {steps} {phase} steps vs oracle: {name} cos {cos:.5f} ratio {ratio:.4f} | oracle self-drift "
              f"split-K {floor[0][0]:.5f} ({floor[0][1]:.4f}) double {floor[1][0]:.5f} ({floor[1][1]:.4f})")
        assert_within_chaos_floor(cos, fcos, f"{name} {phase} {steps}")
        assert abs(ratio - 1) <= spread + 0.1, (name, ratio, floor)
