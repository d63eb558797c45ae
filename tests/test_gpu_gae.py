"""GAE (compute_gae_cuda: csrc/gae.hip's exact segmented scan, Welford triples, normalisation) against
the reference recursion restated in the oracle (ref_gae, reference ppo.cu:326-369) — property tests.

SURVEY §4.3 asks for random done masks, random segment lengths, N not a multiple of the scan tile
(2048 transitions per workgroup) and the all-done / no-done extremes.  V is the identity 1 → 1 network
(W = 1, b = 0: V(s) = s exactly), so v and v′ are exact inputs and the comparison isolates the scan,
the Welford statistics and the normalisation.  Tolerances (stated in DESIGN.md §3): targets
v + A within 1e-5 relative + 1e-5 absolute (values are O(1); the parallel scan re-associates the
γλ-products), normalised advantages within 1e-4 relative + 1e-4 absolute of the exact statistics of
the oracle's advantages (helpers.assert_normalised_close: the reference's fp32 running sums drift by
more than that at N ≳ 1e5, and the oracle restates them faithfully).

Also: "rollout-linked" buffers, where next_state[t] is bitwise state[t+1] inside an episode, run the
V(next_state) reuse (next_value_map_kernel) on every non-terminal row; the production-size GAE pins
(C3, C4 at N = 1,048,576, the C5 shard) are in test_gpu_production.py.
"""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from gpu_internal import gae_device
from helpers import F32, assert_normalised_close, assert_rel_close

pytestmark = pytest.mark.gpu

CHUNK = 2048                      # transitions per scan workgroup (gae.hip CHUNK)
GAMMA, LAM = 0.99, 0.95


def _episode_flags(rng, n, mode, seg_max):
    """terminated / truncated flags of an n-transition buffer.
    segments: random segment lengths in [1, seg_max], each segment ends terminated or truncated;
    no_done: no flag anywhere (one segment, A_N = 0 beyond the end, D6); all_term / all_trunc: every
    transition ends an episode; bernoulli: terminated with p = 1/200 plus truncation every seg_max."""
    term = np.zeros(n, np.uint8)
    trunc = np.zeros(n, np.uint8)
    if mode == "segments":
        t = 0
        while t < n:
            t += int(rng.integers(1, seg_max + 1))
            end = min(t, n) - 1
            if rng.uniform() < 0.5:
                term[end] = 1
            else:
                trunc[end] = 1
    elif mode == "all_term":
        term[:] = 1
    elif mode == "all_trunc":
        trunc[:] = 1
    elif mode == "bernoulli":
        term = (rng.uniform(size=n) < 1 / 200).astype(np.uint8)
        trunc[seg_max - 1::seg_max] = 1
        trunc &= 1 - term
    return term, trunc


def _check(lib, oracle, v, vn, r, term, trunc, what):
    adv_ref, tgt_ref, mean_ref, std_ref = oracle.gae(v, vn, r, term, trunc, GAMMA, LAM)
    adv, tgt = gae_device(lib, v, vn, r, term, trunc, GAMMA, LAM)
    assert_rel_close(tgt, tgt_ref, 1e-5, 1e-5, f"{what}: adv_target")
    assert_normalised_close(adv, adv_ref, mean_ref, std_ref, f"{what}: normalised advantage")
    raw, raw_ref = tgt.astype(np.float64) - v, tgt_ref.astype(np.float64) - v
    assert abs(raw.mean() - raw_ref.mean()) <= 1e-5 * max(1.0, raw_ref.std()), what
    return adv, tgt


def _inputs(rng, n, linked, term, trunc):
    v = rng.normal(size=n).astype(F32)
    if linked:                           # next_state[t] = state[t+1] inside an episode (the rollout layout)
        vn = np.empty(n, F32)
        vn[:-1] = v[1:]
        ends = (term | trunc).astype(bool)
        ends[-1] = True
        vn[ends] = rng.normal(size=int(ends.sum())).astype(F32)
    else:
        vn = rng.normal(size=n).astype(F32)
    r = rng.normal(size=n).astype(F32)
    return v, vn, r


SIZES = [1, 2, 3, 7, 63, 64, 65, 255, 257, CHUNK - 1, CHUNK, CHUNK + 1, 3000, 2 * CHUNK - 1, 3 * CHUNK + 5,
         10_007, 65_537]


@settings(max_examples=40, deadline=None, suppress_health_check=list(HealthCheck), derandomize=True)
@given(n=st.sampled_from(SIZES), mode=st.sampled_from(["segments", "no_done", "all_term", "all_trunc", "bernoulli"]),
       seg_max=st.sampled_from([1, 2, 5, 50, 200, 1000, 5000]), linked=st.booleans(), seed=st.integers(0, 2**31))
def test_gae_properties(lib, oracle, n, mode, seg_max, linked, seed):
    """Random segment lengths / done masks / sizes: the scan, statistics and normalisation vs ref_gae."""
    rng = np.random.default_rng(seed)
    term, trunc = _episode_flags(rng, n, mode, seg_max)
    v, vn, r = _inputs(rng, n, linked, term, trunc)
    _check(lib, oracle, v, vn, r, term, trunc, f"n={n} {mode} seg_max={seg_max} linked={linked}")


@pytest.mark.parametrize("mode,seg_max", [("segments", 4096), ("no_done", 1), ("all_term", 1), ("bernoulli", 1000)])
def test_gae_large_non_power_of_two(lib, oracle, mode, seg_max):
    """N = 1,000,003 (prime: 489 scan workgroups, the last one 627 transitions) in every done regime;
    the no-done buffer chains one segment through every workgroup carry."""
    n = 1_000_003
    rng = np.random.default_rng(7)
    term, trunc = _episode_flags(rng, n, mode, seg_max)
    v, vn, r = _inputs(rng, n, mode != "no_done", term, trunc)
    adv, tgt = _check(lib, oracle, v, vn, r, term, trunc, f"N=1,000,003 {mode}")
    # normalised advantages: population mean 0, σ 1 (ppo.cu:355-368)
    assert abs(float(adv.astype(np.float64).mean())) < 1e-5
    assert abs(float(adv.astype(np.float64).std()) - 1.0) < 1e-4


def test_gae_all_done_is_delta(lib, oracle):
    """Every transition terminated: A_t = δ_t = r_t − v_t exactly (the scan carries nothing)."""
    n = 3000
    rng = np.random.default_rng(11)
    v, vn, r = (rng.normal(size=n).astype(F32) for _ in range(3))
    term, trunc = np.ones(n, np.uint8), np.zeros(n, np.uint8)
    _, tgt = gae_device(lib, v, vn, r, term, trunc, GAMMA, LAM)
    delta = r + np.float32(GAMMA) * vn * np.float32(0) - v
    np.testing.assert_array_equal(tgt, v + delta)


def test_gae_linear_in_rewards(lib, oracle):
    """The unnormalised advantage is linear in the rewards: target(r1 + r2) − v = (target(r1) − v) +
    (target(r2) − v) up to fp32 rounding, at a size with many scan workgroups and segments."""
    n = 5 * CHUNK + 17
    rng = np.random.default_rng(3)
    term, trunc = _episode_flags(rng, n, "segments", 700)
    v = np.zeros(n, F32)
    vn = np.zeros(n, F32)
    r1, r2 = rng.normal(size=n).astype(F32), rng.normal(size=n).astype(F32)
    _, t1 = gae_device(lib, v, vn, r1, term, trunc, GAMMA, LAM)
    _, t2 = gae_device(lib, v, vn, r2, term, trunc, GAMMA, LAM)
    _, t12 = gae_device(lib, v, vn, (r1 + r2).astype(F32), term, trunc, GAMMA, LAM)
    assert_rel_close(t12, t1.astype(np.float64) + t2, 1e-5, 1e-5, "linearity")
