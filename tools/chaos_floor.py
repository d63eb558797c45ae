#!/usr/bin/env python3
"""The oracle's own fp32 chaos floor over long B = 64 runs (reference ppo.cu:398-443, main.c:34).

Long PPO runs amplify rounding: a ReLU mask or a clip branch that flips at z ≈ 0 changes a gradient
outright, Adam normalises each element, and the parameter trajectories separate.  How far two
*equally valid* fp32 implementations drift apart is measured here on the CPU, with the oracle against
itself: the oracle proper (OpenBLAS sgemm, one thread — main.c:18) against the same update with every
product re-associated (split-K halves), evaluated in double and rounded once (the most accurate
fp32-output BLAS), or on 8 OpenBLAS threads.  Same initial state, same buffer, same minibatch order
(Feistel shuffle, seed 9).  The statistic is the one tests/test_gpu_cluster.py asserts on the GPU
paths: cosine and norm ratio of the parameter motion (θ_n − θ_0) against the oracle proper's.

CPU only (test infrastructure: imports the oracle).  Usage: python tools/chaos_floor.py [--steps 512]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle")]
import oracle_ffi  # noqa: E402

C3 = [17, 256, 256, 6]
C4 = [376, 512, 512, 512, 17]
F32 = np.float32


def relu_flags(sizes):
    return [1] * (len(sizes) - 2) + [0]


def make_buffer(sizes, params_mu, log_std, N, E, seed, p_term=1.0 / 200):
    """A synthetic rollout with ppo_fill_synthetic's statistics (host/ppo.c): U(−1, 1) observations,
    env-major segments of T = N/E steps ending truncated, Bernoulli(p) terminations, next_state linked
    to the following row inside an episode, rewards N(0, 0.1²), actions μ(s) + σ·ε and their log-prob."""
    rng = np.random.default_rng(seed)
    S, A = sizes[0], sizes[-1]
    T = N // E
    state = rng.uniform(-1, 1, (N, S)).astype(F32)
    term = (rng.random(N) < p_term).astype(np.uint8)
    trunc = np.zeros(N, np.uint8)
    trunc[T - 1::T] = 1
    trunc[term.astype(bool)] = 0
    nxt = np.empty_like(state)
    nxt[:-1] = state[1:]
    done = (term | trunc).astype(bool)
    nxt[done] = rng.uniform(-1, 1, (int(done.sum()), S)).astype(F32)
    nxt[-1] = rng.uniform(-1, 1, S).astype(F32)
    reward = (rng.standard_normal(N) * 0.1).astype(F32)
    acts = oracle_ffi.mlp_forward(sizes, relu_flags(sizes), params_mu, state)
    mu = oracle_ffi.mlp_layer_outputs(sizes, acts, N)[-1]
    action = (mu + np.exp(log_std) * rng.standard_normal((N, A))).astype(F32)
    logprob = oracle_ffi.log_prob(mu, log_std, action)
    return dict(state=state, next_state=nxt, action=action, reward=reward, logprob=logprob, terminated=term,
                truncated=trunc)


def setup(sizes, N, seed):
    lib = oracle_ffi.load(use_openblas=True)
    oracle_ffi.srand(seed)
    mu0 = oracle_ffi.mlp_init(sizes)
    v0 = oracle_ffi.mlp_init(sizes[:-1] + [1])
    ls0 = np.zeros(sizes[-1], F32)
    buf = make_buffer(sizes, mu0, ls0, N, max(1, N // 256), seed + 1)
    return lib, mu0, v0, ls0, buf


def motion(sizes, mu0, v0, ls0, buf, phase, steps, B=64, mode=0, threads=1):
    lib = oracle_ffi.load(use_openblas=True)
    oracle_ffi.blas_mode(mode)
    lib.ref_blas_threads(threads)
    try:
        lim = (steps, 0) if phase == "value" else (0, steps)
        ref = oracle_ffi.ppo_update(sizes, relu_flags(sizes), mu0, ls0, v0, buf, batch_size=B, n_epochs_policy=4,
                                    n_epochs_value=10, shuffle_mode=1, seed=9, max_value_steps=lim[0],
                                    max_policy_steps=lim[1])
    finally:
        oracle_ffi.blas_mode(0)
        lib.ref_blas_threads(1)
    return (ref["v"] - v0) if phase == "value" else (ref["mu"] - mu0)


def cos_ratio(d, dr):
    d, dr = d.astype(np.float64), dr.astype(np.float64)
    return float(d @ dr / (np.linalg.norm(d) * np.linalg.norm(dr))), float(np.linalg.norm(d) / np.linalg.norm(dr))


VARIANTS = (("split-K halves", 1, 1), ("double products", 2, 1), ("8 BLAS threads", 0, 8))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, nargs="+", default=[16, 64, 256, 512])
    ap.add_argument("--nets", default="c4,c3")
    ap.add_argument("--seeds", type=int, nargs="+", default=[21])
    ap.add_argument("--N", type=int, default=16384)
    args = ap.parse_args()
    oracle_ffi.build()
    nets = {"c3": C3, "c4": C4}
    print(f"# oracle chaos floor: B = 64, N = {args.N}, Feistel minibatch order seed 9; cosine / norm ratio of "
          f"the parameter motion vs the oracle proper (OpenBLAS sgemm, 1 thread)", flush=True)
    for name in args.nets.split(","):
        sizes = nets[name]
        for seed in args.seeds:
            _, mu0, v0, ls0, buf = setup(sizes, args.N, seed)
            for phase in ("value", "policy"):
                for steps in args.steps:
                    t0 = time.time()
                    base = motion(sizes, mu0, v0, ls0, buf, phase, steps)
                    again = motion(sizes, mu0, v0, ls0, buf, phase, steps)
                    rep = "bit-identical" if np.array_equal(base, again) else "NOT reproducible"
                    cols = []
                    for label, mode, thr in VARIANTS:
                        d = motion(sizes, mu0, v0, ls0, buf, phase, steps, mode=mode, threads=thr)
                        c, r = cos_ratio(d, base)
                        same = " (bit-identical)" if np.array_equal(d, base) else ""
                        cols.append(f"{label}: cos {c:.5f} ratio {r:.4f}{same}")
                    print(f"{name} seed {seed} {phase:6s} {steps:4d} steps [{rep}, {time.time() - t0:.0f} s] | "
                          + " | ".join(cols), flush=True)


if __name__ == "__main__":
    main()
