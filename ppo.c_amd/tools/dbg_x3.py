#!/usr/bin/env python3
"""Per-layer policy-gradient error of one policy minibatch step (test_single_policy_step setup), x3 vs exact."""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
for p in ("ppo.c_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import ppo_ffi  # noqa: E402
import oracle_ffi  # noqa: E402
import test_gpu_update as T  # noqa: E402
from helpers import F32, nn_grads_packed  # noqa: E402

oracle_ffi.build()
oracle_ffi.load()
oracle = oracle_ffi
lib = ppo_ffi.load()
lib.ppo_set_device(0)
cfg = sys.argv[1] if len(sys.argv) > 1 else "humanoid"
sizes, N = T.CONFIGS[cfg]["sizes"], T.CONFIGS[cfg]["N"]
for serial in ("0", "1"):
    os.environ["PPO_SERIAL"] = serial
    for eng in (0, 1):
        lib.ppo_gemm_f32_engine(eng)
        ppo = T.make_ppo(lib, oracle, sizes, N, init_std=0.7, ent_coeff=0.01)
        mu0, ls0 = T.policy_state(lib, ppo)
        v0 = T.nn_params_packed(lib, ppo.contents.V)
        buf = T.synthetic_buffer(oracle, sizes, mu0, ls0, N, seed=11)
        buf["logprob"] = (buf["logprob"] + np.random.default_rng(3).normal(scale=0.4, size=N)).astype(F32)
        T.load_buffer(lib, ppo, buf)
        oracle.srand(17)
        lib.ppo_update(ppo, 0.99, N, 1, 0, 0, 9)
        lib.ppo_synchronize()
        gmu = nn_grads_packed(lib, ppo.contents.policy.contents.mu)
        oracle.srand(17)
        ref = oracle.ppo_update(sizes, T.RELU(sizes), mu0, ls0, v0, buf, batch_size=N, n_epochs_policy=1,
                                n_epochs_value=0, ent_coeff=0.01, shuffle_mode=0, seed=9)
        x, a = buf["state"], buf["action"]
        acts = oracle.mlp_forward(sizes, T.RELU(sizes), mu0, x)
        mu = oracle.mlp_layer_outputs(sizes, acts, N)[-1]
        lp = oracle.log_prob(mu, ls0, a)
        _, glp, gent = oracle.policy_loss_and_grad(ref["advantage"], lp, buf["logprob"], oracle.entropy(ls0), 0.01, 0.2)
        gmu_out, _ = oracle.log_prob_backwards(mu, ls0, a, glp)
        g_ref = oracle.mlp_backward(sizes, T.RELU(sizes), mu0, x, acts, gmu_out)
        off = 0
        line = []
        for i in range(len(sizes) - 1):
            for nm, cnt in (("W", sizes[i] * sizes[i + 1]), ("b", sizes[i + 1])):
                e = np.abs(gmu[off:off + cnt] - g_ref[off:off + cnt])
                line.append(f"{nm}{i}:{e.max():.2e}/{np.abs(g_ref[off:off + cnt]).max():.2e}@{int(e.argmax())}")
                off += cnt
        print(f"serial={serial} engine={eng}: " + " ".join(line), flush=True)
        lib.free_ppo(ppo)
