"""Per-tensor error of one C5 bf16 policy minibatch (the test_gpu_production C5 step) against the bf16
emulation and the fp32 oracle: which layer / tensor carries the largest deviation.

    python tools/diag_c5_policy.py [B]
"""
import os
import sys

import numpy as np

R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(R, "ppo.c_amd"), os.path.join(R, "oracle"), os.path.join(R, "tests")]
import oracle_ffi as oracle  # noqa: E402
import ppo_ffi  # noqa: E402
from helpers import F32, nn_grads_packed, nn_params_packed  # noqa: E402
from test_gpu_bf16 import bf16, unpack  # noqa: E402
from test_gpu_production import C5, bench_ppo, emu_backward, emu_forward  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
lib = ppo_ffi.load()
oracle.load(use_openblas=True)
oracle.load().ref_blas_threads(16)
ppo = bench_ppo(lib, oracle, C5, 64, 8192, seed=5151, dtype=1)
N, A, seed = 64 * 8192, 17, 59
b = ppo.contents.buffer.contents
state = ppo_ffi.d2h(lib, b.d_state_p, F32, N * 1024).reshape(N, 1024)
pol = ppo.contents.policy.contents
mu0 = nn_params_packed(lib, pol.mu)
ls0 = ppo_ffi.d2h(lib, pol.d_log_std, F32, A)
lib.ppo_set_step_limit(ppo, 0, 1)
lib.ppo_update(ppo, 0.99, B, 1, 0, 1, seed)
lib.ppo_synchronize()
gmu = nn_grads_packed(lib, pol.mu)
rows = oracle.feistel_perm(N, oracle.splitmix64(seed))[:B]
x = state[rows]
a = ppo_ffi.d2h(lib, b.d_action_p, F32, N * A).reshape(N, A)[rows]
adv = ppo_ffi.d2h(lib, b.d_advantage_p, F32, N)[rows]
old = ppo_ffi.d2h(lib, b.d_logprob_p, F32, N)[rows]
hs, mu = emu_forward(C5, mu0, x)
y_gpu = ppo_ffi.d2h(lib, pol.mu.contents.d_output, F32, B * A).reshape(B, A)
print("mu (network output) vs emulation: max err", float(np.abs(y_gpu - mu).max()), "max |mu|", float(np.abs(mu).max()))
u = y_gpu.view(np.uint32)
print("fraction of outputs exactly bf16:", float(((u & 0xFFFF) == 0).mean()))
for i in range(1, 5):                      # hidden activations (bf16 storage) vs the emulation's
    h16 = ppo_ffi.d2h(lib, pol.mu.contents.layers[i].d_input, np.uint16, B * 1024).reshape(B, 1024)
    h = (h16.astype(np.uint32) << 16).view(F32)
    d = h != hs[i]
    rel = np.abs(h - hs[i]) / np.maximum(np.abs(hs[i]), 1e-30)
    print(f"hidden {i}: {int(d.sum())} of {d.size} differ ({d.mean():.2e}); max rel {float(rel[d].max()) if d.any() else 0:.3g}")
# the output from the GPU's own last hidden activation (isolates the output layer)
W4, b4 = unpack(C5, mu0)[-1]
h16 = ppo_ffi.d2h(lib, pol.mu.contents.layers[4].d_input, np.uint16, B * 1024).reshape(B, 1024)
h = (h16.astype(np.uint32) << 16).view(F32)
y_own = (h.astype(np.float64) @ bf16(W4).astype(np.float64).T + b4).astype(F32)
print("output layer alone (GPU h4): max err", float(np.abs(y_gpu - y_own).max()))
lp = oracle.log_prob(mu, ls0, a)
print("ratio range", float(np.exp(lp - old).min()), float(np.exp(lp - old).max()))
_, glp, gent = oracle.policy_loss_and_grad(adv, lp, old, oracle.entropy(ls0), 0.0, 0.2)
gmu_out, _ = oracle.log_prob_backwards(mu, ls0, a, glp)
g_emu = emu_backward(C5, mu0, hs, gmu_out)
gmax = float(np.abs(g_emu).max())
off = 0
for i, (W, bb) in enumerate(unpack(C5, mu0)):
    for nm, n in (("W", W.size), ("b", bb.size)):
        e = np.abs(gmu[off:off + n] - g_emu[off:off + n])
        j = int(e.argmax())
        print(f"layer {i} {nm}: max err {e.max():.3g} ({e.max() / gmax:.2e} of max|g|) at {j}: got {gmu[off + j]:.6g} "
              f"emu {g_emu[off + j]:.6g}; tensor max|g| {np.abs(g_emu[off:off + n]).max():.3g}")
        off += n
# variant: the top gradient's bias sum from the un-rounded fp32 gradient
print("output bias: emu(bf16 g) vs fp32-g sum:", np.abs(gmu_out.astype(np.float64).sum(0) -
                                                    bf16(gmu_out).astype(np.float64).sum(0)).max())
lib.free_ppo(ppo)
