"""bf16 backward, grad_W slab reduce carried by grad_x (PPO_G16_DEFER=1) vs its own launch: per-layer
differences between two runs of each mode (diagnostic)."""
import os, sys
import numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "ppo.c_amd"), os.path.join(os.path.dirname(__file__), "..", "tests")]
import ppo_ffi
from helpers import F32, dev, nn_grads_packed, nn_set_params_packed
lib = ppo_ffi.load()
assert lib.ppo_set_device(0) == 0
sizes, m = [1024, 1024, 1024, 17], 16384
rng = np.random.default_rng(7)
names = ["relu"] * (len(sizes) - 2) + ["none"]
nn = lib.create_neural_network(ppo_ffi.c_ints(sizes), ppo_ffi.c_strings(names), len(sizes))
params = (rng.uniform(-1, 1, sum(a * b + b for a, b in zip(sizes[:-1], sizes[1:]))) / np.sqrt(max(sizes))).astype(F32)
nn_set_params_packed(lib, nn, params)
assert lib.nn_set_compute_dtype(nn, 1) == 0
dx = dev(lib, rng.uniform(-1, 1, (m, sizes[0])).astype(F32))
dgo = dev(lib, rng.uniform(-1, 1, (m, sizes[-1])).astype(F32))
runs = []
for mode in ("0", "0", "1", "1"):
    os.environ["PPO_G16_DEFER"] = mode
    lib.forward_propagation_cuda(nn, dx.ptr, m)
    lib.backward_propagation_cuda(nn, dgo.ptr, m)
    runs.append((mode, nn_grads_packed(lib, nn)))
offs, o = [], 0
for a, b in zip(sizes[:-1], sizes[1:]):
    offs.append((f"W{len(offs)}", o, o + a * b)); o += a * b
    offs.append((f"b{len(offs)//2}", o, o + b)); o += b
def cmp(x, y, tag):
    print(tag, " ".join(f"{n}:{int((x[s:e] != y[s:e]).sum())}/{e-s} max {float(np.abs(x[s:e]-y[s:e]).max()):.2g}" for n, s, e in offs))
cmp(runs[0][1], runs[1][1], "own-launch run1 vs run2")
cmp(runs[2][1], runs[3][1], "carried run1 vs run2  ")
cmp(runs[0][1], runs[2][1], "own-launch vs carried ")
