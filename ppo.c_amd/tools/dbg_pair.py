import os, sys
sys.path.insert(0, "tests"); sys.path.insert(0, "ppo.c_amd"); sys.path.insert(0, "oracle")
import numpy as np
import ppo_ffi, oracle_ffi as oracle
from helpers import F32, dev, nn_grads_packed, nn_set_params_packed
lib = ppo_ffi.load(); lib.ppo_set_device(0)
sizes, m = [64, 1024, 1024, 8], 16384
rng = np.random.default_rng(1)
relu = [1] * (len(sizes) - 2) + [0]
nn = lib.create_neural_network(ppo_ffi.c_ints(sizes), ppo_ffi.c_strings(["relu"] * (len(sizes) - 2) + ["none"]), len(sizes))
params = (rng.uniform(-1, 1, oracle.mlp_num_params(sizes)) * 0.05).astype(F32)
nn_set_params_packed(lib, nn, params)
x, gout = rng.uniform(-1, 1, (m, sizes[0])).astype(F32), rng.uniform(-1, 1, (m, sizes[-1])).astype(F32)
dx, dgo = dev(lib, x), dev(lib, gout)
res = {}
for flags in (4, 0):
    lib.ppo_gemm_flags(flags)
    lib.forward_propagation_cuda(nn, dx.ptr, m)
    lib.backward_propagation_cuda(nn, dgo.ptr, m)
    gx1 = ppo_ffi.d2h(lib, nn.contents.layers[1].d_grad_x, F32, m * sizes[1])
    res[flags] = (nn_grads_packed(lib, nn), gx1)
g4, g0 = res[4][0], res[0][0]
off = 0
for i in range(len(sizes) - 1):
    nw, nb = sizes[i] * sizes[i + 1], sizes[i + 1]
    for name, n in (("W", nw), ("b", nb)):
        a, b = g4[off:off + n], g0[off:off + n]
        d = np.abs(a - b)
        print(f"layer {i} {name}: max|a| {np.abs(a).max():.4g} max diff {d.max():.4g} n_bad {(d > 1e-3 * np.abs(a).max()).sum()} / {n}", flush=True)
        if name == "W" and d.max() > 1e-3 * np.abs(a).max():
            bad = np.nonzero(d.reshape(sizes[i + 1], sizes[i]) > 1e-3 * np.abs(a).max())
            print("   rows", np.unique(bad[0])[:20], "cols", np.unique(bad[1])[:20], flush=True)
            r0, c0 = bad[0][0], bad[1][0]
            print("   ratio sample", (b.reshape(sizes[i+1], sizes[i])[r0, c0] / a.reshape(sizes[i+1], sizes[i])[r0, c0]))
        off += n
print("gx1 equal:", np.array_equal(res[4][1], res[0][1]), np.abs(res[4][1] - res[0][1]).max())
