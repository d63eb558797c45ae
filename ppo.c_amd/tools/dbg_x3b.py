#!/usr/bin/env python3
"""x3 vs exact: every layer's activations, ReLU' bits, grad_x and grads of one MLP forward/backward."""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
for p in ("ppo.c_amd", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import ppo_ffi  # noqa: E402
from helpers import F32, dev, nn_grads_packed, nn_set_params_packed  # noqa: E402

lib = ppo_ffi.load()
lib.ppo_set_device(0)
sizes = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "376,512,512,512,17").split(",")]
m = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
rng = np.random.default_rng(5)
nn = lib.create_neural_network(ppo_ffi.c_ints(sizes), ppo_ffi.c_strings(["relu"] * (len(sizes) - 2) + ["none"]),
                               len(sizes))
nparams = sum(sizes[i] * sizes[i + 1] + sizes[i + 1] for i in range(len(sizes) - 1))
nn_set_params_packed(lib, nn, (rng.uniform(-1, 1, nparams) * 0.05).astype(F32))
dx = dev(lib, rng.uniform(-1, 1, (m, sizes[0])).astype(F32))
g = rng.uniform(-1, 1, (m, sizes[-1])).astype(F32)
g[rng.uniform(size=g.shape) < 0.5] = 0
dgo = dev(lib, g)
res = {}
for eng, flags in ((0, 0), (1, 0), (1, 4), (1, 32)):
    lib.ppo_gemm_f32_engine(eng)
    lib.ppo_gemm_flags(flags)
    lib.forward_propagation_cuda(nn, dx.ptr, m)
    L = len(sizes) - 1
    c = nn.contents
    acts = [ppo_ffi.d2h(lib, c.layers[i].d_input, F32, m * sizes[i]) for i in range(1, L)]
    acts.append(ppo_ffi.d2h(lib, c.d_output, F32, m * sizes[-1]))
    words = sum(m * ((sizes[i] + 31) // 32) for i in range(L + 1))
    bits = np.ctypeslib.as_array(c.d_act_bits, shape=(1,))  # placeholder (device pointer)
    nb = ppo_ffi.d2h(lib, c.d_act_bits, np.uint32, sum(c.act_cap_m * ((sizes[i] + 31) // 32) for i in range(L + 1)))
    lib.backward_propagation_cuda(nn, dgo.ptr, m)
    gx = [ppo_ffi.d2h(lib, c.layers[i].d_grad_x, F32, m * sizes[i]) for i in range(1, L)]
    res[(eng, flags)] = (acts, nb, gx, nn_grads_packed(lib, nn))
lib.ppo_gemm_flags(0)
base = res[(0, 0)]
for k, (acts, nb, gx, gr) in res.items():
    print(k, "acts", ["%.2e" % np.abs(a - b).max() for a, b in zip(acts, base[0])],
          "bits_diff", int((nb != base[1]).sum()), "/", nb.size,
          "gx", ["%.2e" % np.abs(a - b).max() for a, b in zip(gx, base[2])],
          "grads", "%.2e" % np.abs(gr - base[3]).max(), flush=True)
