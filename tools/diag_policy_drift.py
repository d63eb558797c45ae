#!/usr/bin/env python3
"""Long-run drift of the GPU B = 64 paths against the oracle's own fp32 chaos floor, on the GPU's
buffer (C4 networks, reference ppo.cu:398-443): after n value / policy steps, the cosine of the
parameter motion of the cluster phase (cluster_deep.hip) and of the multi-launch loop against the
oracle proper, next to the oracle re-associated (split-K halves) and in double-precision products.
Per-tensor cosines locate a drift that outruns the floor.  Needs a GPU (tests/test_gpu_cluster.run)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ppo.c_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle_ffi  # noqa: E402
import ppo_ffi  # noqa: E402
from test_gpu_cluster import C4, RELU, run  # noqa: E402


def cos(a, b):
    a, b = a.astype(np.float64), b.astype(np.float64)
    return float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b) + 1e-300))


def tensors(sizes, vec):
    out, off = [], 0
    for i in range(len(sizes) - 1):
        n, l = sizes[i], sizes[i + 1]
        out.append((f"W{i}", vec[off:off + n * l]))
        off += n * l
        out.append((f"b{i}", vec[off:off + l]))
        off += l
    return out


def main():
    lib = ppo_ffi.load()
    assert lib.ppo_set_device(0) == 0
    oracle_ffi.build()
    oracle_ffi.load(use_openblas=True)
    N, B = 16384, 64
    steps_list = [int(s) for s in (sys.argv[1:] or ["64", "128", "256", "512"])]
    for phase in ("policy", "value"):
        for steps in steps_list:
            lim = (steps, 0) if phase == "value" else (0, steps)
            a = run(lib, C4, N, B, 4, 10, 1, cluster=True, limit=lim, ent=0.0)
            b = run(lib, C4, N, B, 4, 10, 1, cluster=False, limit=lim, ent=0.0)
            refs = {}
            for mode in (0, 1, 2):
                oracle_ffi.blas_mode(mode)
                refs[mode] = oracle_ffi.ppo_update(C4, RELU(C4), a["mu0"], a["ls0"], a["v0"], a["buf"], batch_size=B,
                                                   n_epochs_policy=4, n_epochs_value=10, shuffle_mode=1, seed=9,
                                                   max_value_steps=lim[0], max_policy_steps=lim[1])
            oracle_ffi.blas_mode(0)
            k, k0, sizes = ("mu", "mu0", C4) if phase == "policy" else ("v", "v0", C4[:-1] + [1])
            d0 = refs[0][k] - a[k0]
            rows = {"cluster": a[k] - a[k0], "multi": b[k] - b[k0], "oracle split-K": refs[1][k] - a[k0],
                    "oracle double": refs[2][k] - a[k0]}
            line = f"{phase} {steps:4d} steps vs oracle:"
            for name, d in rows.items():
                line += f" | {name} cos {cos(d, d0):.5f} ratio {np.linalg.norm(d) / np.linalg.norm(d0):.4f}"
            print(line, flush=True)
            for name in ("cluster", "multi", "oracle split-K"):
                per = " ".join(f"{t}:{cos(x, y):.4f}" for (t, x), (_, y) in zip(tensors(sizes, rows[name]),
                                                                                tensors(sizes, d0)))
                print(f"    {name:15s} per tensor: {per}", flush=True)
            if phase == "policy":
                dl0 = refs[0]["log_std"] - a["ls0"]
                for name, x in (("cluster", a["ls"]), ("multi", b["ls"]), ("oracle split-K", refs[1]["log_std"]),
                                ("oracle double", refs[2]["log_std"])):
                    dl = x - a["ls0"]
                    print(f"    log σ motion {name:15s} cos {cos(dl, dl0):.5f} max|Δ| {np.abs(dl - dl0).max():.3e} "
                          f"(|motion| {np.abs(dl0).max():.3e})", flush=True)
                print(f"    policy loss sums: cluster {a['stats'][2]:.6f} multi {b['stats'][2]:.6f} "
                      f"oracle {refs[0]['sum_policy_loss']:.6f} split-K {refs[1]['sum_policy_loss']:.6f}", flush=True)


if __name__ == "__main__":
    main()
