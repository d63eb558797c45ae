#!/usr/bin/env python3
"""Drift of the B = 64 multi-workgroup phases from the multi-launch loop over a value phase: the
cosine and norm ratio of the parameter motion after 16 … 2560 steps (C3 and C4 networks), and of
each path against the oracle up to 512 steps — chaos grows smoothly, a defect shows as a jump (e.g. at
the epoch boundary, step 256)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ppo.c_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle_ffi  # noqa: E402
import ppo_ffi  # noqa: E402
from test_gpu_cluster import C3, C4, RELU, run  # noqa: E402


def cosn(da, db):
    return float(da @ db / (np.linalg.norm(da) * np.linalg.norm(db))), float(np.linalg.norm(da) / np.linalg.norm(db))


def main():
    lib = ppo_ffi.load()
    assert lib.ppo_set_device(0) == 0
    oracle_ffi.build()
    oracle_ffi.load(use_openblas=True)
    N, B = 16384, 64
    for name, sizes in (("c3", C3), ("c4", C4)):
        for steps in (16, 64, 255, 257, 512, 1024, 2560):
            a = run(lib, sizes, N, B, 0, 10, 1, cluster=True, limit=(steps, 0))
            b = run(lib, sizes, N, B, 0, 10, 1, cluster=False, limit=(steps, 0))
            c, r = cosn(a["v"] - a["v0"], b["v"] - b["v0"])
            line = f"{name} value steps {steps:5d}: cluster vs multi cos {c:.5f} ratio {r:.4f}"
            if steps <= 512:
                ref = oracle_ffi.ppo_update(sizes, RELU(sizes), a["mu0"], a["ls0"], a["v0"], a["buf"], batch_size=B,
                                            n_epochs_policy=0, n_epochs_value=10, shuffle_mode=1, seed=9,
                                            max_value_steps=steps, max_policy_steps=0)
                ca, ra = cosn(a["v"] - a["v0"], ref["v"] - a["v0"])
                cb, rb = cosn(b["v"] - b["v0"], ref["v"] - b["v0"])
                line += f" | vs oracle: cluster {ca:.5f} ({ra:.4f}) multi {cb:.5f} ({rb:.4f})"
            print(line, flush=True)


if __name__ == "__main__":
    main()
