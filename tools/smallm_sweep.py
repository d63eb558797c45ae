#!/usr/bin/env python3
"""Small-M exact-fp32 products (B = 64 minibatches, rollout steps): the automatic choice (small-M
kernel where it applies) against forced tiled configurations, µs per launch (ppo_bench_gemm).

    python tools/smallm_sweep.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo.c_amd"))
import ppo_ffi  # noqa: E402

SHAPES = [(64, 376, 512), (64, 512, 512), (64, 512, 17), (64, 17, 256), (64, 256, 256), (64, 256, 6),
          (256, 376, 512), (256, 512, 512)]
lib = ppo_ffi.load()
lib.ppo_set_device(0)
old = lib.ppo_gemm_f32_engine(0)
for m, n, l in SHAPES:
    for op in (0, 1, 2):
        row = []
        for cfg in (-1, 0, 2, 3, 4, 5):
            row.append(lib.ppo_bench_gemm(op, m, n, l, 50, cfg))
        print(f"op{op} m={m:4d} n={n:4d} l={l:4d}  auto {row[0]:6.1f}  " +
              "  ".join(f"c{c} {u:6.1f}" for c, u in zip((0, 2, 3, 4, 5), row[1:])), flush=True)
lib.ppo_gemm_f32_engine(old)
