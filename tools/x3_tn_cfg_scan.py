#!/usr/bin/env python3
"""x3 grad_W (op 2) at the C4 shapes per tile configuration and split-K workgroup target (isolated
launches, slab partials when the splits are short): which TN tile the engine should pick."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo.c_amd"))
import ppo_ffi  # noqa: E402

lib = ppo_ffi.load()
lib.ppo_set_device(0)
lib.ppo_bench_gemm_x3(2, 32768, 512, 512, 200, -1, 0)          # settle the clock
for (m, n, l) in [(32768, 512, 512), (32768, 376, 512), (4096, 512, 512)]:
    for cfg in (-1, 0, 2, 3, 4):
        row = []
        for tgt in (0, 256, 512, 1024):
            us = lib.ppo_bench_gemm_x3(2, m, n, l, 30, cfg, tgt)
            row.append(f"t{tgt} {us:6.1f}")
        print(f"op2 m={m} n={n} l={l} cfg {cfg:2d}: " + " | ".join(row), flush=True)
