#!/usr/bin/env python3
"""Exact fp32 MFMA engine vs the x3 engine per launch at the small minibatch shapes (C3 8192 rows,
G = 8 / G = 4 shards 4096 / 8192 rows, C4 32768 for reference): forward, grad_x, grad_W (µs)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo.c_amd"))
import ppo_ffi  # noqa: E402

lib = ppo_ffi.load()
lib.ppo_set_device(0)
shapes = [(8192, 256, 256), (8192, 17, 256), (4096, 512, 512), (4096, 376, 512), (8192, 512, 512),
          (32768, 512, 512)]
names = ["fwd", "grad_x", "grad_W"]
for m, n, l in shapes:
    for op in range(3):
        if op == 1 and n == 17:
            continue
        x3 = lib.ppo_bench_gemm_x3(op, m, n, l, 50, -1, 0) if n % 4 == 0 else float("nan")
        ex = lib.ppo_bench_gemm(op, m, n, l, 50, -1)
        tf = 2.0 * m * n * l / 1e6
        print(f"{names[op]:7s} m={m:6d} n={n:4d} l={l:4d}  exact {ex:7.1f} us ({tf / ex:6.1f} TF/s)  "
              f"x3 {x3:7.1f} us ({tf / x3:6.1f} TF/s)", flush=True)
