#!/usr/bin/env python3
"""bf16 output-layer forward (op 3: no activation) at C5's shape on the skinny-N tiles."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo.c_amd"))
import ppo_ffi  # noqa: E402

lib = ppo_ffi.load()
lib.ppo_set_device(0)
for rep in range(2):
    for (m, n, l) in ((16384, 1024, 17), (16384, 1024, 1), (32768, 512, 17)):
        for cfg in (1, 8):
            us = lib.ppo_bench_gemm16(3, m, n, l, 20, cfg, 0)
            print(f"rep {rep} op3 m={m} n={n} l={l} cfg={cfg} {us:7.1f} us {(m * n * 2 + m * l * 4) / us / 1e3:6.0f} GB/s",
                  flush=True)
