#!/usr/bin/env python3
"""x3 grad_W (op 2, 128x128 tiles) at the C4 shapes over split-K workgroup targets (isolated launches)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo.c_amd"))
import ppo_ffi  # noqa: E402

lib = ppo_ffi.load()
lib.ppo_set_device(0)
for (m, n, l) in [(32768, 512, 512), (32768, 376, 512)]:
    row = []
    for tgt in (0, 256, 384, 512, 768, 1024, 1536, 2048):
        us = lib.ppo_bench_gemm_x3(2, m, n, l, 30, 0, tgt)
        row.append(f"t{tgt} {us:6.1f}us")
    print(f"op2 m={m} n={n} l={l}: " + " | ".join(row), flush=True)
