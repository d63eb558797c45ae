#!/usr/bin/env python3
"""bf16 LDS-DMA kernels (C5 shapes) per launch with the libppo build PPO_LIB points at: forward,
grad_x (op 0 / 1, bf16 DMA tiles) and grad_W (op 2, DMA TN tile).  Used for the asm-issued vs
builtin LDS-DMA A/B (gemm16.hip dma16).

    PPO_LIB=... python tools/dma_ab.py [m n l ...]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo.c_amd"))
import ppo_ffi  # noqa: E402

lib = ppo_ffi.load()
lib.ppo_set_device(0)
args = [int(v) for v in sys.argv[1:]] or [16384, 1024, 1024, 4096, 1024, 1024]
tag = os.path.basename(os.environ.get("PPO_LIB", "libppo.so"))
for i in range(0, len(args), 3):
    m, n, l = args[i:i + 3]
    tf = 2.0 * m * n * l / 1e6
    for op, name in ((0, "fwd"), (1, "grad_x"), (2, "grad_W")):
        lib.ppo_bench_gemm16(op, m, n, l, 100, -1, 0)              # settle the clock
        us = lib.ppo_bench_gemm16(op, m, n, l, 100, -1, 0)
        print(f"{tag} {name} m={m} n={n} l={l}: {us:.1f} us = {tf / us:.0f} TF/s", flush=True)
