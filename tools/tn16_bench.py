#!/usr/bin/env python3
"""bf16 grad_W (C5 shapes) per launch: the LDS-DMA TN tile (width 128 by default; --bn 256 sets it
through ppo_gemm16_tn_width) against the register-staged split-K kernel (cfg 6 forced).

    python tools/tn16_bench.py [--bn 128|256] [m n l ...]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo.c_amd"))
import ppo_ffi  # noqa: E402

lib = ppo_ffi.load()
lib.ppo_set_device(0)
argv = sys.argv[1:]
bn = 128
if argv[:1] == ["--bn"]:
    bn, argv = int(argv[1]), argv[2:]
lib.ppo_gemm16_tn_width(bn)
args = [int(v) for v in argv] or [16384, 1024, 1024, 4096, 1024, 1024, 16384, 384, 512]
for i in range(0, len(args), 3):
    m, n, l = args[i:i + 3]
    lib.ppo_bench_gemm16(2, m, n, l, 200, -1, 0)                 # settle the clock
    dma = lib.ppo_bench_gemm16(2, m, n, l, 100, -1, 0)
    reg = lib.ppo_bench_gemm16(2, m, n, l, 100, 6, 0)
    tf = 2.0 * m * n * l / 1e6
    print(f"grad_W m={m} n={n} l={l} (BN {bn}): DMA TN {dma:.1f} us = {tf / dma:.0f} TF/s, "
          f"register-staged {reg:.1f} us = {tf / reg:.0f} TF/s", flush=True)
