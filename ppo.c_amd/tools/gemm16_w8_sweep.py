#!/usr/bin/env python3
"""bf16 GEMM: 8-wave tiles (cfg 9-11, present only in the build measured in profiles/r01_gemm16_w8_tiles.txt) beside the 4-wave 128x256/BK64 (cfg 6) and 256x128/BK64 (cfg 5) at the C5 / C4 shapes."""
import os, sys
sys.path.insert(0, "ppo.c_amd")
import ppo_ffi
lib = ppo_ffi.load(); lib.ppo_set_device(0)
for (m, n, l) in [(16384, 1024, 1024), (32768, 512, 512)]:
    for op in (0, 1, 2):
        row = []
        for c in (6, 9, 10, 11, 5):
            us = lib.ppo_bench_gemm16(op, m, n, l, 30, c, 0)
            row.append(f"cfg{c} {us:6.1f}us {2.0*m*n*l/us/1e6:5.0f}TF")
        print(f"m={m} n={n} l={l} op{op}: " + " | ".join(row), flush=True)
