#!/usr/bin/env python3
"""x3 engine: BK 16 tiles at 2 / 3 / 4 workgroups per CU (cfg 13 / 14 / 15) beside the 128x128/BK32
tile (cfg 0) and the 8-wave 256x128 tile (cfg 12) at the C4 shapes (isolated launches). cfg 13-15 exist only
in the build measured in profiles/r01_x3_bk16_occupancy.txt."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import ppo_ffi  # noqa: E402

lib = ppo_ffi.load()
lib.ppo_set_device(0)
for (m, n, l) in [(32768, 512, 512), (32768, 376, 512)]:
    for op in (0, 1, 2):
        row = []
        for c in (0, 12, 13, 14, 15):
            us = lib.ppo_bench_gemm_x3(op, m, n, l, 30, c, 0)
            row.append(f"cfg{c} {us:6.1f}us {2.0 * m * n * l / us / 1e6:4.0f}TF")
        print(f"op{op} m={m} n={n} l={l}: " + " | ".join(row), flush=True)
