#!/usr/bin/env python3
"""Per-phase cycles of the x3 forward (C4 512x512, cfg 0) from in-kernel s_memtime stamps
(PPO_X3_ABLATE=32 diagnostic build): prologue, mainloop, epilogue per workgroup."""
import ctypes as C
import os
import sys

import numpy as np

os.environ["PPO_X3_ABLATE"] = "32"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import ppo_ffi  # noqa: E402

lib = ppo_ffi.load()
lib.ppo_set_device(0)
m, n, l = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (32768, 512, 512)))
us = lib.ppo_bench_gemm_x3(0, m, n, l, 20, 0, 0)
buf = (C.c_ulonglong * (8192 * 4))()
lib.ppo_x3_stamps(buf, 8192 * 4)
nwg = ((m + 255) // 256) * ((l + 255) // 256)
st = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 4)[:nwg].astype(np.int64)
t0 = st[:, 0].min()
pro, main, epi = st[:, 1] - st[:, 0], st[:, 2] - st[:, 1], st[:, 3] - st[:, 2]
print(f"forward m={m} n={n} l={l}: {us:.1f} us per launch, {nwg} workgroups")
for name, v in (("start offset", st[:, 0] - t0), ("prologue", pro), ("mainloop", main), ("epilogue", epi),
                ("end offset", st[:, 3] - t0)):
    print(f"{name:13s} cycles: min {v.min():8d}  median {int(np.median(v)):8d}  max {v.max():8d}")
nk = (n + 15) // 16
print(f"mainloop per k-tile (median): {int(np.median(main)) / nk:.0f} cycles; MFMA floor per k-tile at 2 waves/SIMD: {2 * 48 * 32}")
