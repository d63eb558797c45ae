#!/usr/bin/env python3
"""Per-phase cycles of the x3 forward (C4 512x512, cfg 0) from in-kernel stamps (diagnostic build:
`sh tools/build_variant.sh diag -DPPO_X3_DIAG gemm_x3`, run with --lib): prologue, mainloop,
epilogue per workgroup (s_memtime, shader cycles), and from s_memrealtime (100 MHz, common to all
XCDs) the span of the workgroups against the launch's event time and the shader clock."""
import argparse
import ctypes as C
import os
import sys

import numpy as np

os.environ["PPO_X3_ABLATE"] = "32"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo.c_amd"))
import ppo_ffi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--op", type=int, default=0, help="0 forward, 1 grad_x, 2 grad_W (cfg 3)")
ap.add_argument("--cfg", type=int, default=0)
ap.add_argument("--nwg", type=int, default=0, help="workgroups of the launch (default: 256x256 tiles)")
ap.add_argument("--nk", type=int, default=0, help="k-tiles per k-group of one workgroup (default: n/16)")
ap.add_argument("shape", nargs="*", type=int, default=[32768, 512, 512])
args = ap.parse_args()
lib = ppo_ffi.load(args.lib or os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo.c_amd", "lib", "variants", "libppo_diag.so"))
lib.ppo_set_device(0)
m, n, l = args.shape
lib.ppo_bench_gemm_x3(args.op, m, n, l, 400, args.cfg, 0)   # ≥ 2 s of back-to-back launches: settled clock
us = lib.ppo_bench_gemm_x3(args.op, m, n, l, 50, args.cfg, 0)
buf = (C.c_ulonglong * (8192 * 8))()
lib.ppo_x3_stamps(buf, 8192 * 8)
nwg = args.nwg or ((m + 255) // 256) * ((l + 255) // 256)
st = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 8)[:nwg].astype(np.int64)
pro, main, epi = st[:, 1] - st[:, 0], st[:, 2] - st[:, 1], st[:, 3] - st[:, 2]
life = st[:, 3] - st[:, 0]
rt0, rt1 = st[:, 4], st[:, 5]
span_us = (rt1.max() - rt0.min()) / 100.0
clk = life / ((rt1 - rt0) / 100.0) / 1e3                 # GHz per workgroup
print(f"op{args.op} m={m} n={n} l={l}: {us:.1f} us per launch (events), {nwg} workgroups")
for name, v in (("prologue", pro), ("mainloop", main), ("epilogue", epi), ("lifetime", life)):
    print(f"{name:13s} cycles: min {v.min():8d}  median {int(np.median(v)):8d}  max {v.max():8d}")
print(f"start skew {(rt0.max() - rt0.min()) / 100.0:.2f} us, end skew {(rt1.max() - rt1.min()) / 100.0:.2f} us, "
      f"workgroup span {span_us:.1f} us of {us:.1f} us; shader clock median {np.median(clk):.3f} GHz")
nk = args.nk or (n + 15) // 16
floor = 2 * 48 * 32 if args.op != 2 else 2 * 24 * 32
print(f"mainloop per k-tile (median): {int(np.median(main)) / nk:.0f} cycles; MFMA floor per k-tile at 2 waves/SIMD: {floor}")
