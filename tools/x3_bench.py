#!/usr/bin/env python3
"""Time the x3 engine's launches at the C4 (and C3/C5-fp32) layer shapes: µs per launch and TF/s
(fp32-equivalent 2·m·n·l) per tile configuration and split-K target.

    python tools/x3_bench.py [--cfgs 0,1,2] [--splits 0,256,512] [--iters 50]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo.c_amd"))
import ppo_ffi  # noqa: E402

SHAPES = [(0, 32768, 512, 512), (0, 32768, 376, 512), (1, 32768, 512, 512), (2, 32768, 512, 512),
          (2, 32768, 376, 512), (0, 1048576, 376, 512), (0, 8192, 256, 256), (2, 8192, 256, 256)]
OPS = ["fwd", "grad_x", "grad_W", "fwd-noact"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="-1")
    ap.add_argument("--splits", default="0")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--shapes", default="", help="op,m,n,l;... (default: the C4/C3 list)")
    args = ap.parse_args()
    shapes = [tuple(map(int, t.split(","))) for t in args.shapes.split(";")] if args.shapes else SHAPES
    lib = ppo_ffi.load()
    lib.ppo_set_device(0)
    for op, m, n, l in shapes:
        for c in map(int, args.cfgs.split(",")):
            for s in map(int, args.splits.split(",")):
                if op != 2 and s:
                    continue
                if c >= 0 and op == 2 and c not in (1, 3, 4, 5):
                    continue
                us = lib.ppo_bench_gemm_x3(op, m, n, l, args.iters if m < 1 << 20 else 5, c, s)
                tf = 2.0 * m * n * l / (us * 1e-6) / 1e12
                print(f"{OPS[op]:7s} m={m:8d} n={n:4d} l={l:4d} cfg={c:2d} split={s:4d}  {us:9.1f} us  "
                      f"{tf:6.1f} TF/s  frac={tf / 416.67:.3f}", flush=True)


if __name__ == "__main__":
    main()
