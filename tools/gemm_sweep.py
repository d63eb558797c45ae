#!/usr/bin/env python3
"""GEMM tile/split sweep on the MI355X: device µs and TFLOP/s per (op, shape, tile config).

    python tools/gemm_sweep.py [--quick]
op 0 = forward (bias+ReLU), 1 = grad_x, 2 = grad_W (+bias grad, split-K).
"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo.c_amd"))
import ppo_ffi  # noqa: E402

CFG_NAMES = {0: "128x128/bk16", 1: "128x128/bk32", 2: "128x32/bk16", 3: "32x128/bk16", 4: "64x64/bk16",
             5: "128x64/bk16", 6: "256x128/bk16", 7: "128x128/bk16/db", 8: "128x64/bk16/db", 9: "64x64/bk32/db",
             10: "128x32/bk32"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--out", default="")
    ap.add_argument("--kscan", action="store_true", help="forward at fixed M,N over K (edge vs main-loop cost)")
    ap.add_argument("--main", action="store_true", help="C4 minibatch shapes x the large-tile configs only")
    ap.add_argument("--cfgs", default="", help="comma-separated configs for --main (default: a fixed set)")
    ap.add_argument("--lib", default="", help="load this libppo build instead of lib/libppo.so")
    ap.add_argument("--ops", default="0,1,2", help="--main: ops to run")
    ap.add_argument("--skinny", action="store_true", help="output-layer shapes (N = 17 / 1) x every config")
    ap.add_argument("--flags", default="0", help="comma-separated ppo_gemm_flags values to compare (--main)")
    args = ap.parse_args()
    lib = ppo_ffi.load(args.lib) if args.lib else ppo_ffi.load()
    lib.ppo_set_device(0)
    B = 32768
    if args.kscan:
        for (m, l) in ((B, 512), (4096, 4096)):
            for n in (64, 128, 256, 512, 1024, 2048, 4096, 8192):
                us = lib.ppo_bench_gemm(0, m, n, l, 5, -1)
                print(f"kscan fwd m={m} l={l} K={n:5d} {us:9.1f} us {2.0 * m * n * l / (us * 1e-6) / 1e12:7.1f} TF/s",
                      flush=True)
        return
    if args.skinny:
        for (m, n, l) in ((B, 512, 17), (B, 512, 1), (B, 1024, 17)):
            for op in (3, 1, 2):
                for cfg in (range(lib.ppo_gemm_tune(-1, -1)) if not args.cfgs else [int(c) for c in args.cfgs.split(",")]):
                    for tgt in ([256, 512, 1024, 2048] if op == 2 else [0]):
                        for fl in (int(f) for f in args.flags.split(",")):
                            lib.ppo_gemm_tune(-1, tgt)
                            lib.ppo_gemm_flags(fl)
                            us = lib.ppo_bench_gemm(op, m, n, l, 20, cfg)
                            print(f"op{op} m={m:6d} n={n:4d} l={l:3d} {CFG_NAMES[cfg]:16s} split_target={tgt:5d} "
                                  f"flags={fl} {us:8.1f} us {(m * n + m * l) * 4 / (us * 1e-6) / 1e9:7.0f} GB/s",
                                  flush=True)
        lib.ppo_gemm_flags(0)
        lib.ppo_gemm_tune(-1, 0)
        return
    if args.main:
        for (m, n, l) in ((B, 376, 512), (B, 512, 512), (1 << 20, 512, 512)):
            for op in (int(o) for o in args.ops.split(",")):
                if m > B and op:
                    continue
                cfgs = [0, 5, 7] if op != 2 else [0, 4, 5, 7, 9]
                if args.cfgs:
                    cfgs = [int(c) for c in args.cfgs.split(",")]
                for cfg in cfgs:
                    for tgt in ([512, 1024, 2048] if op == 2 else [0]):
                        for fl in (int(f) for f in args.flags.split(",")):
                            lib.ppo_gemm_tune(-1, tgt)
                            lib.ppo_gemm_flags(fl)
                            us = lib.ppo_bench_gemm(op, m, n, l, 10 if m <= B else 3, cfg)
                            tf = 2.0 * m * n * l / (us * 1e-6) / 1e12
                            print(f"op{op} m={m:8d} n={n:4d} l={l:4d} {CFG_NAMES[cfg]:16s} split_target={tgt:5d} "
                                  f"flags={fl} {us:9.1f} us {tf:7.1f} TF/s", flush=True)
                lib.ppo_gemm_flags(0)
        lib.ppo_gemm_tune(-1, 0)
        return
    shapes = [  # (m, n, l) = (batch, in, out) — C4 minibatch layers and the GAE forward
        (B, 376, 512), (B, 512, 512), (B, 512, 17), (B, 512, 1), (1 << 20, 512, 512),
        (8192, 256, 256), (8192, 17, 256),
    ]
    rows = []
    for (m, n, l) in shapes:
        for op in (0, 1, 2):
            if op == 1 and n < 64:
                continue
            cfgs = [-1, 0, 1, 5, 6] if min(n, l) > 32 else [-1, 2, 3, 4]
            if args.quick:
                cfgs = [-1]
            targets = [512] if op != 2 else [256, 512, 1024, 2048]
            for cfg in cfgs:
                for tgt in targets:
                    lib.ppo_gemm_tune(-1, tgt)
                    us = lib.ppo_bench_gemm(op, m, n, l, 10 if m < (1 << 20) else 3, cfg)
                    tf = 2.0 * m * n * l / (us * 1e-6) / 1e12
                    rows.append(dict(op=op, m=m, n=n, l=l, cfg=CFG_NAMES.get(cfg, "auto"), splitk=tgt, us=us,
                                     tflops=tf))
                    print(f"op{op} m={m:8d} n={n:4d} l={l:4d} {CFG_NAMES.get(cfg, 'auto'):14s} "
                          f"split_target={tgt:5d} {us:9.1f} us {tf:7.1f} TF/s", flush=True)
    lib.ppo_gemm_tune(-1, 0)
    if args.out:
        json.dump(rows, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
