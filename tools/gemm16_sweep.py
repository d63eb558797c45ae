#!/usr/bin/env python3
"""bf16 GEMM (gemm16.hip) sweep on the MI355X: device µs and TFLOP/s per (op, shape, config, split-K).

    python tools/gemm16_sweep.py [--cfgs 0,4] [--shape M,N,L]
op 0 = forward (bias+ReLU+bits), 1 = grad_x (bit mask), 2 = grad_W (split-K, fp32 atomics).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo.c_amd"))
import ppo_ffi  # noqa: E402

NAMES = {0: "128x128/bk32", 1: "128x32/bk32", 2: "32x128/bk32", 3: "64x64/bk32", 4: "128x128/bk64",
         5: "256x128/bk64", 6: "128x256/bk64", 7: "256x128/bk32", 8: "128x32/bk64", 9: "256x256/bk64 db", 10: "256x256 db 4w"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="0,3,4")
    ap.add_argument("--shape", default="16384,1024,1024")
    args = ap.parse_args()
    lib = ppo_ffi.load()
    lib.ppo_set_device(0)
    m, n, l = (int(v) for v in args.shape.split(","))
    for op in (0, 1) if os.environ.get("NO_GRADW") else (0, 1, 2):
        for cfg in (int(c) for c in args.cfgs.split(",")):
            for tgt in ([128, 256, 512, 1024] if op == 2 else [0]):
                us = lib.ppo_bench_gemm16(op, m, n, l, 20, cfg, tgt)
                tf = 2.0 * m * n * l / (us * 1e-6) / 1e12
                print(f"op{op} m={m} n={n} l={l} {NAMES[cfg]:14s} split={tgt:5d} {us:9.1f} us {tf:8.1f} TF/s",
                      flush=True)


if __name__ == "__main__":
    main()
