#!/usr/bin/env python3
"""x3-engine GEMM sweep (fp32 operands on the bf16 MFMA, gemm16.hip P = 3) next to the exact
fp32-MFMA engine, on the MI355X: device µs and algorithmic fp32 TFLOP/s per (op, shape, config).

    python ppo.c_amd/tools/gemm_x3_sweep.py [--shapes 32768,512,512;32768,376,512] [--cfgs -1,0,3]
op 0 = forward (bias+ReLU+bits), 1 = grad_x (bit mask), 2 = grad_W (split-K), 3 = forward, no activation,
4 = grad_x as an NT product against a transposed fp32 weight copy;
op + 10 = the same with pre-split (three bf16 plane) operands and outputs, the update path's storage.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import ppo_ffi  # noqa: E402

NAMES = {-1: "auto", 0: "128x128/bk32", 1: "128x32/bk32", 2: "32x128/bk32", 3: "64x64/bk32", 4: "128x128/bk64",
         5: "128x128 fp32img", 6: "128x128 fp32img db", 7: "128x128 pingpong", 8: "fp32img pipelined", 9: "pingpong fp32img pipe", 10: "producer/consumer", 11: "128x256 8 waves", 12: "256x128 8 waves"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="32768,512,512;32768,376,512;32768,512,17;32768,512,1")
    ap.add_argument("--cfgs", default="-1")
    ap.add_argument("--splits", default="0")
    ap.add_argument("--ops", default="0,1,2")
    args = ap.parse_args()
    lib = ppo_ffi.load()
    lib.ppo_set_device(0)
    for shape in args.shapes.split(";"):
        m, n, l = (int(v) for v in shape.split(","))
        for op in (int(o) for o in args.ops.split(",")):
            if op == 0 and l < 32:
                op = 3
            flop = 2.0 * m * n * l
            ex = lib.ppo_bench_gemm(1 if op % 10 == 4 else op % 10, m, n, l, 20, -1)
            print(f"op{op} m={m} n={n} l={l} exact-f32 auto        {ex:9.1f} us {flop / ex / 1e6:8.1f} TF/s", flush=True)
            for cfg in (int(c) for c in args.cfgs.split(",")):
                for tgt in ([int(s) for s in args.splits.split(",")] if op == 2 else [0]):
                    us = lib.ppo_bench_gemm_x3(op, m, n, l, 20, cfg, tgt)
                    print(f"op{op} m={m} n={n} l={l} x3 {NAMES[cfg]:14s} split={tgt:5d} {us:9.1f} us "
                          f"{flop / us / 1e6:8.1f} TF/s  ({ex / us:.2f}x)", flush=True)


if __name__ == "__main__":
    main()
