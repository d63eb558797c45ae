#!/bin/sh
# fold_bench.sh — isolated x3 timings of the value-head fold variants (ops 4-6) against the plain
# kernels (ops 0-2) at the C4, G = 8 shard and C3 shapes
for s in "32768 512 512" "4096 512 512" "8192 256 256"; do
    for op in 0 4 1 5 2 6; do
        GEMM_ENGINE=x3 timeout -k 5 60 python tools/gemm_one.py $op $s -1 100 || exit 1
    done
done
