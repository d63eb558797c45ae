#!/usr/bin/env python3
"""x3 forward / grad_x per launch with W split in the kernel (ops 0 / 1) against W pre-split into
three bf16 planes and staged by LDS-DMA (ops 4 / 5), interleaved, at the C4 and shard shapes.

    python tools/x3_wplanes_ab.py [reps]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo.c_amd"))
import ppo_ffi  # noqa: E402

lib = ppo_ffi.load()
lib.ppo_set_device(0)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
SHAPES = [(32768, 512, 512), (32768, 376, 512), (4096, 512, 512), (8192, 512, 512), (8192, 256, 256)]
for rep in range(reps):
    for m, n, l in SHAPES:
        tf = 2.0 * m * n * l / 1e6
        for base, pre, name in ((0, 4, "fwd"), (1, 5, "grad_x")):
            if name == "grad_x" and n == 376:
                continue
            lib.ppo_bench_gemm_x3(base, m, n, l, 50, -1, 0)
            t0 = lib.ppo_bench_gemm_x3(base, m, n, l, 50, -1, 0)
            t1 = lib.ppo_bench_gemm_x3(pre, m, n, l, 50, -1, 0)
            print(f"{name} {m}x{n}x{l}: split-in-kernel {t0:.1f} us ({tf / t0:.0f} TF/s), "
                  f"pre-split W by DMA {t1:.1f} us ({tf / t1:.0f} TF/s)", flush=True)
