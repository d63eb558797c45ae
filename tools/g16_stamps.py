#!/usr/bin/env python3
"""Per-phase cycles of the double-buffered bf16 GEMM (cfg 9, C5 16384x1024x1024) from in-kernel
stamps (diagnostic build: `sh tools/build_variant.sh g16ab32 -DPPO_G16_ABLATE=32 gemm16`):
mainloop, epilogue issue, store drain per workgroup (s_memtime), and from s_memrealtime the span of
the workgroups against the launch's event time."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo.c_amd"))
import ppo_ffi  # noqa: E402

lib = ppo_ffi.load(os.environ.get("PPO_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo.c_amd", "lib",
                                                             "variants", "libppo_g16ab32.so"))
lib.ppo_set_device(0)
m, n, l = 16384, 1024, 1024
for op in (0, 1):
    lib.ppo_bench_gemm16(op, m, n, l, 200, 9, 0)
    us = lib.ppo_bench_gemm16(op, m, n, l, 20, 9, 0)
    buf = (C.c_ulonglong * (8192 * 8))()
    lib.ppo_g16_stamps(buf, 8192 * 8)
    nwg = (m // 256) * (l // 256)
    st = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 8)[:nwg].astype(np.int64)
    main, epi, drain, life = st[:, 1] - st[:, 0], st[:, 2] - st[:, 1], st[:, 3] - st[:, 2], st[:, 3] - st[:, 0]
    rt0, rt1 = st[:, 4], st[:, 5]
    clk = life / ((rt1 - rt0) / 100.0) / 1e3
    print(f"op{op} m={m} n={n} l={l}: {us:.1f} us per launch (events), {nwg} workgroups")
    for name, v in (("mainloop", main), ("epilogue", epi), ("drain", drain), ("lifetime", life)):
        print(f"  {name:9s} cycles: min {v.min():8d}  median {int(np.median(v)):8d}  max {v.max():8d}")
    print(f"  start skew {(rt0.max() - rt0.min()) / 100.0:.2f} us, end skew {(rt1.max() - rt1.min()) / 100.0:.2f} us, "
          f"span {(rt1.max() - rt0.min()) / 100.0:.1f} us; shader clock median {np.median(clk):.3f} GHz")
