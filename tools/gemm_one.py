#!/usr/bin/env python3
"""Run one GEMM shape/op/config repeatedly (a target for rocprofv3 --pmc passes).

    python tools/gemm_one.py OP M N L [CFG] [ITERS] [SPLITK_TARGET]
env GEMM_ENGINE=x3 runs the x3 engine (fp32 operands on the bf16 MFMA) instead of the exact fp32 one.
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo.c_amd"))
import ppo_ffi  # noqa: E402

op, m, n, l = (int(v) for v in sys.argv[1:5])
cfg = int(sys.argv[5]) if len(sys.argv) > 5 else -1
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 20
tgt = int(sys.argv[7]) if len(sys.argv) > 7 else 0
lib = ppo_ffi.load()
lib.ppo_set_device(0)
if os.environ.get("GEMM_ENGINE") == "x3":
    us = lib.ppo_bench_gemm_x3(op, m, n, l, iters, cfg, tgt)
else:
    lib.ppo_gemm_tune(-1, tgt)
    us = lib.ppo_bench_gemm(op, m, n, l, iters, cfg)
print(f"op{op} m={m} n={n} l={l} cfg={cfg} {us:.1f} us {2.0 * m * n * l / (us * 1e-6) / 1e12:.1f} TF/s")
