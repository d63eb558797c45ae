#!/usr/bin/env python3
"""libppo's GEMM kernels beside the vendor library at the PPO layer shapes (context for the roofline).

    python tools/vendor_gemm_ref.py > profiles/r01_vendor_gemm_ref.txt

Per shape and op (0 forward y = x·Wᵀ, 1 grad_x = g·W, 2 grad_W = gᵀ·x): torch.matmul (hipBLASLt /
rocBLAS) in bf16 and fp32, libppo's bf16 kernel (C5 mode) and its x3 engine (fp32 on the bf16 MFMA).
Plain products only: libppo's launches also carry their fused epilogues (bias, ReLU, ReLU′ bits,
bias gradient, split-K atomics), torch's do not.  Not a test: torch is the measuring stick here.
"""
import os
import sys

import torch  # first: libppo binds to the HIP runtime torch already loaded

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo.c_amd"))
import ppo_ffi  # noqa: E402

SHAPES = [("c4 512->512", 32768, 512, 512), ("c4 376->512", 32768, 376, 512), ("c5 1024->1024", 16384, 1024, 1024)]
ITERS = 30


def torch_us(op, m, n, l, dtype):
    dev = "cuda"
    x = torch.randn(m, n, device=dev, dtype=dtype)
    W = torch.randn(l, n, device=dev, dtype=dtype)
    g = torch.randn(m, l, device=dev, dtype=dtype)
    f = {0: lambda: x @ W.t(), 1: lambda: g @ W, 2: lambda: g.t() @ x}[op]
    for _ in range(5):
        f()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(ITERS):
        f()
    b.record()
    torch.cuda.synchronize()
    return 1000.0 * a.elapsed_time(b) / ITERS


def main():
    torch.backends.cuda.matmul.allow_tf32 = False
    lib = ppo_ffi.load()
    lib.ppo_set_device(0)
    print(f"# {ITERS} launches each, HIP events; TF/s = 2·m·n·l / time (fp32-equivalent for x3)")
    print(f"# {'shape':14s} op  {'torch bf16':>16s} {'libppo bf16':>16s} {'torch fp32':>16s} {'libppo x3':>16s}")
    for name, m, n, l in SHAPES:
        for op in (0, 1, 2):
            fl = 2.0 * m * n * l
            r = [torch_us(op, m, n, l, torch.bfloat16), lib.ppo_bench_gemm16(op, m, n, l, ITERS, -1, 0),
                 torch_us(op, m, n, l, torch.float32), lib.ppo_bench_gemm_x3(op, m, n, l, ITERS, -1, 0)]
            cells = " ".join(f"{us:7.1f}us {fl / us / 1e6:5.0f}TF" for us in r)
            print(f"  {name:14s} {op}   {cells}", flush=True)


if __name__ == "__main__":
    main()
