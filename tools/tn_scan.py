#!/usr/bin/env python3
"""grad_W (op 2) at the C4 batch over input widths around 376, per tile config and split target."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo.c_amd"))
import ppo_ffi  # noqa: E402

lib = ppo_ffi.load()
lib.ppo_set_device(0)
for rep in range(2):
    for n in (376, 384, 512):
        for cfg, tgts in ((0, (512, 1024)), (4, (1024, 2048)), (5, (1024, 2048))):
            for t in tgts:
                lib.ppo_gemm_tune(-1, t)
                us = lib.ppo_bench_gemm(2, 32768, n, 512, 20, cfg)
                print(f"rep {rep} op2 n={n} cfg={cfg} target={t} {us:7.1f} us {2 * 32768 * n * 512 / us / 1e6:6.1f} TF/s",
                      flush=True)
lib.ppo_gemm_tune(-1, 0)
