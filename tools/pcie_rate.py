#!/usr/bin/env python3
"""PCIe-inclusive C4 rate: the reference API hands the rollout over in host memory (train_ppo_epoch
→ buffer_to_device, pageable malloc'd arrays), so one update costs the H2D copy of the buffer plus
the update itself.  Reported in DESIGN §5 beside bench.py's HBM-resident `value` (never as it).

    python tools/pcie_rate.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo.c_amd"))
import ppo_ffi  # noqa: E402

S, H, A, T, E, B = 376, [512, 512, 512], 17, 4096, 256, 32768
N = T * E
lib = ppo_ffi.load()
lib.ppo_set_device(0)
sizes = [S] + H + [A]
ppo = lib.create_ppo(ppo_ffi.c_strings(["relu"] * len(H) + ["none"]), ppo_ffi.c_ints(sizes), len(sizes), N, 3e-4,
                     3e-4, 0.95, 0.2, 0.0, 1.0, True)
lib.ppo_fill_synthetic(ppo, E, T, 1234, 1.0 / 500)
buf = ppo.contents.buffer
lib.buffer_to_host(buf)                      # rollout now lives in host memory, as after a CPU rollout
lib.ppo_synchronize()
nbytes = N * (4 * (2 * S + A + 4) + 2)
res = []
for it in range(4):
    t0 = time.perf_counter()
    lib.buffer_to_device(buf)
    lib.ppo_synchronize()
    t1 = time.perf_counter()
    lib.ppo_update(ppo, 0.99, B, 4, 10, 1, 1234)
    lib.ppo_synchronize()
    t2 = time.perf_counter()
    lib.buffer_to_host(buf)
    lib.ppo_synchronize()
    if it:                                   # first iteration warms up
        res.append((t1 - t0, t2 - t1))
h2d = sum(r[0] for r in res) / len(res)
upd = sum(r[1] for r in res) / len(res)
print(f"C4 host buffer {nbytes / 1e9:.2f} GB: H2D {1e3 * h2d:.1f} ms ({nbytes / h2d / 1e9:.1f} GB/s), update "
      f"{1e3 * upd:.1f} ms; PCIe-inclusive {N / (h2d + upd) / 1e6:.2f} M env-steps/s vs HBM-resident "
      f"{N / upd / 1e6:.2f} M")
lib.free_ppo(ppo)
