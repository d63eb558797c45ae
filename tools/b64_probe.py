#!/usr/bin/env python3
"""Small-minibatch probe (the reference's own B = 64): wall µs per minibatch step of a
step-limited update at CONFIG's network, host-issue vs GPU time.

    python tools/b64_probe.py [c4|c3] [B] [value_steps] [policy_steps]
Prints µs per step with both loops concurrent and with PPO_SERIAL=1 semantics (serial run last).
"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo.c_amd"))
import ppo_ffi  # noqa: E402

NETS = {"c4": (376, [512, 512, 512], 17, 4096, 256), "c3": (17, [256, 256], 6, 4096, 64)}
cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
nv = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
npol = int(sys.argv[4]) if len(sys.argv) > 4 else 800
S, H, A, T, E = NETS[cfg]
lib = ppo_ffi.load()
lib.ppo_set_device(0)
sizes = [S] + H + [A]
ppo = lib.create_ppo(ppo_ffi.c_strings(["relu"] * len(H) + ["none"]), ppo_ffi.c_ints(sizes), len(sizes), T * E,
                     3e-4, 3e-4, 0.95, 0.2, 0.0, 1.0, True)
lib.ppo_fill_synthetic(ppo, E, T, 7, 1.0 / 500)
lib.ppo_set_step_limit(ppo, nv, npol)
for serial in (False, True):
    if serial:
        os.environ["PPO_SERIAL"] = "1"
    lib.ppo_update(ppo, 0.99, B, 4, 10, 1, 3)               # warm
    lib.ppo_synchronize()
    t0 = time.perf_counter()
    lib.ppo_update(ppo, 0.99, B, 4, 10, 1, 3)
    t1 = time.perf_counter()
    lib.ppo_synchronize()
    t2 = time.perf_counter()
    print(f"{cfg} B={B} {'serial' if serial else 'concurrent'}: {nv}+{npol} steps, host issue "
          f"{(t1 - t0) * 1e6 / (nv + npol):.1f} us/step, wall {(t2 - t0) * 1e6 / (nv + npol):.1f} us/step", flush=True)
lib.free_ppo(ppo)
