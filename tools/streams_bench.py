import os, sys
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "ppo.c_amd"))
import ppo_ffi
lib = ppo_ffi.load(); lib.ppo_set_device(0)
for B in (32768,):
    for two in (0, 1, 0, 1):
        us = lib.ppo_bench_streams(two, 10, B, 17)
        print(f"B={B} two={two} total {us/1000:.2f} ms  per step-pair {us/10:.1f} us", flush=True)
