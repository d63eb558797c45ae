"""C2 tiny kernels vs the multi-launch path: max |Δ| of value / policy grads after one value step and
after one policy step (specialised kernel, generic kernel, multi-launch)."""
import os
import sys

R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(R, "ppo.c_amd"), os.path.join(R, "oracle"), os.path.join(R, "tests")]
import numpy as np  # noqa: E402
import oracle_ffi as oracle  # noqa: E402
import ppo_ffi  # noqa: E402
from test_gpu_tiny import run  # noqa: E402

lib = ppo_ffi.load()
lib.ppo_set_device(0)
SEG = [("W0", 0, 192), ("b0", 192, 256), ("W1", 256, 4352), ("b1", 4352, 4416), ("W2", 4416, 4480), ("b2", 4480, 4481)]
for shuffle in (0, 1):
    for n_pol, n_val in ((0, 1), (1, 0)):
        os.environ.pop("PPO_TINY_GENERIC", None)
        a = run(lib, oracle, [3, 64, 64, 1], 256, 64, n_pol, n_val, shuffle, tiny=True)
        os.environ["PPO_TINY_GENERIC"] = "1"
        g = run(lib, oracle, [3, 64, 64, 1], 256, 64, n_pol, n_val, shuffle, tiny=True)
        os.environ.pop("PPO_TINY_GENERIC", None)
        b = run(lib, oracle, [3, 64, 64, 1], 256, 64, n_pol, n_val, shuffle, tiny=False)
        for k in ("gv", "gmu", "v", "mu", "ls"):
            print(f"shuffle {shuffle} pol {n_pol} val {n_val} {k}: c2-multi {np.abs(a[k] - b[k]).max():.3g} "
                  f"generic-multi {np.abs(g[k] - b[k]).max():.3g} max|ref| {np.abs(b[k]).max():.3g} "
                  f"argmax {int(np.abs(a[k] - b[k]).argmax())}")
        print("stats", a["stats"], g["stats"], b["stats"])
        k = "gmu" if n_pol else "gv"
        for nm, lo, hi in SEG:
            e = np.abs(a[k][lo:hi] - b[k][lo:hi])
            print(f"   {k} {nm}: max err {e.max():.3g} at {lo + int(e.argmax())}, #>1e-6 {int((e > 1e-6).sum())}, "
                  f"max|ref| {np.abs(b[k][lo:hi]).max():.3g}")
