"""The data-parallel replica check (replicated Adam "verified with a periodic checksum
all-reduce"; reference optimiser order ppo.cu:440-442, run on every rank).

Every rank hashes its HBM parameters (μ, log σ, V: Σ mix(index, bits) mod 2^64, so equal bits give
equal hashes and one changed bit changes it), the hashes are all-gathered and compared with rank 0's.
One GPU stands in for two ranks through PPO_COMM_LOOPBACK=2: the other rank's hash is registered
(ppo_comm_loopback_peer_hash), so a drifted peer is rank 1 of a real two-rank job.
"""
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

import ppo_ffi
from helpers import F32
from test_gpu_update import make_ppo

pytestmark = pytest.mark.gpu

SIZES = [17, 256, 256, 6]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _poke(lib, d_ptr, index, delta):
    """Add `delta` to one float of a device array (the drift a diverged replica would carry)."""
    v = ppo_ffi.d2h(lib, d_ptr, F32, index + 1)
    v[index] = np.float32(v[index] + delta)
    addr = ppo_ffi.C.cast(d_ptr, ppo_ffi.C.c_void_p).value + 4 * index
    lib.ppo_h2d(ppo_ffi.C.c_void_p(addr), v[index:].ctypes.data_as(ppo_ffi.C.c_void_p), 4)


def test_param_hash_is_a_function_of_the_bits(lib, oracle):
    """Equal parameters hash equal (same srand seed → bit-identical initialisation); one ulp in any of μ,
    log σ or V changes the hash; undoing it restores it."""
    a = make_ppo(lib, oracle, SIZES, 256, seed=77)
    b = make_ppo(lib, oracle, SIZES, 256, seed=77)
    c = make_ppo(lib, oracle, SIZES, 256, seed=78)
    ha, hb, hc = lib.ppo_param_hash(a), lib.ppo_param_hash(b), lib.ppo_param_hash(c)
    assert ha == hb and ha != hc
    pb = b.contents.policy.contents
    for ptr, idx in ((pb.mu.contents.d_params, 1234), (pb.d_log_std, 3), (b.contents.V.contents.d_params, 5000)):
        old = ppo_ffi.d2h(lib, ptr, F32, idx + 1)[idx]
        _poke(lib, ptr, idx, np.spacing(np.float32(old)))
        assert lib.ppo_param_hash(b) != ha
        _poke(lib, ptr, idx, -np.spacing(np.float32(old)))
        assert ppo_ffi.d2h(lib, ptr, F32, idx + 1)[idx] == old
        assert lib.ppo_param_hash(b) == ha
    for p in (a, b, c):
        lib.free_ppo(p)


def test_replica_check_names_the_diverged_rank(lib, oracle, monkeypatch):
    """Two in-process ranks: the check passes when the peer holds the same parameters (identical
    replicas, or the peer's registered hash equal to ours) and returns −1 naming rank 1 when the peer's
    parameters differ by one ulp."""
    monkeypatch.setenv("PPO_COMM_LOOPBACK", "2")
    assert lib.ppo_comm_init(0, 1, None) == 0
    try:
        a = make_ppo(lib, oracle, SIZES, 256, seed=91)
        peer = make_ppo(lib, oracle, SIZES, 256, seed=91)
        assert lib.ppo_comm_check_replicas(a) == 0                   # unregistered peer: identical replicas
        h = (ppo_ffi.C.c_ulonglong * 1)(lib.ppo_param_hash(peer))
        assert lib.ppo_comm_loopback_peer_hash(h, 1) == 0
        assert lib.ppo_comm_check_replicas(a) == 0
        pv = peer.contents.V.contents
        old = ppo_ffi.d2h(lib, pv.d_params, F32, 11)[10]
        _poke(lib, pv.d_params, 10, np.spacing(np.float32(old)))
        h[0] = lib.ppo_param_hash(peer)
        assert lib.ppo_comm_loopback_peer_hash(h, 1) == 0
        assert lib.ppo_last_error() in (b"", None), lib.ppo_last_error()
        assert lib.ppo_comm_check_replicas(a) == -1
        err = lib.ppo_last_error().decode()
        assert "replica check" in err and "rank 1" in err, err
        lib.free_ppo(a)
        lib.free_ppo(peer)
    finally:
        lib.ppo_clear_error()                 # the mismatch was this test's own: later tests expect no error
        lib.ppo_comm_loopback_clear()
        lib.ppo_comm_finalize()


def test_update_with_diverged_replica_fails_loudly(tmp_path):
    """ppo_update at world > 1 runs the replica check after the update (PPO_REPLICA_CHECK=1, the
    default) and ends the process with status 1 and a message naming the rank when a peer's parameters
    differ — a drifted replica must not keep training on its own weights.  Run in a child process (the
    failure is fatal by design, as the reference's checks are: cuda_helper.h:4-16)."""
    script = tmp_path / "diverged.py"
    script.write_text(textwrap.dedent(f"""
        import ctypes as C, sys
        sys.path.insert(0, {os.path.join(ROOT, 'ppo.c_amd')!r})
        import ppo_ffi
        lib = ppo_ffi.load()
        assert lib.ppo_comm_init(0, 1, None) == 0
        C.CDLL("libc.so.6").srand(5)
        sizes = [17, 64, 64, 6]
        acts = ["relu", "relu", "none"]
        ppo = lib.create_ppo(ppo_ffi.c_strings(acts), ppo_ffi.c_ints(sizes), 4, 1024, 3e-4, 3e-4, 0.95, 0.2,
                             0.0, 1.0, True)
        lib.ppo_fill_synthetic(ppo, 4, 256, 1, 1.0 / 500)
        lib.ppo_update(ppo, 0.99, 256, 1, 1, 1, 3)                  # identical replicas: passes
        lib.ppo_synchronize()
        print("first update ok", flush=True)
        h = (C.c_ulonglong * 1)(lib.ppo_param_hash(ppo) ^ 1)       # rank 1 drifted
        assert lib.ppo_comm_loopback_peer_hash(h, 1) == 0
        lib.ppo_update(ppo, 0.99, 256, 1, 1, 1, 3)
        lib.ppo_synchronize()
        print("second update returned", flush=True)
    """))
    env = dict(os.environ, PPO_COMM_LOOPBACK="2", PPO_REPLICA_CHECK="1", PPO_NO_TINY="1")
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=120, env=env)
    assert "first update ok" in r.stdout, (r.stdout, r.stderr)
    assert "second update returned" not in r.stdout, (r.stdout, r.stderr)
    assert r.returncode == 1, (r.returncode, r.stdout, r.stderr)
    assert "replica check" in r.stderr and "rank 1" in r.stderr, r.stderr
