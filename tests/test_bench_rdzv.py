"""bench.py's torch-free rendezvous: rank 0 publishes the RCCL unique id through a file, the other ranks
read it (CPU test: fake id bytes, world_size 4 processes started at once, some before rank 0)."""
import multiprocessing as mp
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rank(rank, world, path, q):
    sys.path.insert(0, ROOT)
    import bench
    uid = bench.exchange_unique_id(rank, world, lambda: bytes(range(128)), timeout_s=30, path=path)
    q.put((rank, uid))


def test_exchange_unique_id(tmp_path):
    path = str(tmp_path / "uid")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, 4, path, q)) for r in (3, 1, 2, 0)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=60) for _ in procs)
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    assert sorted(got) == [0, 1, 2, 3]
    assert all(v == bytes(range(128)) for v in got.values())
    assert not [f for f in os.listdir(tmp_path) if ".tmp" in f]      # published by an atomic rename


def test_uid_path_names_one_launch(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setenv("MASTER_PORT", "29511")
    a = bench.uid_path(8)
    monkeypatch.setenv("MASTER_PORT", "29512")
    assert bench.uid_path(8) != a and str(os.getppid()) in a
