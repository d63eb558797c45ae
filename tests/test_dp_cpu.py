"""CPU, world_size 2 over gloo: the env-sharded data-parallel update math libppo uses.

Each rank owns a contiguous block of environments.  Per minibatch it computes mean-over-local-rows
gradients, sums them with an all-reduce and scales by 1/world (libppo: RCCL all-reduce of the flat
gradient buffer + Adam grad_scale = 1/world); advantage statistics come from an all-gather of Welford
triples (n, mean, M2) combined pairwise.  Both must equal the single-process computation on the
concatenated global minibatch / buffer — checked here with the oracle's kernels.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

F32 = np.float32


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _welford(x):
    x = np.asarray(x, np.float64)
    m = x.mean()
    return np.array([x.size, m, ((x - m) ** 2).sum()])


def _combine(parts):
    n = mean = m2 = 0.0
    for nb, mb, m2b in parts:
        if nb <= 0:
            continue
        nn = n + nb
        d = mb - mean
        mean += d * nb / nn
        m2 += m2b + d * d * n * nb / nn
        n = nn
    return n, mean, m2


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "oracle"))
    import oracle_ffi as oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(0)                 # identical global data on every rank
        sizes, relu = [5, 32, 32, 1], [1, 1, 0]
        oracle.srand(9)
        params = oracle.mlp_init(sizes)
        B_global, E, T = 64, 4, 32
        x_all = rng.uniform(-1, 1, (E * T, sizes[0])).astype(F32)
        t_all = rng.normal(size=E * T).astype(F32)
        # shard: rank r owns envs [r·E/world, (r+1)·E/world); like libppo's sampler each rank draws
        # B_global/world rows of its own shard per minibatch
        shard = (E // world) * T
        picks = [k * shard + rng.permutation(shard)[:B_global // world] for k in range(world)]
        lo, hi = rank * shard, (rank + 1) * shard
        mine = picks[rank]
        x, t = x_all[mine], t_all[mine]
        acts = oracle.mlp_forward(sizes, relu, params, x)
        y = oracle.mlp_layer_outputs(sizes, acts, len(mine))[-1].ravel()
        # local mean-gradient scaled as libppo does: grad = 2(y−t)/B_local, then Σ_ranks / world.
        # With equal shard sizes this equals the global mean gradient.
        _, g = oracle.mse(y, t)
        grads = oracle.mlp_backward(sizes, relu, params, x, acts, g)
        gt = torch.from_numpy(grads.astype(np.float64))
        dist.all_reduce(gt)
        dp_grad = gt.numpy() / world
        # global statistics of a sharded advantage buffer via all-gathered Welford triples
        adv_all = rng.normal(loc=0.3, scale=2.0, size=E * T)
        trip = torch.from_numpy(_welford(adv_all[lo:hi]))
        gathered = [torch.zeros(3, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(gathered, trip)
        n, mean, m2 = _combine([g_.numpy() for g_ in gathered])
        if rank == 0:
            # single-process reference on the same global minibatch (rows ordered by shard)
            order = np.concatenate(picks)
            xa, ta = x_all[order], t_all[order]
            acts_g = oracle.mlp_forward(sizes, relu, params, xa)
            yg = oracle.mlp_layer_outputs(sizes, acts_g, len(order))[-1].ravel()
            _, gg = oracle.mse(yg, ta)
            ref_grad = oracle.mlp_backward(sizes, relu, params, xa, acts_g, gg)
            q.put(dict(dp=dp_grad, ref=ref_grad, n_local=[len(mine)], stats=(n, mean, np.sqrt(m2 / n)),
                       ref_stats=(adv_all.size, adv_all.mean(), adv_all.std())))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_gradient_allreduce_and_global_advantage_stats():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n, mean, std = res["stats"]
    rn, rmean, rstd = res["ref_stats"]
    assert n == rn and abs(mean - rmean) < 1e-12 and abs(std - rstd) < 1e-12
    # all-reduce-sum / world of per-shard mean gradients == gradient of the global minibatch
    np.testing.assert_allclose(res["dp"], res["ref"], rtol=1e-5, atol=1e-6)


@pytest.mark.timeout(300)
def test_two_rank_equal_shards_reproduce_global_mean_gradient():
    """With B/world rows per rank (libppo's sampler), all-reduce-sum / world == global mean gradient."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "oracle"))
    import oracle_ffi as oracle

    rng = np.random.default_rng(1)
    sizes, relu, world, B_local = [5, 32, 32, 1], [1, 1, 0], 2, 32
    oracle.srand(4)
    params = oracle.mlp_init(sizes)
    xs = [rng.uniform(-1, 1, (B_local, 5)).astype(F32) for _ in range(world)]
    ts = [rng.normal(size=B_local).astype(F32) for _ in range(world)]
    local = []
    for x, t in zip(xs, ts):
        acts = oracle.mlp_forward(sizes, relu, params, x)
        y = oracle.mlp_layer_outputs(sizes, acts, B_local)[-1].ravel()
        _, g = oracle.mse(y, t)
        local.append(oracle.mlp_backward(sizes, relu, params, x, acts, g).astype(np.float64))
    dp = sum(local) / world
    xa, ta = np.concatenate(xs), np.concatenate(ts)
    acts = oracle.mlp_forward(sizes, relu, params, xa)
    y = oracle.mlp_layer_outputs(sizes, acts, world * B_local)[-1].ravel()
    _, g = oracle.mse(y, ta)
    ref = oracle.mlp_backward(sizes, relu, params, xa, acts, g)
    np.testing.assert_allclose(dp, ref, rtol=1e-5, atol=1e-6)
