#!/usr/bin/env python3
"""Generate tests/golden/*.npz — independent float64 known answers for the oracle.

The reference (cube1324/ppo.c) ships no tests, fixtures or golden vectors, and its CPU path cannot be
built here (it needs CUDA/cuBLAS/CBLAS headers).  These fixtures therefore restate the reference's
math independently of oracle/ref_cpu.c: float64 numpy loops, torch autograd and torch.optim.Adam
(CPU), and a Python model of glibc's rand() (TYPE_3 additive feedback generator).  Every fixture
names the reference lines it encodes.  Inputs are small and seeded; rerun to regenerate:

    python tests/golden/make_golden.py
"""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def glibc_rand(seed, count):
    """glibc random()/rand() with the default TYPE_3 state (the libc the reference links)."""
    r = [0] * (34 + 310 + count)
    r[0] = seed & 0xFFFFFFFF
    if r[0] == 0:
        r[0] = 1
    for i in range(1, 31):
        hi, lo = divmod(r[i - 1], 127773)
        word = 16807 * lo - 2836 * hi
        if word < 0:
            word += 2147483647
        r[i] = word
    for i in range(31, 34):
        r[i] = r[i - 31]
    for i in range(34, 344 + count):
        r[i] = (r[i - 31] + r[i - 3]) & 0xFFFFFFFF
    return [r[i] >> 1 for i in range(344, 344 + count)]


def linear(rng):
    m, n, l = 33, 7, 5
    x, W, b, g = rng.normal(size=(m, n)), rng.normal(size=(l, n)), rng.normal(size=l), rng.normal(size=(m, l))
    # mat_mul.cu:39-80 — out = x·Wᵀ + b; grad_x = g·W; grad_W = gᵀ·x
    return dict(x=x, W=W, b=b, g=g, y=x @ W.T + b, gx=g @ W, gW=g.T @ x)


def mlp(rng):
    import torch

    sizes, relu = [3, 16, 16, 2], [1, 1, 0]
    m = 20
    params = []
    for a, b in zip(sizes[:-1], sizes[1:]):
        params += [rng.normal(scale=0.5, size=(b, a)), rng.normal(scale=0.1, size=b)]
    x = rng.normal(size=(m, sizes[0]))
    go = rng.normal(size=(m, sizes[-1]))
    tp = [torch.tensor(p, dtype=torch.float64, requires_grad=True) for p in params]
    h = torch.tensor(x)
    acts = []
    for i in range(len(sizes) - 1):                      # neural_network.cu:163-189
        h = h @ tp[2 * i].T + tp[2 * i + 1]
        if relu[i]:
            h = torch.relu(h)
        acts.append(h.detach().numpy().copy())
    (h * torch.tensor(go)).sum().backward()               # backward of Σ go·y (neural_network.cu:192-231)
    flat = np.concatenate([p.ravel() for p in params])
    grads = np.concatenate([t.grad.numpy().ravel() for t in tp])
    return dict(sizes=np.array(sizes), relu=np.array(relu), params=flat, x=x, grad_out=go,
                out=acts[-1], acts=np.concatenate([a.ravel() for a in acts]), grads=grads)


def policy(rng):
    import torch

    m, A = 25, 3
    mu = rng.normal(size=(m, A))
    log_std = rng.normal(scale=0.3, size=A)
    action = mu + rng.normal(size=(m, A)) * np.exp(log_std)
    gin = rng.normal(size=m)
    tmu = torch.tensor(mu, requires_grad=True)
    tls = torch.tensor(log_std, requires_grad=True)
    ta = torch.tensor(action)
    # policy.cu:67-74: log π = −½·A·log 2π − Σ_j [log σ_j + ½((a−μ)/σ_j)²]
    lp = -0.5 * A * np.log(2 * np.pi) - (tls + 0.5 * ((ta - tmu) / torch.exp(tls)) ** 2).sum(1)
    (lp * torch.tensor(gin)).sum().backward()
    ent = A * 0.5 * (1 + np.log(2 * np.pi)) + log_std.sum()   # policy.cu:171-178
    return dict(mu=mu, log_std=log_std, action=action, grad_in=gin, log_prob=lp.detach().numpy(),
                grad_mu=tmu.grad.numpy(), grad_log_std=tls.grad.numpy(), entropy=np.array(ent))


def surrogate(rng):
    import torch

    m, eps, c = 40, 0.2, 0.01
    adv = rng.normal(size=m)
    adv[::7] = 0.0
    old = rng.normal(size=m)
    lp = old + rng.normal(scale=0.4, size=m)
    tlp = torch.tensor(lp, requires_grad=True)
    ratio = torch.exp(tlp - torch.tensor(old))
    ta = torch.tensor(adv)
    pos = ta > 0
    # ppo.cu:82-107: A > 0: r > 1+ε → 1+ε else r;  A ≤ 0: r < 1−ε → 1−ε else r
    val = torch.where(pos, torch.where(ratio > 1 + eps, torch.full_like(ratio, 1 + eps), ratio),
                      torch.where(ratio < 1 - eps, torch.full_like(ratio, 1 - eps), ratio))
    entropy = 1.2345
    loss = -(ta * val).mean() - c * entropy
    loss.backward()
    return dict(adv=adv, lp=lp, old_lp=old, epsilon=np.array(eps), ent_coeff=np.array(c),
                entropy=np.array(entropy), loss=np.array(loss.item()), grad_lp=tlp.grad.numpy())


def gae(rng):
    n, gamma, lam = 64, 0.99, 0.95
    v, vn, r = rng.normal(size=n), rng.normal(size=n), rng.normal(size=n)
    term = (rng.uniform(size=n) < 0.08).astype(np.uint8)
    trunc = np.zeros(n, np.uint8)
    trunc[15::16] = 1
    trunc &= 1 - term
    adv = np.zeros(n)
    nxt = 0.0
    for t in range(n - 1, -1, -1):                       # ppo.cu:340-349
        delta = r[t] + gamma * vn[t] * (1 - term[t]) - v[t]
        nxt = delta + gamma * lam * (1 - (term[t] | trunc[t])) * nxt
        adv[t] = nxt
    target = v + adv                                     # ppo.cu:351-353
    mean, std = adv.mean(), adv.std()                    # population σ (ppo.cu:355-362)
    return dict(v=v, v_next=vn, reward=r, terminated=term, truncated=trunc, gamma=np.array(gamma),
                lam=np.array(lam), adv_target=target, advantage=(adv - mean) / (std + 1e-8),
                mean=np.array(mean), std=np.array(std))


def adam(rng):
    import torch

    n, lr, steps = 37, 3e-4, 5
    p0 = rng.normal(size=n)
    grads = rng.normal(size=(steps, n))
    grads[:, :3] = 1e-9                                   # tiny gradients: the sign-amplified corner
    t = torch.tensor(p0, requires_grad=True)
    opt = torch.optim.Adam([t], lr=lr, betas=(0.9, 0.999), eps=1e-8)   # == adam.cu:53-74
    out = []
    for k in range(steps):
        t.grad = torch.tensor(grads[k])
        opt.step()
        out.append(t.detach().numpy().copy())
    return dict(p0=p0, grads=grads, lr=np.array(lr), params=np.array(out))


def rand_vectors():
    seeds = [1, 42, 1234]
    seq = np.array([glibc_rand(s, 64) for s in seeds], dtype=np.int64)
    # trajectory_buffer.cu:126-146 — swap(i, rand() % N) shuffle of 0..N−1 after srand(seed)
    n = 50
    r = glibc_rand(7, n)
    perm = list(range(n))
    for i in range(n):
        j = r[i] % n
        perm[i], perm[j] = perm[j], perm[i]
    return dict(seeds=np.array(seeds), rand=seq, shuffle_seed=np.array(7), shuffle=np.array(perm))


def init_vectors():
    # neural_network.cu:40-51 for sizes {3, 4, 2} from srand(5), float32 arithmetic as in C
    sizes = [3, 4, 2]
    r = glibc_rand(5, 64)
    k = 0
    out = []
    f = np.float32
    RAND_MAX = f(2147483647)
    for i in range(len(sizes) - 1):
        a, b = sizes[i], sizes[i + 1]
        gain = f(1) if i == len(sizes) - 2 else np.sqrt(f(2.0))
        std = f(gain * np.sqrt(f(2.0 / (a + b))))
        for _ in range(a * b):
            out.append(f((f(2) * f(r[k]) / RAND_MAX - f(1)) * np.sqrt(f(3.0)) * std))
            k += 1
        for _ in range(b):
            # float expression times the DOUBLE (1. / sqrtf(in)), rounded once to float
            out.append(f(np.float64(f(2) * f(r[k]) / RAND_MAX - f(1)) * (1.0 / np.float64(np.sqrt(f(a))))))
            k += 1
    return dict(sizes=np.array(sizes), seed=np.array(5), params=np.array(out, np.float32))


def main():
    rng = np.random.default_rng(20250404)
    for name, fn in (("linear", linear), ("mlp", mlp), ("policy", policy), ("surrogate", surrogate),
                     ("gae", gae), ("adam", adam)):
        np.savez(os.path.join(HERE, f"{name}.npz"), **fn(rng))
    np.savez(os.path.join(HERE, "rand.npz"), **rand_vectors())
    np.savez(os.path.join(HERE, "init.npz"), **init_vectors())
    print("wrote", sorted(f for f in os.listdir(HERE) if f.endswith(".npz")))


if __name__ == "__main__":
    main()
