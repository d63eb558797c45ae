#!/usr/bin/env python3
"""bench.py — PPO-update throughput of libppo on MI355X (BASELINE.json metric).

A "step" is ONE PPO update over a device-resident synthetic rollout: GAE (two value
forwards over the whole buffer + exact scan + global normalisation), then 10 value
epochs and 4 policy epochs of ⌊N/B⌋ minibatches each (reference defaults, main.c:39-40).
Workload (config C4 of BASELINE.json): Humanoid-shaped 376 → 3×512 → 17 MLPs, ONE 4096-step ×
256-env rollout, B = N/32 = 32768, fp32.  Data-parallel runs split that rollout by whole
environments (SURVEY §8(e), strong scaling — the default): rank r owns envs [r·E/G, (r+1)·E/G)
and draws B/G rows per minibatch step, gradients are all-reduced with RCCL inside libppo each
step (÷G: the gradient of the global B-row minibatch), advantage statistics are global.  `--weak`
(opt-in, labelled "weak") gives every rank a whole 4096×256 rollout instead.  `--emulate-world G`
runs rank 0's shard of a G-way split on one GPU (E/G envs, B/G rows), for tuning the shard shapes.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4|c3|c2|c5|c5f32] [--batch B] [--weak]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N
    (torch.distributed.run is only the launcher: this process never imports torch)

Prints ONE JSON line (rank 0).  `value` = learner env-steps/s over all ranks = world·N / t_update.
"""
import argparse
import ctypes as C
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ppo.c_amd"))

# No torch in this process: libppo owns the device, the stream and RCCL, so the process maps ONE HIP
# runtime (torch's wheel bundles a second one).  torch.distributed.run is only the
# launcher; ranks exchange the RCCL unique id through a file (exchange_unique_id) and the barrier /
# max-over-ranks timing run over libppo's communicator.
import numpy as np  # noqa: E402

import ppo_ffi  # noqa: E402

LIB = ppo_ffi.load() if __name__ == "__main__" else None

CONFIGS = {
    # name: (S, hidden, A, T, E, batch)   — BASELINE.json configs
    "c2": (3, [64, 64], 1, 4096, 1, 64),
    "c3": (17, [256, 256], 6, 4096, 64, 8192),
    "c4": (376, [512, 512, 512], 17, 4096, 256, 32768),
    "c5": (1024, [1024, 1024, 1024, 1024], 17, 8192, 64, 16384),        # bf16 MFMA (8-GPU shard of 8192×512)
    "c5f32": (1024, [1024, 1024, 1024, 1024], 17, 8192, 64, 16384),
}
METRIC = "PPO updates/sec + env-steps/sec on 4096×256 synthetic rollout, 1/2/4/8 MI355X"
PEAK_FP32_MFMA_TFLOPS = 157.3          # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 (spec; 155 measured)
PEAK_BF16_MFMA_TFLOPS = 2500.0         # MI355X_MICROARCH.md: dense bf16 MFMA (spec, no sparsity)
DTYPE = {"c5": "bf16"}                 # compute precision per config (default fp32)
# configs whose CONFIGS entry is ONE rank's shard of BASELINE.json's rollout: C5 is 8192 × 512 envs over
# 8 MI355X (B = 131072 global), i.e. 8192 × 64 envs and B / 8 = 16384 rows per rank per step
SHARD_OF = {"c5": 8, "c5f32": 8}
PEAK_HBM_GBPS = 8000.0
# x3 engine (fp32 mode's default GEMMs): six bf16-MFMA products per fp32 product, so the MFMA bound
# of the fp32 algorithmic FLOPs is the dense bf16 peak / 6
PEAK_X3_TFLOPS = PEAK_BF16_MFMA_TFLOPS / 6


def algorithmic_flops(S, H, A, N, B, n_v=10, n_p=4):
    """F = 4·N·P_V + n_v·⌊N/B⌋·B·(6P_V − 2·S·H1) + n_p·⌊N/B⌋·B·(6P_μ − 2·S·H1)."""
    def P(sizes):
        return sum(a * b for a, b in zip(sizes[:-1], sizes[1:]))
    P_mu, P_v = P([S] + H + [A]), P([S] + H + [1])
    nb = (N // B) * B
    return 4 * N * P_v + n_v * nb * (6 * P_v - 2 * S * H[0]) + n_p * nb * (6 * P_mu - 2 * S * H[0])


def uid_path(world):
    """Rendezvous file of one launch: torch.distributed.run starts every local rank as a child of one
    agent process, so (agent pid, master port, run id) names this launch and nothing else."""
    tag = f"{os.getppid()}_{os.environ.get('MASTER_PORT', '0')}_{os.environ.get('TORCHELASTIC_RUN_ID', 'none')}"
    return os.path.join(os.environ.get("PPO_RDZV_DIR", "/tmp"), f"ppo_rccl_uid_{tag}_w{world}")


def exchange_unique_id(rank, world, make_id, timeout_s=300.0, path=None):
    """Rank 0 publishes the RCCL unique id (atomic rename); the other ranks poll for it."""
    path = path or uid_path(world)
    if rank == 0:
        uid = make_id()
        tmp = f"{path}.tmp{os.getpid()}"
        with open(tmp, "wb") as f:
            f.write(uid)
        os.replace(tmp, path)
        return uid
    t0 = time.time()
    while True:
        try:
            with open(path, "rb") as f:
                uid = f.read()
            if uid:
                return uid
        except FileNotFoundError:
            pass
        if time.time() - t0 > timeout_s:
            raise SystemExit(f"rank {rank}: no RCCL unique id at {path} after {timeout_s:.0f}s")
        time.sleep(0.01)


def pmc_traffic():
    """HBM bytes per GEMM launch from the newest committed PMC pass (profiles/rNN_pmc_gemm.json:
    separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of this bench, (2·FETCH + WRITE)·1 KiB)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_gemm.json")))
    if not files:
        return {}, None
    d = json.load(open(files[-1]))
    return d, os.path.relpath(files[-1], ROOT)


def cpu_info():
    """CPU model (/proc/cpuinfo), the machine's logical CPUs and the ones this process may use."""
    model = platform.machine()
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = os.cpu_count() or 1
    return model, os.cpu_count() or 1, usable


def cpu_baseline(lib, ppo, S, H, A, N, B, sample_envs=16, steps=2):
    """The oracle (plain-C restatement of the reference CPU path, OpenBLAS sgemm, 1 thread) on a bounded
    sample of the same workload; extrapolated to one full update with the update formula."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_ffi

    oracle_ffi.build()
    olib = oracle_ffi.load(use_openblas=True)
    blas = olib.ref_blas_name().decode()
    T = N // 256 if N >= 256 else N
    Ns = min(N, sample_envs * T)                          # whole envs → whole GAE segments
    Bs = min(B, Ns)
    b = ppo.contents.buffer.contents
    buf = {
        "state": ppo_ffi.d2h(lib, b.d_state_p, np.float32, Ns * S).reshape(Ns, S),
        "next_state": ppo_ffi.d2h(lib, b.d_next_state_p, np.float32, Ns * S).reshape(Ns, S),
        "action": ppo_ffi.d2h(lib, b.d_action_p, np.float32, Ns * A).reshape(Ns, A),
        "reward": ppo_ffi.d2h(lib, b.d_reward_p, np.float32, Ns),
        "logprob": ppo_ffi.d2h(lib, b.d_logprob_p, np.float32, Ns),
        "terminated": ppo_ffi.d2h(lib, b.d_terminated_p, np.uint8, Ns),
        "truncated": ppo_ffi.d2h(lib, b.d_truncated_p, np.uint8, Ns),
    }
    sizes = [S] + H + [A]

    def packed(nn_ptr):
        nn = nn_ptr.contents
        out = []
        for i in range(nn.num_layers - 1):
            ly = nn.layers[i]
            out.append(ppo_ffi.d2h(lib, ly.d_weights, np.float32, ly.input_size * ly.output_size))
            out.append(ppo_ffi.d2h(lib, ly.d_biases, np.float32, ly.output_size))
        return np.concatenate(out)

    pol = ppo.contents.policy.contents
    mu0 = packed(pol.mu)
    ls0 = ppo_ffi.d2h(lib, pol.d_log_std, np.float32, A)
    v0 = packed(ppo.contents.V)
    nb = N // B

    def timed(threads):
        olib.ref_blas_threads(threads)
        try:
            r = oracle_ffi.ppo_update(sizes, [1] * len(H) + [0], mu0, ls0, v0, buf, batch_size=Bs, shuffle_mode=1,
                                      seed=1, max_value_steps=steps, max_policy_steps=steps)
        finally:
            olib.ref_blas_threads(1)
        t = r["t_gae"] * (N / Ns) + 10 * nb * (r["t_value"] / max(1, r["n_v"])) * (B / Bs) \
            + 4 * nb * (r["t_policy"] / max(1, r["n_p"])) * (B / Bs)
        return r, t, r["t_gae"] + r["t_value"] + r["t_policy"]

    r, t_update, sample_s = timed(1)
    # SURVEY §8d also asks for an all-cores run: the same sample with OpenBLAS on every core this
    # process may use (the box's share: OMP_NUM_THREADS; GAE and the element-wise code stay serial C)
    model, nproc, usable = cpu_info()
    cores = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, usable)
    _, t_all, sample_all = timed(cores)
    return {
        "value": N / t_update, "unit": "env-steps/s", "cores": 1, "kind": "port",
        "sample": (f"oracle (C restatement of the reference CPU path, {blas}, 1 thread): GAE over {Ns} "
                   f"transitions + {r['n_v']} value + {r['n_p']} policy minibatches at B={Bs}, "
                   f"extrapolated to a full update (t={t_update:.1f}s); sample took {sample_s:.1f}s"),
        "cpu": model, "nproc": nproc, "usable_cpus": usable,
        "all_cores": {"value": N / t_all, "unit": "env-steps/s", "cores": cores,
                      "sample": f"same sample, OpenBLAS on {cores} threads (the process's share: OMP_NUM_THREADS "
                                f"or min(16, usable CPUs); the machine has {nproc}) (t={t_all:.1f}s extrapolated; "
                                f"sample took {sample_all:.1f}s)"},
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--weak", action="store_true",
                    help="weak scaling (opt-in): every rank owns a whole rollout of the config; default splits ONE "
                         "rollout over the ranks (SURVEY §8(e))")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="one GPU runs rank 0's shard of a G-way split (E/G envs, B/G rows per step); the line is "
                         "then a per-rank shard measurement, not the metric")
    ap.add_argument("--shuffle", type=int, default=1, help="1 = device Feistel shuffle, 0 = reference host rand()")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-events", action="store_true")
    ap.add_argument("--gemm-flags", type=int, default=0, help="ppo_gemm_flags experiment bits (A/B runs)")
    ap.add_argument("--no-rollout", action="store_true", help="skip the rollout env-steps/s measurement")
    ap.add_argument("--step-limit", default="", help="V,P: cap each update at V value and P policy minibatch steps "
                    "(profiling passes only: a bounded sample of the same launches; the line is then not the metric)")
    ap.add_argument("--event-stride", type=int, default=7,
                    help="HIP events around every k-th launch of each kernel class (1 = all; each event pair "
                         "costs a few µs of stream time, so the throughput run samples)")
    ap.add_argument("--seed", type=int, default=1234)
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        if world == 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one process per GPU)")
    if LIB.ppo_set_device(local) != 0:
        raise SystemExit(f"libppo: cannot select device {local}: {LIB.ppo_last_error().decode()}")

    if world > 1:
        def make_id():
            buf = C.create_string_buffer(256)
            n = LIB.ppo_comm_unique_id(buf, 256)
            return bytes(buf.raw[:n])

        uid = exchange_unique_id(rank, world, make_id)
        if LIB.ppo_comm_init(rank, world, uid) != 0:                      # RCCL over xGMI for the data path
            raise SystemExit(f"ppo_comm_init failed: {LIB.ppo_last_error().decode()}")
        if rank == 0:                                                    # every rank has joined: tidy up
            try:
                os.remove(uid_path(world))
            except OSError:
                pass
    comm_self = world == 1 and os.environ.get("PPO_COMM_SELF", "0") not in ("", "0")
    if comm_self:
        # rehearsal of the data-parallel path on one GPU: a one-rank RCCL communicator, so every
        # gradient all-reduce goes through the comm stream exactly as at world > 1
        if LIB.ppo_comm_init(0, 1, None) != 0:
            raise SystemExit(f"ppo_comm_init (self) failed: {LIB.ppo_last_error().decode()}")

    S, H, A, T, E, B = CONFIGS[args.config]
    shard_of = SHARD_OF.get(args.config, 1)
    split = world if world > 1 else max(1, args.emulate_world)
    if args.weak:
        split = 1
    if split > 1:
        if E % split or B % split:
            raise SystemExit(f"config {args.config}: E={E}, B={B} do not split over {split} ranks")
        E = E // split
        B = B // split
    if args.batch:
        B = args.batch
    N = T * E
    sizes = [S] + H + [A]
    acts = ["relu"] * len(H) + ["none"]

    if args.gemm_flags:
        LIB.ppo_gemm_flags(args.gemm_flags)
    C.CDLL("libc.so.6").srand(args.seed)                                 # identical init on every rank
    ppo = LIB.create_ppo(ppo_ffi.c_strings(acts), ppo_ffi.c_ints(sizes), len(sizes), N, 3e-4, 3e-4, 0.95, 0.2, 0.0,
                         1.0, True)
    dtype = DTYPE.get(args.config, "fp32")
    engine = "bf16" if dtype == "bf16" else ("x3" if LIB.ppo_gemm_f32_engine(-1) == 1 else "exact")
    peak = {"bf16": PEAK_BF16_MFMA_TFLOPS, "x3": PEAK_X3_TFLOPS, "exact": PEAK_FP32_MFMA_TFLOPS}[engine]
    if LIB.ppo_set_compute_dtype(ppo, 1 if dtype == "bf16" else 0) != 0:
        raise SystemExit("ppo_set_compute_dtype failed")
    LIB.ppo_fill_synthetic(ppo, E, T, args.seed * 1000 + rank, 1.0 / 500)
    if args.step_limit:
        lv, lp = (int(v) for v in args.step_limit.split(","))
        LIB.ppo_set_step_limit(ppo, lv, lp)
    LIB.ppo_synchronize()

    def barrier():
        LIB.ppo_synchronize()
        LIB.ppo_comm_barrier()

    for _ in range(args.warmup):
        LIB.ppo_update(ppo, 0.99, B, 4, 10, args.shuffle, args.seed)
    barrier()
    LIB.ppo_reset_stats(ppo)
    LIB.ppo_prof_reset()
    # the timed region only counts launches and their algorithmic work (a stride this large records
    # one event pair per class); kernel timing is the serialised pass below
    LIB.ppo_prof_enable(1 << 30)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        LIB.ppo_update(ppo, 0.99, B, 4, 10, args.shuffle, args.seed)
    barrier()
    elapsed = time.perf_counter() - t0
    LIB.ppo_prof_enable(0)
    elapsed = LIB.ppo_comm_max_f64(elapsed)                              # max over ranks

    # batched device rollout of the same E x T (SURVEY §8d "rollout env-steps/s", reported beside
    # the learner throughput; not part of `value`): one warm call, then one timed call
    env_kind = 0 if (S, A) == (3, 1) else 1
    t_rollout = None
    if not args.no_rollout:
        LIB.ppo_rollout_device(ppo, E, T, env_kind, args.seed + rank)
        barrier()
        r0 = time.perf_counter()
        LIB.ppo_rollout_device(ppo, E, T, env_kind, args.seed + rank)
        barrier()
        t_rollout = time.perf_counter() - r0
        t_rollout = LIB.ppo_comm_max_f64(t_rollout)

    def prof_snapshot():
        ms, work, launches = (C.c_double * 7)(), (C.c_double * 7)(), (C.c_long * 7)()
        LIB.ppo_prof_read(ms, work, launches)
        issued, issued_work = (C.c_long * 7)(), (C.c_double * 7)()
        LIB.ppo_prof_counts(issued)
        LIB.ppo_prof_issued_work(issued_work)
        return list(ms), list(work), list(launches), list(issued), list(issued_work)

    ms, work, launches, issued, issued_work = prof_snapshot()
    stats = (C.c_double * 7)()
    LIB.ppo_read_stats(ppo, stats, 7)

    # Kernel pass for the roofline (not part of `value`): in the timed region the value and policy
    # minibatch loops overlap on two streams, so a launch's event time there includes the share of
    # the chip the other stream held.  One more update with the loops serialised (PPO_SERIAL=1)
    # times every event_stride-th launch running alone.
    serial = None
    shapes = []
    if not args.no_kernel_events:
        os.environ["PPO_SERIAL"] = "1"
        LIB.ppo_prof_reset()
        LIB.ppo_prof_kernel_events(1)          # GEMMs: the kernel's own duration (dispatch-stamped)
        LIB.ppo_prof_enable(max(1, args.event_stride))
        barrier()
        s0 = time.perf_counter()
        LIB.ppo_update(ppo, 0.99, B, 4, 10, args.shuffle, args.seed)
        barrier()
        serial_s = time.perf_counter() - s0
        LIB.ppo_prof_enable(0)
        LIB.ppo_prof_kernel_events(0)
        del os.environ["PPO_SERIAL"]
        serial = list(prof_snapshot()) + [serial_s]
        cap = 256
        keys, kms, kl, kw = (C.c_longlong * cap)(), (C.c_double * cap)(), (C.c_long * cap)(), (C.c_double * cap)()
        n_sh = min(cap, LIB.ppo_prof_shapes(keys, kms, kl, kw, cap))
        ops = ["forward", "grad_x", "grad_W", "grad_W+grad_x", "forward+head+grad_W+grad_x"]
        engines = ["exact-fp32", "x3", "bf16"]
        issued_sh = (C.c_long * cap)()
        LIB.ppo_prof_shape_issued(keys, issued_sh, n_sh)
        for i in range(n_sh):
            k = keys[i]
            avg_ms = kms[i] / kl[i]
            # the sampled average of the shape × the launches of it the update really issued: one
            # sampled launch of a rare shape (the 1M-row GAE forward) cannot outweigh a frequent one
            shapes.append({"op": ops[(k >> 60) & 0xF], "engine": engines[(k >> 56) & 0xF], "m": (k >> 32) & 0xFFFFFF,
                           "n": (k >> 16) & 0xFFFF, "l": k & 0xFFFF, "sampled_launches": kl[i],
                           "launches": issued_sh[i], "ms": avg_ms * issued_sh[i], "avg_us": 1000.0 * avg_ms,
                           "work_per_launch": kw[i] / kl[i], "tflops": kw[i] / (kms[i] * 1e-3) / 1e12})
        shapes.sort(key=lambda d: -d["ms"])

    t_update = elapsed / args.steps
    # algorithmic FLOPs of the update: SURVEY §8(d)'s formula counts two full-buffer value forwards for
    # GAE; V(next_state[t]) = V(state[t+1]) is reused wherever the rows are equal, so only the rows of
    # the own next-state forward (stats[7]) are work the update does
    stats_all = (C.c_double * 8)()
    LIB.ppo_read_stats(ppo, stats_all, 8)
    gae_own = int(stats_all[7])
    sv = [S] + H + [1]
    P_v = sum(a * b for a, b in zip(sv[:-1], sv[1:]))
    flops = algorithmic_flops(S, H, A, N, B) - 2.0 * (N - gae_own) * P_v
    # sampled launches: class time per update = mean sampled launch time × launches issued
    # per-class breakdown from the serialised kernel pass (one update) when it ran
    k_ms, k_launches, k_issued, k_updates = (serial[0], serial[2], serial[3], 1) if serial else \
        (ms, launches, issued, args.steps)
    kernels = {k: {"ms_per_update": k_ms[i] / k_launches[i] * k_issued[i] / k_updates,
                   "launches_per_update": k_issued[i] / k_updates, "avg_launch_us": 1000.0 * k_ms[i] / k_launches[i],
                   "sampled_launches": k_launches[i]}
               for i, k in enumerate(["gemm", "gae", "adam", "gather", "head", "comm", "other"]) if k_launches[i]}
    result = {
        "metric": METRIC,
        "value": world * N / t_update,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1000.0 * t_update,
        "higher_is_better": True,
        "scaling": "weak" if args.weak else "strong",
        "vs_baseline": None,
        "dtype": dtype,
        "data": "synthetic (seeded device generator: obs U(-1,1), actions from the policy, rewards 0.1·N(0,1), "
                "terminated Bernoulli(1/500), truncated at env-segment ends); random-init weights",
        "config": {"workload": f"{args.config}: {S}->{'x'.join(map(str, H))}->{A} MLP (policy + value), " + (
                               f"{T} steps x {E} envs = one rank's shard of the {T}x{E * shard_of} rollout split "
                               f"over {shard_of} ranks (B/{shard_of}={B} rows per rank per step, global B="
                               f"{B * shard_of}), measured as one GPU's share of that job"
                               if shard_of > 1 and split == 1 and world == 1 else
                               f"{T} steps x {E * split} envs" + (f" split over {split} ranks ({E} envs, B/{split}="
                               f"{B} rows per rank per step)" if split > 1 else "") +
                               (" per GPU (weak scaling)" if args.weak else "") +
                               f", global B={B * (world if args.weak else split)}") + ", 10 value + 4 policy epochs",
                   "global_batch": B * (world if args.weak else split) * (shard_of if split == 1 and world == 1 else 1),
                   "rollout_per_gpu": N,
                   "per_rank_shard_of": shard_of if shard_of > 1 else None,
                   "parallelism": f"dp{world}",
                   "emulated_world": args.emulate_world if (world == 1 and args.emulate_world > 1) else None,
                   "comm": ("rccl-self (1-rank rehearsal)" if comm_self else ("rccl" if world > 1 else "none")) +
                           (f"; gradient all-reduce {LIB.ppo_comm_mode().decode()}" if world > 1 or comm_self else ""),
                   "shuffle": "device-feistel" if args.shuffle else "host-rand"},
        "updates_per_sec": 1.0 / t_update,
        "rollout_env_steps_per_sec": (world * N / t_rollout) if t_rollout else None,
        "iteration_env_steps_per_sec": (world * N / (t_rollout + t_update)) if t_rollout else None,
        "rollout": {"env": "pendulum-v1" if env_kind == 0 else "synthetic", "envs_per_gpu": E, "horizon": T,
                    "ms": 1000.0 * t_rollout if t_rollout else None},
        "minibatch_steps_per_sec": 14 * (N // B) / t_update,
        "algorithmic_tflop_per_update": flops / 1e12,
        "gae_next_state_forward_rows": gae_own,
        "mfma_frac_whole_update": flops / t_update / (peak * 1e12),
        "kernels": kernels,
        "loss": {"value_mean": stats[0] / max(1.0, stats[1]), "policy_mean": stats[2] / max(1.0, stats[3])},
    }
    if serial and serial[2][0] and serial[0][0] > 0:
        s_ms, s_work, s_launches = serial[0][0], serial[1][0], serial[2][0]
        # the GEMM class over one serial update: Σ_shape issued·work ÷ Σ_shape issued·(sampled average
        # duration) — the rate a rocprofv3 trace of the same serial update gives (every launch timed)
        tot_work = sum(sh["launches"] * sh["work_per_launch"] for sh in shapes)
        tot_ms = sum(sh["ms"] for sh in shapes)
        achieved = tot_work / (tot_ms * 1e-3) / 1e12 if tot_ms > 0 else s_work / (s_ms * 1e-3) / 1e12
        pmc, traffic_src = pmc_traffic() if args.config == "c4" else ({}, None)   # PMC passes are of c4
        traffic = pmc.get("hbm_bytes_per_launch")
        # dominant kernel = the kernel TEMPLATE (op × engine: one compiled kernel family, e.g. the x3
        # grad_W TN) with the most time in the serialised update (each shape's sampled average × its
        # issued launches), over all its shapes: Σ 2mnl ÷ Σ time; shapes as [m, n, l, launches, avg µs]
        groups = {}
        for sh in shapes:
            g = groups.setdefault((sh["op"], sh["engine"]), {"op": sh["op"], "engine": sh["engine"], "launches": 0,
                                                           "ms": 0.0, "work": 0.0, "bytes": 0.0, "shapes": []})
            g["launches"] += sh["launches"]
            g["ms"] += sh["ms"]
            g["work"] += sh["work_per_launch"] * sh["launches"]
            m_, n_, l_ = sh["m"], sh["n"], sh["l"]
            # operands read once, output written once (fp32; grad_W: + its bias-gradient vector)
            g["bytes"] += sh["launches"] * 4 * (m_ * n_ + n_ * l_ + m_ * l_ + (l_ if sh["op"] == "grad_W" else 0))
            g["shapes"].append([m_, n_, l_, sh["launches"], round(sh["avg_us"], 2)])
        dom = None
        if groups:
            g = max(groups.values(), key=lambda v: v["ms"])
            dom = {"op": g["op"], "engine": g["engine"], "template": {"forward": "NT", "grad_x": "NN", "grad_W": "TN",
                                                                      "grad_W+grad_x": "pair",
                                                                      "forward+head+grad_W+grad_x": "fused"}.get(g["op"]),
                   "launches": g["launches"], "ms": g["ms"], "avg_us": 1000.0 * g["ms"] / g["launches"],
                   "tflops": g["work"] / (g["ms"] * 1e-3) / 1e12,
                   "algorithmic_bytes": g["bytes"] / g["launches"], "shapes": g["shapes"]}
            dom["frac"] = dom["tflops"] / peak
            # the PMC pass's kernel of this op (template's first parameter) with the most launches
            # in the traced update: for C4 the 512-wide hidden-layer instance of the dominant op
            code = {"forward": "0", "grad_x": "1", "grad_W": "2"}.get(dom["op"])
            cand = [(v.get("launches_in_update", 0), k, v) for k, v in (pmc.get("by_kernel") or {}).items()
                    if k.startswith(f"gemm<{code}, ") and "true" not in k and "false" not in k   # x3 template
                    and dom.get("engine") == "x3"]
            if cand:
                _, k, v = max(cand)
                dom["traffic"] = v.get("hbm_bytes_per_launch")
                dom["traffic_kernel"] = k
        # lower bound of the GEMM class rate in the timed (concurrent) region: every GEMM launch's
        # algorithmic FLOPs over the whole wall time (non-GEMM time counted as GEMM-idle)
        conc = issued_work[0] / elapsed / 1e12
        result["roofline"] = {"bound": "mfma", "achieved": achieved, "peak": peak,
                              "unit": "TFLOP/s", "frac": achieved / peak, "traffic": traffic,
                              "traffic_source": traffic_src,
                              "kernel": {"bf16": "gemm_bf16_kernel / gemm_bf16_db_kernel",
                                         "x3": "gemm_x3_kernel (x3 engine: hidden and input layers) + "
                                               "gemm_f32_kernel / gemm_pair_kernel (1- and A-wide output layers)",
                                         "exact": "gemm_f32_kernel"}[engine] +
                                        " (every linear-layer launch of one serialised update after the timed "
                                        "region; Σ 2MNK / Σ kernel duration, each duration stamped by the "
                                        "kernel's own dispatch (hipExtLaunchKernel events), as rocprofv3 "
                                        "--kernel-trace measures it)",
                              "dominant": dom,
                              "by_shape": shapes[:12],
                              "gemm_engine": engine,
                              "peak_basis": {"bf16": "dense bf16 MFMA spec",
                                             "x3": "dense bf16 MFMA spec / 6 (six bf16 products per fp32 product)",
                                             "exact": "fp32 MFMA spec (v_mfma_f32_32x32x2_f32)"}[engine],
                              "fp32_mfma_peak": PEAK_FP32_MFMA_TFLOPS,
                              "launches": sum(sh["launches"] for sh in shapes), "sampled_launches": s_launches,
                              "event_stride": args.event_stride,
                              "avg_launch_us": 1000.0 * tot_ms / max(1, sum(sh["launches"] for sh in shapes)),
                              "algorithmic_flop_per_launch": tot_work / max(1, sum(sh["launches"] for sh in shapes)),
                              "serial_update_ms": 1000.0 * serial[5],
                              "concurrent_class_tflops": conc, "concurrent_class_frac": conc / peak}
    if (world > 1 or comm_self) and "comm" in kernels:
        # the gradient all-reduce as the serialised pass timed it (issuing stream ready -> collective
        # done, per minibatch step): at world > 1 this is the exposed xGMI time SCALE runs pay per step
        steps = 14 * (N // B)
        result["comm"] = {"mode": LIB.ppo_comm_mode().decode(),
                          "ms_per_update": kernels["comm"]["ms_per_update"],
                          "us_per_minibatch_step": 1000.0 * kernels["comm"]["ms_per_update"] / steps,
                          "collectives_per_update": kernels["comm"]["launches_per_update"],
                          "replica_check": os.environ.get("PPO_REPLICA_CHECK", "1") != "0" and world > 1}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(LIB, ppo, S, H, A, N, B)
        result["cpu_baseline"]["gpu_over_cpu"] = result["value"] / result["cpu_baseline"]["value"]
    LIB.free_ppo(ppo)
    LIB.ppo_comm_finalize()
    if rank == 0:
        print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
