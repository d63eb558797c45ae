/*
 * ppo_ext.h — libppo exports beyond the reference API (additive only).
 *
 * None of these exist in cube1324/ppo.c; they expose what the MI355X build
 * adds: device selection and error reporting (SURVEY §8b "Errors"), the
 * device-resident PPO update over an already-filled buffer (the hot path of
 * reference ppo.cu:479-539 without the host rollout), the batched sampler,
 * the env-sharded data-parallel communicator (RCCL over xGMI),
 * a seeded synthetic rollout generator and kernel timing.
 */
#ifndef PPO_EXT_H
#define PPO_EXT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* PPO / GaussianPolicy objects are passed as void* so this header stands alone. */

/* ---------------- device & errors ----------------
 * Fatal errors (a failed HIP/RCCL call, a grid-barrier timeout of the B = 64 phases, a replica-check
 * mismatch, a stalled collective past PPO_COMM_TIMEOUT_S) END THE EMBEDDING PROCESS with status 1, as
 * the reference's checks do (cuda_helper.h:4-16, exit(1)) — but through _exit(1): after a device fault
 * the HIP runtime's own teardown can hang, so atexit handlers and buffered stdio of the host language
 * (e.g. Python's) do not run.  libppo prints the message to stderr and records it for ppo_last_error
 * first.  Callers that must decide for themselves use the entry points that return a status
 * (ppo_comm_init, ppo_comm_check_replicas, ppo_set_device, …). */
int         ppo_device_count(void);              /* HIP devices visible (0 without a GPU) */
int         ppo_set_device(int device);          /* 0 on success */
const char* ppo_last_error(void);                /* first HIP/RCCL error recorded, "" if none */
void        ppo_clear_error(void);               /* forget it (after a status-returning call the caller handled) */
void        ppo_synchronize(void);               /* drain libppo's stream */
const char* ppo_build_info(void);                /* offload arch, compiler, kernel list */
/* sizeof of the API structs, for FFI layout checks: Layer, NeuralNetwork,
 * GaussianPolicy, TrajectoryBuffer, Adam, PPO, Env (no GPU needed) */
int         ppo_struct_sizes(long* out, int n);

/* raw device memory helpers (tests, bench) */
void* ppo_dev_alloc(size_t bytes);
void  ppo_dev_free(void* p);
void  ppo_h2d(void* dst, const void* src, size_t bytes);
void  ppo_d2h(void* dst, const void* src, size_t bytes);
void  ppo_d2d(void* dst, const void* src, size_t bytes);
void  ppo_dev_memset(void* dst, int value, size_t bytes);

/* ---------------- data parallel (RCCL) ---------------- */
int  ppo_comm_unique_id(unsigned char* out, int cap);   /* returns id size (128) */
int  ppo_comm_init(int rank, int world, const unsigned char* id);  /* 0 on success */
int  ppo_comm_rank(void);
int  ppo_comm_world(void);
void ppo_comm_finalize(void);
/* sum-all-reduce of n floats in place on libppo's stream (no-op at world 1) */
void ppo_comm_allreduce_f32(float* d_buf, long n);
/* host-synchronous helpers over the communicator (identity at world 1): a barrier (every rank's
 * queued work drained, then one collective), and the max over ranks of a host double */
void   ppo_comm_barrier(void);
double ppo_comm_max_f64(double v);
/* the advantage-statistics combine after the all-gather: `count` device triples (n, mean, M2) in
 * double → one triple (Chan et al. pairwise combine; empty parts skipped).  Synchronises. */
void ppo_welford_combine(const double* d_parts, int count, double* d_out);
/* PPO_COMM_LOOPBACK=k (one process standing in for k ranks, tests): the other ranks' contributions,
 * so rank 0 of a k-rank job whose shards DIFFER runs in one process.  welford: host [(k−1)·3]
 * (n, mean, M2) triples of ranks 1…k−1, delivered by the all-gather after the local one; limits: host
 * [k−1] buffer limits for the empty-shard agreement (min over ranks); either may be NULL.  Returns
 * 0, or −1 outside loopback mode or for count ≠ k − 1. */
int  ppo_comm_loopback_peers(const double* welford, const int* limits, int count);
/* an all-reduce of a span inside [d_local_base, d_local_base + n) adds the peers' values at the same
 * offset from d_peers (device, [k−1][n], rank order) instead of the k-fold identical sum; ≤ 4 spans */
int  ppo_comm_loopback_peer_grads(const float* d_local_base, const float* d_peers, long n);
/* the parameter hashes of ranks 1…k−1 for the replica check (host [k−1]) */
int  ppo_comm_loopback_peer_hash(const unsigned long long* hashes, int count);
void ppo_comm_loopback_clear(void);                      /* forget every registered peer contribution */
/* the gradient all-reduce form in use: "none", "inline: …" (default: one all-reduce per step in each
 * loop's stream, a communicator per loop) or "bucketed: …" (PPO_COMM_ASYNC=1, or after a failed split) */
const char* ppo_comm_mode(void);
/* Replica check (SURVEY §8e "verify with a periodic checksum all-reduce"): every rank hashes its
 * parameters (μ, log σ, V: 64-bit, bit-exact), the hashes are all-gathered and compared.  Returns 0
 * when every rank holds rank 0's parameters, −1 otherwise (ppo_last_error names the ranks).
 * Synchronises (bounded: PPO_COMM_TIMEOUT_S).  ppo_update runs it at world > 1 after every
 * PPO_REPLICA_CHECK-th update (default 1; 0 = off) and ends the process on a mismatch. */
int  ppo_comm_check_replicas(void* ppo);
/* this rank's parameter hash (as the replica check computes it; synchronises) */
unsigned long long ppo_param_hash(void* ppo);

/* ---------------- the PPO update ---------------- */
enum { PPO_SHUFFLE_HOST_RAND = 0,   /* reference shuffle_buffer: swap(i, rand()%N), host rand() */
       PPO_SHUFFLE_DEVICE   = 1 };  /* device Feistel bijection, seeded, no host work */

/* One PPO update over the device-resident buffer (limit = full ? capacity : idx):
 * compute_gae_cuda, then n_epochs_value value epochs and n_epochs_policy policy
 * epochs of ⌊limit/batch_size⌋ minibatches (reference ppo.cu:487-533).  With
 * ppo_comm_world() > 1 every rank holds its own env shard; gradients are
 * all-reduced (mean over the global minibatch) and advantage statistics are
 * global.  Asynchronous: nothing is read back to the host — except after the multi-workgroup
 * B = 64 phases (cluster.hip), which synchronise once at the end to check their grid barriers
 * (a timeout ends the process with status 1: the phase's state is incomplete). */
void ppo_update(void* ppo, float gamma, int batch_size, int n_epochs_policy, int n_epochs_value,
                int shuffle_mode, unsigned long long seed);

/* stats accumulated by ppo_update since the last reset (synchronises):
 * out[0]=Σ value loss, out[1]=#value steps, out[2]=Σ policy loss,
 * out[3]=#policy steps, out[4]=entropy, out[5]=advantage mean, out[6]=advantage std,
 * out[7]=rows of the last GAE's own V(next_state) forward (those not reused from V(state[t+1])),
 * out[8]=minibatch steps replayed from captured graphs (PPO_GRAPH=1) */
void ppo_read_stats(void* ppo, double* out, int n);
void ppo_reset_stats(void* ppo);
/* the last GAE's state (compute_gae_cuda / ppo_update; synchronises): welford (may be NULL) ← the
 * (n, mean, M2) triple the normalisation used (global at world > 1; out[3..5] the local triple);
 * v / v_next (may be NULL) ← the first n values of V(state) and V(next_state) the scan read.
 * Returns the number of transitions of that GAE. */
long ppo_gae_state(double* welford, float* v, float* v_next, long n);
/* Parity testing at full size: cap the value / policy minibatch steps of the following ppo_update
 * calls (−1 = no cap).  GAE, the shuffles and their rand() consumption are unchanged; only the
 * loops stop early (so one step of a 1M-row, B = 32768 update can be checked against the oracle). */
void ppo_set_step_limit(void* ppo, long max_value_steps, long max_policy_steps);

/* Batched policy sample on device: a = μ(s) + σ·ε, ε ~ N(0,1) (counter-based
 * Philox + Box–Muller), log_prob per row.  d_* are device pointers. */
void ppo_sample_action_device(void* policy, float* d_state, float* d_action, float* d_log_prob, int m,
                              unsigned long long seed, unsigned long long offset);

/* Seeded synthetic rollout written straight into the device buffer
 * (SURVEY §8d): n_envs env-major segments of `horizon` steps, obs ~ U(−1,1),
 * actions sampled from the current policy, rewards 0.1·N(0,1),
 * terminated ~ Bernoulli(p_terminate), truncated at each segment end. */
void ppo_fill_synthetic(void* ppo, int n_envs, int horizon, unsigned long long seed, float p_terminate);

/* Batched on-device rollout: `horizon` steps of all `n_envs` environments — μ forward
 * over the E current observations, Gaussian sampling (Philox), one environment step — written
 * env-major into the device buffer (transition (e, t) at row e·horizon + t; each segment ends
 * truncated), ready for ppo_update.  env_kind 0 = Pendulum-v1 (S = 3, A = 1; gymnasium dynamics),
 * 1 = synthetic (any S, A).  Episodes continue across calls; the first call (or a change of
 * n_envs / env_kind) resets every environment from `seed`. */
void ppo_rollout_device(void* ppo, int n_envs, int horizon, int env_kind, unsigned long long seed);

/* layer 0's input of the last device forward of a NeuralNetwork*, m rows × input_size fp32, to the
 * host: the gathered minibatch rows the GEMMs read (NeuralNetwork.d_x0) — for parity tests;
 * synchronises.  bf16 copies (x0_dtype 1) are not converted: returns −1 for them and for m beyond the
 * last forward, else 0. */
int ppo_nn_input_rows(void* nn, float* out, int m);

/* ---------------- compute precision ---------------- */
/* 0 = fp32 (default: exact fp32 MFMA GEMMs), 1 = bf16 MFMA GEMMs with fp32 accumulation, fp32
 * master parameters / Adam / heads / GAE, bf16 storage of hidden activations and their gradients
 * (BASELINE config C5).  Returns 0, or −1 for an invalid dtype. */
int ppo_set_compute_dtype(void* ppo, int dtype);
int nn_set_compute_dtype(void* nn, int dtype);          /* NeuralNetwork* */

/* ---------------- GEMM tuning utilities ---------------- */
/* force a tile configuration (−1 = automatic) and the split-K workgroup target of grad_W
 * (0 = per-shape automatic, < 0 keeps the current setting); returns the number of tile configurations */
int    ppo_gemm_tune(int force_cfg, int splitk_target);
/* experiment switches of the fp32 tiled GEMM (bit 0: invert the s_setprio default around the MFMA block; bit 2 (value 4): grad_W and grad_x of a layer as two launches instead of one paired launch); flags < 0
 * only queries; returns the previous value */
int    ppo_gemm_flags(int flags);
/* average device µs of one launch: op 0 = forward (bias+ReLU), 1 = grad_x, 2 = grad_W (+bias grad),
 * 3 = forward without activation (output layer);
 * m = batch, n = in, l = out; cfg −1 = automatic */
double ppo_bench_gemm(int op, int m, int n, int l, int iters, int cfg);
/* two independent C4-shaped minibatch GEMM chains (B rows, `out` outputs), `steps` steps each,
 * interleaved on one stream (two = 0) or two streams (two = 1); total device µs */
double ppo_bench_streams(int two, int steps, int B, int out);
/* bf16 GEMMs: force a tile configuration (−1 = automatic); returns the number of configurations */
int    ppo_gemm16_tune(int force_cfg);
/* average device µs of one bf16 launch (op as ppo_bench_gemm: 0 forward+ReLU, 1 grad_x, 2 grad_W, 3 forward to fp32 without activation; bf16 operands); splitk_target 0 = automatic */
double ppo_bench_gemm16(int op, int m, int n, int l, int iters, int cfg, int splitk_target);

/* fp32 GEMM engine of fp32 mode: 0 = exact fp32 MFMA (v_mfma_f32_32x32x2_f32), 1 = "x3": fp32
 * operands split exactly into three bf16 planes, the six plane products with pa + pb <= 2 on the
 * bf16 MFMA, fp32 accumulation (fp32-accurate, 6/16 of the fp32 MFMA cycles).  engine < 0 only
 * queries; returns the previous engine.  Env PPO_F32_GEMM=exact|x3 sets the initial value. */
int    ppo_gemm_f32_engine(int engine);
/* bf16 mode's LDS-DMA GEMM kernel (forward / grad_x with bf16 operands, gemm16.hip): on = 1 / 0
 * sets, −1 queries; returns the previous setting (initially PPO_G16_DMA, else on) */
int    ppo_gemm16_dma(int on);
/* bf16 mode's LDS-DMA grad_W tile width: 128 (256 × 128 tiles, default) or 256 (256 × 256, for
 * n % 256 = 0); other values query; returns the previous width */
int    ppo_gemm16_tn_width(int bn);
/* x3 engine tuning: force a tile configuration (−1 = automatic) and the grad_W split-K workgroup
 * target (0 = automatic, < 0 keeps); returns the number of configurations */
int    ppo_gemm_x3_tune(int force_cfg, int splitk_target);
/* diagnostic (libppo built with -DPPO_X3_DIAG): 8 slots per workgroup of the last x3 forward
 * launched with PPO_X3_ABLATE=32 — s_memtime at start, after the prologue, after the mainloop, at
 * the end; s_memrealtime (100 MHz, one clock for every XCD) at start and end; returns the slots */
int    ppo_x3_stamps(unsigned long long* out, int n);
/* diagnostic: the same for the double-buffered bf16 GEMM (gemm16.hip, -DPPO_G16_ABLATE=32 builds; else 0) */
int    ppo_g16_stamps(unsigned long long* out, int n);
/* average device µs of one x3 launch (fp32 operands; op as ppo_bench_gemm) */
double ppo_bench_gemm_x3(int op, int m, int n, int l, int iters, int cfg, int splitk_target);

/* ---------------- kernel timing ---------------- */
enum { PPO_K_GEMM = 0, PPO_K_GAE = 1, PPO_K_ADAM = 2, PPO_K_GATHER = 3, PPO_K_HEAD = 4,
       PPO_K_COMM = 5, PPO_K_OTHER = 6, PPO_K_COUNT = 7 };
/* stride > 0: record HIP events around every stride-th launch of each class on libppo's stream
 * (1 = every launch; an event pair costs a few µs of stream time, so throughput runs sample);
 * 0 = off */
void ppo_prof_enable(int stride);
void ppo_prof_reset(void);
/* per class: out_ms[k] = Σ kernel time (ms), out_work[k] = Σ algorithmic FLOPs (GEMM) or bytes,
 * out_launches[k] = launches.  Synchronises. */
void ppo_prof_read(double* out_ms, double* out_work, long* out_launches);
/* on != 0: sampled GEMM launches are timed by events the kernel dispatch itself stamps
 * (hipExtLaunchKernel) instead of event packets around the launch — the kernel's own duration, as
 * rocprofv3 --kernel-trace reports it (default off: event pairs around every sampled launch) */
void ppo_prof_kernel_events(int on);
/* per GEMM shape since the last reset: key = op<<58 | engine<<54 | m<<24 | n<<12 | l (op 0 forward,
 * 1 grad_x, 2 grad_W, 3 paired grad_W + grad_x; engine 0 exact fp32, 1 x3, 2 bf16), Σ ms, sampled
 * launches and Σ algorithmic FLOPs.  Returns the number of shapes (fills at most cap).  Synchronises. */
int  ppo_prof_shapes(long long* keys, double* ms, long* launches, double* work, int cap);
/* per GEMM shape key (as ppo_prof_shapes returns them): launches issued while profiling was enabled,
 * sampled or not — so a sampled average can be weighted by how often the shape really runs.
 * Returns how many of the n keys were seen. */
int  ppo_prof_shape_issued(const long long* keys, long* issued, int n);
/* per class: launches issued while profiling was enabled (sampled or not) */
void ppo_prof_counts(long* out_total);
/* per class: Σ algorithmic work of every launch issued while profiling was enabled */
void ppo_prof_issued_work(double* out_work);

#ifdef __cplusplus
}
#endif
#endif /* PPO_EXT_H */
