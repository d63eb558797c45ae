/*
 * ppo_hip.h — the thin C ABI between libppo's plain-C host code (ppo.c_amd/host)
 * and its hand-written gfx950 HIP kernels (ppo.c_amd/csrc).
 *
 * All pointers named d_* / device arrays are HBM pointers; every launch goes to
 * libppo's single stream and is asynchronous unless stated.  Shapes follow the
 * reference (row-major, W is [out, in]).  No function here allocates per call.
 */
#ifndef PPO_HIP_H
#define PPO_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- runtime / memory ---------------- */
void  phip_init(void);                     /* select device, create stream; abort without a GPU */
void* phip_malloc(size_t bytes);           /* zero-filled, 256-B aligned */
void  phip_free(void* p);
void  phip_h2d(void* dst, const void* src, size_t bytes);   /* completes before return */
void  phip_d2h(void* dst, const void* src, size_t bytes);   /* completes before return */
void  phip_d2d(void* dst, const void* src, size_t bytes);   /* async */
void  phip_memset(void* dst, int value, size_t bytes);      /* async */
void  phip_sync(void);                     /* both queues */
/* a second queue for independent work: fork = the side queue waits for everything issued so far on
 * the main queue; use(1) routes launches to the side queue until use(0); join = the main queue
 * waits for everything issued so far on the side queue */
void  phip_side_fork(void);
void  phip_side_use(int on);
int   phip_comm_inline(void);   /* gradient all-reduces in stream order, one per step (comm.hip) */
int   phip_side_active(void);   /* 1 while launches go to the side stream */
void  phip_side_join(void);
void  phip_record_error(const char* msg);
void  phip_drain(void);                 /* synchronise both streams, ignoring errors (before a fatal exit) */

/* ---------------- dense layers (gemm.hip) ---------------- */
/* y[m,l] = x[m,n]·W[l,n]ᵀ + b[l], optional ReLU (mat_mul.cu:132-163 + K1/K5 fused) */
void phip_linear_fwd(float* y, const float* x, const float* W, const float* b, int m, int n, int l, int relu);
/* same, and (relu) writes the ReLU′ mask as bits: word (row, c/32) bit c%32 = y[row, c] > 0,
 * ⌈l/32⌉ words per row — 1/32 of the bytes the float mask costs the backward */
void phip_linear_fwd_bits(float* y, const float* x, const float* W, const float* b, int m, int n, int l, int relu,
                          unsigned* bits);
/* gx[m,n] = g[m,l]·W[l,n]; if mask: gx = (mask > 0) ? gx : 0 (K3 + K6 fused) */
void phip_linear_bwd_x(float* gx, const float* g, const float* W, const float* mask, int m, int n, int l);
/* forward whose input row r is x[ridx[r]] (the minibatch gather fused into layer 0); the gathered
 * rows are also written to xcopy[m, n] (for the layer's grad_W) when xcopy != NULL */
void phip_linear_fwd_gather(float* y, const float* x, const int* ridx, float* xcopy, const float* W, const float* b,
                            int m, int n, int l, int relu, unsigned* bits);
/* same with the mask given as bits (phip_linear_fwd_bits layout, ⌈n/32⌉ words per row) */
void phip_linear_bwd_x_bits(float* gx, const float* g, const float* W, const float* mask, const unsigned* bits, int m,
                            int n, int l);
/* gW[l,n] = g[m,l]ᵀ·x[m,n] and gb[l] = Σ_m g[m,l] (K4 + K7 fused); overwrites */
void phip_linear_bwd_w(float* gW, float* gb, const float* g, const float* x, int m, int n, int l);
/* same, with gW/gb already zero on entry when `zeroed` (one memset per backward instead of two per layer) */
/* grad_W (+ bias) and grad_x ⊙ ReLU′(bits) of one layer, one launch when the shapes allow */
void phip_linear_bwd_pair(float* gW, float* gb, float* gx, const float* g, const float* x, const float* W,
                          const unsigned* bits, int m, int n, int l, int zeroed);
void phip_linear_bwd_w_ex(float* gW, float* gb, const float* g, const float* x, int m, int n, int l, int zeroed);

/* ---------------- bf16-MFMA dense layers (gemm16.hip) ---------------- */
/* dtype codes t*: 0 = fp32 storage, 1 = bf16 storage; W16 = bf16 shadow of W [l, n]; fp32 accumulation.
 * forward (optional fused gather: ridx / bf16 copy of the gathered rows in xcopy16) */
void phip_linear16_fwd(void* y, int ty, const void* x, int tx, const int* ridx, void* xcopy16, const void* W16,
                       const float* b, int m, int n, int l, int relu, unsigned* bits);
/* gx = (g·W) ⊙ bits (bits may be NULL: no mask) */
void phip_linear16_bwd_x(void* gx, int tgx, const void* g, int tg, const void* W16, const unsigned* bits, int m,
                         int n, int l);
/* gW[l,n] (+)= gᵀ·x, gb (+)= Σ g in fp32 (zeroed != 0: outputs already zero) */
void phip_linear16_bwd_w(float* gW, float* gb, const void* g, int tg, const void* x, int tx, int m, int n, int l,
                         int zeroed);
/* fp32-accurate products on the bf16 MFMA (gemm_x3.hip, the "x3" engine of fp32 mode): every fp32
 * operand splits exactly into three bf16 planes on its way into LDS, six plane products, fp32
 * accumulation.  Forward with optional fused gather (xcopy = fp32 copy of the gathered rows) +
 * bias/ReLU/ReLU' bits; grad_x with the bit mask; grad_W (+gb) split-K. */
int  phip_x3_supported(int op, int m, int n, int l);
void phip_x3_fwd(float* y, const float* x, const int* ridx, float* xcopy, const float* W, const float* b, int m,
                 int n, int l, int relu, unsigned* bits);
/* the next phip_x3_bwd_w(_fold) leaves its split-K slab reduce to the next phip_x3_bwd_x(_fold) on the same
 * stream (extra workgroups of that launch) — the caller guarantees grad_x follows */
void phip_x3_defer_reduce(int on);
void phip_x3_bwd_x(float* gx, const float* g, const float* W, const unsigned* bits, int m, int n, int l);
void phip_x3_bwd_w(float* gW, float* gb, const float* g, const float* x, int m, int n, int l, int zeroed);
/* value-head fold (nn_value_fold_step): forward partial y dots (returns ypart slots); backward with the
 * upper gradient g·w·1[h > 0] applied as the 0/1 mask of h with g, w as row / column scales (grad_x:
 * W pre-scaled by w) and the output layer's gW */
int  phip_x3_fwd_vhead(float* y, const float* x, const int* ridx, float* xcopy, const float* W, const float* b, int m,
                       int n, int l, int relu, unsigned* bits, const float* ydot, float* ypart);
void phip_x3_bwd_x_fold(float* gx, const float* g, const unsigned* fold_bits, const float* fold_g, const float* fold_w,
                        const float* W, const unsigned* bits, int m, int n, int l);
void phip_x3_bwd_w_fold(float* gW, float* gb, const float* h, const float* fold_g, const float* fold_w, float* fold_gw,
                        const float* x, int m, int n, int l, int zeroed);
/* phip_x3_bwd_w_fold carrying the value head: g (into fold_g) from the forward's partial dots ypart [slots][m]
 * + b against tgt, y, the output bias gradient gb_out and loss_accum (+= loss / m) — value_head_kernel's work */
void phip_x3_bwd_w_vhead(float* gW, float* gb, const float* h, float* fold_g, const float* fold_w, float* fold_gw,
                         const float* x, int m, int n, int l, int zeroed, const float* ypart, int slots, const float* b,
                         const float* tgt, float* y, float* gb_out, float* loss_accum);
/* dst[i, :] = bf16(src[rows[i], :]) for i < m (S % 4 == 0): layer 0's gather in bf16 mode */
void phip_gather_rows_bf16(unsigned short* dst, const float* src, const int* rows, int m, int S);
void phip_f32_to_bf16(unsigned short* dst, const float* src, long count);

/* ---------------- batched device rollout (rollout.hip) ---------------- */
/* env kinds: 0 = Pendulum-v1 (S = 3, A = 1), 1 = synthetic (any S, A) */
void phip_rollout_rows(int* rows, int E, int T);             /* rows[t·E + e] = e·T + t */
void phip_env_reset(int kind, float* env_state, float* state, int E, int T, int S, uint64_t seed);
void phip_env_first_obs(int kind, const float* env_state, float* state, int E, int T, int S);
void phip_sample_rows(const float* mu, const float* log_std, const int* rows, float* action, float* logprob, int E,
                      int A, uint64_t seed, uint64_t step);
void phip_env_step(int kind, float* env_state, float* state, const float* action, float* next_state, float* reward,
                   uint8_t* term, uint8_t* trunc, int E, int T, int t, int S, int A, uint64_t seed);

/* ---------------- single-workgroup update phase for small networks (tiny.hip) ---------------- */
typedef struct {
    int L;                          /* linear layers (≤ 8) */
    int sizes[9];                   /* widths (≤ 128; output ≤ 32) */
    int relu[8];
    long woff[8], boff[8];          /* offsets of W_l / b_l in params / grads */
    float *params, *grads, *m, *v;  /* flat parameter / gradient buffers, the network's Adam moments */
    long span;                      /* floats the network's Adam updates */
    float *log_std, *log_std_grad, *m_ls, *v_ls;   /* policy: log σ and its Adam (entropy) state */
    float* wt; long wt_cap;         /* scratch for the transposed weights (Σ in·out floats) */
} PhipTinyNet;
typedef struct {
    int policy;                     /* 0 = value epochs (MSE), 1 = policy epochs (clipped surrogate) */
    const float *state, *action, *logprob, *adv, *adv_target;   /* device buffer arrays */
    int limit, B, num_batches, n_epochs;        /* n_epochs ≤ 16 */
    long max_steps;                 /* ≤ 0: every step of the n_epochs; else the first max_steps */
    const int* perms;               /* [n_epochs][limit] permutations, or NULL: device Feistel */
    uint32_t feistel_k[64];         /* per epoch, 4 round keys (when perms == NULL) */
    const float *steps, *steps_ls;  /* device [n_steps][2] = {lr/bc1, bc2} per Adam step */
    float b1, b2, eps, ent_coeff;
    float* stats;                   /* device [0] Σ value loss, [1] Σ policy loss */
} PhipTinyPhase;
/* runs every minibatch step of the phase in one workgroup; returns −1 (nothing launched) when the
 * network or minibatch does not fit */
int phip_tiny_update(const PhipTinyNet* net, const PhipTinyPhase* ph);
/* the same phase for S → 256 → 256 → O networks (S ≤ 20, O ≤ 16) at B = 64 on 8 cooperating
 * workgroups (cluster.hip; net->wt unused); −1 when it does not fit, −2 after an earlier timeout */
int phip_cluster_update(const PhipTinyNet* net, const PhipTinyPhase* ph);
int phip_cluster_error(void);          /* nonzero: a cluster barrier timed out */
void phip_cluster_report(void);        /* PPO_CLUSTER_STAMPS: print the joined phases' sub-phase means */
/* S → 512 → 512 → 512 → O (S ≤ 380, S % 4 = 0, O ≤ 20) at B = 64 on 32 cooperating workgroups
 * (cluster_deep.hip); phip_cluster_update dispatches 4-layer networks here */
int phip_cluster_deep_update(const PhipTinyNet* net, const PhipTinyPhase* ph);
unsigned* phip_cluster_err_dev(void);  /* device pointer of the shared error word (NULL: already set) */

/* ---------------- element-wise / heads (kernels.hip) ---------------- */
void phip_relu(float* x, long count);
void phip_relu_bwd(const float* y, float* g, long count);
/* y += x (host-pointer API: the reference's CPU backward accumulates, mat_mul.cu:67,79) */
void phip_axpy(float* y, const float* x, long count);
/* d_loss[0] = Σ(t−y)²/count (written), d_loss_accum[0] += same (if non-NULL);
 * grad = 2(y−t)/count (if non-NULL).  loss.cu:25-83 fused, no host sync. */
void phip_mse(const float* y, const float* t, long count, float* grad, float* d_loss, float* d_loss_accum);
/* the folded value head (kernels.hip): y = Σ ypart slots + b, loss += Σ(t−y)²/m, g = 2(y−t)/m, gb += Σ g;
 * and Ws = diag(w)·W for the hidden layer's grad_x (W [l][n], w [l]) */
void phip_value_head(const float* ypart, int slots, const float* b, const float* tgt, int m, float* y, float* g,
                     float* gb, float* d_loss_accum);
/* out_head.hip: output layer forward + loss head + output-layer backward in one pass (ppo_update;
 * head 0 = value, A = 1, MSE against tgt; 1 = policy, clipped surrogate); gW / gb / grad_log_std
 * accumulated into zeroed outputs, loss into loss_accum; widths 64…1024, A ∈ {1, 6}; bf16 != 0:
 * x, W and gx stored bf16 (bf16 compute mode, value head) */
int  phip_out_head_supported(int head, int n, int A);
/* gemm.hip: 1 when ppo_gemm_tune(·, 1) asked for atomic-free (deterministic) gradient products */
int  phip_gemm_deterministic(void);
/* out_head.hip: the backward of a wide output layer (A = 17, n = 512 / 256, fp32) in one pass over the
 * rows — gx = (g·W) ⊙ 1[x > 0] (relu_in) and gW = gᵀ·x, gb = Σ g through per-workgroup partials;
 * gb must follow gW in memory (the flat gradient layout); returns 0 when the shape is not taken */
/* 1 when the wide pass takes (m rows, width n, A outputs; head: the fused policy head too) */
int  phip_out_bwd_wide_ok(int m, int n, int A, int head);
int  phip_out_bwd_wide(float* gW, float* gb, float* gx, const float* g, const float* x, const float* W, int relu_in,
                       int m, int n, int A);
/* the same pass with the policy head (kernels.hip policy_head_tiled_kernel's arithmetic) computed from μ
 * first: ∂/∂log σ (+ −c_ent) and the loss accumulated into grad_log_std / loss_accum (atomics) */
int  phip_policy_out_fused(const float* x, const float* W, const float* b, float* mu, const float* log_std,
                           const float* action, const float* adv, const float* old_lp, float eps, float ent_coeff,
                           float* grad_log_std, float* loss_accum, int relu_in, float* gW, float* gb, float* gx,
                           int m, int n, int A);
int  phip_policy_head_bwd_wide(const float* mu, const float* log_std, const float* action, const float* adv,
                               const float* old_lp, float eps, float ent_coeff, float* grad_log_std,
                               float* loss_accum, const float* x, const float* W, int relu_in, float* gW, float* gb,
                               float* gx, int m, int n, int A);
void phip_out_head(int head, int bf16, const void* x, int relu_in, const void* W, const float* b, int m, int n,
                   int A, const float* tgt, const float* log_std, const float* action, const float* adv,
                   const float* old_lp, float eps, float ent_coeff, float* y, void* gx, float* gW, float* gb,
                   float* grad_log_std, float* loss_accum);
void phip_log_prob(const float* mu, const float* log_std, const float* action, float* out, int m, int A);
void phip_log_prob_bwd(const float* mu, const float* log_std, const float* action, const float* grad_in,
                       float* grad_mu, float* grad_log_std, int m, int A);
/* d_out[0] = A·½(1+log 2π) + Σ log_std */
void phip_entropy(const float* log_std, int A, float* d_out);
/* clipped surrogate (ppo.cu:82-107): grad_lp[i], d_loss[0] = loss incl. −c·H (H from d_entropy) */
void phip_policy_loss(const float* adv, const float* lp, const float* old_lp, float* grad_lp, int m,
                      float epsilon, float ent_coeff, const float* d_entropy, float* d_loss, float* d_loss_accum);
/* fused policy head for the update: log-prob, ratio/clip, grad_lp, grad_mu, grad_log_std
 * (+ −ent_coeff, ppo.cu:436-438); loss accumulated into d_loss_accum; ls_zeroed: grad_log_std
 * already holds zeros (cleared by the previous entropy Adam step), else it is cleared first. */
void phip_policy_head(const float* mu, const float* log_std, const float* action, const float* adv,
                      const float* old_lp, int m, int A, float epsilon, float ent_coeff,
                      float* grad_mu, float* grad_log_std, float* d_loss_accum,
                      int ls_zeroed);

/* ---------------- GAE + normalisation (gae.hip) ---------------- */
/* advantages and targets by an exact segmented reverse scan; d_welford[0..2] =
 * (n, mean, M2) in double for this shard.  Then normalise with the (global)
 * statistics held in d_welford. */
void phip_gae_scan(const float* v, const float* v_next, const float* reward, const uint8_t* term,
                   const uint8_t* trunc, int n, float gamma, float lambda, float* adv, float* adv_target,
                   double* d_welford);
/* vn[t] = v[t+1] wherever next_state[t] == state[t+1] bit for bit; every other t is written to
 * own[0, count) (any order).  Returns count (synchronises). */
int phip_next_value_map(const float* next_state, const float* state, const float* v, float* vn, int* own, int n,
                        int S);
/* vn[own[i]] = vals[i] */
void phip_scatter_values(float* vn, const int* own, const float* vals, int m);
/* d_welford_all holds `world` triples; combine them into d_welford (3 doubles) */
void phip_welford_combine(const double* d_welford_all, int world, double* d_welford);
/* adv = (adv − mean)/(σ_pop + 1e-8); d_stats_out (optional) = {mean, std} as float */
void phip_normalize(float* adv, int n, const double* d_welford, float* d_stats_out);

/* ---------------- buffer (buffer.hip) ---------------- */
/* minibatch gather: row i ← perm[(offset+i) % limit] (perm != NULL) or
 * feistel((offset+i) % limit, limit, key) (perm == NULL).  Any dst may be NULL. */
/* phip_gather that also (or, with states == NULL, instead of copying states) writes each slot's
 * source row to rows[batch] — for layer 0's fused gather (phip_linear_fwd_gather) */
void phip_gather_rows(const int* perm, uint64_t key, int offset, int limit, int batch, int S, int A,
                      const float* state, const float* action, const float* logprob, const float* advantage,
                      const float* adv_target, float* states, float* actions, float* logprobs, float* advs,
                      float* adv_targets, int* rows);
void phip_gather(const int* perm, uint64_t key, int offset, int limit, int batch, int S, int A,
                 const float* state, const float* action, const float* logprob,
                 const float* advantage, const float* adv_target,
                 float* states, float* actions, float* logprobs, float* advs, float* adv_targets);

/* ---------------- Adam (adam.hip) ---------------- */
void phip_adam_flat(float* p, const float* g, float* m, float* v, long n, float lr, float beta1,
                    float beta2, float bias_correction1, float bias_correction2, float grad_scale);
/* the same, also writing bf16(p) into w16[0, n16) (bf16 mode's parameter shadow); zero_g: g is
 * cleared once read (the next backward accumulates into it without a memset) */
/* ---- launch-free minibatch steps (hipGraph replay with a device step table) ----
 * One minibatch step is captured once as a graph whose per-step arguments — the gather's
 * permutation offset / Feistel round keys and row offset, the Adam step sizes — live in a device
 * table indexed by a device step counter; the network's Adam kernel advances the counter (its last
 * workgroup to finish), so every replay of the same graph performs the next step. */
typedef struct {
    long perm_off;                  /* ≥ 0: host-rand permutation at perm_base + perm_off; −1: Feistel */
    unsigned fk[4];                 /* Feistel round keys of the epoch */
    unsigned fhalf, fmask, fn;      /* Feistel domain (the buffer's limit) */
    int offset;                     /* k·B: the minibatch's first position in the epoch order */
    float step, bc2;                /* the network Adam's lr / (1 − β1^t) and 1 − β2^t */
    float step_ls, bc2_ls;          /* the entropy Adam's (policy log σ) */
} PhipStepArgs;
void phip_step_feistel(PhipStepArgs* s, unsigned long long key, int limit);   /* fills fk / fhalf / fmask / fn */
void phip_gather_rows_tab(const PhipStepArgs* tab, const int* ctr, const int* perm_base, int limit, int batch, int A,
                          const float* action, const float* logprob, const float* advantage,
                          const float* adv_target, float* actions, float* logprobs, float* advs, float* adv_targets,
                          int* rows);
/* which = 0: the network's Adam (step / bc2; advances *ctr); 1: the entropy Adam (step_ls / bc2_ls) */
void phip_adam_flat_tab(float* p, float* g, float* m, float* v, long n, const PhipStepArgs* tab, int* ctr,
                        unsigned* ticket, int which, float beta1, float beta2, float grad_scale, unsigned short* w16,
                        long n16, int zero_g);
int  phip_graph_begin(void);                 /* capture the current stream's launches (returns 0 on success) */
void* phip_graph_end(void);                  /* → instantiated executable graph (NULL on failure) */
void phip_graph_launch(void* exec);          /* replay on the current stream */
void phip_graph_destroy(void* exec);
const char* phip_graph_error(void);         /* why the last capture failed (warning text) */
int  phip_capturing(void);                   /* 1 while a capture is open (profiling scopes stay out) */

void phip_adam_flat_w16(float* p, float* g, float* m, float* v, long n, float lr, float beta1, float beta2,
                        float bias_correction1, float bias_correction2, float grad_scale, unsigned short* w16,
                        long n16, int zero_g);
/* the same for a network span (16-B aligned) plus a small second span (≤ 256 floats, any alignment:
 * the policy step's entropy Adam) with its own step size, in one launch */
void phip_adam_flat_pair(float* p, float* g, float* m, float* v, long n, float lr, float beta1, float beta2,
                         float bias_correction1, float bias_correction2, float grad_scale, unsigned short* w16,
                         long n16, int zero_g, float* p2, float* g2, float* m2, float* v2, int n2, float lr2,
                         float bias_correction1_2, float bias_correction2_2, float grad_scale2, int zero_g2);
/* multi-tensor: ptrs/lengths are HOST arrays describing device tensors; m/v are flat */
void phip_adam_multi(float* const* params, float* const* grads, const int* lengths, int num_tensors,
                     float* m, float* v, float lr, float beta1, float beta2,
                     float bias_correction1, float bias_correction2, float grad_scale);

/* ---------------- sampling / synthetic data (sample.hip) ---------------- */
void phip_sample(const float* mu, const float* log_std, float* action, float* logprob, int m, int A,
                 uint64_t seed, uint64_t offset);
/* same with caller-supplied noise ε[m·A] (host rand() Box–Muller in the reference API path) */
void phip_sample_noise(const float* mu, const float* log_std, const float* noise, float* action, float* logprob,
                       int m, int A);
void phip_fill_uniform(float* p, long n, uint64_t seed, float lo, float hi);
void phip_fill_normal(float* p, long n, uint64_t seed, float scale);
void phip_fill_rollout_flags(uint8_t* term, uint8_t* trunc, int n_envs, int horizon, float p_term, uint64_t seed);
/* next_state[t] = state[t+1] inside an env segment when not terminated (else fresh U(−1,1)) */
void phip_link_next_state(float* next_state, const float* state, const uint8_t* term, int n_envs,
                          int horizon, int S, uint64_t seed);

/* ---------------- data parallel (comm.hip, RCCL) ---------------- */
int  phip_comm_world(void);
int  phip_comm_rank(void);
int  phip_comm_min_i32(int v);      /* min over ranks (synchronous); identity at world 1 */
/* a communicator is up (world > 1, the PPO_COMM_SELF one-rank rehearsal, or the loopback) */
int  phip_comm_active(void);
void phip_allreduce_sum_f32(float* d_buf, long n);
/* gradient bucket: queued behind the issuing stream's work, which does not wait for it;
 * phip_allreduce_join() makes the issuing stream wait for every bucket queued so far */
void phip_allreduce_sum_f32_async(float* d_buf, long n);
void phip_allreduce_join(void);
void phip_allgather_f64(const double* d_send, double* d_recv, long n_per_rank);
/* bounded host wait for every libppo stream (PPO_COMM_TIMEOUT_S, RCCL async errors polled): a stall
 * or an RCCL error aborts the communicators and fails loudly, naming `what` */
void phip_comm_wait(const char* what);
/* replica check: this rank's parameter hash into a device word (Σ mix(index, bits) over the spans,
 * indices running on across spans), then an all-gather over ranks, a bounded wait and the comparison —
 * 0 if every rank's hash equals rank 0's, −1 with the differing ranks in msg; own ← this rank's hash */
void phip_param_hash(const float* const* spans, const long* lens, int nspans);
int  phip_comm_check_hash(int gather, unsigned long long* own, char* msg, int cap);   /* gather 0: own only */

/* ---------------- profiling ---------------- */
/* host C wrappers bracket launches: slot = phip_prof_begin(cls, work); ...; phip_prof_end(slot) */
int  phip_prof_begin(int cls, double work);
int  phip_prof_begin_key(int cls, double work, long long key);
void phip_prof_end(int slot);

#ifdef __cplusplus
}
#endif
#endif /* PPO_HIP_H */
