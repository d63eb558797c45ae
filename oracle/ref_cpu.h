/*
 * ref_cpu.h — ORACLE (test infrastructure only; never linked into libppo).
 *
 * A plain-C restatement of cube1324/ppo.c's CPU path for the PPO update
 * (reference /root/reference/src/ppo.cu:326-448 and the modules it calls).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load liboracle.so, and only as the checker / CPU baseline.
 *
 * Parity status: UNPINNED by reference outputs.  The reference ships no
 * tests, fixtures or golden vectors, and its CPU path cannot be compiled here
 * without stand-in CUDA/cuBLAS/CBLAS headers (forbidden), so oracle/_ref is
 * not built.  The restatement is instead cross-checked against independent
 * float64 known answers (torch autograd / torch.optim.Adam / direct loops)
 * committed under tests/golden/ — see DESIGN.md §Oracle.
 *
 * Interfaces are flat host arrays so ctypes tests can drive them:
 *   MLP parameters: one packed array [W0 (out0×in0), b0, W1, b1, …] in the
 *   reference's per-layer order (adam.cu:25-42 flattens in the same order).
 */
#ifndef PPO_ORACLE_REF_CPU_H
#define PPO_ORACLE_REF_CPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- BLAS plumbing: optional OpenBLAS (dlopen), else blocked C ---- */
int  ref_blas_load(const char* openblas_path);   /* 1 if OpenBLAS sgemm was bound */
void ref_blas_threads(int n);
const char* ref_blas_name(void);
/* chaos-floor perturbations of the product arithmetic (0 = oracle proper, 1 = split-K halves,
 * 2 = double-precision products rounded once); -1 if unavailable */
int  ref_blas_mode(int mode);

/* ---- ops (mat_mul.cu:39-80, activation_function.cu:5-15, loss.cu:5-23) ---- */
void  ref_mat_mul(float* out, const float* x, const float* W, const float* b, int m, int n, int l);
void  ref_mat_mul_backwards(float* gx, float* gW, const float* gin, const float* x, const float* W, int m, int n, int l);
void  ref_relu(float* x, long count);
void  ref_relu_derivative(const float* x, float* g, long count);
float ref_mse(const float* y, const float* t, int m, int n);
void  ref_mse_derivative(float* g, const float* y, const float* t, int m, int n);

/* ---- MLP (neural_network.cu:6-72,163-231) ---- */
long ref_mlp_num_params(int num_sizes, const int* sizes);
void ref_mlp_init(int num_sizes, const int* sizes, float* params);         /* consumes rand() */
/* acts receives every layer's post-activation output back to back:
 * [m×sizes[1]] [m×sizes[2]] … ; relu[i] applies after linear layer i. */
void ref_mlp_forward(int num_sizes, const int* sizes, const int* relu, const float* params,
                     const float* x, int m, float* acts);
/* grads (packed like params) are overwritten; grad_x (m×sizes[0]) optional */
void ref_mlp_backward(int num_sizes, const int* sizes, const int* relu, const float* params,
                      const float* x, const float* acts, const float* grad_out, int m,
                      float* grads, float* grad_x);

/* ---- Gaussian policy (policy.cu:46-111,171-178) ---- */
float ref_entropy(const float* log_std, int A);
void  ref_log_prob(const float* mu, const float* log_std, const float* action, int m, int A, float* out);
void  ref_log_prob_backwards(const float* mu, const float* log_std, const float* action,
                             const float* grad_in, int m, int A, float* grad_mu, float* grad_log_std);
void  ref_gaussian_noise(float* out, int n);                               /* consumes rand() */
float ref_policy_loss_and_grad(float* grad_lp, float* grad_entropy, const float* adv, const float* lp,
                               const float* old_lp, float entropy, float ent_coeff, float epsilon, int m);

/* ---- GAE after the two value forwards (ppo.cu:326-369) ---- */
void ref_gae(const float* v, const float* v_next, const float* reward, const uint8_t* term,
             const uint8_t* trunc, int n, float gamma, float lambda,
             float* adv, float* adv_target, float* mean_out, float* std_out);

/* ---- buffer (trajectory_buffer.cu:126-146,202-220) ---- */
void ref_shuffle(int* perm, int n);                                        /* consumes rand() */
uint32_t ref_feistel_index(uint32_t i, uint32_t n, uint64_t key);          /* libppo device shuffle */
void ref_feistel_perm(int* perm, int n, uint64_t key);
void ref_get_batch(const int* perm, int n, int batch_idx, int batch_size, int S, int A,
                   const float* state, const float* action, const float* logprob,
                   const float* advantage, const float* adv_target,
                   float* states, float* actions, float* logprobs, float* advs, float* adv_targets);

/* ---- Adam (adam.cu:53-74) ---- */
void ref_adam_update(float* params, const float* grads, float* m, float* v, long size,
                     int* time_step, float beta1, float beta2, float lr);

/* ---- one PPO update = ppo.cu:395-443 (CPU branch) without the rollout ---- */
typedef struct {
    int num_sizes;            /* layer sizes incl. input/output, ≤ 8 */
    int sizes_mu[8];          /* {S, H…, A} */
    int relu[8];              /* per linear layer */
    int N;                    /* transitions in the buffer (limit) */
    int batch_size;
    int n_epochs_policy, n_epochs_value;
    float gamma, lambda, epsilon, ent_coeff, lr_policy, lr_v;
    int shuffle_mode;         /* 0 = rand() swap shuffle (reference), 1 = Feistel (libppo device) */
    uint64_t seed;            /* Feistel key base when shuffle_mode == 1 */
    int max_value_steps;      /* <0: all; else stop after this many value minibatches (CPU-baseline sampling) */
    int max_policy_steps;
    int capacity;             /* buffer capacity (0: N, a full buffer); minibatches per epoch = capacity / B
                                 (D13) even when only N = idx < capacity rows are filled — rows wrap mod N */
} RefUpdateCfg;

typedef struct {
    float* mu_params;  float* log_std;  float* v_params;          /* in/out */
    float* m_mu; float* v_mu; int t_mu;                           /* Adam state, in/out */
    float* m_v;  float* v_v;  int t_v;
    float* m_ent; float* v_ent; int t_ent;
    const float* state; const float* next_state; const float* action; const float* reward;
    const float* logprob; const uint8_t* terminated; const uint8_t* truncated;
    float* advantage; float* adv_target;                          /* out (GAE) */
    double sum_v_loss; double sum_policy_loss; long n_v; long n_p;  /* out */
    float adv_mean, adv_std;                                      /* out */
    double t_gae, t_value, t_policy;                              /* out: seconds */
} RefUpdateState;

void ref_ppo_update(const RefUpdateCfg* cfg, RefUpdateState* st);

#ifdef __cplusplus
}
#endif
#endif
