/*
 * ppo.h — PPO trainer: rollout, GAE, clipped-surrogate update.
 *
 * Drop-in for /root/reference/include/ppo.h:15-47; the reference main.c
 * (/root/reference/src/main.c) compiles against this header set unchanged and
 * links against libppo.so.
 *
 * The PPO update (train_ppo_epoch minus the rollout: GAE → normalisation →
 * n_epochs_value × ⌊N/B⌋ value steps → n_epochs_policy × ⌊N/B⌋ policy steps,
 * reference ppo.cu:373-550) runs entirely on the MI355X with no host
 * round-trips per minibatch.  Numerics follow the reference's CPU path
 * (ppo.cu:373-448), including log_std_grad += −ent_coeff and a
 * single entropy term in the loss (D5).  `use_cuda` is accepted for ABI
 * compatibility: libppo has no CPU compute path, both values run the HIP
 * path (the plain-C restatement lives in oracle/ as test infrastructure).
 */
#ifndef PPO_H
#define PPO_H

#include "trajectory_buffer.h"
#include "policy.h"
#include "neural_network.h"
#include "env.h"
#include "loss.h"
#include "adam.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    TrajectoryBuffer* buffer;
    GaussianPolicy* policy;
    NeuralNetwork* V;
    Adam* adam_policy;
    Adam* adam_V;
    Adam* adam_entropy;
    float lambda;
    float epsilon;
    float ent_coeff;
    float lr_policy;
    float lr_V;
    bool use_cuda;

    /* ---- libppo extension ---- */
    void* dev;              /* device-side workspaces for the fused update (opaque) */
} PPO;

PPO* create_ppo(char** activation_functions, int* layer_sizes, int num_layers, int buffer_size, float lr_policy, float lr_v, float lambda, float epsilon, float ent_coeff, float init_std, bool use_cuda);

void free_ppo(PPO* ppo);

void collect_trajectories(TrajectoryBuffer* buffer, Env* env, GaussianPolicy* policy, int steps);
void compute_gae(NeuralNetwork* V, TrajectoryBuffer* buffer, float gamma, float lambda);

float policy_loss_and_grad(float* grad_logprob, float* grad_entropy, float* adv, float* logprobs, float* old_logprobs, float entropy, float ent_coeff, float epsilon, int m);

void compute_gae_cuda(NeuralNetwork* V, TrajectoryBuffer* buffer, float gamma, float lambda, int horizon);
float policy_loss_and_grad_cuda(float* grad_logprob, float* grad_entropy, float* adv, float* logprobs, float* old_logprobs, float entropy, float ent_coeff, float epsilon, int m);

void train_ppo_epoch(PPO* ppo, Env* env, int steps_per_epoch, int batch_size, int n_epochs_policy, int n_epochs_value);
void eval_ppo(PPO* ppo, Env* env, int steps);

void save_ppo(PPO* ppo, const char* filename);

PPO* load_ppo(const char* filename, bool use_cuda);

/* The reference main.c calls this OpenBLAS function without declaring it
 * (main.c:18).  libppo exports it: it sets the thread count of host-side
 * helpers and is otherwise a no-op (there is no BLAS in libppo). */
void openblas_set_num_threads(int num_threads);

#ifdef __cplusplus
}
#endif

#include "ppo_ext.h"

#endif /* PPO_H */
