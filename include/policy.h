/*
 * policy.h — state-independent diagonal Gaussian policy over an MLP mean.
 *
 * Drop-in for /root/reference/include/policy.h:12-41.
 *   μ = mu(s) (MLP),  σ_j = exp(log_std[j]),  a = μ + σ·ε.
 *   log π(a|s) = −½·A·log 2π − Σ_j [log σ_j + ½((a_j−μ_j)/σ_j)²]   (policy.cu:67-74)
 *
 * Deliberate fixes of reference defects:
 *   D1/D2  log-prob forward/backward are correct for every action size A
 *          (the reference is only correct for A=1: policy.cu:106,116-122);
 *          grad_in is indexed per SAMPLE, grad_in[i].
 *   D3     all noise elements are filled (policy.cu:53-64 leaves holes).
 *   D14    input_action / d_input_action are BORROWED and never freed.
 */
#ifndef POLICY_H
#define POLICY_H

#include "neural_network.h"
#include <math.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    NeuralNetwork* mu;
    float* log_std;         /* host [A] */
    float* log_std_grad;    /* host [A] */
    float* d_log_std;       /* device [A] */
    float* d_log_std_grad;  /* device [A] */
    int state_size;
    int action_size;

    float* input_action;    /* borrowed host pointer recorded by compute_log_prob */
    float* d_input_action;  /* borrowed device pointer recorded by compute_log_prob_cuda */
} GaussianPolicy;

GaussianPolicy* create_gaussian_policy(int* layer_sizes, char** activation_functions, int num_layers, float init_std);
void free_gaussian_policy(GaussianPolicy* policy);

void sample_action(GaussianPolicy* policy, float* state, float* action, float* log_prob, int m);
void compute_log_prob(GaussianPolicy* policy, float* out, float* state, float* action, int m);
void log_prob_backwards(GaussianPolicy* policy, float* grad_in, float* grad_mu, float* grad_log_std, int m);

void compute_log_prob_cuda(GaussianPolicy* policy, float* out, float* state, float* action, int m);
void log_prob_backwards_cuda(GaussianPolicy* policy, float* grad_in, float* grad_mu, float* grad_log_std, int m);
float compute_entropy_cuda(GaussianPolicy* policy);

float compute_entropy(GaussianPolicy* policy);
void policy_to_host(GaussianPolicy* policy);

void save_policy(GaussianPolicy* policy, FILE* file);
GaussianPolicy* load_policy(FILE* file, int state_size, int action_size);

#ifdef __cplusplus
}
#endif
#endif /* POLICY_H */
