/*
 * policy.c — state-independent diagonal Gaussian policy.
 *
 * Reference: /root/reference/src/policy.cu.  log_std lives in HBM directly
 * behind μ's flat parameters (and its gradient behind μ's gradients), so one
 * all-reduce covers every policy gradient in data-parallel training.
 */
#include "internal.h"

#include <math.h>

NeuralNetwork* nn_load_ex(FILE* file, long extra_floats);

static void attach_log_std(GaussianPolicy* p) {
    p->d_log_std = p->mu->d_params + p->mu->num_params;
    p->d_log_std_grad = p->mu->d_grads + p->mu->num_params;
}

GaussianPolicy* policy_create_ex(int* layer_sizes, char** activation_functions, int num_layers, float init_std,
                                 int init_from_rand) {
    GaussianPolicy* p = (GaussianPolicy*)xcalloc(1, sizeof(GaussianPolicy));
    p->state_size = layer_sizes[0];
    p->action_size = layer_sizes[num_layers - 1];
    p->mu = nn_create_ex(layer_sizes, activation_functions, num_layers, p->action_size, init_from_rand);
    p->log_std = (float*)xmalloc(sizeof(float) * (size_t)p->action_size);
    p->log_std_grad = (float*)xcalloc((size_t)p->action_size, sizeof(float));
    attach_log_std(p);
    for (int i = 0; i < p->action_size; i++) p->log_std[i] = logf(init_std);      /* policy.cu:22-24 */
    phip_h2d(p->d_log_std, p->log_std, sizeof(float) * (size_t)p->action_size);
    nn_sync_extra_snapshot(p->mu, p->log_std);
    p->input_action = NULL;
    p->d_input_action = NULL;
    return p;
}

GaussianPolicy* create_gaussian_policy(int* layer_sizes, char** activation_functions, int num_layers, float init_std) {
    return policy_create_ex(layer_sizes, activation_functions, num_layers, init_std, 1);
}

/* input_action / d_input_action are borrowed (D14): never freed here. */
void free_gaussian_policy(GaussianPolicy* policy) {
    if (!policy) return;
    free_neural_network(policy->mu);       /* owns d_log_std / d_log_std_grad */
    free(policy->log_std);
    free(policy->log_std_grad);
    free(policy);
}

/* policy.cu:46-65 Box–Muller on libc rand(), every element filled (D3). */
static void gaussian_noise_from_rand(float* out, int n) {
    if (n == 1) {
        out[0] = sqrtf(-2 * logf((float)rand() / RAND_MAX)) * cosf(2 * M_PI * (float)rand() / RAND_MAX);
        return;
    }
    int i = 0;
    for (; i + 1 < n; i += 2) {
        float u1 = (float)rand() / RAND_MAX;
        float u2 = (float)rand() / RAND_MAX;
        float r = sqrtf(-2 * logf(u1));
        float theta = 2 * M_PI * u2;
        out[i] = r * cosf(theta);
        out[i + 1] = r * sinf(theta);
    }
    if (i < n) out[n - 1] = sqrtf(-2 * logf((float)rand() / RAND_MAX)) * cosf(2 * M_PI * (float)rand() / RAND_MAX);
}

/* policy.cu:76-89 — host pointers; μ and the sample run on the GPU, the noise keeps the
 * reference's seeded rand() stream. */
void sample_action(GaussianPolicy* policy, float* state, float* action, float* log_prob, int m) {
    const int A = policy->action_size;
    policy_host_sync(policy);
    forward_propagation(policy->mu, state, m);
    float* noise = (float*)xmalloc(sizeof(float) * (size_t)m * A);
    gaussian_noise_from_rand(noise, m * A);
    float* d_noise = stage_up(ST_E, noise, (size_t)m * A);
    float* d_act = (float*)stage(ST_F, sizeof(float) * (size_t)m * A);
    float* d_lp = (float*)stage(ST_G, sizeof(float) * (size_t)m);
    phip_sample_noise(policy->mu->d_output, policy->d_log_std, d_noise, d_act, d_lp, m, A);
    phip_d2h(action, d_act, sizeof(float) * (size_t)m * A);
    phip_d2h(log_prob, d_lp, sizeof(float) * (size_t)m);
    free(noise);
}

/* policy.cu:91-99 */
void compute_log_prob(GaussianPolicy* policy, float* out, float* state, float* action, int m) {
    const int A = policy->action_size;
    policy->input_action = action;
    policy_host_sync(policy);
    forward_propagation(policy->mu, state, m);
    float* d_act = stage_up(ST_E, action, (size_t)m * A);
    float* d_out = (float*)stage(ST_F, sizeof(float) * (size_t)m);
    phip_log_prob(policy->mu->d_output, policy->d_log_std, d_act, d_out, m, A);
    phip_d2h(out, d_out, sizeof(float) * (size_t)m);
}

/* policy.cu:101-111 with D2 (grad_in per sample) */
void log_prob_backwards(GaussianPolicy* policy, float* grad_in, float* grad_mu, float* grad_log_std, int m) {
    const int A = policy->action_size;
    policy_host_sync(policy);
    float* d_act = stage_up(ST_E, policy->input_action, (size_t)m * A);
    float* d_g = stage_up(ST_F, grad_in, (size_t)m);
    float* d_gmu = (float*)stage(ST_G, sizeof(float) * (size_t)m * A);
    float* d_gls = (float*)stage(ST_H, sizeof(float) * (size_t)A);
    phip_log_prob_bwd(policy->mu->d_output, policy->d_log_std, d_act, d_g, d_gmu, d_gls, m, A);
    phip_d2h(grad_mu, d_gmu, sizeof(float) * (size_t)m * A);
    phip_d2h(grad_log_std, d_gls, sizeof(float) * (size_t)A);
}

/* policy.cu:113-139 (K11), correct for any action size (D1) */
void compute_log_prob_cuda(GaussianPolicy* policy, float* out, float* state, float* action, int m) {
    policy->d_input_action = action;
    forward_propagation_cuda(policy->mu, state, m);
    phip_log_prob(policy->mu->d_output, policy->d_log_std, action, out, m, policy->action_size);
}

/* policy.cu:141-169 (K12) */
void log_prob_backwards_cuda(GaussianPolicy* policy, float* grad_in, float* grad_mu, float* grad_log_std, int m) {
    phip_log_prob_bwd(policy->mu->d_output, policy->d_log_std, policy->d_input_action, grad_in, grad_mu,
                      grad_log_std, m, policy->action_size);
}

/* policy.cu:180-193 */
float compute_entropy_cuda(GaussianPolicy* policy) {
    float* d = (float*)stage(ST_H, 16);
    phip_entropy(policy->d_log_std, policy->action_size, d);
    float e = 0.f;
    phip_d2h(&e, d, sizeof(float));
    return e;
}

/* policy.cu:171-178 — reads the host log_std mirror, evaluated on the GPU */
float compute_entropy(GaussianPolicy* policy) {
    policy_host_sync(policy);
    float* d_ls = stage_up(ST_G, policy->log_std, (size_t)policy->action_size);
    float* d = (float*)stage(ST_H, 16);
    phip_entropy(d_ls, policy->action_size, d);
    float e = 0.f;
    phip_d2h(&e, d, sizeof(float));
    return e;
}

void policy_to_host(GaussianPolicy* policy) {
    nn_write_weights_to_host(policy->mu);
    phip_d2h(policy->log_std, policy->d_log_std, sizeof(float) * (size_t)policy->action_size);
    nn_sync_extra_snapshot(policy->mu, policy->log_std);
    policy->mu->host_version = policy->mu->host_version_w = policy->mu->dev_version;
}

/* before a host-pointer entry point: μ's mirrors and log_std reconciled with HBM (nn_host_sync) */
void policy_host_sync(GaussianPolicy* policy) { nn_host_sync(policy->mu, policy->log_std); }

/* policy.cu:201-227 */
void save_policy(GaussianPolicy* policy, FILE* file) {
    policy_host_sync(policy);
    fwrite(policy->log_std, sizeof(float), (size_t)policy->action_size, file);
    save_neural_network(policy->mu, file);
}

GaussianPolicy* load_policy(FILE* file, int state_size, int action_size) {
    GaussianPolicy* p = (GaussianPolicy*)xcalloc(1, sizeof(GaussianPolicy));
    p->state_size = state_size;
    p->action_size = action_size;
    p->log_std = (float*)xmalloc(sizeof(float) * (size_t)action_size);
    p->log_std_grad = (float*)xcalloc((size_t)action_size, sizeof(float));
    if (fread(p->log_std, sizeof(float), (size_t)action_size, file) != (size_t)action_size)
        die("checkpoint: unexpected end of file");
    p->mu = nn_load_ex(file, action_size);
    attach_log_std(p);
    phip_h2d(p->d_log_std, p->log_std, sizeof(float) * (size_t)action_size);
    nn_sync_extra_snapshot(p->mu, p->log_std);
    p->mu->host_version = p->mu->host_version_w = p->mu->dev_version;
    return p;
}
