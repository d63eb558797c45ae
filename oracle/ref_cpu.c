/*
 * ref_cpu.c — ORACLE: plain-C restatement of cube1324/ppo.c's CPU update path.
 *
 * TEST INFRASTRUCTURE ONLY.  Never linked into libppo; loaded by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker.
 * Parity status: unpinned by reference outputs (see ref_cpu.h header).
 *
 * Each function restates the reference's arithmetic, including its C type
 * promotions (float vs double temporaries), so that results are comparable
 * at the tolerances stated in tests/.  Citations are /root/reference paths.
 * Documented deviations: D2 log_prob_backwards indexes
 * grad_in per sample; D3 every noise element is filled; D6 A[N] := 0;
 * D16/D17 heap buffers instead of stack VLAs / per-call malloc.
 */
#define _GNU_SOURCE
#include "ref_cpu.h"

#include <dlfcn.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* ------------------------------------------------------------------ */
/* BLAS plumbing                                                       */
/* ------------------------------------------------------------------ */
/* OpenBLAS ILP64 cblas_sgemm as bundled with numpy (scipy_openblas64_). */
typedef void (*sgemm64_fn)(int order, int ta, int tb, int64_t M, int64_t N, int64_t K, float alpha,
                           const float* A, int64_t lda, const float* B, int64_t ldb, float beta,
                           float* C, int64_t ldc);
typedef void (*setthreads_fn)(int);
typedef void (*dgemm64_fn)(int order, int ta, int tb, int64_t M, int64_t N, int64_t K, double alpha,
                           const double* A, int64_t lda, const double* B, int64_t ldb, double beta,
                           double* C, int64_t ldc);
static sgemm64_fn g_sgemm = NULL;
static dgemm64_fn g_dgemm = NULL;
static setthreads_fn g_setthreads = NULL;
/* Perturbation modes (chaos-floor measurements only, tools/chaos_floor.py; 0 = the oracle proper):
 * 1 = every product's K range summed as two halves (sgemm over the first half, then β = 1 over the
 *     second: a split-K re-association of the same fp32 arithmetic);
 * 2 = products evaluated in double (dgemm on widened operands), rounded once to fp32 on store
 *     (β·C added in double) — the most accurate fp32-output BLAS. */
static int g_blas_mode = 0;

int ref_blas_load(const char* path) {
    if (!path || !*path) return 0;
    void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h) return 0;
    g_sgemm = (sgemm64_fn)dlsym(h, "scipy_cblas_sgemm64_");
    if (!g_sgemm) g_sgemm = (sgemm64_fn)dlsym(h, "cblas_sgemm64_");
    g_dgemm = (dgemm64_fn)dlsym(h, "scipy_cblas_dgemm64_");
    if (!g_dgemm) g_dgemm = (dgemm64_fn)dlsym(h, "cblas_dgemm64_");
    g_setthreads = (setthreads_fn)dlsym(h, "scipy_openblas_set_num_threads64_");
    if (!g_setthreads) g_setthreads = (setthreads_fn)dlsym(h, "openblas_set_num_threads");
    if (g_setthreads) g_setthreads(1);       /* main.c:18 pins OpenBLAS to one thread */
    return g_sgemm != NULL;
}
void ref_blas_threads(int n) { if (g_setthreads) g_setthreads(n); }
const char* ref_blas_name(void) { return g_sgemm ? "openblas(scipy_openblas64_)" : "blocked-C"; }
int ref_blas_mode(int mode) {
    if (mode == 2 && !g_dgemm) return -1;
    if (mode < 0 || mode > 2 || (mode && !g_sgemm)) return -1;
    g_blas_mode = mode;
    return 0;
}

static void sgemm_rm(int ta, int tb, int M, int N, int K, float alpha, const float* A, int lda,
                     const float* B, int ldb, float beta, float* C, int ldc);

/* mode 2: C = round_f32(α·op(A)·op(B) + β·C) with every operation in double */
static void sgemm_rm_wide(int ta, int tb, int M, int N, int K, float alpha, const float* A, int lda,
                          const float* B, int ldb, float beta, float* C, int ldc) {
    const long ar = ta ? K : M, ac = ta ? M : K, br = tb ? N : K, bc = tb ? K : N;
    double* a = (double*)malloc(sizeof(double) * (size_t)(ar * ac));
    double* b = (double*)malloc(sizeof(double) * (size_t)(br * bc));
    double* c = (double*)malloc(sizeof(double) * (size_t)M * N);
    for (long i = 0; i < ar; i++)
        for (long j = 0; j < ac; j++) a[i * ac + j] = A[i * lda + j];
    for (long i = 0; i < br; i++)
        for (long j = 0; j < bc; j++) b[i * bc + j] = B[i * ldb + j];
    for (long i = 0; i < M; i++)
        for (long j = 0; j < N; j++) c[i * N + j] = (double)C[i * ldc + j];
    g_dgemm(101, ta ? 112 : 111, tb ? 112 : 111, M, N, K, alpha, a, ac, b, bc, beta, c, N);
    for (long i = 0; i < M; i++)
        for (long j = 0; j < N; j++) C[i * ldc + j] = (float)c[i * N + j];
    free(a);
    free(b);
    free(c);
}

/* Row-major C[M,N] = alpha·op(A)·op(B) + beta·C, op = transpose if t != 0. */
static void sgemm_rm(int ta, int tb, int M, int N, int K, float alpha, const float* A, int lda,
                     const float* B, int ldb, float beta, float* C, int ldc) {
    if (g_blas_mode == 2) {
        sgemm_rm_wide(ta, tb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc);
        return;
    }
    if (g_blas_mode == 1 && K >= 2) {
        /* the first ⌊K/2⌋ terms, then the rest accumulated on top */
        const int k1 = K / 2;
        const float* A2 = ta ? A + (size_t)k1 * lda : A + k1;
        const float* B2 = tb ? B + k1 : B + (size_t)k1 * ldb;
        g_sgemm(101, ta ? 112 : 111, tb ? 112 : 111, M, N, k1, alpha, A, lda, B, ldb, beta, C, ldc);
        g_sgemm(101, ta ? 112 : 111, tb ? 112 : 111, M, N, K - k1, alpha, A2, lda, B2, ldb, 1.0f, C, ldc);
        return;
    }
    if (g_sgemm) {   /* CblasRowMajor=101, NoTrans=111, Trans=112 */
        g_sgemm(101, ta ? 112 : 111, tb ? 112 : 111, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc);
        return;
    }
    /* blocked fallback: accumulate op(A)·op(B) into a float row, then C = α·acc + β·C */
    float* acc = (float*)malloc(sizeof(float) * (size_t)N);
    for (int i = 0; i < M; i++) {
        memset(acc, 0, sizeof(float) * (size_t)N);
        for (int k = 0; k < K; k++) {
            float a = ta ? A[(size_t)k * lda + i] : A[(size_t)i * lda + k];
            if (!tb) {
                const float* brow = B + (size_t)k * ldb;
                for (int j = 0; j < N; j++) acc[j] += a * brow[j];
            } else {
                for (int j = 0; j < N; j++) acc[j] += a * B[(size_t)j * ldb + k];
            }
        }
        float* crow = C + (size_t)i * ldc;
        for (int j = 0; j < N; j++) crow[j] = alpha * acc[j] + beta * crow[j];
    }
    free(acc);
}

/* ------------------------------------------------------------------ */
/* ops                                                                 */
/* ------------------------------------------------------------------ */
/* mat_mul.cu:39-55: bias pre-fill, then sgemm(NoTrans, Trans) with beta = 1.
 * (The m==1 sgemv branch computes the same product.) */
void ref_mat_mul(float* out, const float* x, const float* W, const float* b, int m, int n, int l) {
    for (int i = 0; i < m; i++)
        for (int j = 0; j < l; j++) out[(size_t)i * l + j] = b[j];
    sgemm_rm(0, 1, m, l, n, 1.0f, x, n, W, n, 1.0f, out, l);
}

/* mat_mul.cu:57-80: both products ACCUMULATE (beta = 1). */
void ref_mat_mul_backwards(float* gx, float* gW, const float* gin, const float* x, const float* W,
                           int m, int n, int l) {
    if (gx) sgemm_rm(0, 0, m, n, l, 1.0f, gin, l, W, n, 1.0f, gx, n);
    sgemm_rm(1, 0, l, n, m, 1.0f, gin, l, x, n, 1.0f, gW, n);
}

/* activation_function.cu:5-15 */
void ref_relu(float* x, long count) {
    for (long i = 0; i < count; i++) x[i] = x[i] > 0 ? x[i] : 0;
}
void ref_relu_derivative(const float* x, float* g, long count) {
    for (long i = 0; i < count; i++) g[i] = x[i] > 0 ? g[i] : 0;
}

/* loss.cu:5-23 — pow() is the double libm pow, accumulated into a float. */
float ref_mse(const float* y, const float* t, int m, int n) {
    float loss = 0.0f;
    for (int i = 0; i < m; i++)
        for (int j = 0; j < n; j++) loss += pow(t[i * n + j] - y[i * n + j], 2);
    return loss / (m * n);
}
void ref_mse_derivative(float* g, const float* y, const float* t, int m, int n) {
    for (int i = 0; i < m; i++)
        for (int j = 0; j < n; j++) g[i * n + j] = 2 * (y[i * n + j] - t[i * n + j]) / (m * n);
}

/* ------------------------------------------------------------------ */
/* MLP                                                                 */
/* ------------------------------------------------------------------ */
long ref_mlp_num_params(int num_sizes, const int* sizes) {
    long p = 0;
    for (int i = 0; i + 1 < num_sizes; i++) p += (long)sizes[i] * sizes[i + 1] + sizes[i + 1];
    return p;
}

/* neural_network.cu:40-51: He-uniform hidden layers (gain √2), Xavier-uniform
 * output layer (gain 1); biases U(−1,1)/√in.  Draw order: W then b per layer. */
void ref_mlp_init(int num_sizes, const int* sizes, float* params) {
    long off = 0;
    for (int i = 0; i + 1 < num_sizes; i++) {
        int in = sizes[i], out = sizes[i + 1];
        float gain = i == num_sizes - 2 ? 1 : sqrtf(2.0);
        float std = gain * sqrtf(2.0 / (in + out));
        for (long j = 0; j < (long)in * out; j++)
            params[off + j] = (2 * (float)rand() / RAND_MAX - 1) * sqrtf(3.0) * std;
        off += (long)in * out;
        for (int j = 0; j < out; j++)
            params[off + j] = (2 * (float)rand() / RAND_MAX - 1) * (1. / sqrtf(in));
        off += out;
    }
}

/* neural_network.cu:163-189 */
void ref_mlp_forward(int num_sizes, const int* sizes, const int* relu, const float* params,
                     const float* x, int m, float* acts) {
    const float* in = x;
    long poff = 0, aoff = 0;
    for (int i = 0; i + 1 < num_sizes; i++) {
        int n = sizes[i], l = sizes[i + 1];
        float* out = acts + aoff;
        ref_mat_mul(out, in, params + poff, params + poff + (long)n * l, m, n, l);
        if (relu[i]) ref_relu(out, (long)m * l);
        poff += (long)n * l + l;
        aoff += (long)m * l;
        in = out;
    }
}

/* neural_network.cu:192-231 */
void ref_mlp_backward(int num_sizes, const int* sizes, const int* relu, const float* params,
                      const float* x, const float* acts, const float* grad_out, int m,
                      float* grads, float* grad_x) {
    int L = num_sizes - 1;
    long* poff = (long*)malloc(sizeof(long) * (size_t)(L + 1));
    long* aoff = (long*)malloc(sizeof(long) * (size_t)(L + 1));
    poff[0] = 0; aoff[0] = 0;
    for (int i = 0; i < L; i++) {
        poff[i + 1] = poff[i] + (long)sizes[i] * sizes[i + 1] + sizes[i + 1];
        aoff[i + 1] = aoff[i] + (long)m * sizes[i + 1];
    }
    int outsz = sizes[L];
    float* layer_grad = (float*)malloc(sizeof(float) * (size_t)m * outsz);
    memcpy(layer_grad, grad_out, sizeof(float) * (size_t)m * outsz);
    if (relu[L - 1]) ref_relu_derivative(acts + aoff[L - 1], layer_grad, (long)m * outsz);

    for (int i = L - 1; i >= 0; i--) {
        int n = sizes[i], l = sizes[i + 1];
        const float* input = i == 0 ? x : acts + aoff[i - 1];
        float* gW = grads + poff[i];
        float* gb = gW + (long)n * l;
        memset(gW, 0, sizeof(float) * (size_t)n * l);
        memset(gb, 0, sizeof(float) * (size_t)l);
        for (int j = 0; j < l; j++)
            for (int k = 0; k < m; k++) gb[j] += layer_grad[(size_t)k * l + j];
        int want_gx = i > 0 || grad_x != NULL;
        float* tgx = want_gx ? (float*)calloc((size_t)m * n, sizeof(float)) : NULL;
        ref_mat_mul_backwards(tgx, gW, layer_grad, input, params + poff[i], m, n, l);
        free(layer_grad);
        layer_grad = tgx;
        if (i > 0 && relu[i - 1]) ref_relu_derivative(input, layer_grad, (long)m * n);
    }
    if (grad_x && layer_grad) memcpy(grad_x, layer_grad, sizeof(float) * (size_t)m * sizes[0]);
    free(layer_grad);
    free(poff);
    free(aoff);
}

/* ------------------------------------------------------------------ */
/* Gaussian policy                                                     */
/* ------------------------------------------------------------------ */
/* policy.cu:171-178 */
float ref_entropy(const float* log_std, int A) {
    float entropy = A * 0.5 * (1 + log(2 * M_PI));
    for (int j = 0; j < A; j++) entropy += log_std[j];
    return entropy;
}

/* policy.cu:67-74 */
static float log_prob_row(const float* mu, const float* log_std, const float* a, int A) {
    float lp = -0.5 * A * logf(2 * M_PI);
    for (int i = 0; i < A; i++) lp -= log_std[i] + 0.5 * powf((a[i] - mu[i]) / expf(log_std[i]), 2);
    return lp;
}

/* policy.cu:91-99 */
void ref_log_prob(const float* mu, const float* log_std, const float* action, int m, int A, float* out) {
    for (int i = 0; i < m; i++) out[i] = log_prob_row(mu + (size_t)i * A, log_std, action + (size_t)i * A, A);
}

/* policy.cu:101-111 with D2: grad_in is one value per SAMPLE (identical at A = 1). */
void ref_log_prob_backwards(const float* mu, const float* log_std, const float* action,
                            const float* grad_in, int m, int A, float* grad_mu, float* grad_log_std) {
    memset(grad_log_std, 0, sizeof(float) * (size_t)A);
    for (int i = 0; i < m; i++)
        for (int j = 0; j < A; j++) {
            size_t k = (size_t)i * A + j;
            grad_mu[k] = (action[k] - mu[k]) * expf(-2 * log_std[j]) * grad_in[i];
            grad_log_std[j] += (-1 + powf(action[k] - mu[k], 2) * expf(-2 * log_std[j])) * grad_in[i];
        }
}

/* policy.cu:46-65 Box–Muller on rand(), with D3 (every element filled). */
void ref_gaussian_noise(float* out, int n) {
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
    if (i < n)
        out[n - 1] = sqrtf(-2 * logf((float)rand() / RAND_MAX)) * cosf(2 * M_PI * (float)rand() / RAND_MAX);
}

/* ppo.cu:82-107 (exp() is the double libm exp). */
float ref_policy_loss_and_grad(float* grad_lp, float* grad_entropy, const float* adv, const float* lp,
                               const float* old_lp, float entropy, float ent_coeff, float epsilon, int m) {
    float loss = 0;
    for (int i = 0; i < m; i++) {
        float ratio = exp(lp[i] - old_lp[i]);
        int adv_pos = adv[i] > 0;
        int ratio_pos = ratio > 1 + epsilon;
        int ratio_neg = ratio < 1 - epsilon;
        loss -= adv[i] * (adv_pos * (ratio_pos * (1 + epsilon) + !ratio_pos * ratio) +
                          !adv_pos * (ratio_neg * (1 - epsilon) + !ratio_neg * ratio));
        grad_lp[i] = -(adv_pos * !ratio_pos + !adv_pos * !ratio_neg) * adv[i] * ratio / m;
    }
    loss /= m;
    loss -= ent_coeff * entropy;
    *grad_entropy = -ent_coeff;
    return loss;
}

/* ------------------------------------------------------------------ */
/* GAE (ppo.cu:326-369, after the two value forwards)                  */
/* ------------------------------------------------------------------ */
void ref_gae(const float* v, const float* v_next, const float* reward, const uint8_t* term,
             const uint8_t* trunc, int n, float gamma, float lambda,
             float* adv, float* adv_target, float* mean_out, float* std_out) {
    float* delta = (float*)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
    for (int i = 0; i < n; i++) delta[i] = reward[i] + gamma * v_next[i] * !term[i] - v[i];
    float sum = 0;
    float next = 0;                        /* D6: A[N] := 0 (the reference reads one past the end) */
    for (int i = n - 1; i >= 0; i--) {
        adv[i] = delta[i] + gamma * lambda * !(trunc[i] || term[i]) * next;
        next = adv[i];
        sum += adv[i];
    }
    for (int i = 0; i < n; i++) adv_target[i] = v[i] + adv[i];
    float mean = sum / n;
    float std = 0;
    for (int i = 0; i < n; i++) std += pow(adv[i] - mean, 2);
    std = sqrt(std / n);
    for (int i = 0; i < n; i++) adv[i] = (adv[i] - mean) / (std + 1e-8);
    if (mean_out) *mean_out = mean;
    if (std_out) *std_out = std;
    free(delta);
}

/* ------------------------------------------------------------------ */
/* buffer                                                              */
/* ------------------------------------------------------------------ */
/* trajectory_buffer.cu:126-146 — swap(i, rand() % N), a biased shuffle (D12). */
void ref_shuffle(int* perm, int n) {
    for (int i = 0; i < n; i++) perm[i] = i;
    for (int i = 0; i < n; i++) {
        int j = rand() % n;
        int t = perm[i];
        perm[i] = perm[j];
        perm[j] = t;
    }
}

/* libppo's device shuffle: a 4-round Feistel bijection on the smallest even
 * power-of-two domain ≥ n, cycle-walked into [0, n).  Restated here so tests
 * reproduce the device permutation bit-exactly (ppo.c_amd/csrc/buffer.hip). */
static uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
uint32_t ref_feistel_index(uint32_t i, uint32_t n, uint64_t key) {
    int bits = 2;
    while ((1ULL << bits) < n) bits++;
    int half = (bits + 1) / 2;
    uint32_t mask = (1u << half) - 1u;
    uint32_t k[4];
    for (int r = 0; r < 4; r++) k[r] = (uint32_t)splitmix64(key + (uint64_t)r);
    uint32_t x = i;
    do {
        uint32_t L = x >> half, R = x & mask;
        for (int r = 0; r < 4; r++) {
            uint32_t nl = R;
            R = L ^ (mix32(R ^ k[r]) & mask);
            L = nl;
        }
        x = (L << half) | R;
    } while (x >= n);
    return x;
}
void ref_feistel_perm(int* perm, int n, uint64_t key) {
    for (int i = 0; i < n; i++) perm[i] = (int)ref_feistel_index((uint32_t)i, (uint32_t)n, key);
}

/* trajectory_buffer.cu:202-220 */
void ref_get_batch(const int* perm, int n, int batch_idx, int batch_size, int S, int A,
                   const float* state, const float* action, const float* logprob,
                   const float* advantage, const float* adv_target,
                   float* states, float* actions, float* logprobs, float* advs, float* adv_targets) {
    int offset = batch_idx * batch_size;
    for (int i = 0; i < batch_size; i++) {
        int idx = perm[(offset + i) % n];
        memcpy(states + (size_t)i * S, state + (size_t)idx * S, sizeof(float) * (size_t)S);
        memcpy(actions + (size_t)i * A, action + (size_t)idx * A, sizeof(float) * (size_t)A);
        logprobs[i] = logprob[idx];
        advs[i] = advantage[idx];
        adv_targets[i] = adv_target[idx];
    }
}

/* ------------------------------------------------------------------ */
/* Adam (adam.cu:53-74)                                                */
/* ------------------------------------------------------------------ */
void ref_adam_update(float* params, const float* grads, float* m, float* v, long size,
                     int* time_step, float beta1, float beta2, float lr) {
    *time_step += 1;
    float bias_correction1 = 1 - powf(beta1, *time_step);
    float bias_correction2 = 1 - powf(beta2, *time_step);
    float step_size = lr / bias_correction1;
    for (long i = 0; i < size; i++) {
        m[i] = beta1 * m[i] + (1 - beta1) * grads[i];
        v[i] = beta2 * v[i] + (1 - beta2) * powf(grads[i], 2);
        float denom = sqrtf(v[i] / bias_correction2) + 1e-8;
        params[i] -= step_size * m[i] / denom;
    }
}

/* ------------------------------------------------------------------ */
/* one PPO update (ppo.cu:395-443, CPU branch, without collect_trajectories) */
/* ------------------------------------------------------------------ */
static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

void ref_ppo_update(const RefUpdateCfg* c, RefUpdateState* st) {
    const int ns = c->num_sizes, L = ns - 1;
    const int S = c->sizes_mu[0], A = c->sizes_mu[L], N = c->N, B = c->batch_size;
    int sizes_v[8];
    memcpy(sizes_v, c->sizes_mu, sizeof(int) * (size_t)ns);
    sizes_v[L] = 1;                                   /* ppo.cu:12-16 */
    long acts_mu = 0, acts_v = 0, acts_big = 0;
    for (int i = 1; i < ns; i++) {
        acts_mu += (long)B * c->sizes_mu[i];
        acts_v += (long)B * sizes_v[i];
        acts_big += (long)N * sizes_v[i];
    }
    long np_mu = ref_mlp_num_params(ns, c->sizes_mu), np_v = ref_mlp_num_params(ns, sizes_v);

    double t0 = now_s();
    /* compute_gae: V(next_state), V(state), then the recursion (ppo.cu:326-369) */
    float* big = (float*)malloc(sizeof(float) * (size_t)acts_big);
    float* vn = (float*)malloc(sizeof(float) * (size_t)N);
    float* vv = (float*)malloc(sizeof(float) * (size_t)N);
    ref_mlp_forward(ns, sizes_v, c->relu, st->v_params, st->next_state, N, big);
    memcpy(vn, big + acts_big - N, sizeof(float) * (size_t)N);
    ref_mlp_forward(ns, sizes_v, c->relu, st->v_params, st->state, N, big);
    memcpy(vv, big + acts_big - N, sizeof(float) * (size_t)N);
    free(big);
    ref_gae(vv, vn, st->reward, st->terminated, st->truncated, N, c->gamma, c->lambda,
            st->advantage, st->adv_target, &st->adv_mean, &st->adv_std);
    free(vn);
    free(vv);
    double t1 = now_s();

    float* states = (float*)malloc(sizeof(float) * (size_t)B * S);
    float* actions = (float*)malloc(sizeof(float) * (size_t)B * A);
    float* lp_old = (float*)malloc(sizeof(float) * (size_t)B);
    float* lp = (float*)malloc(sizeof(float) * (size_t)B);
    float* adv = (float*)malloc(sizeof(float) * (size_t)B);
    float* tgt = (float*)malloc(sizeof(float) * (size_t)B);
    float* g_lp = (float*)malloc(sizeof(float) * (size_t)B);
    float* g_mu = (float*)malloc(sizeof(float) * (size_t)B * A);
    float* g_v = (float*)malloc(sizeof(float) * (size_t)B);
    float* acts = (float*)malloc(sizeof(float) * (size_t)(acts_mu > acts_v ? acts_mu : acts_v));
    float* grads = (float*)malloc(sizeof(float) * (size_t)(np_mu > np_v ? np_mu : np_v));
    float* g_logstd = (float*)malloc(sizeof(float) * (size_t)A);
    int* perm = (int*)malloc(sizeof(int) * (size_t)N);
    /* D13: ceilf(capacity / batch_size) with integer division inside (ppo.cu:387-388); get_batch
     * wraps the rows modulo limit = N (trajectory_buffer.cu:168-200) */
    int num_batches = (c->capacity > 0 ? c->capacity : c->N) / B;
    uint64_t epoch_key = splitmix64(c->seed);
    int vsteps = 0, psteps = 0;

    for (int j = 0; j < c->n_epochs_value; j++) {
        if (c->shuffle_mode == 0) ref_shuffle(perm, N);
        else ref_feistel_perm(perm, N, epoch_key++);
        for (int k = 0; k < num_batches; k++) {
            if (c->max_value_steps >= 0 && vsteps >= c->max_value_steps) break;
            ref_get_batch(perm, N, k, B, S, A, st->state, st->action, st->logprob, st->advantage,
                          st->adv_target, states, actions, lp_old, adv, tgt);
            ref_mlp_forward(ns, sizes_v, c->relu, st->v_params, states, B, acts);
            const float* y = acts + acts_v - B;
            st->sum_v_loss += ref_mse(y, tgt, B, 1);
            ref_mse_derivative(g_v, y, tgt, B, 1);
            ref_mlp_backward(ns, sizes_v, c->relu, st->v_params, states, acts, g_v, B, grads, NULL);
            ref_adam_update(st->v_params, grads, st->m_v, st->v_v, np_v, &st->t_v, 0.9f, 0.999f, c->lr_v);
            st->n_v++;
            vsteps++;
        }
    }
    double t2 = now_s();
    for (int j = 0; j < c->n_epochs_policy; j++) {
        if (c->shuffle_mode == 0) ref_shuffle(perm, N);
        else ref_feistel_perm(perm, N, epoch_key++);
        for (int k = 0; k < num_batches; k++) {
            if (c->max_policy_steps >= 0 && psteps >= c->max_policy_steps) break;
            ref_get_batch(perm, N, k, B, S, A, st->state, st->action, st->logprob, st->advantage,
                          st->adv_target, states, actions, lp_old, adv, tgt);
            ref_mlp_forward(ns, c->sizes_mu, c->relu, st->mu_params, states, B, acts);
            const float* mu = acts + acts_mu - (long)B * A;
            ref_log_prob(mu, st->log_std, actions, B, A, lp);
            float entropy = ref_entropy(st->log_std, A);
            float g_ent;
            st->sum_policy_loss += ref_policy_loss_and_grad(g_lp, &g_ent, adv, lp, lp_old, entropy,
                                                            c->ent_coeff, c->epsilon, B);
            ref_log_prob_backwards(mu, st->log_std, actions, g_lp, B, A, g_mu, g_logstd);
            ref_mlp_backward(ns, c->sizes_mu, c->relu, st->mu_params, states, acts, g_mu, B, grads, NULL);
            for (int a = 0; a < A; a++) g_logstd[a] += g_ent;          /* ppo.cu:436-438 */
            ref_adam_update(st->log_std, g_logstd, st->m_ent, st->v_ent, A, &st->t_ent, 0.9f, 0.999f,
                            c->lr_policy);
            ref_adam_update(st->mu_params, grads, st->m_mu, st->v_mu, np_mu, &st->t_mu, 0.9f, 0.999f,
                            c->lr_policy);
            st->n_p++;
            psteps++;
        }
    }
    double t3 = now_s();
    st->t_gae = t1 - t0;
    st->t_value = t2 - t1;
    st->t_policy = t3 - t2;
    free(states); free(actions); free(lp_old); free(lp); free(adv); free(tgt);
    free(g_lp); free(g_mu); free(g_v); free(acts); free(grads); free(g_logstd); free(perm);
}
