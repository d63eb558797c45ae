// sample.hip — batched Gaussian policy sampling and seeded synthetic rollouts.
//
// Reference sample_action (policy.cu:76-89) draws Box–Muller noise from libc rand() on the host
// for one environment at a time.  Here the noise is counter-based (Philox-4x32-10, keyed by a
// seed, counter = element index + offset) so any number of environments sample in one launch,
// deterministically and independently of launch geometry:
//   a = μ + ε·exp(log_std),   log π(a) as in policy.cu:67-74.
// The synthetic-rollout fills implement SURVEY §8d's generator on the device.
#include "dev.h"

#include <cmath>

namespace {

constexpr int TPB = 256;

struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox(uint64_t counter, uint64_t offset, uint64_t seed) {
    uint32_t c0 = (uint32_t)counter, c1 = (uint32_t)(counter >> 32);
    uint32_t c2 = (uint32_t)offset, c3 = (uint32_t)(offset >> 32);
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return u32x4{c0, c1, c2, c3};
}

// uniform in (0, 1): 24 random bits, centred in their bucket
__device__ __forceinline__ float u01(uint32_t x) { return ((x >> 8) + 0.5f) * (1.0f / 16777216.0f); }

__device__ __forceinline__ float normal_at(uint64_t idx, uint64_t offset, uint64_t seed) {
    const u32x4 r = philox(idx, offset, seed);
    const float u1 = u01(r.x), u2 = u01(r.y);
    return sqrtf(-2.f * logf(u1)) * cosf(2.f * (float)M_PI * u2);
}

__device__ __forceinline__ float log_prob_row(const float* mu, const float* log_std, const float* a, int A) {
    const float c = (float)(-0.5 * A * (double)logf((float)(2 * M_PI)));
    float lp = c;
    for (int j = 0; j < A; ++j) {
        const float z = (a[j] - mu[j]) / expf(log_std[j]);
        lp = (float)((double)lp - ((double)log_std[j] + 0.5 * (double)(z * z)));
    }
    return lp;
}

__global__ void sample_kernel(const float* __restrict__ mu, const float* __restrict__ log_std,
                              float* __restrict__ action, float* __restrict__ logprob, int m, int A, uint64_t seed,
                              uint64_t offset) {
    const int i = blockIdx.x * TPB + threadIdx.x;
    if (i >= m) return;
    const float* mr = mu + (long)i * A;
    float* ar = action + (long)i * A;
    for (int j = 0; j < A; ++j) ar[j] = mr[j] + normal_at((uint64_t)i * A + j, offset, seed) * expf(log_std[j]);
    if (logprob) logprob[i] = log_prob_row(mr, log_std, ar, A);
}

__global__ void sample_noise_kernel(const float* __restrict__ mu, const float* __restrict__ log_std,
                                    const float* __restrict__ noise, float* __restrict__ action,
                                    float* __restrict__ logprob, int m, int A) {
    const int i = blockIdx.x * TPB + threadIdx.x;
    if (i >= m) return;
    const float* mr = mu + (long)i * A;
    float* ar = action + (long)i * A;
    for (int j = 0; j < A; ++j) ar[j] = mr[j] + noise[(long)i * A + j] * expf(log_std[j]);   // policy.cu:84
    if (logprob) logprob[i] = log_prob_row(mr, log_std, ar, A);
}

__global__ void fill_uniform_kernel(float* __restrict__ p, long n, uint64_t seed, float lo, float hi) {
    for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < n; i += (long)gridDim.x * TPB)
        p[i] = lo + (hi - lo) * u01(philox((uint64_t)i, 0x5EED, seed).x);
}

__global__ void fill_normal_kernel(float* __restrict__ p, long n, uint64_t seed, float scale) {
    for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < n; i += (long)gridDim.x * TPB)
        p[i] = scale * normal_at((uint64_t)i, 0xA11CE, seed);
}

__global__ void fill_flags_kernel(uint8_t* __restrict__ term, uint8_t* __restrict__ trunc, int n_envs, int T,
                                  float p_term, uint64_t seed) {
    const long n = (long)n_envs * T;
    for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < n; i += (long)gridDim.x * TPB) {
        const int t = (int)(i % T);
        const uint8_t te = u01(philox((uint64_t)i, 0x7E4, seed).x) < p_term;
        term[i] = te;
        trunc[i] = (t == T - 1) && !te;          // ppo.cu:70-74: last step truncated unless terminated
    }
}

__global__ void link_next_kernel(float* __restrict__ next_state, const float* __restrict__ state,
                                 const uint8_t* __restrict__ term, int n_envs, int T, int S, uint64_t seed) {
    const long n = (long)n_envs * T * S;
    for (long k = blockIdx.x * (long)TPB + threadIdx.x; k < n; k += (long)gridDim.x * TPB) {
        const long row = k / S;
        const int t = (int)(row % T);
        if (t + 1 < T && !term[row]) next_state[k] = state[k + S];
        else next_state[k] = -1.f + 2.f * u01(philox((uint64_t)k, 0x4E57, seed).x);
    }
}

int grid_for(long n) {
    long g = (n + TPB - 1) / TPB;
    if (g < 1) g = 1;
    if (g > 8192) g = 8192;
    return (int)g;
}

}  // namespace

extern "C" {

void phip_sample(const float* mu, const float* log_std, float* action, float* logprob, int m, int A, uint64_t seed,
                 uint64_t offset) {
    if (m <= 0) return;
    ppo::ProfScope ps(PPO_K_OTHER, 4.0 * m * (2 * A + 1));
    hipLaunchKernelGGL(sample_kernel, dim3(ppo_divup(m, TPB)), dim3(TPB), 0, ppo::stream(), mu, log_std, action,
                       logprob, m, A, seed, offset);
    PPO_LAUNCH_CHECK();
}

void phip_sample_noise(const float* mu, const float* log_std, const float* noise, float* action, float* logprob,
                       int m, int A) {
    if (m <= 0) return;
    hipLaunchKernelGGL(sample_noise_kernel, dim3(ppo_divup(m, TPB)), dim3(TPB), 0, ppo::stream(), mu, log_std, noise,
                       action, logprob, m, A);
    PPO_LAUNCH_CHECK();
}

void phip_fill_uniform(float* p, long n, uint64_t seed, float lo, float hi) {
    if (n <= 0) return;
    hipLaunchKernelGGL(fill_uniform_kernel, dim3(grid_for(n)), dim3(TPB), 0, ppo::stream(), p, n, seed, lo, hi);
    PPO_LAUNCH_CHECK();
}

void phip_fill_normal(float* p, long n, uint64_t seed, float scale) {
    if (n <= 0) return;
    hipLaunchKernelGGL(fill_normal_kernel, dim3(grid_for(n)), dim3(TPB), 0, ppo::stream(), p, n, seed, scale);
    PPO_LAUNCH_CHECK();
}

void phip_fill_rollout_flags(uint8_t* term, uint8_t* trunc, int n_envs, int horizon, float p_term, uint64_t seed) {
    const long n = (long)n_envs * horizon;
    if (n <= 0) return;
    hipLaunchKernelGGL(fill_flags_kernel, dim3(grid_for(n)), dim3(TPB), 0, ppo::stream(), term, trunc, n_envs,
                       horizon, p_term, seed);
    PPO_LAUNCH_CHECK();
}

void phip_link_next_state(float* next_state, const float* state, const uint8_t* term, int n_envs, int horizon, int S,
                          uint64_t seed) {
    const long n = (long)n_envs * horizon * S;
    if (n <= 0) return;
    hipLaunchKernelGGL(link_next_kernel, dim3(grid_for(n)), dim3(TPB), 0, ppo::stream(), next_state, state, term,
                       n_envs, horizon, S, seed);
    PPO_LAUNCH_CHECK();
}

}  // extern "C"
