// rollout.hip — batched on-device rollout: all E environments step together.
//
// Reference collect_trajectories (ppo.cu:54-79) steps ONE environment on the host: policy sgemv
// (m = 1), rand()-Box–Muller noise (policy.cu:46-89), a gymnasium step through CPython.  Here one
// rollout step for E environments is: the μ forward over E rows (the buffer rows e·T + t read
// through the GEMM's row indirection), one sampling kernel that writes action / log-prob straight
// into the buffer rows, and one environment kernel.  Buffer layout is the env-major convention of
// ppo.cu:70-74: transition (e, t) at row e·T + t, every segment ending with truncated = 1.
//
// Environments (device, per-env state in HBM):
//   kind 0 — Pendulum-v1 (S = 3, A = 1): gymnasium classic_control dynamics as restated in
//            host/env.c (g = 10, m = l = 1, dt = 0.05, max speed 8, max torque 2, 200-step limit);
//            reset θ ~ U(−π, π), θ̇ ~ U(−1, 1) from Philox.
//   kind 1 — synthetic (any S, A): o' = clip(0.95·o + 0.05·tanh(a[j mod A]) +
//            0.05·ε, −1, 1); r = −0.01·mean(a²) + 0.1·ε; terminated ~ Bernoulli(1/500), reset
//            o ~ U(−1, 1).
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

__device__ __forceinline__ float u01(uint32_t x) { return ((x >> 8) + 0.5f) * (1.0f / 16777216.0f); }

__device__ __forceinline__ float normal_at(uint64_t idx, uint64_t offset, uint64_t seed) {
    const u32x4 r = philox(idx, offset, seed);
    return sqrtf(-2.f * logf(u01(r.x))) * cosf(2.f * (float)M_PI * u01(r.y));
}

// Streams of the Philox key space used here (offset high bits): policy noise, env noise, resets.
constexpr uint64_t kNoise = 1ull << 40, kEnv = 2ull << 40, kReset = 3ull << 40;

// a = μ + ε·σ written to buffer row rows[e]; log π(a) as policy.cu:67-74 (same as sample.hip)
__global__ void sample_rows_kernel(const float* __restrict__ mu, const float* __restrict__ log_std,
                                   const int* __restrict__ rows, float* __restrict__ action,
                                   float* __restrict__ logprob, int E, int A, uint64_t seed, uint64_t step) {
    const int e = blockIdx.x * TPB + threadIdx.x;
    if (e >= E) return;
    const float* mr = mu + (long)e * A;
    float* ar = action + (long)rows[e] * A;
    const float c = (float)(-0.5 * A * (double)logf((float)(2 * M_PI)));
    float lp = c;
    for (int j = 0; j < A; ++j) {
        const float a = mr[j] + normal_at((uint64_t)e * A + j, kNoise + step, seed) * expf(log_std[j]);
        ar[j] = a;
        const float z = (a - mr[j]) / expf(log_std[j]);
        lp = (float)((double)lp - ((double)log_std[j] + 0.5 * (double)(z * z)));
    }
    logprob[rows[e]] = lp;
}

__device__ __forceinline__ float angle_normalize(float x) {
    const float two_pi = 2.f * (float)M_PI;
    float y = fmodf(x + (float)M_PI, two_pi);
    if (y < 0.f) y += two_pi;
    return y - (float)M_PI;
}

// Pendulum-v1: env state (θ, θ̇, steps) in es[3e .. 3e+2]
__global__ void pendulum_step_kernel(float* __restrict__ es, float* __restrict__ state,
                                     const float* __restrict__ action, float* __restrict__ next_state,
                                     float* __restrict__ reward, uint8_t* __restrict__ term,
                                     uint8_t* __restrict__ trunc, int E, int T, int t, uint64_t seed) {
    const int e = blockIdx.x * TPB + threadIdx.x;
    if (e >= E) return;
    const long row = (long)e * T + t;
    float th = es[3 * e], thdot = es[3 * e + 1];
    float steps = es[3 * e + 2];
    const float u = fminf(fmaxf(action[row], -2.f), 2.f);
    const float an = angle_normalize(th);
    const float cost = an * an + 0.1f * thdot * thdot + 0.001f * u * u;
    float nthdot = thdot + (3.f * 10.f / 2.f * sinf(th) + 3.f * u) * 0.05f;
    nthdot = fminf(fmaxf(nthdot, -8.f), 8.f);
    th = th + nthdot * 0.05f;
    thdot = nthdot;
    steps += 1.f;
    next_state[3 * row] = cosf(th);
    next_state[3 * row + 1] = sinf(th);
    next_state[3 * row + 2] = thdot;
    reward[row] = -cost;
    const bool limit = steps >= 200.f;
    term[row] = 0;
    trunc[row] = (limit || t == T - 1) ? 1 : 0;
    if (limit) {                                         // TimeLimit reset
        const u32x4 r = philox((uint64_t)e, kReset + (uint64_t)t, seed);
        th = -(float)M_PI + 2.f * (float)M_PI * u01(r.x);
        thdot = -1.f + 2.f * u01(r.y);
        steps = 0.f;
    }
    es[3 * e] = th;
    es[3 * e + 1] = thdot;
    es[3 * e + 2] = steps;
    if (t + 1 < T) {
        state[3 * (row + 1)] = cosf(th);
        state[3 * (row + 1) + 1] = sinf(th);
        state[3 * (row + 1) + 2] = thdot;
    }
}

// synthetic env: one thread per (env, obs element); the reward / done decision per env is taken
// by every thread of the env identically (same Philox draw), so no cross-thread exchange
__global__ void synth_step_kernel(float* __restrict__ es, float* __restrict__ state, const float* __restrict__ action,
                                  float* __restrict__ next_state, float* __restrict__ reward,
                                  uint8_t* __restrict__ term, uint8_t* __restrict__ trunc, int E, int T, int t,
                                  int S, int A, uint64_t seed) {
    const long k = (long)blockIdx.x * TPB + threadIdx.x;
    if (k >= (long)E * S) return;
    const int e = (int)(k / S), j = (int)(k % S);
    const long row = (long)e * T + t;
    const float* ar = action + row * A;
    const u32x4 d = philox((uint64_t)e, kEnv + 2 * (uint64_t)t, seed);
    const bool done = u01(d.z) < 1.f / 500.f;
    const float o = es[k];
    const float eps = normal_at((uint64_t)k, kEnv + 2 * (uint64_t)t + 1, seed);
    float o2 = 0.95f * o + 0.05f * tanhf(ar[j % A]) + 0.05f * eps;
    o2 = fminf(fmaxf(o2, -1.f), 1.f);
    next_state[row * S + j] = o2;
    if (j == 0) {
        float ss = 0.f;
        for (int q = 0; q < A; ++q) ss += ar[q] * ar[q];
        reward[row] = -0.01f * ss / (float)A + 0.1f * sqrtf(-2.f * logf(u01(d.x))) * cosf(2.f * (float)M_PI * u01(d.y));
        term[row] = done ? 1 : 0;
        trunc[row] = (!done && t == T - 1) ? 1 : 0;
    }
    const float nxt = done ? -1.f + 2.f * u01(philox((uint64_t)k, kReset + (uint64_t)t, seed).x) : o2;
    es[k] = nxt;
    if (t + 1 < T) state[(row + 1) * S + j] = nxt;
}

// reset every env; write row e·T (t = 0) of the buffer
__global__ void env_reset_kernel(int kind, float* __restrict__ es, float* __restrict__ state, int E, int T, int S,
                                 uint64_t seed) {
    const long k = (long)blockIdx.x * TPB + threadIdx.x;
    if (kind == 0) {
        if (k >= E) return;
        const u32x4 r = philox((uint64_t)k, kReset - 1, seed);
        const float th = -(float)M_PI + 2.f * (float)M_PI * u01(r.x), thdot = -1.f + 2.f * u01(r.y);
        es[3 * k] = th; es[3 * k + 1] = thdot; es[3 * k + 2] = 0.f;
        return;
    }
    if (k >= (long)E * S) return;
    es[k] = -1.f + 2.f * u01(philox((uint64_t)k, kReset - 1, seed).x);
}

// first row of each segment from the persistent env state (episodes continue across rollouts)
__global__ void env_obs_kernel(int kind, const float* __restrict__ es, float* __restrict__ state, int E, int T,
                               int S) {
    const long k = (long)blockIdx.x * TPB + threadIdx.x;
    if (k >= (long)E * S) return;
    const int e = (int)(k / S), j = (int)(k % S);
    float v;
    if (kind == 0) v = j == 0 ? cosf(es[3 * e]) : (j == 1 ? sinf(es[3 * e]) : es[3 * e + 1]);
    else v = es[k];
    state[(long)e * T * S + j] = v;
}

__global__ void rows_kernel(int* __restrict__ rows, int E, int T) {
    const long k = (long)blockIdx.x * TPB + threadIdx.x;     // k = t·E + e
    if (k >= (long)E * T) return;
    const int t = (int)(k / E), e = (int)(k % E);
    rows[k] = e * T + t;
}

}  // namespace

extern "C" {

void phip_rollout_rows(int* rows, int E, int T) {
    const long n = (long)E * T;
    hipLaunchKernelGGL(rows_kernel, dim3(ppo_divup(n, TPB)), dim3(TPB), 0, ppo::stream(), rows, E, T);
    PPO_LAUNCH_CHECK();
}

void phip_env_reset(int kind, float* env_state, float* state, int E, int T, int S, uint64_t seed) {
    const long n = kind == 0 ? E : (long)E * S;
    hipLaunchKernelGGL(env_reset_kernel, dim3(ppo_divup(n, TPB)), dim3(TPB), 0, ppo::stream(), kind, env_state, state,
                       E, T, S, seed);
    PPO_LAUNCH_CHECK();
}

void phip_env_first_obs(int kind, const float* env_state, float* state, int E, int T, int S) {
    const long n = (long)E * S;
    hipLaunchKernelGGL(env_obs_kernel, dim3(ppo_divup(n, TPB)), dim3(TPB), 0, ppo::stream(), kind, env_state, state,
                       E, T, S);
    PPO_LAUNCH_CHECK();
}

void phip_sample_rows(const float* mu, const float* log_std, const int* rows, float* action, float* logprob, int E,
                      int A, uint64_t seed, uint64_t step) {
    ppo::ProfScope ps(PPO_K_OTHER, 4.0 * E * (2 * A + 1));
    hipLaunchKernelGGL(sample_rows_kernel, dim3(ppo_divup(E, TPB)), dim3(TPB), 0, ppo::stream(), mu, log_std, rows,
                       action, logprob, E, A, seed, step);
    PPO_LAUNCH_CHECK();
}

void phip_env_step(int kind, float* env_state, float* state, const float* action, float* next_state, float* reward,
                   uint8_t* term, uint8_t* trunc, int E, int T, int t, int S, int A, uint64_t seed) {
    ppo::ProfScope ps(PPO_K_OTHER, 4.0 * E * (3 * S + A + 2));
    if (kind == 0) {
        PPO_REQUIRE(S == 3 && A == 1, "phip_env_step: Pendulum-v1 needs S = 3, A = 1");
        hipLaunchKernelGGL(pendulum_step_kernel, dim3(ppo_divup(E, TPB)), dim3(TPB), 0, ppo::stream(), env_state,
                           state, action, next_state, reward, term, trunc, E, T, t, seed);
    } else {
        hipLaunchKernelGGL(synth_step_kernel, dim3(ppo_divup((long)E * S, TPB)), dim3(TPB), 0, ppo::stream(),
                           env_state, state, action, next_state, reward, term, trunc, E, T, t, S, A, seed);
    }
    PPO_LAUNCH_CHECK();
}

}  // extern "C"
