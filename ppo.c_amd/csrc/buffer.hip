// buffer.hip — minibatch gather from the HBM-resident trajectory buffer.
//
// Reference: get_batch_kernel (trajectory_buffer.cu:168-200, K18): one thread per sample looping
// over state_size — uncoalesced.  Here one wave owns one minibatch row, so every row copy is a
// contiguous, coalesced read of state (S floats) and action (A floats).
//
// Row index of minibatch slot i:  list = (offset + i) mod limit, then either
//   perm[list]                            — a permutation in HBM (host rand() shuffle, the
//                                           reference's shuffle_buffer semantics), or
//   feistel(list)                         — libppo's device shuffle: a 4-round Feistel
//                                           bijection on 2^(2h) ≥ limit, cycle-walked into
//                                           [0, limit); no storage, no host work.  Restated
//                                           bit-exactly in oracle/ref_cpu.c (ref_feistel_index).
#include "dev.h"

namespace {

constexpr int TPB = 256;

struct Feistel { uint32_t k[4]; uint32_t half, mask, n; };

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

__device__ __forceinline__ uint32_t feistel_index(uint32_t i, const Feistel& f) {
    uint32_t x = i;
    do {
        uint32_t L = x >> f.half, R = x & f.mask;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t nl = R;
            R = L ^ (mix32(R ^ f.k[r]) & f.mask);
            L = nl;
        }
        x = (L << f.half) | R;
    } while (x >= f.n);
    return x;
}

__global__ void gather_kernel(const int* __restrict__ perm, Feistel f, int offset, int limit, int batch, int S,
                              int A, const float* __restrict__ state, const float* __restrict__ action,
                              const float* __restrict__ logprob, const float* __restrict__ advantage,
                              const float* __restrict__ adv_target, float* __restrict__ states,
                              float* __restrict__ actions, float* __restrict__ logprobs, float* __restrict__ advs,
                              float* __restrict__ adv_targets, int* __restrict__ rows) {
    const int lane = threadIdx.x & 63;
    const int waves = gridDim.x * (TPB / 64);
    for (int i = blockIdx.x * (TPB / 64) + (threadIdx.x >> 6); i < batch; i += waves) {
        const int list = (int)(((long)offset + i) % limit);
        const int src = perm ? perm[list] : (int)feistel_index((uint32_t)list, f);
        if (states) {
            const float* sp = state + (long)src * S;
            float* dp = states + (long)i * S;
            for (int c = lane; c < S; c += 64) dp[c] = sp[c];
        }
        if (actions) {
            const float* sp = action + (long)src * A;
            float* dp = actions + (long)i * A;
            for (int c = lane; c < A; c += 64) dp[c] = sp[c];
        }
        if (lane == 0) {
            if (rows) rows[i] = src;
            if (logprobs) logprobs[i] = logprob[src];
            if (advs) advs[i] = advantage[src];
            if (adv_targets) adv_targets[i] = adv_target[src];
        }
    }
}

// No state rows to copy (layer 0 gathers them itself): one thread per minibatch slot writes the
// slot's source row and its small per-row fields — one pass, every slot's loads in flight together.
__global__ void gather_small_kernel(const int* __restrict__ perm, Feistel f, int offset, int limit, int batch, int A,
                                    const float* __restrict__ action, const float* __restrict__ logprob,
                                    const float* __restrict__ advantage, const float* __restrict__ adv_target,
                                    float* __restrict__ actions, float* __restrict__ logprobs,
                                    float* __restrict__ advs, float* __restrict__ adv_targets,
                                    int* __restrict__ rows) {
    const int i = blockIdx.x * TPB + threadIdx.x;
    if (i >= batch) return;
    const int list = (int)(((long)offset + i) % limit);
    const int src = perm ? perm[list] : (int)feistel_index((uint32_t)list, f);
    if (rows) rows[i] = src;
    if (logprobs) logprobs[i] = logprob[src];
    if (advs) advs[i] = advantage[src];
    if (adv_targets) adv_targets[i] = adv_target[src];
    if (actions) {
        const float* sp = action + (long)src * A;
        float* dp = actions + (long)i * A;
        for (int c = 0; c < A; ++c) dp[c] = sp[c];
    }
}

// the same gather with its per-step arguments from the step table (graph replay)
__global__ void gather_small_tab_kernel(const PhipStepArgs* __restrict__ tab, const int* __restrict__ ctr,
                                        const int* __restrict__ perm_base, int limit, int batch, int A,
                                        const float* __restrict__ action, const float* __restrict__ logprob,
                                        const float* __restrict__ advantage, const float* __restrict__ adv_target,
                                        float* __restrict__ actions, float* __restrict__ logprobs,
                                        float* __restrict__ advs, float* __restrict__ adv_targets,
                                        int* __restrict__ rows) {
    const int i = blockIdx.x * TPB + threadIdx.x;
    if (i >= batch) return;
    const PhipStepArgs& s = tab[*ctr];
    Feistel f;
#pragma unroll
    for (int r = 0; r < 4; ++r) f.k[r] = s.fk[r];
    f.half = s.fhalf; f.mask = s.fmask; f.n = s.fn;
    const int list = (int)(((long)s.offset + i) % limit);
    const int src = s.perm_off >= 0 ? perm_base[s.perm_off + list] : (int)feistel_index((uint32_t)list, f);
    if (rows) rows[i] = src;
    if (logprobs) logprobs[i] = logprob[src];
    if (advs) advs[i] = advantage[src];
    if (adv_targets) adv_targets[i] = adv_target[src];
    if (actions) {
        const float* sp = action + (long)src * A;
        float* dp = actions + (long)i * A;
        for (int c = 0; c < A; ++c) dp[c] = sp[c];
    }
}

uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

}  // namespace

extern "C" {

void phip_gather_rows(const int* perm, uint64_t key, int offset, int limit, int batch, int S, int A,
                      const float* state, const float* action, const float* logprob, const float* advantage,
                      const float* adv_target, float* states, float* actions, float* logprobs, float* advs,
                      float* adv_targets, int* rows) {
    if (batch <= 0) return;
    PPO_REQUIRE(limit > 0, "phip_gather: empty buffer");
    Feistel f{};
    int bits = 2;
    while ((1ULL << bits) < (unsigned long long)limit) bits++;
    f.half = (uint32_t)((bits + 1) / 2);
    f.mask = (1u << f.half) - 1u;
    f.n = (uint32_t)limit;
    for (int r = 0; r < 4; ++r) f.k[r] = (uint32_t)splitmix64(key + (uint64_t)r);
    ppo::ProfScope ps(PPO_K_GATHER, 8.0 * batch * ((states ? S : 0) + (actions ? A : 0) + 3));
    if (!states && (!actions || A <= 32)) {
        hipLaunchKernelGGL(gather_small_kernel, dim3(ppo_divup(batch, TPB)), dim3(TPB), 0, ppo::stream(), perm, f,
                           offset, limit, batch, A, action, logprob, advantage, adv_target, actions, logprobs, advs,
                           adv_targets, rows);
        PPO_LAUNCH_CHECK();
        return;
    }
    int grid = ppo_divup(batch, TPB / 64);
    if (grid > 8192) grid = 8192;
    hipLaunchKernelGGL(gather_kernel, dim3(grid), dim3(TPB), 0, ppo::stream(), perm, f, offset, limit, batch, S, A,
                       state, action, logprob, advantage, adv_target, states, actions, logprobs, advs, adv_targets,
                       rows);
    PPO_LAUNCH_CHECK();
}

void phip_step_feistel(PhipStepArgs* s, unsigned long long key, int limit) {
    int bits = 2;
    while ((1ULL << bits) < (unsigned long long)limit) bits++;
    s->fhalf = (unsigned)((bits + 1) / 2);
    s->fmask = (1u << s->fhalf) - 1u;
    s->fn = (unsigned)limit;
    for (int r = 0; r < 4; ++r) s->fk[r] = (unsigned)splitmix64(key + (uint64_t)r);
}

void phip_gather_rows_tab(const PhipStepArgs* tab, const int* ctr, const int* perm_base, int limit, int batch, int A,
                          const float* action, const float* logprob, const float* advantage,
                          const float* adv_target, float* actions, float* logprobs, float* advs, float* adv_targets,
                          int* rows) {
    if (batch <= 0) return;
    PPO_REQUIRE(limit > 0 && (!actions || A <= 32), "phip_gather_rows_tab: unsupported shape");
    hipLaunchKernelGGL(gather_small_tab_kernel, dim3(ppo_divup(batch, TPB)), dim3(TPB), 0, ppo::stream(), tab, ctr,
                       perm_base, limit, batch, A, action, logprob, advantage, adv_target, actions, logprobs, advs,
                       adv_targets, rows);
    PPO_LAUNCH_CHECK();
}

void phip_gather(const int* perm, uint64_t key, int offset, int limit, int batch, int S, int A,
                 const float* state, const float* action, const float* logprob, const float* advantage,
                 const float* adv_target, float* states, float* actions, float* logprobs, float* advs,
                 float* adv_targets) {
    phip_gather_rows(perm, key, offset, limit, batch, S, A, state, action, logprob, advantage, adv_target, states,
                     actions, logprobs, advs, adv_targets, nullptr);
}

}  // extern "C"
