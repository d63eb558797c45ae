// cluster_common.h — device primitives shared by the multi-workgroup phase kernels (cluster.hip,
// cluster_deep.hip): the device Feistel order, the sc1 hand-off primitives and the split barrier
// (MI355X_MICROARCH.md § inter-workgroup visibility, the first row of the sc1 table), fixed-order
// column sums, the 16×16×4 fp32 MFMA tile from LDS, and the per-row PPO head / Adam arithmetic.
#pragma once
#include "dev.h"

#include <cmath>
#include <cstdint>

#ifndef CLU_REPL
#define CLU_REPL 8                                   // barrier counter replicas (128-B lines; ≤ 64)
#endif
#ifndef CLU_RSTRIDE
#define CLU_RSTRIDE 32                               // words between replicas (32: adjacent 128-B lines)
#endif
constexpr int CLU_CTR_BYTES = 4 * CLU_RSTRIDE * CLU_REPL;
#ifndef CLU_SLEEP
#define CLU_SLEEP 4                                  // s_sleep between barrier polls (× 64 clocks): 32 pollers
                                                     // at 1 slowed every barrier (C4 value step 75 → 69 µs at 4)
#endif

namespace clu {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int TPB = 512, NWAVE = TPB / 64;   // eight waves per workgroup
constexpr int BB = 64;                       // minibatch rows (the reference's B, main.c:34)

struct Feistel { uint32_t k[4]; uint32_t half, mask, n; };

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
// identical to buffer.hip's feistel_index (restated in oracle/ref_cpu.c: ref_feistel_index)
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

// ---- hand-off primitives (sc1: write-through stores, L1-bypassing loads) ----
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* p, long floats) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, (int)(floats * 4), 0x00020000);
}
__device__ __forceinline__ void st16_sc1(__amdgpu_buffer_rsrc_t r, int off_floats, f32x4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off_floats * 4, 0, 16);
}
__device__ __forceinline__ f32x4 ld16_sc1(__amdgpu_buffer_rsrc_t r, int off_floats) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off_floats * 4, 0, 16));
}
__device__ __forceinline__ float ld4_sc1(__amdgpu_buffer_rsrc_t r, int off_floats) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off_floats * 4, 0, 16));
}

// The arrival counter is kept in CLU_REPL replicas, each on a 128-B line of its own (ctr + 32·r;
// MI355X_MICROARCH.md's replicated-counter row): every workgroup adds to every replica with ONE wave
// instruction (lanes 0 … CLU_REPL−1, one replica each) and polls only its own replica, so the polls of
// 32 workgroups spread over CLU_REPL lines instead of loading the line every arrival lands on.
// Arrival: the workgroup's published stores are complete (every wave drained, then a workgroup
// barrier), then the adds.  Work that publishes nothing may run between cluster_arrive and
// cluster_wait (it overlaps the other workgroups' arrival skew).
__device__ __forceinline__ void cluster_arrive(unsigned* ctr) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x < CLU_REPL)
        __hip_atomic_fetch_add(ctr + CLU_RSTRIDE * threadIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Wait until all `nwg` workgroups have arrived for barrier number `n` (counting from 0 within the
// launch; `rank` = the workgroup's index in the phase, picks its replica): the arriving lane polls
// (sc1 loads + s_sleep), the other waves wait at the workgroup barrier it then joins.  The wait is
// bounded in wall-clock time (`timeout` ticks of the constant 100 MHz realtime counter, from the first
// unsuccessful poll) and ends early when another workgroup has already set the error word.  Returns
// false on timeout (error word set), uniformly for the workgroup.
__device__ __forceinline__ bool cluster_wait(unsigned* ctr, unsigned* err, unsigned n, int nwg, int* flag_lds, int rank,
                                             unsigned long long timeout) {
    if (threadIdx.x == 0) {
        ctr += CLU_RSTRIDE * (rank % CLU_REPL);                         // this workgroup's replica
        const unsigned target = (unsigned)nwg * (n + 1);
        int ok = 1;
        if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            const unsigned long long t0 = wall_clock64();
            while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                __builtin_amdgcn_s_sleep(CLU_SLEEP);
                if (wall_clock64() - t0 > timeout ||
                    __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) {
                    __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    ok = 0;
                    break;
                }
            }
        }
        *flag_lds = ok;
    }
    __syncthreads();
    return *flag_lds != 0;
}

// Σ_b M[b][col] over the 64 minibatch rows for columns [0, NC) by ONE wave, in a fixed order: lane
// (col = lane / P, part = lane % P) adds rows part·R … part·R + R − 1 in order, then the P parts are
// combined by xor shuffles (commutative pairs: every lane of a column, and every workgroup, gets the
// same bits).  out[col] = sum + add for col < ncols.
template <int NC>
__device__ __forceinline__ void colsum64(const float* M, int pitch, int ncols, float add, float* out,
                                         int tid = (int)threadIdx.x) {
    constexpr int P = 64 / NC, R = 64 / P;
    const int lane = tid & 63, col = lane / P, part = lane % P;
    float v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = M[(part * R + r) * pitch + col];
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < R; ++r) s += v[r];
#pragma unroll
    for (int o = 1; o < P; o <<= 1) s += __shfl_xor(s, o, 64);
    if (part == 0 && col < ncols) out[col] = s + add;
}

// One 16×16 output tile: acc(i, j) = Σ_k A(i, k)·B(k, j), A(i, k) = A[i·as_i + k·as_k],
// B(k, j) = B[k·bs_k + j·bs_j] (pointers at the tile's origin, LDS).  Lane (c = l&15, q = l>>4)
// loads A(c, k0+q), B(k0+q, c) and receives acc rows 4q..4q+3 of column c.  K ≥ 1; a k-tail
// (K % 4) is zeroed.  Eight MFMAs' operands are loaded before their MFMAs issue.
__device__ __forceinline__ f32x4 mm_tile(const float* A, int as_i, int as_k, const float* B, int bs_k, int bs_j,
                                         int K, int tid = (int)threadIdx.x) {
    const int lane = tid & 63, c = lane & 15, q = lane >> 4;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const float* Ar = A + c * as_i;
    const float* Bc = B + c * bs_j;
    for (int k0 = 0; k0 < K; k0 += 32) {
        float av[8], bv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int k = min(k0 + 4 * u + q, K - 1);
            av[u] = Ar[k * as_k];
            bv[u] = Bc[k * bs_k];
        }
        asm("" : "+v"(av[0]), "+v"(av[1]), "+v"(av[2]), "+v"(av[3]), "+v"(av[4]), "+v"(av[5]), "+v"(av[6]),
                 "+v"(av[7]), "+v"(bv[0]), "+v"(bv[1]), "+v"(bv[2]), "+v"(bv[3]), "+v"(bv[4]), "+v"(bv[5]),
                 "+v"(bv[6]), "+v"(bv[7]));
        const int nu = K - k0 >= 32 ? 8 : (K - k0 + 3) >> 2;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const bool kin = k0 + 4 * u + q < K;
            if (u < nu) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(kin ? av[u] : 0.f, kin ? bv[u] : 0.f, acc, 0, 0, 0);
        }
    }
    return acc;
}

__device__ __forceinline__ float log_prob_row(const float* mu, const float* log_std, const float* a, int A) {
    const float cst = (float)(-0.5 * A * (double)logf((float)(2 * M_PI)));
    float lp = cst;
    for (int j = 0; j < A; ++j) {
        const float z = (a[j] - mu[j]) / expf(log_std[j]);
        lp = (float)((double)lp - ((double)log_std[j] + 0.5 * (double)(z * z)));
    }
    return lp;
}

__device__ __forceinline__ float surrogate(float adv, float lp, float old_lp, float eps, int m, float* grad) {
    const float ratio = (float)exp((double)(lp - old_lp));
    const int adv_pos = adv > 0;
    const int ratio_pos = ratio > 1 + eps;
    const int ratio_neg = ratio < 1 - eps;
    *grad = -(adv_pos * !ratio_pos + !adv_pos * !ratio_neg) * adv * ratio / m;
    return adv * (adv_pos * (ratio_pos * (1 + eps) + !ratio_pos * ratio) +
                  !adv_pos * (ratio_neg * (1 - eps) + !ratio_neg * ratio));
}

// adam.cu:53-74 / tiny.hip adam_elem
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float step, float b1, float b2,
                                          float bc2) {
    m = b1 * m + (1 - b1) * g;
    v = b2 * v + (1 - b2) * (g * g);
    const float denom = (float)((double)sqrtf(v / bc2) + 1e-8);
    p -= step * m / denom;
}

// stamp buffer layout (PPO_CLUSTER_STAMPS): [64 steps][≤ 32] s_memrealtime | [64] placement words |
// [64 steps][≤ 32] s_memtime (the shader clock beside the wall clock, at the same points)
constexpr int CLU_STAMP_CLK = 64 * 32 + 64;

// ---- host side, shared by both phase kernels (defined in cluster.hip) ----
// Barrier wait bound in realtime ticks: 2 s (PPO_CLUSTER_TEST_TIMEOUT=1, a test hook, makes it 0 so
// the first barrier that is not already complete times out and the error path runs).
unsigned long long host_timeout_ticks();
// Co-residency guard: the phase spins at grid barriers, so every workgroup of the launch — and of the
// other phase running beside it on the side stream — must be resident at once.  True when
// `2 × grid` blocks of `kfn` with `lds` bytes fit the device's CUs at its occupancy.
bool host_grid_fits(const void* kfn, size_t lds, int grid);
// Per-stream diagnostics (PPO_CLUSTER_STAMPS): the stamp buffer of the calling stream, and a pending
// report printed by phip_cluster_report() after the phases joined (no mid-phase synchronisation).
unsigned long long* host_stamps(int nstamp, const char* kind, const char* const* names, int policy, int total_steps,
                                int nwg);
// PPO_CLUSTER_STAMPS=2 (cluster_deep): every workgroup's arrival and exit time at each of the ≤ 6 barriers of
// steps 0 … 63 ([64][6][2][nwg], zeroed); phip_cluster_report prints the arrival skew, the exit latency
// after the last arrival and the workgroups that arrive last
unsigned long long* host_barrier_stamps(int nwg);

}  // namespace clu
