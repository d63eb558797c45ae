// gae.hip — GAE as an exact segmented reverse scan, Welford statistics, normalisation.
//
// Reference: compute_gae (ppo.cu:326-369) and its CUDA twin (K14-K17, ppo.cu:171-323,
// welford_var.h:13-69).  The reference GPU path bounds its look-ahead to horizon/512 blocks
// (D7) and its Welford kernel races on shared memory (D8); this one is exact and race-free.
//
// Recurrence (right to left):  A_t = δ_t + c_t·A_{t+1},  A_N = 0   (D6)
//   δ_t = r_t + γ·v′_t·!term_t − v_t,   c_t = γλ·!(term_t ∨ trunc_t)
// Each step is the affine map T_t(x) = δ_t + c_t·x; maps compose associatively:
//   T_a∘T_b = (c_a·c_b, δ_a + c_a·δ_b).  c_t = 0 at every episode end, so segments never mix.
//
// Three passes over HBM-resident inputs (≈18 B read per transition per pass):
//   1. gae_block_kernel   each workgroup composes its 2048 transitions → (C, D) aggregate
//   2. gae_carry_kernel   right-to-left over the aggregates → the A entering each workgroup
//   3. gae_apply_kernel   recompute with the true carry; write A and target = v + A; emit a
//                         per-workgroup Welford triple (n, mean, M2) in double
// then welford_combine (Chan et al. parallel combine, double) and normalise:
//   A ← (A − μ) / (σ_pop + 1e-8)                                        (ppo.cu:355-368)
#include "dev.h"

namespace {

constexpr int TPB = 256;
constexpr int EPT = 8;                    // transitions per thread
constexpr int CHUNK = TPB * EPT;          // transitions per workgroup

struct Affine { float c, d; };            // x ↦ d + c·x

__device__ __forceinline__ Affine compose(Affine a, Affine b) {   // a ∘ b  (b is applied first)
    return Affine{a.c * b.c, a.d + a.c * b.d};
}

__device__ __forceinline__ float delta_at(const float* v, const float* vn, const float* r, const uint8_t* term,
                                          float gamma, long t) {
    return r[t] + gamma * vn[t] * (float)(!term[t]) - v[t];
}

// Thread-local transform over its EPT transitions [t0, t0+EPT) ∩ [0, n)
__device__ __forceinline__ Affine thread_transform(const float* v, const float* vn, const float* r,
                                                   const uint8_t* term, const uint8_t* trunc, long t0, long n,
                                                   float gamma, float gl) {
    Affine T{1.f, 0.f};
#pragma unroll
    for (int e = EPT - 1; e >= 0; --e) {
        const long t = t0 + e;
        if (t < n) {
            const float c = gl * (float)(!(trunc[t] || term[t]));
            T = compose(Affine{c, delta_at(v, vn, r, term, gamma, t)}, T);
        }
    }
    return T;
}

// Exclusive right-to-left scan of per-thread transforms inside the workgroup.
// Returns the composition of all LATER threads of the block (identity for the last thread);
// *block_total receives the composition of the whole block.
__device__ __forceinline__ Affine block_suffix_exclusive(Affine T, Affine* wave_tot, Affine* block_total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // inclusive suffix within the wave: lane l ← T_l ∘ T_{l+1} ∘ … ∘ T_63
    Affine inc = T;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        Affine other{__shfl_down(inc.c, o, 64), __shfl_down(inc.d, o, 64)};
        if (lane + o < 64) inc = compose(inc, other);
    }
    Affine excl{__shfl_down(inc.c, 1, 64), __shfl_down(inc.d, 1, 64)};
    if (lane == 63) excl = Affine{1.f, 0.f};
    if (lane == 0) wave_tot[w] = inc;
    __syncthreads();
    // compositions of the waves after w
    Affine after{1.f, 0.f};
    for (int k = TPB / 64 - 1; k > w; --k) after = compose(wave_tot[k], after);
    Affine tot{1.f, 0.f};
    for (int k = TPB / 64 - 1; k >= 0; --k) tot = compose(wave_tot[k], tot);
    *block_total = tot;
    return compose(excl, after);
}

__global__ void gae_block_kernel(const float* __restrict__ v, const float* __restrict__ vn,
                                 const float* __restrict__ r, const uint8_t* __restrict__ term,
                                 const uint8_t* __restrict__ trunc, long n, float gamma, float gl,
                                 float2* __restrict__ agg) {
    __shared__ Affine wave_tot[TPB / 64];
    const long t0 = (long)blockIdx.x * CHUNK + (long)threadIdx.x * EPT;
    const Affine T = thread_transform(v, vn, r, term, trunc, t0, n, gamma, gl);
    Affine tot;
    block_suffix_exclusive(T, wave_tot, &tot);
    if (threadIdx.x == 0) agg[blockIdx.x] = make_float2(tot.c, tot.d);
}

// carry[b] = A entering block b from the right = T_{b+1}(carry[b+1]),  carry[last] = 0
__global__ void gae_carry_kernel(const float2* __restrict__ agg, float* __restrict__ carry, int nblocks) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    float x = 0.f;
    for (int b = nblocks - 1; b >= 0; --b) {
        carry[b] = x;
        x = agg[b].y + agg[b].x * x;
    }
}

__global__ void gae_apply_kernel(const float* __restrict__ v, const float* __restrict__ vn,
                                 const float* __restrict__ r, const uint8_t* __restrict__ term,
                                 const uint8_t* __restrict__ trunc, long n, float gamma, float gl,
                                 const float* __restrict__ carry, float* __restrict__ adv,
                                 float* __restrict__ adv_target, double* __restrict__ wpart) {
    __shared__ Affine wave_tot[TPB / 64];
    __shared__ double red[TPB / 64];
    const long t0 = (long)blockIdx.x * CHUNK + (long)threadIdx.x * EPT;
    const Affine T = thread_transform(v, vn, r, term, trunc, t0, n, gamma, gl);
    Affine tot;
    const Affine S = block_suffix_exclusive(T, wave_tot, &tot);
    float x = S.d + S.c * carry[blockIdx.x];          // A entering this thread's last transition
    float a[EPT];
    int cnt = 0;
    double sum = 0.0;
#pragma unroll
    for (int e = EPT - 1; e >= 0; --e) {
        const long t = t0 + e;
        a[e] = 0.f;
        if (t < n) {
            const float c = gl * (float)(!(trunc[t] || term[t]));
            x = delta_at(v, vn, r, term, gamma, t) + c * x;
            a[e] = x;
            adv[t] = x;
            adv_target[t] = v[t] + x;
            sum += x;
            cnt++;
        }
    }
    // per-workgroup Welford triple (n, mean, M2): two-pass over registers, double accumulation
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double s = sum;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    int c_tot = cnt;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c_tot += __shfl_xor(c_tot, o, 64);
    __syncthreads();
    if (lane == 0) { red[w] = s; wave_tot[w].c = (float)c_tot; }
    __syncthreads();
    double bs = 0.0; long bn = 0;
    for (int k = 0; k < TPB / 64; ++k) { bs += red[k]; bn += (long)wave_tot[k].c; }
    const double mean = bn > 0 ? bs / (double)bn : 0.0;
    double m2 = 0.0;
#pragma unroll
    for (int e = 0; e < EPT; ++e)
        if (t0 + e < n) { const double d = (double)a[e] - mean; m2 += d * d; }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m2 += __shfl_xor(m2, o, 64);
    __syncthreads();
    if (lane == 0) red[w] = m2;
    __syncthreads();
    if (threadIdx.x == 0) {
        double bm2 = 0.0;
        for (int k = 0; k < TPB / 64; ++k) bm2 += red[k];
        wpart[3 * blockIdx.x + 0] = (double)bn;
        wpart[3 * blockIdx.x + 1] = mean;
        wpart[3 * blockIdx.x + 2] = bm2;
    }
}

// Chan/Golub/LeVeque pairwise combine of `count` triples (n, mean, M2), one thread (count ≤ a few 1000)
// Chan et al. combine of two (n, mean, M2) triples; an empty side leaves the other as is
__device__ __forceinline__ void chan(double& n, double& mean, double& m2, double nb, double mb, double m2b) {
    if (nb <= 0.0) return;
    if (n <= 0.0) { n = nb; mean = mb; m2 = m2b; return; }
    const double nn = n + nb, d = mb - mean;
    mean += d * nb / nn;
    m2 += m2b + d * d * n * nb / nn;
    n = nn;
}

// one 256-thread workgroup: each thread combines a contiguous run of parts in order, then a
// pairwise tree over the threads (was one thread over every part: 116 µs for C4's 512 parts)
constexpr int WF_T = 256;
__global__ __launch_bounds__(WF_T) void welford_combine_kernel(const double* __restrict__ parts, int count,
                                                                double* __restrict__ out) {
    __shared__ double sn[WF_T], sm[WF_T], s2[WF_T];
    const int t = threadIdx.x;
    const int per = (count + WF_T - 1) / WF_T;
    double n = 0.0, mean = 0.0, m2 = 0.0;
    for (int i = t * per; i < min(count, (t + 1) * per); ++i) chan(n, mean, m2, parts[3 * i], parts[3 * i + 1], parts[3 * i + 2]);
    sn[t] = n; sm[t] = mean; s2[t] = m2;
    __syncthreads();
    for (int off = 1; off < WF_T; off <<= 1) {
        if ((t & (2 * off - 1)) == 0) {
            double a = sn[t], am = sm[t], a2 = s2[t];
            chan(a, am, a2, sn[t + off], sm[t + off], s2[t + off]);
            sn[t] = a; sm[t] = am; s2[t] = a2;
        }
        __syncthreads();
    }
    if (t == 0) { out[0] = sn[0]; out[1] = sm[0]; out[2] = s2[0]; }
}

__global__ void normalize_kernel(float* __restrict__ adv, long n, const double* __restrict__ wf,
                                 float* __restrict__ stats) {
    const float mean = (float)wf[1];
    const float std = (float)sqrt(wf[0] > 0.0 ? wf[2] / wf[0] : 0.0);
    if (stats && blockIdx.x == 0 && threadIdx.x == 0) { stats[0] = mean; stats[1] = std; }
    const double den = (double)std + 1e-8;
    for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < n; i += (long)gridDim.x * TPB)
        adv[i] = (float)((double)(adv[i] - mean) / den);
}

// workspace (grow-only, owned here): aggregates, carries, Welford partials
float2* g_agg = nullptr;
float*  g_carry = nullptr;
double* g_wpart = nullptr;
int     g_cap_blocks = 0;

void ensure_ws(int nb) {
    if (nb <= g_cap_blocks) return;
    if (g_agg) { phip_free(g_agg); phip_free(g_carry); phip_free(g_wpart); }
    g_cap_blocks = nb + 64;
    g_agg = (float2*)phip_malloc(sizeof(float2) * g_cap_blocks);
    g_carry = (float*)phip_malloc(sizeof(float) * g_cap_blocks);
    g_wpart = (double*)phip_malloc(sizeof(double) * 3 * g_cap_blocks);
}

// V(next_state) reuse.  In a rollout buffer next_state[t] is state[t+1] unless the episode ended at
// t (or t is the last row), so V(next_state[t]) = V(state[t+1]) — already computed by the state
// forward.  One wave per transition compares the two rows bit for bit; equal rows take v[t+1],
// the others are listed for their own forward (≈ N/500 + E rows at C4).  A buffer filled any other
// way is handled exactly: every row that differs is evaluated.
__global__ void next_value_map_kernel(const uint32_t* __restrict__ ns, const uint32_t* __restrict__ st,
                                      const float* __restrict__ v, float* __restrict__ vn, int* __restrict__ own,
                                      int* __restrict__ count, long n, int S) {
    const int lane = threadIdx.x & 63;
    const long waves = (long)gridDim.x * (TPB / 64);
    for (long t = blockIdx.x * (long)(TPB / 64) + (threadIdx.x >> 6); t < n; t += waves) {
        bool diff = t + 1 >= n;
        if (!diff) {
            const uint32_t* a = ns + t * S;
            const uint32_t* b = st + (t + 1) * S;
            for (int c = lane; c < S; c += 64) diff |= a[c] != b[c];
        }
        const bool any = __ballot(diff) != 0;
        if (lane == 0) {
            if (!any) vn[t] = v[t + 1];
            else own[atomicAdd(count, 1)] = (int)t;
        }
    }
}

__global__ void scatter_values_kernel(float* __restrict__ vn, const int* __restrict__ own,
                                      const float* __restrict__ vals, int m) {
    const int i = blockIdx.x * TPB + threadIdx.x;
    if (i < m) vn[own[i]] = vals[i];
}

int* g_count = nullptr;

}  // namespace

extern "C" {

void phip_gae_scan(const float* v, const float* v_next, const float* reward, const uint8_t* term,
                   const uint8_t* trunc, int n, float gamma, float lambda, float* adv, float* adv_target,
                   double* d_welford) {
    if (n <= 0) { phip_memset(d_welford, 0, 3 * sizeof(double)); return; }
    const int nb = ppo_divup(n, CHUNK);
    ensure_ws(nb);
    const float gl = gamma * lambda;
    hipStream_t s = ppo::stream();
    {
        ppo::ProfScope ps(PPO_K_GAE, 18.0 * n);
        hipLaunchKernelGGL(gae_block_kernel, dim3(nb), dim3(TPB), 0, s, v, v_next, reward, term, trunc, (long)n,
                           gamma, gl, g_agg);
        PPO_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(gae_carry_kernel, dim3(1), dim3(64), 0, s, g_agg, g_carry, nb);
    PPO_LAUNCH_CHECK();
    {
        ppo::ProfScope ps(PPO_K_GAE, 26.0 * n);
        hipLaunchKernelGGL(gae_apply_kernel, dim3(nb), dim3(TPB), 0, s, v, v_next, reward, term, trunc, (long)n,
                           gamma, gl, g_carry, adv, adv_target, g_wpart);
        PPO_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(welford_combine_kernel, dim3(1), dim3(WF_T), 0, s, g_wpart, nb, d_welford);
    PPO_LAUNCH_CHECK();
}

void phip_welford_combine(const double* d_welford_all, int world, double* d_welford) {
    hipLaunchKernelGGL(welford_combine_kernel, dim3(1), dim3(WF_T), 0, ppo::stream(), d_welford_all, world,
                       d_welford);
    PPO_LAUNCH_CHECK();
}

void ppo_welford_combine(const double* d_parts, int count, double* d_out) {
    phip_welford_combine(d_parts, count, d_out);
    phip_sync();
}

void phip_normalize(float* adv, int n, const double* d_welford, float* d_stats_out) {
    if (n <= 0) return;
    int g = ppo_divup(n, TPB * 4);
    if (g > 2048) g = 2048;
    ppo::ProfScope ps(PPO_K_GAE, 8.0 * n);
    hipLaunchKernelGGL(normalize_kernel, dim3(g), dim3(TPB), 0, ppo::stream(), adv, (long)n, d_welford,
                       d_stats_out);
    PPO_LAUNCH_CHECK();
}

int phip_next_value_map(const float* next_state, const float* state, const float* v, float* vn, int* own, int n,
                        int S) {
    if (n <= 0) return 0;
    if (!g_count) g_count = (int*)phip_malloc(sizeof(int));
    phip_memset(g_count, 0, sizeof(int));
    long g = ((long)n + TPB / 64 - 1) / (TPB / 64);
    if (g > 8192) g = 8192;
    {
        ppo::ProfScope ps(PPO_K_GAE, 8.0 * n * S);
        hipLaunchKernelGGL(next_value_map_kernel, dim3((int)g), dim3(TPB), 0, ppo::stream(),
                           reinterpret_cast<const uint32_t*>(next_state), reinterpret_cast<const uint32_t*>(state), v,
                           vn, own, g_count, (long)n, S);
        PPO_LAUNCH_CHECK();
    }
    int count = 0;
    phip_d2h(&count, g_count, sizeof(int));
    return count;
}

void phip_scatter_values(float* vn, const int* own, const float* vals, int m) {
    if (m <= 0) return;
    hipLaunchKernelGGL(scatter_values_kernel, dim3(ppo_divup(m, TPB)), dim3(TPB), 0, ppo::stream(), vn, own, vals, m);
    PPO_LAUNCH_CHECK();
}

}  // extern "C"
