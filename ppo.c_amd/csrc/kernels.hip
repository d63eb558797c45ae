// kernels.hip — element-wise and head kernels of the PPO update (gfx950).
//
//   ReLU / ReLU′                  activation_function.cu:17-43   (K5, K6 when not fused)
//   MSE loss + derivative         loss.cu:25-83                  (K8 + K9 fused, no host sync)
//   Gaussian log-prob / backward  policy.cu:67-74,101-169        (K11, K12; correct for any A)
//   entropy                       policy.cu:171-193
//   clipped surrogate             ppo.cu:82-169                  (K13; entropy counted once, D5)
//   fused policy head             K11 + K13 + K12 + ppo.cu:436-438 in ONE pass over the minibatch
//
// Arithmetic mirrors the reference's C promotions (its double exp/pow temporaries) so results
// match the oracle to a few ulps; reductions use wave shuffles + one f32 atomic per workgroup.
#include "dev.h"

#include <algorithm>

#include <cmath>

namespace {

constexpr int TPB = 256;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// block-wide sum: every thread gets the result
__device__ __forceinline__ float block_sum(float v, float* red) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    float s = 0.f;
    for (int i = 0; i < nw; ++i) s += red[i];
    return s;
}

inline int grid_for(long n, int per_thread = 1) {
    long g = (n + (long)TPB * per_thread - 1) / ((long)TPB * per_thread);
    if (g < 1) g = 1;
    if (g > 4096) g = 4096;
    return (int)g;
}

__global__ void relu_kernel(float* __restrict__ x, long n) {
    for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < n; i += (long)gridDim.x * TPB) {
        const float v = x[i];
        x[i] = v > 0.f ? v : 0.f;
    }
}

__global__ void relu_bwd_kernel(const float* __restrict__ y, float* __restrict__ g, long n) {
    for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < n; i += (long)gridDim.x * TPB)
        if (!(y[i] > 0.f)) g[i] = 0.f;
}

// fp32 → bf16 (round to nearest even, NaN preserved: the plain cast lowers to v_cvt_pk_bf16_f32)
__global__ void f32_to_bf16_kernel(__bf16* __restrict__ dst, const float* __restrict__ src, long n) {
    for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < n; i += (long)gridDim.x * TPB) dst[i] = (__bf16)src[i];
}

// dst[i, :] = bf16(src[rows[i], :]) — layer 0's minibatch gather in bf16 mode, done once before the
// GEMM so the forward's column tiles all read a compact bf16 copy (the fused fp32 gather re-read
// each 4-byte row once per column tile: 175 µs vs 52 µs at C5).  Four columns per thread.
__global__ void rows_to_bf16_kernel(__bf16* __restrict__ dst, const float* __restrict__ src,
                                    const int* __restrict__ rows, int m, int S) {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    const int q = S >> 2;
    const long n = (long)m * q;
    for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < n; i += (long)gridDim.x * TPB) {
        const int r = (int)(i / q), c = (int)(i - (long)r * q);
        const float4 v = reinterpret_cast<const float4*>(src + (long)rows[r] * S)[c];
        bf16x4 o = {(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
        *reinterpret_cast<bf16x4*>(dst + (long)r * S + 4 * c) = o;
    }
}

__global__ void axpy_kernel(float* __restrict__ y, const float* __restrict__ x, long n) {
    for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < n; i += (long)gridDim.x * TPB) y[i] += x[i];
}

// loss.cu:5-23 semantics: L = Σ(t−y)²/count, grad = 2(y−t)/count
__global__ void mse_kernel(const float* __restrict__ y, const float* __restrict__ t, long n,
                           float* __restrict__ grad, float* d_loss, float* d_loss_accum) {
    __shared__ float red[TPB / 64];
    float s = 0.f;
    const float inv = 1.0f / (float)n;
    for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < n; i += (long)gridDim.x * TPB) {
        const float d = t[i] - y[i];
        s += d * d;
        if (grad) grad[i] = 2 * (y[i] - t[i]) / (float)n;
    }
    s = block_sum(s, red);
    if (threadIdx.x == 0) {
        if (d_loss) atomicAdd(d_loss, s * inv);
        if (d_loss_accum) atomicAdd(d_loss_accum, s * inv);
    }
}

// The folded value head (loss.cu:5-23 on y = h·w + b, nn_value_fold_step): y from the last hidden
// layer's per-wave partial dots (gemm_x3 forward epilogue, `slots` partials summed in slot order),
// the MSE loss (Σ(t − y)² / m, as mse_kernel) and its gradient g = 2(y − t)/m, the output bias gradient
// Σ g; the output layer's weight gradient and the hidden layer's ∂L/∂z follow in the x3 backward
// kernels, which take g and w as row / column scales of the 0/1 mask of h.  Since round 5 the hidden
// layer's grad_W launch carries this head (gemm_x3.hip X3Args vh_*, the same arithmetic per row); this
// kernel runs only when that launch has no LDS room for its split's g.
__global__ void value_head_kernel(const float* __restrict__ ypart, int slots, const float* __restrict__ b,
                                  const float* __restrict__ t, int m, float* __restrict__ y, float* __restrict__ g,
                                  float* gb, float* d_loss_accum) {
    __shared__ float red[TPB / 64];
    const float bias = b[0];
    float s = 0.f, sg = 0.f;
    for (int i = blockIdx.x * TPB + threadIdx.x; i < m; i += gridDim.x * TPB) {
        float yv = 0.f;
        for (int q = 0; q < slots; ++q) yv += ypart[(long)q * m + i];
        yv += bias;
        const float tv = t[i];
        const float d = tv - yv;
        s += d * d;
        const float gv = 2 * (yv - tv) / (float)m;
        y[i] = yv;
        g[i] = gv;
        sg += gv;
    }
    s = block_sum(s, red);
    sg = block_sum(sg, red);
    if (threadIdx.x == 0) {
        atomicAdd(gb, sg);
        if (d_loss_accum) atomicAdd(d_loss_accum, s * (1.0f / (float)m));
    }
}

// policy.cu:67-74 with the reference's double temporaries
__device__ __forceinline__ float log_prob_row(const float* mu, const float* log_std, const float* a, int A) {
    const float c = (float)(-0.5 * A * (double)logf((float)(2 * M_PI)));
    float lp = c;
    for (int j = 0; j < A; ++j) {
        const float z = (a[j] - mu[j]) / expf(log_std[j]);
        lp = (float)((double)lp - ((double)log_std[j] + 0.5 * (double)(z * z)));
    }
    return lp;
}

__global__ void log_prob_kernel(const float* __restrict__ mu, const float* __restrict__ log_std,
                                const float* __restrict__ action, float* __restrict__ out, int m, int A) {
    const int i = blockIdx.x * TPB + threadIdx.x;
    if (i < m) out[i] = log_prob_row(mu + (long)i * A, log_std, action + (long)i * A, A);
}

// policy.cu:101-111 (D2: grad_in per sample).  grad_log_std pre-zeroed; one atomic per (block, j).
__global__ void log_prob_bwd_kernel(const float* __restrict__ mu, const float* __restrict__ log_std,
                                    const float* __restrict__ action, const float* __restrict__ grad_in,
                                    float* __restrict__ grad_mu, float* grad_log_std, int m, int A) {
    extern __shared__ float sacc[];   // [A]
    for (int j = threadIdx.x; j < A; j += TPB) sacc[j] = 0.f;
    __syncthreads();
    const int i = blockIdx.x * TPB + threadIdx.x;
    const float g = i < m ? grad_in[i] : 0.f;
    for (int j = 0; j < A; ++j) {          // column sums: wave shuffle, then one LDS add per wave
        float c = 0.f;
        if (i < m) {
            const long k = (long)i * A + j;
            const float d = action[k] - mu[k];
            const float e = expf(-2 * log_std[j]);
            grad_mu[k] = d * e * g;
            c = (-1 + d * d * e) * g;
        }
        c = wave_sum(c);
        if ((threadIdx.x & 63) == 0) atomicAdd(&sacc[j], c);
    }
    __syncthreads();
    for (int j = threadIdx.x; j < A; j += TPB) atomicAdd(grad_log_std + j, sacc[j]);
}

__global__ void entropy_kernel(const float* __restrict__ log_std, int A, float* out) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        float e = (float)(A * 0.5 * (1 + log(2 * M_PI)));
        for (int j = 0; j < A; ++j) e += log_std[j];
        out[0] = e;
    }
}

// ppo.cu:82-107, per sample
__device__ __forceinline__ float surrogate(float adv, float lp, float old_lp, float eps, int m, float* grad) {
    const float ratio = (float)exp((double)(lp - old_lp));
    const int adv_pos = adv > 0;
    const int ratio_pos = ratio > 1 + eps;
    const int ratio_neg = ratio < 1 - eps;
    *grad = -(adv_pos * !ratio_pos + !adv_pos * !ratio_neg) * adv * ratio / m;
    return adv * (adv_pos * (ratio_pos * (1 + eps) + !ratio_pos * ratio) +
                  !adv_pos * (ratio_neg * (1 - eps) + !ratio_neg * ratio));
}

__global__ void policy_loss_kernel(const float* __restrict__ adv, const float* __restrict__ lp,
                                   const float* __restrict__ old_lp, float* __restrict__ grad_lp, int m,
                                   float eps, float ent_coeff, const float* d_entropy, float* d_loss,
                                   float* d_loss_accum) {
    __shared__ float red[TPB / 64];
    float s = 0.f;
    for (int i = blockIdx.x * TPB + threadIdx.x; i < m; i += gridDim.x * TPB) {
        float g;
        s += surrogate(adv[i], lp[i], old_lp[i], eps, m, &g);
        grad_lp[i] = g;
    }
    s = block_sum(s, red);
    if (threadIdx.x == 0) {
        float contrib = -s / m;
        if (blockIdx.x == 0) contrib -= ent_coeff * d_entropy[0];     // once (D5)
        if (d_loss) atomicAdd(d_loss, contrib);
        if (d_loss_accum) atomicAdd(d_loss_accum, contrib);
    }
}

// Fused policy head: per row i  lp_i → ratio/clip → grad_lp_i → grad_mu[i,:], and the per-column
// grad_log_std sums, in one pass over μ and the action rows.  grad_log_std must be pre-zeroed.
__global__ void policy_head_kernel(const float* __restrict__ mu, const float* __restrict__ log_std,
                                   const float* __restrict__ action, const float* __restrict__ adv,
                                   const float* __restrict__ old_lp, int m, int A, float eps, float ent_coeff,
                                   float* __restrict__ grad_mu, float* grad_log_std, float* d_loss_accum) {
    extern __shared__ float smem[];          // [A] inv-var, [A] grad_log_std partials, [4] reduction
    float* e2 = smem;
    float* gls = smem + A;
    float* red = smem + 2 * A;
    for (int j = threadIdx.x; j < A; j += TPB) {
        e2[j] = expf(-2 * log_std[j]);
        gls[j] = 0.f;
    }
    __syncthreads();
    float s = 0.f, g = 0.f;
    const int i = blockIdx.x * TPB + threadIdx.x;
    const float* mr = mu + (long)i * A;
    const float* ar = action + (long)i * A;
    if (i < m) {
        const float lp = log_prob_row(mr, log_std, ar, A);
        s = surrogate(adv[i], lp, old_lp[i], eps, m, &g);
    }
    for (int j = 0; j < A; ++j) {          // column sums: wave shuffle, then one LDS add per wave
        float c = 0.f;
        if (i < m) {
            const float d = ar[j] - mr[j];
            grad_mu[(long)i * A + j] = d * e2[j] * g;
            c = (-1 + d * d * e2[j]) * g;
        }
        c = wave_sum(c);
        if ((threadIdx.x & 63) == 0) atomicAdd(&gls[j], c);
    }
    s = block_sum(s, red);
    __syncthreads();
    for (int j = threadIdx.x; j < A; j += TPB) {
        float v = gls[j];
        if (blockIdx.x == 0) v += -ent_coeff;                     // ppo.cu:436-438 (D4)
        atomicAdd(grad_log_std + j, v);
    }
    if (threadIdx.x == 0 && d_loss_accum) {
        float contrib = -s / m;
        if (blockIdx.x == 0) {
            float ent = (float)(A * 0.5 * (1 + log(2 * M_PI)));
            for (int j = 0; j < A; ++j) ent += log_std[j];
            contrib -= ent_coeff * ent;
        }
        atomicAdd(d_loss_accum, contrib);
    }
}

// The same head for A ≤ 32 over ROWS-row tiles: μ and action rows staged through LDS by coalesced
// loads (the one-thread-per-row form reads them at a 4·A-byte lane stride), the per-row log-prob /
// surrogate chain unchanged (log_prob_row, surrogate: identical values), grad_μ stored coalesced,
// the log σ column sums from the staged tile (8 partial sums per column, then one f32 atomic per
// column per workgroup).  Grid: ⌈m / ROWS⌉ (512 workgroups at C4's B = 32768, every CU busy).
template <int ROWS>
__global__ __launch_bounds__(TPB) void policy_head_tiled_kernel(
    const float* __restrict__ mu, const float* __restrict__ log_std, const float* __restrict__ action,
    const float* __restrict__ adv, const float* __restrict__ old_lp, int m, int A, float eps, float ent_coeff,
    float* __restrict__ grad_mu, float* grad_log_std, float* d_loss_accum) {
    extern __shared__ float smem[];
    float* e2 = smem;                    // [32] exp(−2 log σ)
    float* lsd = smem + 32;              // [32] log σ
    float* mt = smem + 64;               // [ROWS][A] μ
    float* at = mt + ROWS * A;           // [ROWS][A] actions
    float* gr = at + ROWS * A;           // [ROWS] ∂L/∂lp
    float* cp = gr + ROWS;               // [8][32] column partial sums
    float* red = cp + 8 * 32;            // [TPB/64]
    const int tid = threadIdx.x;
    const int r0 = blockIdx.x * ROWS;
    const int nr = min(ROWS, m - r0);
    if (tid < A) {
        e2[tid] = expf(-2 * log_std[tid]);
        lsd[tid] = log_std[tid];
    }
    const long base = (long)r0 * A;
    for (int e = tid; e < nr * A; e += TPB) {
        mt[e] = mu[base + e];
        at[e] = action[base + e];
    }
    __syncthreads();
    float s = 0.f;
    if (tid < nr) {
        float g;
        const float lp = log_prob_row(mt + tid * A, lsd, at + tid * A, A);
        s = surrogate(adv[r0 + tid], lp, old_lp[r0 + tid], eps, m, &g);
        gr[tid] = g;
    }
    __syncthreads();
    for (int e = tid; e < nr * A; e += TPB) {
        const int row = e / A, j = e - row * A;
        const float d = at[e] - mt[e];
        grad_mu[base + e] = d * e2[j] * gr[row];
    }
    if (tid < 8 * A) {
        const int j = tid % A, q = tid / A;
        float c = 0.f;
        for (int row = q; row < nr; row += 8) {
            const float d = at[row * A + j] - mt[row * A + j];
            c += (-1 + d * d * e2[j]) * gr[row];
        }
        cp[q * 32 + j] = c;
    }
    s = block_sum(s, red);
    if (tid < A) {
        float v = 0.f;
        for (int q = 0; q < 8; ++q) v += cp[q * 32 + tid];
        if (blockIdx.x == 0) v += -ent_coeff;                     // ppo.cu:436-438 (D4)
        atomicAdd(grad_log_std + tid, v);
    }
    if (tid == 0 && d_loss_accum) {
        float contrib = -s / m;
        if (blockIdx.x == 0) {
            float ent = (float)(A * 0.5 * (1 + log(2 * M_PI)));
            for (int j = 0; j < A; ++j) ent += log_std[j];
            contrib -= ent_coeff * ent;
        }
        atomicAdd(d_loss_accum, contrib);
    }
}

}  // namespace

extern "C" {

void phip_relu(float* x, long count) {
    if (count <= 0) return;
    ppo::ProfScope ps(PPO_K_OTHER, 8.0 * count);
    hipLaunchKernelGGL(relu_kernel, dim3(grid_for(count, 4)), dim3(TPB), 0, ppo::stream(), x, count);
    PPO_LAUNCH_CHECK();
}

void phip_relu_bwd(const float* y, float* g, long count) {
    if (count <= 0) return;
    ppo::ProfScope ps(PPO_K_OTHER, 12.0 * count);
    hipLaunchKernelGGL(relu_bwd_kernel, dim3(grid_for(count, 4)), dim3(TPB), 0, ppo::stream(), y, g, count);
    PPO_LAUNCH_CHECK();
}

void phip_f32_to_bf16(unsigned short* dst, const float* src, long count) {
    if (count <= 0) return;
    ppo::ProfScope ps(PPO_K_OTHER, 6.0 * count);
    hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(grid_for(count, 4)), dim3(TPB), 0, ppo::stream(),
                       reinterpret_cast<__bf16*>(dst), src, count);
    PPO_LAUNCH_CHECK();
}

void phip_gather_rows_bf16(unsigned short* dst, const float* src, const int* rows, int m, int S) {
    if (m <= 0) return;
    PPO_REQUIRE(S % 4 == 0, "phip_gather_rows_bf16: row width must be a multiple of 4");
    ppo::ProfScope ps(PPO_K_GATHER, 6.0 * m * S);
    hipLaunchKernelGGL(rows_to_bf16_kernel, dim3(grid_for((long)m * S / 4, 1)), dim3(TPB), 0, ppo::stream(),
                       reinterpret_cast<__bf16*>(dst), src, rows, m, S);
    PPO_LAUNCH_CHECK();
}

void phip_axpy(float* y, const float* x, long count) {
    if (count <= 0) return;
    hipLaunchKernelGGL(axpy_kernel, dim3(grid_for(count, 4)), dim3(TPB), 0, ppo::stream(), y, x, count);
    PPO_LAUNCH_CHECK();
}

void phip_value_head(const float* ypart, int slots, const float* b, const float* tgt, int m, float* y, float* g,
                     float* gb, float* d_loss_accum) {
    if (m <= 0) return;
    ppo::ProfScope ps(PPO_K_HEAD, 4.0 * m * (slots + 3));
    const int hb = std::min(ppo_divup(m, TPB), 256);
    hipLaunchKernelGGL(value_head_kernel, dim3(hb), dim3(TPB), 0, ppo::stream(), ypart, slots, b, tgt, m, y, g, gb,
                       d_loss_accum);
    PPO_LAUNCH_CHECK();
}

void phip_mse(const float* y, const float* t, long count, float* grad, float* d_loss, float* d_loss_accum) {
    if (count <= 0) return;
    if (d_loss) phip_memset(d_loss, 0, sizeof(float));
    ppo::ProfScope ps(PPO_K_HEAD, 12.0 * count);
    hipLaunchKernelGGL(mse_kernel, dim3(grid_for(count, 8)), dim3(TPB), 0, ppo::stream(), y, t, count, grad,
                       d_loss, d_loss_accum);
    PPO_LAUNCH_CHECK();
}

void phip_log_prob(const float* mu, const float* log_std, const float* action, float* out, int m, int A) {
    if (m <= 0) return;
    ppo::ProfScope ps(PPO_K_HEAD, 4.0 * m * (2 * A + 1));
    hipLaunchKernelGGL(log_prob_kernel, dim3(ppo_divup(m, TPB)), dim3(TPB), 0, ppo::stream(), mu, log_std, action,
                       out, m, A);
    PPO_LAUNCH_CHECK();
}

void phip_log_prob_bwd(const float* mu, const float* log_std, const float* action, const float* grad_in,
                       float* grad_mu, float* grad_log_std, int m, int A) {
    phip_memset(grad_log_std, 0, sizeof(float) * (size_t)A);
    if (m <= 0) return;
    ppo::ProfScope ps(PPO_K_HEAD, 4.0 * m * (3 * A + 1));
    hipLaunchKernelGGL(log_prob_bwd_kernel, dim3(ppo_divup(m, TPB)), dim3(TPB), sizeof(float) * A, ppo::stream(),
                       mu, log_std, action, grad_in, grad_mu, grad_log_std, m, A);
    PPO_LAUNCH_CHECK();
}

void phip_entropy(const float* log_std, int A, float* d_out) {
    hipLaunchKernelGGL(entropy_kernel, dim3(1), dim3(64), 0, ppo::stream(), log_std, A, d_out);
    PPO_LAUNCH_CHECK();
}

void phip_policy_loss(const float* adv, const float* lp, const float* old_lp, float* grad_lp, int m, float epsilon,
                      float ent_coeff, const float* d_entropy, float* d_loss, float* d_loss_accum) {
    if (d_loss) phip_memset(d_loss, 0, sizeof(float));
    if (m <= 0) return;
    ppo::ProfScope ps(PPO_K_HEAD, 16.0 * m);
    hipLaunchKernelGGL(policy_loss_kernel, dim3(grid_for(m, 4)), dim3(TPB), 0, ppo::stream(), adv, lp, old_lp,
                       grad_lp, m, epsilon, ent_coeff, d_entropy, d_loss, d_loss_accum);
    PPO_LAUNCH_CHECK();
}

void phip_policy_head(const float* mu, const float* log_std, const float* action, const float* adv,
                      const float* old_lp, int m, int A, float epsilon, float ent_coeff, float* grad_mu,
                      float* grad_log_std, float* d_loss_accum, int ls_zeroed) {
    if (!ls_zeroed) phip_memset(grad_log_std, 0, sizeof(float) * (size_t)A);
    if (m <= 0) return;
    PPO_REQUIRE(A > 0 && A <= 4096, "phip_policy_head: action size out of range");
    ppo::ProfScope ps(PPO_K_HEAD, 4.0 * m * (3 * A + 2));
    if (A <= 32) {
        constexpr int ROWS = 64;
        const size_t lds = sizeof(float) * (64 + 2 * ROWS * A + ROWS + 8 * 32 + TPB / 64);
        hipLaunchKernelGGL(policy_head_tiled_kernel<ROWS>, dim3(ppo_divup(m, ROWS)), dim3(TPB), lds, ppo::stream(),
                           mu, log_std, action, adv, old_lp, m, A, epsilon, ent_coeff, grad_mu, grad_log_std,
                           d_loss_accum);
    } else {
        hipLaunchKernelGGL(policy_head_kernel, dim3(ppo_divup(m, TPB)), dim3(TPB), sizeof(float) * (2 * A + 4),
                           ppo::stream(), mu, log_std, action, adv, old_lp, m, A, epsilon, ent_coeff, grad_mu,
                           grad_log_std, d_loss_accum);
    }
    PPO_LAUNCH_CHECK();
}

}  // extern "C"
