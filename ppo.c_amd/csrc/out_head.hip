// out_head.hip — the output layer of a minibatch step in one pass over its input rows (gfx950).
//
// Replaces, inside ppo_update, four launches per minibatch step:
//   output-layer forward    y = x·Wᵀ + b               mat_mul.cu:122-163 (K1+K2)
//   loss head               value: MSE + derivative     loss.cu:25-83 (K8+K9)
//                           policy: log-prob, ratio/clip, grad_μ, grad_logσ   ppo.cu:82-169, policy.cu:67-169
//   output-layer backward   gx = (g·W) ⊙ 1[x > 0], gW = gᵀ·x, gb = Σ g        mat_mul.cu:165-217,
//                                                                            neural_network.cu:108-118
// The last hidden activation x [m, n] is read once and grad_x written once (the separate kernels
// read x twice and round-trip y and g through HBM): ≈ 2·m·n·4 B per step.
//
// One wave owns one row at a time; lane l holds x[row, l·NPL … l·NPL+NPL) (NPL = n/64).  W sits in
// LDS.  y_j is a wave sum of the lanes' partial dots; the head runs on the full y row (every lane
// computes it, identical to the standalone head kernels' arithmetic given y); g·W and gᵀ·x use the
// lane's NPL columns.  grad_W / grad_b: per-lane accumulators, summed over the workgroup's waves
// in LDS in wave order and written as one partial per workgroup; out_reduce_kernel adds the
// partials in workgroup order — deterministic, no float atomics on parameter gradients.
#include "dev.h"

#include <algorithm>
#include <cmath>

namespace {

constexpr int NTH = 256;             // 4 waves per workgroup

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// policy.cu:67-74 with the reference's double temporaries (as kernels.hip log_prob_row)
template <int A>
__device__ __forceinline__ float log_prob_row_r(const float (&mu)[A], const float* log_std, const float* a) {
    const float c = (float)(-0.5 * A * (double)logf((float)(2 * M_PI)));
    float lp = c;
#pragma unroll
    for (int j = 0; j < A; ++j) {
        const float z = (a[j] - mu[j]) / expf(log_std[j]);
        lp = (float)((double)lp - ((double)log_std[j] + 0.5 * (double)(z * z)));
    }
    return lp;
}

// ppo.cu:82-107, per sample (as kernels.hip surrogate)
__device__ __forceinline__ float surrogate_r(float adv, float lp, float old_lp, float eps, int m, float* grad) {
    const float ratio = (float)exp((double)(lp - old_lp));
    const int adv_pos = adv > 0;
    const int ratio_pos = ratio > 1 + eps;
    const int ratio_neg = ratio < 1 - eps;
    *grad = -(adv_pos * !ratio_pos + !adv_pos * !ratio_neg) * adv * ratio / m;
    return adv * (adv_pos * (ratio_pos * (1 + eps) + !ratio_pos * ratio) +
                  !adv_pos * (ratio_neg * (1 - eps) + !ratio_neg * ratio));
}

struct OutArgs {
    const float* x; const float* W; const float* b; const unsigned* bits;   // bits: ReLU′ of x or null
    int m, n, wpr;
    const float* tgt;                                                       // HEAD 0 (value)
    const float* log_std; const float* action; const float* adv; const float* old_lp;   // HEAD 1
    float eps, ent_coeff;
    float* y; float* gx; float* part; float* grad_log_std; float* loss_accum;
};

template <int NPL, int A, int HEAD>
__global__ __launch_bounds__(NTH) void out_fused_kernel(OutArgs p) {
    extern __shared__ float sm[];                 // W [A·n] | wave-ordered gW/gb sum [A·n + A]
    const int n = p.n, AN = A * n;
    float* Ws = sm;
    float* red = sm + AN;
    for (int i = threadIdx.x * 4; i < AN; i += NTH * 4)
        *reinterpret_cast<float4*>(Ws + i) = *reinterpret_cast<const float4*>(p.W + i);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = NTH / 64;
    const int c0 = lane * NPL;
    float e2[A];
    if (HEAD == 1) {
#pragma unroll
        for (int j = 0; j < A; ++j) e2[j] = expf(-2 * p.log_std[j]);
    }
    __syncthreads();

    float acc[A][NPL], accb[A], gls[A];
#pragma unroll
    for (int j = 0; j < A; ++j) {
        accb[j] = 0.f;
        gls[j] = 0.f;
#pragma unroll
        for (int e = 0; e < NPL; ++e) acc[j][e] = 0.f;
    }
    float lsum = 0.f;
    const float inv_m = 1.0f / (float)p.m;

    for (int row = blockIdx.x * nw + wv; row < p.m; row += gridDim.x * nw) {
        float xv[NPL];
        const float* xr = p.x + (long)row * n + c0;
#pragma unroll
        for (int e = 0; e < NPL; e += 4) {
            const float4 v = *reinterpret_cast<const float4*>(xr + e);
            xv[e] = v.x; xv[e + 1] = v.y; xv[e + 2] = v.z; xv[e + 3] = v.w;
        }
        float y[A];
#pragma unroll
        for (int j = 0; j < A; ++j) {
            float s = 0.f;
#pragma unroll
            for (int e = 0; e < NPL; ++e) s = fmaf(xv[e], Ws[j * n + c0 + e], s);
            y[j] = wsum(s) + p.b[j];
        }
#pragma unroll
        for (int j = 0; j < A; ++j)
            if (lane == j) p.y[(long)row * A + j] = y[j];

        float g[A];
        if (HEAD == 0) {
            // loss.cu:25-83 as mse_kernel: loss term (t − y)², derivative 2(y − t)/m (one output)
            const float t = p.tgt[row];
            const float d = t - y[0];
            lsum += d * d;
            g[0] = 2 * (y[0] - t) / (float)p.m;
        } else {
            float a[A];
#pragma unroll
            for (int j = 0; j < A; ++j) a[j] = p.action[(long)row * A + j];
            const float lp = log_prob_row_r<A>(y, p.log_std, a);
            float glp;
            lsum += surrogate_r(p.adv[row], lp, p.old_lp[row], p.eps, p.m, &glp);
#pragma unroll
            for (int j = 0; j < A; ++j) {
                const float d = a[j] - y[j];
                g[j] = d * e2[j] * glp;
                gls[j] += (-1 + d * d * e2[j]) * glp;
            }
        }

        // grad_x = (g·W) ⊙ ReLU′(x); grad_W += gᵀ·x; grad_b += g
        unsigned word = ~0u;
        if (p.bits) word = p.bits[(long)row * p.wpr + (c0 >> 5)] >> (c0 & 31);
        float gxv[NPL];
#pragma unroll
        for (int e = 0; e < NPL; ++e) {
            float s = 0.f;
#pragma unroll
            for (int j = 0; j < A; ++j) s = fmaf(g[j], Ws[j * n + c0 + e], s);
            gxv[e] = ((word >> e) & 1u) ? s : 0.f;
        }
        float* gr = p.gx + (long)row * n + c0;
#pragma unroll
        for (int e = 0; e < NPL; e += 4)
            *reinterpret_cast<float4*>(gr + e) = make_float4(gxv[e], gxv[e + 1], gxv[e + 2], gxv[e + 3]);
#pragma unroll
        for (int j = 0; j < A; ++j) {
            accb[j] += g[j];
#pragma unroll
            for (int e = 0; e < NPL; ++e) acc[j][e] = fmaf(g[j], xv[e], acc[j][e]);
        }
    }

    // loss and grad_logσ: one atomic per wave (statistics / the policy's logσ gradient, as the
    // standalone head kernels)
    if (lane == 0) {
        if (HEAD == 0) {
            if (p.loss_accum) atomicAdd(p.loss_accum, lsum * inv_m);
        } else {
            float contrib = -lsum / p.m;
            if (blockIdx.x == 0 && wv == 0) {
                float ent = (float)(A * 0.5 * (1 + log(2 * M_PI)));
                for (int j = 0; j < A; ++j) ent += p.log_std[j];
                contrib -= p.ent_coeff * ent;
            }
            if (p.loss_accum) atomicAdd(p.loss_accum, contrib);
#pragma unroll
            for (int j = 0; j < A; ++j) {
                float v = gls[j];
                if (blockIdx.x == 0 && wv == 0) v += -p.ent_coeff;           // ppo.cu:436-438 (D4)
                atomicAdd(p.grad_log_std + j, v);
            }
        }
    }

    // workgroup partial of grad_W / grad_b, summed over waves in wave order
    for (int w = 0; w < nw; ++w) {
        if (wv == w) {
#pragma unroll
            for (int j = 0; j < A; ++j) {
#pragma unroll
                for (int e = 0; e < NPL; ++e) {
                    float* d = red + j * n + c0 + e;
                    *d = w == 0 ? acc[j][e] : *d + acc[j][e];
                }
                if (lane == 0) red[AN + j] = w == 0 ? accb[j] : red[AN + j] + accb[j];
            }
        }
        __syncthreads();
    }
    float* dst = p.part + (long)blockIdx.x * (AN + A);
    for (int i = threadIdx.x; i < AN + A; i += NTH) dst[i] = red[i];
}

// gW[k] (k < A·n) and gb[j]: Σ over workgroups of the partials in a fixed order (deterministic).
// 64 columns per workgroup; wave q sums partials q, q+4, …, and the four wave sums add in wave order.
__global__ __launch_bounds__(256) void out_reduce_kernel(const float* __restrict__ part, int nwg, int AN, int A,
                                                         float* __restrict__ gW, float* __restrict__ gb) {
    __shared__ float red[4][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int k = blockIdx.x * 64 + lane, K = AN + A;
    float s = 0.f;
    if (k < K)
        for (int w = wv; w < nwg; w += 4) s += part[(long)w * K + k];
    red[wv][lane] = s;
    __syncthreads();
    if (wv == 0 && k < K) {
        const float t = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
        if (k < AN) gW[k] = t;
        else gb[k - AN] = t;
    }
}

template <int NPL, int A, int HEAD>
void launch_h(const OutArgs& p, int grid, size_t lds) {
    auto kern = out_fused_kernel<NPL, A, HEAD>;
    static size_t attr = 0;                          // dynamic LDS above 64 KiB: once per instantiation
    if (lds > 64 * 1024 && attr < lds) {
        PPO_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        attr = lds;
    }
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NTH), lds, ppo::stream(), p);
}

template <int NPL, int A>
bool launch_a(const OutArgs& p, int head, int grid, size_t lds) {
    if (head == 0) launch_h<NPL, A, 0>(p, grid, lds);
    else launch_h<NPL, A, 1>(p, grid, lds);
    return true;
}

template <int NPL>
bool launch_n(const OutArgs& p, int A, int head, int grid, size_t lds) {
    switch (A) {
        case 1: return launch_a<NPL, 1>(p, head, grid, lds);
        case 6: return launch_a<NPL, 6>(p, head, grid, lds);
        case 17: return launch_a<NPL, 17>(p, head, grid, lds);
        default: return false;
    }
}

constexpr int kGrid = 512;           // workgroups (2 per CU); 16 rows per wave at B = 32768

float* g_part = nullptr;             // [kGrid][A·n + A] partials (grow-only, per stream slot)
size_t g_part_cap = 0;
float* g_part_side = nullptr;
size_t g_part_side_cap = 0;

}  // namespace

extern "C" {

int phip_out_fused_supported(int n, int A) {
    if (A != 1 && A != 6 && A != 17) return 0;
    if (n != 256 && n != 512) return 0;              // A·n/64 grad_W accumulators per lane ≤ 136
    const size_t lds = sizeof(float) * (2 * (size_t)A * n + A);
    return lds <= 160 * 1024;
}

// head 0: value (A = 1, targets tgt); head 1: policy (clipped surrogate over the Gaussian log-prob).
// gW / gb are overwritten; grad_log_std (head 1) is accumulated and must be pre-zeroed.
void phip_out_fused(int head, const float* x, const unsigned* bits, const float* W, const float* b, int m, int n,
                    int A, const float* tgt, const float* log_std, const float* action, const float* adv,
                    const float* old_lp, float eps, float ent_coeff, float* y, float* gx, float* gW, float* gb,
                    float* grad_log_std, float* loss_accum) {
    PPO_REQUIRE(phip_out_fused_supported(n, A), "phip_out_fused: unsupported shape");
    PPO_REQUIRE(head == 0 ? (A == 1 && tgt) : (log_std && action && adv && old_lp && grad_log_std),
                "phip_out_fused: missing head inputs");
    PPO_REQUIRE(((uintptr_t)x & 15u) == 0 && ((uintptr_t)gx & 15u) == 0 && ((uintptr_t)W & 15u) == 0,
                "phip_out_fused: x, gx and W must be 16-byte aligned");
    if (m <= 0) return;
    ppo::ProfScope ps(PPO_K_GEMM, 2.0 * 3 * (double)m * n * A);
    const int AN = A * n;
    const int grid = (int)std::min<long>(kGrid, ((long)m + 3) / 4);
    const size_t need = sizeof(float) * (size_t)grid * (AN + A);
    const bool side = phip_side_active();
    float*& part = side ? g_part_side : g_part;
    size_t& cap = side ? g_part_side_cap : g_part_cap;
    if (cap < need) {
        if (part) phip_free(part);
        part = (float*)phip_malloc(need);
        cap = need;
    }
    OutArgs p{};
    p.x = x; p.W = W; p.b = b; p.bits = bits; p.m = m; p.n = n; p.wpr = ppo_divup(n, 32);
    p.tgt = tgt; p.log_std = log_std; p.action = action; p.adv = adv; p.old_lp = old_lp;
    p.eps = eps; p.ent_coeff = ent_coeff;
    p.y = y; p.gx = gx; p.part = part; p.grad_log_std = grad_log_std; p.loss_accum = loss_accum;
    const size_t lds = sizeof(float) * (2 * (size_t)AN + A);
    bool ok = false;
    if (n == 256) ok = launch_n<4>(p, A, head, grid, lds);
    else ok = launch_n<8>(p, A, head, grid, lds);
    PPO_REQUIRE(ok, "phip_out_fused: no instantiation");
    PPO_LAUNCH_CHECK();
    hipLaunchKernelGGL(out_reduce_kernel, dim3(ppo_divup(AN + A, 64)), dim3(256), 0, ppo::stream(), part, grid, AN,
                       A, gW, gb);
    PPO_LAUNCH_CHECK();
}

}  // extern "C"
