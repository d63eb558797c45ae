// out_head.hip — a minibatch step's output layer fused with its loss head, for narrow outputs
// (value networks A = 1, small action spaces): fp32 storage, and bf16 storage for value networks.
//
// Replaces four launches per step inside ppo_update:
//   output-layer forward    y = x·Wᵀ + b                         mat_mul.cu:122-163 (K1+K2)
//   loss head               value: MSE + derivative                 loss.cu:5-83 (K8+K9)
//                           policy: log-prob, ratio/clip, ∂/∂μ, ∂/∂logσ (+ −c_ent)
//                                                                  ppo.cu:82-107,436-438, policy.cu:67-111
//   output-layer backward   gx = (g·W) ⊙ 1[x > 0], gW += gᵀ·x, gb += Σ g
//                                                                  mat_mul.cu:165-217, neural_network.cu:108-118
// The last hidden activation x [m, n] is read once and gx written once: ≈ 8·m·n bytes per step (the
// separate launches read x twice and round-trip y and g through HBM, and their GEMM grids were
// latency-bound at these shapes).
//
// One wave per row (rows strided over every wave of the grid); lane l owns the NPL = n/64 columns
// [l·NPL, l·NPL + NPL): its slice of W (A·NPL values) and its gW accumulators sit in registers.
// y_a is a wave sum of the lanes' partial dots; every lane then evaluates the head on the full row
// (the same arithmetic as kernels.hip's mse_kernel / policy_head_kernel given y), and g·W, gᵀ·x use
// the lane's columns.  gW / gb / grad_logσ / loss: summed over the workgroup's waves through LDS,
// then one f32 atomic per element per workgroup into outputs that are zero on entry (as the split-K
// grad_W GEMMs).  The wide policy output (A = 17) does not fit this layout: one wave per row would
// need 2·17·8 registers for its weights and accumulators alone (the round-1 fused kernel spilled,
// 10× slower), and splitting each row over two waves (4 columns per lane, 256 VGPRs, one wave per
// SIMD) measured slower than the separate launches (C4 update 330 -> 347 ms,
// profiles/r02_out_head_ab.txt).  It takes out_bwd_wide_kernel (head + backward, thread per column)
// after the forward GEMM, or policy_out_fused_kernel (forward + head + backward) up to 8192 rows.
#include "dev.h"

#include <algorithm>
#include <cmath>

namespace {

constexpr int NTH = 256;                   // 4 waves
constexpr int NW = NTH / 64;

__device__ __forceinline__ float wsum(float v) { return ppo::wave_sum64(v); }   // DPP rows + scalar reads

// policy.cu:67-74 with the reference's double temporaries (kernels.hip log_prob_row); es[j] =
// expf(log_std[j]), computed once per wave (the same value the per-element expf gave)
template <int A>
__device__ __forceinline__ float log_prob_row(const float (&mu)[A], const float (&log_std)[A], const float (&es)[A],
                                              const float (&a)[A]) {
    const float c = (float)(-0.5 * A * (double)logf((float)(2 * M_PI)));
    float lp = c;
#pragma unroll
    for (int j = 0; j < A; ++j) {
        const float z = (a[j] - mu[j]) / es[j];
        lp = (float)((double)lp - ((double)log_std[j] + 0.5 * (double)(z * z)));
    }
    return lp;
}

// ppo.cu:82-107 per sample (kernels.hip surrogate)
__device__ __forceinline__ float surrogate(float adv, float lp, float old_lp, float eps, int m, float* grad) {
    const float ratio = (float)exp((double)(lp - old_lp));
    const int adv_pos = adv > 0;
    const int ratio_pos = ratio > 1 + eps;
    const int ratio_neg = ratio < 1 - eps;
    *grad = -(adv_pos * !ratio_pos + !adv_pos * !ratio_neg) * adv * ratio / m;
    return adv * (adv_pos * (ratio_pos * (1 + eps) + !ratio_pos * ratio) +
                  !adv_pos * (ratio_neg * (1 - eps) + !ratio_neg * ratio));
}

struct OutArgs {
    const void* x; const void* W; const float* b;     // x [m, n] (the last hidden activation), W [A, n], b [A]
    int m, n, relu_in;                                // relu_in: gx masked by x > 0
    const float* tgt;                                 // value head: targets [m]
    const float* log_std; const float* action; const float* adv; const float* old_lp;   // policy head
    float eps, ent_coeff;
    float* y; void* gx; float* gW; float* gb; float* grad_log_std; float* loss_accum;
};

// bf16 storage (bf16 compute mode): NPL elements of 2 B, widened to fp32 exactly
__device__ __forceinline__ float bf(unsigned short h) { return __builtin_bit_cast(float, (unsigned)h << 16); }
__device__ __forceinline__ unsigned short to_bf(float f) {          // round to nearest even (as gemm16.hip)
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    bf16x2 p = {(__bf16)f, (__bf16)0.f};
    return (unsigned short)(__builtin_bit_cast(unsigned, p) & 0xffffu);
}

template <int NPL>
__device__ __forceinline__ void load_cols(const unsigned short* __restrict__ p, float (&v)[NPL]) {
    if constexpr (NPL % 8 == 0) {
#pragma unroll
        for (int c = 0; c < NPL / 8; ++c) {
            const uint4 a = reinterpret_cast<const uint4*>(p)[c];
            const unsigned w[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                v[8 * c + 2 * q] = bf((unsigned short)(w[q] & 0xffffu));
                v[8 * c + 2 * q + 1] = bf((unsigned short)(w[q] >> 16));
            }
        }
    } else if constexpr (NPL == 4) {
        const uint2 a = *reinterpret_cast<const uint2*>(p);
        v[0] = bf((unsigned short)(a.x & 0xffffu)); v[1] = bf((unsigned short)(a.x >> 16));
        v[2] = bf((unsigned short)(a.y & 0xffffu)); v[3] = bf((unsigned short)(a.y >> 16));
    } else {
#pragma unroll
        for (int q = 0; q < NPL; ++q) v[q] = bf(p[q]);
    }
}

template <int NPL>
__device__ __forceinline__ void store_cols(unsigned short* __restrict__ p, const float (&v)[NPL]) {
    if constexpr (NPL % 8 == 0) {
#pragma unroll
        for (int c = 0; c < NPL / 8; ++c) {
            unsigned w[4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                w[q] = (unsigned)to_bf(v[8 * c + 2 * q]) | ((unsigned)to_bf(v[8 * c + 2 * q + 1]) << 16);
            reinterpret_cast<uint4*>(p)[c] = uint4{w[0], w[1], w[2], w[3]};
        }
    } else if constexpr (NPL == 4) {
        const unsigned a = (unsigned)to_bf(v[0]) | ((unsigned)to_bf(v[1]) << 16);
        const unsigned b = (unsigned)to_bf(v[2]) | ((unsigned)to_bf(v[3]) << 16);
        *reinterpret_cast<uint2*>(p) = uint2{a, b};
    } else {
#pragma unroll
        for (int q = 0; q < NPL; ++q) p[q] = to_bf(v[q]);
    }
}

template <int NPL>
__device__ __forceinline__ void load_cols(const float* __restrict__ p, float (&v)[NPL]) {
    if constexpr (NPL == 8) {
        const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else if constexpr (NPL == 4) {
        const float4 a = *reinterpret_cast<const float4*>(p);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    } else if constexpr (NPL == 2) {
        const float2 a = *reinterpret_cast<const float2*>(p);
        v[0] = a.x; v[1] = a.y;
    } else {
        v[0] = p[0];
    }
}

template <int NPL>
__device__ __forceinline__ void store_cols(float* __restrict__ p, const float (&v)[NPL]) {
    if constexpr (NPL == 8) {
        *reinterpret_cast<float4*>(p) = float4{v[0], v[1], v[2], v[3]};
        *reinterpret_cast<float4*>(p + 4) = float4{v[4], v[5], v[6], v[7]};
    } else if constexpr (NPL == 4) {
        *reinterpret_cast<float4*>(p) = float4{v[0], v[1], v[2], v[3]};
    } else if constexpr (NPL == 2) {
        *reinterpret_cast<float2*>(p) = float2{v[0], v[1]};
    } else {
        p[0] = v[0];
    }
}

// HEAD 0: value (A = 1, MSE against tgt); HEAD 1: policy (clipped surrogate + Gaussian log-prob).
// WPR waves share a row (WPR = 2 for wide outputs: each lane then holds half the weights and
// accumulators); their partial dot products meet in LDS, one barrier per row step.
// T: storage of x, W and gx — float (fp32 mode) or unsigned short (bf16 mode: x and gx bf16, W the
// bf16 parameter shadow, and the head gradient rounded to bf16 before its products, as the separate
// bf16 GEMMs round the fp32 operand they stage)
#ifndef OUTHEAD_PF
#define OUTHEAD_PF 4                                 // rows in flight per wave (one wave per row)
#endif

template <int NPL, int A, int HEAD, int WPR, typename T>
__global__ __launch_bounds__(NTH) void out_head_kernel(OutArgs p) {
    constexpr bool B16 = sizeof(T) == 2;
    const T* __restrict__ X = static_cast<const T*>(p.x);
    const T* __restrict__ Wp = static_cast<const T*>(p.W);
    T* __restrict__ GX = static_cast<T*>(p.gx);
    static_assert(HEAD == 1 || A == 1, "value head: one output");
    constexpr int N = 64 * NPL * WPR;                  // the layer's input width
    constexpr int SLOTS = NW / WPR;                    // rows in flight per workgroup
    extern __shared__ float sm[];
    float* red = sm;                                   // [SLOTS][A·N] gW partials (after the row loop)
    float* xch = sm;                                   // [2][SLOTS][WPR][A] partial dots (row loop)
    __shared__ float redb[NW][2 * A + 1];              // gb, grad_logσ partials, loss
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int slot = w / WPR, part = w % WPR;
    const int c0 = (part * 64 + lane) * NPL;
    const int m = p.m;

    float Wr[A][NPL], bias[A], e2[A], ls[A], es[A];
#pragma unroll
    for (int a = 0; a < A; ++a) {
        load_cols<NPL>(Wp + (long)a * N + c0, Wr[a]);
        bias[a] = p.b[a];
        if (HEAD == 1) {
            ls[a] = p.log_std[a];
            e2[a] = expf(-2 * ls[a]);
            es[a] = expf(ls[a]);
        }
    }
    float gWacc[A][NPL], gbacc[A], glsacc[A];
#pragma unroll
    for (int a = 0; a < A; ++a) {
        gbacc[a] = glsacc[a] = 0.f;
#pragma unroll
        for (int q = 0; q < NPL; ++q) gWacc[a][q] = 0.f;
    }
    float loss = 0.f;

    int it = 0;
    const int stride = gridDim.x * SLOTS;
    // rows in flight per wave: PF rows' slices are loaded ahead (a ring of registers, statically
    // indexed by unrolling PF rows per iteration); one wave per row keeps up to PF·NPL loads in
    // flight instead of one row's (3.5 -> ≈5 TB/s of x read + gx written at C4's value head)
    constexpr int PF = WPR == 1 ? OUTHEAD_PF : 1;
    float xr[PF][NPL];
    const int first = blockIdx.x * SLOTS + slot;
#pragma unroll
    for (int f = 0; f < PF; ++f) {
        const int r0 = first + f * stride;
        if (r0 < m) load_cols<NPL>(X + (long)r0 * N + c0, xr[f]);
    }
    for (int base = blockIdx.x * SLOTS; base < m; base += PF * stride) {
#pragma unroll
    for (int f = 0; f < PF; ++f, ++it) {
        const int row = base + f * stride + slot;
        if (WPR == 1 && base + f * stride >= m) break;  // (WPR > 1: PF = 1, the loop condition)
        const bool valid = row < m;                    // every wave reaches the barrier
        float xv[NPL];
#pragma unroll
        for (int q = 0; q < NPL; ++q) xv[q] = valid ? xr[f][q] : 0.f;
        if (row + PF * stride < m) load_cols<NPL>(X + (long)(row + PF * stride) * N + c0, xr[f]);
        float yv[A];
#pragma unroll
        for (int a = 0; a < A; ++a) {
            float part_s = 0.f;
#pragma unroll
            for (int q = 0; q < NPL; ++q) part_s += xv[q] * Wr[a][q];
            yv[a] = wsum(part_s);
        }
        if constexpr (WPR > 1) {
            float* x2 = xch + (it & 1) * (SLOTS * WPR * A);
            if (lane == 0)
#pragma unroll
                for (int a = 0; a < A; ++a) x2[(slot * WPR + part) * A + a] = yv[a];
            __syncthreads();
#pragma unroll
            for (int a = 0; a < A; ++a) {
                float t = 0.f;
#pragma unroll
                for (int q = 0; q < WPR; ++q) t += x2[(slot * WPR + q) * A + a];
                yv[a] = t;
            }
        }
#pragma unroll
        for (int a = 0; a < A; ++a) yv[a] += bias[a];
        if (!valid) continue;
        const bool owner = part == 0;                  // one wave per row counts the row-wide sums
        float g[A];
        if (HEAD == 0) {                                   // loss.cu:5-23 (kernels.hip mse_kernel)
            const float t = p.tgt[row];
            const float d = t - yv[0];
            if (owner) loss += d * d;
            g[0] = 2 * (yv[0] - t) / (float)m;
        } else {                                           // kernels.hip policy_head_kernel, per row
            float act[A];
#pragma unroll
            for (int a = 0; a < A; ++a) act[a] = p.action[(long)row * A + a];
            const float lp = log_prob_row<A>(yv, ls, es, act);
            float glp;
            const float sv = surrogate(p.adv[row], lp, p.old_lp[row], p.eps, m, &glp);
            if (owner) loss += sv;
#pragma unroll
            for (int a = 0; a < A; ++a) {
                const float d = act[a] - yv[a];
                g[a] = d * e2[a] * glp;
                if (owner) glsacc[a] += (-1 + d * d * e2[a]) * glp;
            }
        }
        if (owner && lane == 0) {
#pragma unroll
            for (int a = 0; a < A; ++a) p.y[(long)row * A + a] = yv[a];
        }
        if constexpr (B16) {
#pragma unroll
            for (int a = 0; a < A; ++a) g[a] = bf(to_bf(g[a]));
        }
        float gxv[NPL];
#pragma unroll
        for (int q = 0; q < NPL; ++q) {
            float s = 0.f;
#pragma unroll
            for (int a = 0; a < A; ++a) s += g[a] * Wr[a][q];
            gxv[q] = (!p.relu_in || xv[q] > 0.f) ? s : 0.f;
        }
        store_cols<NPL>(GX + (long)row * N + c0, gxv);
#pragma unroll
        for (int a = 0; a < A; ++a) {
            if (owner) gbacc[a] += g[a];
#pragma unroll
            for (int q = 0; q < NPL; ++q) gWacc[a][q] += g[a] * xv[q];
        }
    }
    }

    // workgroup sums (row slots in order), then one atomic per element
    __syncthreads();                                   // the exchange buffer is reused below
#pragma unroll
    for (int a = 0; a < A; ++a)
#pragma unroll
        for (int q = 0; q < NPL; ++q) red[slot * (A * N) + a * N + c0 + q] = gWacc[a][q];
    if (lane == 0) {
#pragma unroll
        for (int a = 0; a < A; ++a) {
            redb[w][a] = gbacc[a];
            redb[w][A + a] = glsacc[a];
        }
        redb[w][2 * A] = loss;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < A * N; i += NTH) {
        float s = 0.f;
#pragma unroll
        for (int v = 0; v < SLOTS; ++v) s += red[v * (A * N) + i];
        atomicAdd(p.gW + i, s);
    }
    if (threadIdx.x < A) {
        float s = 0.f, l = 0.f;
#pragma unroll
        for (int v = 0; v < NW; ++v) { s += redb[v][threadIdx.x]; l += redb[v][A + threadIdx.x]; }
        atomicAdd(p.gb + threadIdx.x, s);
        if (HEAD == 1) {
            if (blockIdx.x == 0) l += -p.ent_coeff;                        // ppo.cu:436-438 (D4)
            atomicAdd(p.grad_log_std + threadIdx.x, l);
        }
    }
    if (threadIdx.x == 0 && p.loss_accum) {
        float s = 0.f;
#pragma unroll
        for (int v = 0; v < NW; ++v) s += redb[v][2 * A];
        if (HEAD == 0) {
            atomicAdd(p.loss_accum, s * (1.0f / (float)m));
        } else {
            float contrib = -s / m;
            if (blockIdx.x == 0) {
                float ent = (float)(A * 0.5 * (1 + log(2 * M_PI)));
                for (int j = 0; j < A; ++j) ent += ls[j];
                contrib -= p.ent_coeff * ent;
            }
            atomicAdd(p.loss_accum, contrib);
        }
    }
}

template <int NPL, int A, int HEAD, int WPR, typename T>
void launch(const OutArgs& a) {
    constexpr int N = 64 * NPL * WPR, SLOTS = NW / WPR;
    const size_t lds = sizeof(float) * (size_t)std::max(SLOTS * A * N, 2 * SLOTS * WPR * A);
    static_assert(sizeof(float) * SLOTS * A * N <= 150 * 1024, "out_head: LDS");
    auto kern = out_head_kernel<NPL, A, HEAD, WPR, T>;
    if (lds > 64 * 1024) {
        static bool attr = false;
        if (!attr) {
            PPO_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            attr = true;
        }
    }
    // about 16 rows per wave slot (32 / 64 measured slower at C3, C4 and the shard: r04_outhead_rps_*),
    // at most 1024 workgroups
    constexpr int rps = 16;
    int grid = ppo_divup(a.m, SLOTS * rps);
    if (grid > 1024) grid = 1024;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NTH), lds, ppo::stream(), a);
    PPO_LAUNCH_CHECK();
}

// one wave per row up to width 512; at width 1024 (value networks) two waves per row in fp32
// storage, one (16 columns per lane) in bf16 storage (C5 fused head 35.2 µs with two waves per row)
template <int A, int HEAD, typename T>
bool launch_n(const OutArgs& a) {
    switch (a.n) {
        case 64: launch<1, A, HEAD, 1, T>(a); return true;
        case 128: launch<2, A, HEAD, 1, T>(a); return true;
        case 256: launch<4, A, HEAD, 1, T>(a); return true;
        case 512: launch<8, A, HEAD, 1, T>(a); return true;
        case 1024:
            if constexpr (A == 1) {
                if constexpr (sizeof(T) == 2) launch<16, A, HEAD, 1, T>(a);   // bf16: one wave per row
                else launch<8, A, HEAD, 2, T>(a);
                return true;
            }
            return false;
        default: return false;
    }
}

// Backward of a wide output layer (policy A = 17 at C4) in one pass over the rows: a 256-thread
// workgroup takes a chunk of rows; thread t owns columns NPT·t .. NPT·t+NPT-1 — their A weights and
// A gW accumulators in registers — and per row reads x (NPT floats), the row's A head gradients as
// wave-uniform scalar loads, and writes gx = (g·W) ⊙ 1[x > 0]; lanes a < A of wave 0 also sum gb.
// Each workgroup's gW / gb partial goes to its slab and ppo::slab_reduce sums them in order.  Replaces
// the paired grad_W + grad_x GEMM launch (x read once for both; HBM ≈ 8·n bytes per row).
struct WideArgs {
    const float* g; const float* x; const float* W; float* gx; float* slab; long slab_stride;
    int m, rows_per_wg, relu_in;
    // HEAD: the policy head computed here from μ (the forward's output) — kernels.hip
    // policy_head_tiled_kernel's per-row arithmetic and its 8 partial sums per column of ∂/∂log σ
    const float* mu; const float* log_std; const float* action; const float* adv; const float* old_lp;
    float eps, ent_coeff; float* grad_log_std; float* loss_accum;
};

// kernels.hip log_prob_row (policy.cu:67-74, double temporaries), on LDS rows; es[j] = expf(log_std[j])
// computed once per workgroup (the same value the per-element expf gave)
__device__ __forceinline__ float log_prob_row_p(const float* mu, const float* log_std, const float* es, const float* a,
                                                int A) {
    const float c = (float)(-0.5 * A * (double)logf((float)(2 * M_PI)));
    float lp = c;
    for (int j = 0; j < A; ++j) {
        const float z = (a[j] - mu[j]) / es[j];
        lp = (float)((double)lp - ((double)log_std[j] + 0.5 * (double)(z * z)));
    }
    return lp;
}

template <int A, int NPT, int U, bool HEAD>
__global__ __launch_bounds__(256) void out_bwd_wide_kernel(WideArgs p) {
    constexpr int N = 256 * NPT;
    extern __shared__ float gs[];                        // this workgroup's rows of g [rows][A] (+ μ, actions)
    __shared__ float e2s[32], lss[32], ess[32], cps[8][32], redl[4];
    const int t = threadIdx.x, k0 = t * NPT;
    const int m = p.m;
    const int r0 = blockIdx.x * p.rows_per_wg;
    const int nr = min(m, r0 + p.rows_per_wg) - r0;
    // the weights and the first U rows' x in flight before the head (they do not depend on it)
    float Wr[A][NPT], acc[A][NPT], xpre[U][NPT];
#pragma unroll
    for (int a = 0; a < A; ++a) {
        load_cols<NPT>(p.W + (long)a * N + k0, Wr[a]);
#pragma unroll
        for (int q = 0; q < NPT; ++q) acc[a][q] = 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (u < nr) load_cols<NPT>(p.x + (long)(r0 + u) * N + k0, xpre[u]);
    if constexpr (HEAD) {
        float* mus = gs + p.rows_per_wg * A;
        float* acts = mus + p.rows_per_wg * A;
        float* grs = acts + p.rows_per_wg * A;           // ∂L/∂lp per row
        const float adv0 = t < nr ? p.adv[r0 + t] : 0.f, olp0 = t < nr ? p.old_lp[r0 + t] : 0.f;   // first row's
        for (int e = t; e < nr * A; e += 256) {
            mus[e] = p.mu[(long)r0 * A + e];
            acts[e] = p.action[(long)r0 * A + e];
        }
        if (t < A) {
            lss[t] = p.log_std[t];
            e2s[t] = expf(-2 * p.log_std[t]);
            ess[t] = expf(p.log_std[t]);
        }
        __syncthreads();
        float sv = 0.f;
        for (int row = t; row < nr; row += 256) {
            float glp;
            const float lp = log_prob_row_p(mus + row * A, lss, ess, acts + row * A, A);
            const float ad = row == t ? adv0 : p.adv[r0 + row], ol = row == t ? olp0 : p.old_lp[r0 + row];
            sv += surrogate(ad, lp, ol, p.eps, m, &glp);
            grs[row] = glp;
        }
        sv = ppo::wave_sum64(sv);
        if ((t & 63) == 0) redl[t >> 6] = sv;
        __syncthreads();
        for (int e = t; e < nr * A; e += 256) {
            const int row = e / A, j = e - row * A;
            gs[e] = (acts[e] - mus[e]) * e2s[j] * grs[row];
        }
        if (t < 8 * A) {                                 // ∂/∂log σ: 8 partial sums per column
            const int j = t % A, qq = t / A;
            float c = 0.f;
            for (int row = qq; row < nr; row += 8) {
                const float d = acts[row * A + j] - mus[row * A + j];
                c += (-1 + d * d * e2s[j]) * grs[row];
            }
            cps[qq][j] = c;
        }
        __syncthreads();
        if (t < A) {
            float v = 0.f;
            for (int q = 0; q < 8; ++q) v += cps[q][t];
            if (blockIdx.x == 0) v += -p.ent_coeff;                           // ppo.cu:436-438 (D4)
            atomicAdd(p.grad_log_std + t, v);
        }
        if (t == 0 && p.loss_accum) {
            const float sl = ((redl[0] + redl[1]) + redl[2]) + redl[3];
            float contrib = -sl / m;
            if (blockIdx.x == 0) {
                float ent = (float)(A * 0.5 * (1 + log(2 * M_PI)));
                for (int j = 0; j < A; ++j) ent += lss[j];
                contrib -= p.ent_coeff * ent;
            }
            atomicAdd(p.loss_accum, contrib);
        }
    } else {
        for (int e = t; e < nr * A; e += 256) gs[e] = p.g[(long)r0 * A + e];
    }
    __syncthreads();
    for (int rb = 0; rb < nr; rb += U) {
        float xv[U][NPT];                                // U rows in flight
        if (rb == 0) {
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int q = 0; q < NPT; ++q) xv[u][q] = xpre[u][q];
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (rb + u < nr) load_cols<NPT>(p.x + (long)(r0 + rb + u) * N + k0, xv[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int r = rb + u;
            if (r >= nr) break;                          // workgroup-uniform
            float gv[A];
#pragma unroll
            for (int a = 0; a < A; ++a) gv[a] = gs[r * A + a];   // uniform address: LDS broadcast
            // fused multiply-adds (this file is built with -ffp-contract=off): the two 17-term products
            // are GEMM-shaped sums, held to the GEMM tolerance; packed they are one v_pk_fma_f32 per
            // term and column pair instead of a v_pk_mul + v_pk_add (the loop was VALU-bound)
            float o[NPT];
#pragma unroll
            for (int q = 0; q < NPT; ++q) {
                float sacc = 0.f;
#pragma unroll
                for (int a = 0; a < A; ++a) sacc = __builtin_fmaf(gv[a], Wr[a][q], sacc);
                o[q] = (!p.relu_in || xv[u][q] > 0.f) ? sacc : 0.f;
            }
            store_cols<NPT>(p.gx + (long)(r0 + r) * N + k0, o);
#pragma unroll
            for (int a = 0; a < A; ++a)
#pragma unroll
                for (int q = 0; q < NPT; ++q) acc[a][q] = __builtin_fmaf(gv[a], xv[u][q], acc[a][q]);
        }
    }
    float* __restrict__ out = p.slab + (long)blockIdx.x * p.slab_stride;
#pragma unroll
    for (int a = 0; a < A; ++a) store_cols<NPT>(out + a * N + k0, acc[a]);
    if (t < A) {                                         // gb partial: the rows in order
        float sb = 0.f;
        for (int r = 0; r < nr; ++r) sb += gs[r * A + t];
        out[A * N + t] = sb;
    }
}


// ---------------------------------------------------------------------------------------------------
// The A = 17 policy network's whole output layer for one minibatch step in ONE pass over the last hidden
// activation h (round 6; replaces the exact-fp32 forward GEMM and out_bwd_wide_kernel<HEAD>):
//   μ = h·W3ᵀ + b3 — exact fp32 MFMA (v_mfma_f32_16x16x4_f32) on 16-row blocks of h staged in LDS, K split
//       over the four waves and their partial tiles summed in a fixed order (mat_mul.cu:122-163);
//   the policy head on μ — out_bwd_wide_kernel<HEAD>'s per-row arithmetic (policy.cu:67-111, ppo.cu:82-107);
//   gx = (g·W3) ⊙ 1[h > 0], gW3 += gᵀ·h, gb3 += Σ g (mat_mul.cu:165-217) — thread t owns columns
//       t·NPT … t·NPT + NPT − 1 with their W3 values and gW3 accumulators in registers, h read from LDS.
// h leaves HBM once (the separate forward and backward read it twice and round-trip μ): ≈ 8·n bytes per
// row.  Each workgroup loops over 16-row blocks; its gW3 / gb3 partial goes to its slab (ppo::slab_reduce
// sums them in order), log σ's gradient and the loss get one f32 atomic per workgroup (as the HEAD path).
struct FusedArgs {
    const float* x; const float* W; const float* b; float* mu;    // h [m, n], W3 [A, n], b3 [A], μ out [m, A]
    float* gx; float* slab; long slab_stride;
    int m, relu_in, nblk;                                          // nblk: 16-row blocks of the minibatch
    const float* log_std; const float* action; const float* adv; const float* old_lp;
    float eps, ent_coeff; float* grad_log_std; float* loss_accum;
};

constexpr int FR = 16;                                             // rows per block
#ifndef PPO_FUSED_ABL
#define PPO_FUSED_ABL 0        // diagnostic builds only: 1 no μ MFMA, 2 no head, 4 no gx / gW3 rows, 8 no h loads
#endif

template <int NPT>
constexpr size_t fused_lds_floats() {
    constexpr int N = 256 * NPT, HPs = N + 4;                      // pitch ≡ 4 (mod 32): 2-way = optimal for
    return (size_t)FR * HPs + 17 * HPs + 4 * 2 * 256               // the MFMA operand reads
           + 3 * FR * 20 + 3 * FR;                                 // μ / g, actions, log σ terms; ∂L/∂lp, adv, old lp
}

template <int NPT>
__global__ __launch_bounds__(256, 2) void policy_out_fused_kernel(FusedArgs p) {
    typedef float f32x4v __attribute__((ext_vector_type(4)));
    constexpr int A = 17, AP = 20, N = 256 * NPT, HPs = N + 4, KW = N / 4;   // KW: k range of one wave
    constexpr int NPF = FR * (N / 4) / 256;                        // float4 loads of h per thread per block
    extern __shared__ __attribute__((aligned(16))) float smf[];
    float* hs = smf;                                               // [FR][HPs] the block's rows of h
    float* ws = hs + FR * HPs;                                     // [A][HPs] W3
    float* red = ws + A * HPs;                                     // [wave][tile][lane] f32x4 partial μ tiles
    float* mus = red + 4 * 2 * 256;                                // [FR][AP] μ, then ∂L/∂μ in place
    float* acts = mus + FR * AP;                                   // [FR][AP] actions
    float* lst = acts + FR * AP;                                   // [FR][AP] ∂/∂log σ row terms
    float* grs = lst + FR * AP;                                    // [FR] ∂L/∂lp
    float* advs = grs + FR;                                        // [FR] advantage | old log-prob (2 × FR)
    double* dterm = reinterpret_cast<double*>(red);                // [FR][A] log-prob terms, over the μ tiles
    __shared__ float lss[32], ess[32], e2s[32], b3s[32];
    static_assert(sizeof(float) * fused_lds_floats<NPT>() + 4 * 32 * 4 <= 80 * 1024, "two workgroups per CU");
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, k0 = t * NPT;
    const int c = lane & 15, q = lane >> 4;
    float Wr[A][NPT], acc[A][NPT];
#pragma unroll
    for (int a = 0; a < A; ++a) {
        load_cols<NPT>(p.W + (long)a * N + k0, Wr[a]);
#pragma unroll
        for (int u = 0; u < NPT; ++u) acc[a][u] = 0.f;
    }
    for (int e = t; e < A * (N / 4); e += 256) {
        const int a = e / (N / 4), cq = e % (N / 4);
        *reinterpret_cast<f32x4v*>(ws + a * HPs + 4 * cq) = *reinterpret_cast<const f32x4v*>(p.W + (long)a * N + 4 * cq);
    }
    if (t < A) {
        lss[t] = p.log_std[t];
        e2s[t] = expf(-2 * p.log_std[t]);
        ess[t] = expf(p.log_std[t]);
        b3s[t] = p.b[t];
    }
    // the next block's operands in registers while this block computes: h rows, actions, adv / old log-prob
    f32x4v hpf[NPF];
    float apf[2], xpf = 0.f;
    auto prefetch = [&](int blk) {
        const int r0 = blk * FR, nr = blk < p.nblk ? min(FR, p.m - r0) : 0;
#pragma unroll
        for (int v = 0; v < NPF; ++v) {
            const int e = t + 256 * v, r = e / (N / 4), cq = e % (N / 4);
            hpf[v] = r < nr ? *reinterpret_cast<const f32x4v*>(p.x + (long)(r0 + r) * N + 4 * cq)
                            : f32x4v{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int v = 0; v < 2; ++v) {
            const int e = t + 256 * v;
            apf[v] = e < nr * A ? p.action[(long)r0 * A + e] : 0.f;
        }
        xpf = t < nr ? p.adv[r0 + t] : (t >= 32 && t < 32 + nr ? p.old_lp[r0 + t - 32] : 0.f);
    };
    float gls = 0.f, gbs = 0.f, sv = 0.f;     // threads j < A: log σ and gb3 partials; wave 0's rows: loss terms
    prefetch(blockIdx.x);
    for (int blk = blockIdx.x; blk < p.nblk; blk += gridDim.x) {
        const int r0 = blk * FR, nr = min(FR, p.m - r0);
        __syncthreads();                                           // the previous block is done with the LDS
#pragma unroll
        for (int v = 0; v < NPF; ++v) {
            const int e = t + 256 * v, r = e / (N / 4), cq = e % (N / 4);
            if (!(PPO_FUSED_ABL & 8)) *reinterpret_cast<f32x4v*>(hs + r * HPs + 4 * cq) = hpf[v];
        }
#pragma unroll
        for (int v = 0; v < 2; ++v) {
            const int e = t + 256 * v;
            if (e < FR * A) acts[(e / A) * AP + e % A] = apf[v];
        }
        if (t < FR) advs[t] = xpf;
        else if (t >= 32 && t < 32 + FR) advs[FR + t - 32] = xpf;
        __syncthreads();
        if (blk + (int)gridDim.x < p.nblk) prefetch(blk + gridDim.x);
        {   // μ partial tiles of this wave's k range (two interleaved chains per tile): tile 0 = columns
            // 0 … 15, tile 1 = column 16
            f32x4v a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, b0 = a0, b1 = a0;
            const float* Ar = hs + c * HPs + w * KW + q;
            const float* B0 = ws + c * HPs + w * KW + q;
            const float* B1 = ws + 16 * HPs + w * KW + q;
#pragma unroll 4
            for (int kk = 0; kk < KW && !(PPO_FUSED_ABL & 1); kk += 8) {
                const float av = Ar[kk], bv = Ar[kk + 4];
                a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, B0[kk], a0, 0, 0, 0);
                b0 = __builtin_amdgcn_mfma_f32_16x16x4f32(bv, B0[kk + 4], b0, 0, 0, 0);
                a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, c == 0 ? B1[kk] : 0.f, a1, 0, 0, 0);
                b1 = __builtin_amdgcn_mfma_f32_16x16x4f32(bv, c == 0 ? B1[kk + 4] : 0.f, b1, 0, 0, 0);
            }
            f32x4v* rp = reinterpret_cast<f32x4v*>(red) + w * 2 * 64 + lane;
            rp[0] = a0 + b0;
            rp[64] = a1 + b1;
        }
        __syncthreads();
        // μ = Σ over the waves in order + b3; tile element (row r, column cc) sits in lane cc + 16·(r / 4),
        // component r % 4.  Then each (row, j) term of the log-prob in parallel (the sum stays sequential)
        for (int e = t; e < FR * A; e += 256) {
            const int r = e / A, j = e % A, tile = j >> 4, cc = j & 15;
            const int ln = cc + 16 * (r >> 2), comp = r & 3;
            float sacc = red[((0 * 2 + tile) * 64 + ln) * 4 + comp];
#pragma unroll
            for (int ww = 1; ww < 4; ++ww) sacc += red[((ww * 2 + tile) * 64 + ln) * 4 + comp];
            const float muv = sacc + b3s[j];
            mus[r * AP + j] = muv;
            if (r < nr) p.mu[(long)(r0 + r) * A + j] = muv;       // the network's output
        }
        __syncthreads();
        for (int e = t; e < FR * A; e += 256) {
            const int r = e / A, j = e % A;
            const float z = (acts[r * AP + j] - mus[r * AP + j]) / ess[j];
            dterm[e] = (double)lss[j] + 0.5 * (double)(z * z);     // policy.cu:67-74 (log_prob_row_p)
        }
        __syncthreads();
        if (t < nr && !(PPO_FUSED_ABL & 2)) {                     // the head, one row per thread (wave 0)
            float lp = (float)(-0.5 * A * (double)logf((float)(2 * M_PI)));
#pragma unroll
            for (int j = 0; j < A; ++j) lp = (float)((double)lp - dterm[t * A + j]);
            float glp;
            sv += surrogate(advs[t], lp, advs[FR + t], p.eps, p.m, &glp);
            grs[t] = glp;
        }
        __syncthreads();
        for (int e = t; e < FR * A; e += 256) {                    // log σ row terms; μ → ∂L/∂μ in place
            const int r = e / A, j = e % A;
            const float d = acts[r * AP + j] - mus[r * AP + j], gr = r < nr ? grs[r] : 0.f;
            lst[r * AP + j] = (-1 + d * d * e2s[j]) * gr;
            mus[r * AP + j] = d * e2s[j] * gr;
        }
        __syncthreads();
        if (t < A && !(PPO_FUSED_ABL & 2)) {                      // ordered sums over the block's rows
            for (int r = 0; r < nr; ++r) gls += lst[r * AP + t];
        } else if (t >= 32 && t < 32 + A) {
            for (int r = 0; r < nr; ++r) gbs += mus[r * AP + t - 32];
        }
        for (int r = 0; r < nr && !(PPO_FUSED_ABL & 4); r += 2) {  // two rows at a time (independent chains)
            const bool two = r + 1 < nr;
            float gv0[A], gv1[A], xv0[NPT], xv1[NPT];
#pragma unroll
            for (int a = 0; a < A; ++a) {
                gv0[a] = mus[r * AP + a];                          // uniform address: LDS broadcast
                gv1[a] = two ? mus[(r + 1) * AP + a] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < NPT; ++u) {
                xv0[u] = hs[r * HPs + k0 + u];
                xv1[u] = two ? hs[(r + 1) * HPs + k0 + u] : 0.f;
            }
            float o0[NPT], o1[NPT];
#pragma unroll
            for (int u = 0; u < NPT; ++u) {
                float s0 = 0.f, s1 = 0.f;
#pragma unroll
                for (int a = 0; a < A; ++a) {
                    s0 = __builtin_fmaf(gv0[a], Wr[a][u], s0);
                    s1 = __builtin_fmaf(gv1[a], Wr[a][u], s1);
                }
                o0[u] = (!p.relu_in || xv0[u] > 0.f) ? s0 : 0.f;
                o1[u] = (!p.relu_in || xv1[u] > 0.f) ? s1 : 0.f;
            }
            store_cols<NPT>(p.gx + (long)(r0 + r) * N + k0, o0);
            if (two) store_cols<NPT>(p.gx + (long)(r0 + r + 1) * N + k0, o1);
#pragma unroll
            for (int a = 0; a < A; ++a)
#pragma unroll
                for (int u = 0; u < NPT; ++u)
                    acc[a][u] = __builtin_fmaf(gv1[a], xv1[u], __builtin_fmaf(gv0[a], xv0[u], acc[a][u]));
        }
    }
    float* __restrict__ out = p.slab + (long)blockIdx.x * p.slab_stride;
#pragma unroll
    for (int a = 0; a < A; ++a) store_cols<NPT>(out + a * N + k0, acc[a]);
    if (t < A) atomicAdd(p.grad_log_std + t, gls + (blockIdx.x == 0 ? -p.ent_coeff : 0.f));     // ppo.cu:436-438 (D4)
    else if (t >= 32 && t < 32 + A) out[A * N + t - 32] = gbs;
    if (w == 0) {
        const float sl = ppo::wave_sum64(sv);
        if (lane == 0 && p.loss_accum) {
            float contrib = -sl / p.m;
            if (blockIdx.x == 0) {
                float ent = (float)(A * 0.5 * (1 + log(2 * M_PI)));
                for (int j = 0; j < A; ++j) ent += lss[j];
                contrib -= p.ent_coeff * ent;
            }
            atomicAdd(p.loss_accum, contrib);
        }
    }
}

}  // namespace

extern "C" {

// workgroups of the one-pass wide backward (512: ≥ 16 rows each)
static int wide_nwg_cap() { return 512; }

int phip_out_bwd_wide_ok(int m, int n, int A, int head) {
    if (A != 17 || (n != 512 && n != 256) || m <= 0 || getenv("PPO_NO_WIDE_BWD")) return 0;
    const int U = 8;
    const int nwg = std::min(wide_nwg_cap(), ppo_divup(m, 16));
    const long rows = (long)ppo_divup(ppo_divup(m, nwg), U) * U;
    return sizeof(float) * rows * (head ? 3 * A + 1 : A) <= 64 * 1024;
}

static int out_bwd_wide_launch(WideArgs w, float* gW, float* gb, int n, int A, bool head) {
    const int m = w.m;
    if (!phip_out_bwd_wide_ok(m, n, A, head) || gb != gW + (long)A * n) return 0;
    if ((((uintptr_t)w.x | (uintptr_t)w.gx | (uintptr_t)w.W | (uintptr_t)gW) & 15u) != 0) return 0;
    ppo::ProfScope ps(PPO_K_GEMM, 4.0 * m * n * A, ppo::gemm_key(3, 1, m, n, A));
    constexpr int U = 8;
    int nwg = std::min(wide_nwg_cap(), ppo_divup(m, 16));     // ≥ 16 rows per workgroup
    const int rows = ppo_divup(ppo_divup(m, nwg), U) * U;
    nwg = ppo_divup(m, rows);
    w.rows_per_wg = rows;
    w.slab_stride = ((long)A * n + A + 3) & ~3L;              // slab rows 16-B aligned
    const size_t lds = sizeof(float) * (size_t)rows * (head ? 3 * A + 1 : A);
    if (lds > 64 * 1024) return 0;                            // (m > 512 · 315 rows: the separate launches)
    w.slab = ppo::slab_scratch((size_t)nwg * w.slab_stride);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const bool timed = ppo::take_kernel_events(&e0, &e1);      // one duration: kernel start → reduce end
    auto go = [&](auto kern) {
        if (timed) hipExtLaunchKernelGGL(kern, dim3(nwg), dim3(256), lds, ppo::stream(), e0, nullptr, 0, w);
        else hipLaunchKernelGGL(kern, dim3(nwg), dim3(256), lds, ppo::stream(), w);
    };
    if (n == 512) head ? go(out_bwd_wide_kernel<17, 2, U, true>) : go(out_bwd_wide_kernel<17, 2, U, false>);
    else head ? go(out_bwd_wide_kernel<17, 1, U, true>) : go(out_bwd_wide_kernel<17, 1, U, false>);
    PPO_LAUNCH_CHECK();
    ppo::slab_reduce(w.slab, gW, (long)A * n + A, w.slab_stride, nwg, timed ? e1 : nullptr);
    return 1;
}

int phip_out_bwd_wide(float* gW, float* gb, float* gx, const float* g, const float* x, const float* W, int relu_in,
                      int m, int n, int A) {
    WideArgs w{};
    w.g = g; w.x = x; w.W = W; w.gx = gx; w.m = m; w.relu_in = relu_in;
    return out_bwd_wide_launch(w, gW, gb, n, A, false);
}

// the fused policy output layer (policy_out_fused_kernel): 1 when it ran, 0 when the shape is not its
// (A = 17, n = 256 or 512, the flat gradient layout gb = gW + A·n, 16-B aligned operands)
int phip_policy_out_fused(const float* x, const float* W, const float* b, float* mu, const float* log_std,
                          const float* action, const float* adv, const float* old_lp, float eps, float ent_coeff,
                          float* grad_log_std, float* loss_accum, int relu_in, float* gW, float* gb, float* gx, int m,
                          int n, int A) {
    if (A != 17 || (n != 512 && n != 256) || m <= 0 || !b || !mu || !log_std || !action || !adv || !old_lp ||
        !grad_log_std || gb != gW + (long)A * n)
        return 0;
    if ((((uintptr_t)x | (uintptr_t)gx | (uintptr_t)W | (uintptr_t)gW) & 15u) != 0) return 0;
    ppo::ProfScope ps(PPO_K_GEMM, 6.0 * m * n * A, ppo::gemm_key(4, 0, m, n, A));
    FusedArgs f{};
    f.x = x; f.W = W; f.b = b; f.mu = mu; f.gx = gx; f.m = m; f.relu_in = relu_in;
    f.log_std = log_std; f.action = action; f.adv = adv; f.old_lp = old_lp;
    f.eps = eps; f.ent_coeff = ent_coeff; f.grad_log_std = grad_log_std; f.loss_accum = loss_accum;
    f.nblk = ppo_divup(m, FR);
    // two workgroups per CU (C4: 256 / 512 / 1024 / 2048 workgroups 107 / 74 / 87 / 104 µs)
    const int nwg = std::min(512, f.nblk);
    f.slab_stride = ((long)A * n + A + 3) & ~3L;
    f.slab = ppo::slab_scratch((size_t)nwg * f.slab_stride);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const bool timed = ppo::take_kernel_events(&e0, &e1);          // one duration: kernel start → reduce end
    auto go = [&](auto kern, size_t lds) {
        static bool attr[2] = {false, false};
        bool& at = attr[n == 512 ? 1 : 0];
        if (!at) {
            PPO_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            at = true;
        }
        if (timed) hipExtLaunchKernelGGL(kern, dim3(nwg), dim3(256), lds, ppo::stream(), e0, nullptr, 0, f);
        else hipLaunchKernelGGL(kern, dim3(nwg), dim3(256), lds, ppo::stream(), f);
    };
    if (n == 512) go(policy_out_fused_kernel<2>, sizeof(float) * fused_lds_floats<2>());
    else go(policy_out_fused_kernel<1>, sizeof(float) * fused_lds_floats<1>());
    PPO_LAUNCH_CHECK();
    ppo::slab_reduce(f.slab, gW, (long)A * n + A, f.slab_stride, nwg, timed ? e1 : nullptr);
    return 1;
}

int phip_policy_head_bwd_wide(const float* mu, const float* log_std, const float* action, const float* adv,
                              const float* old_lp, float eps, float ent_coeff, float* grad_log_std, float* loss_accum,
                              const float* x, const float* W, int relu_in, float* gW, float* gb, float* gx, int m,
                              int n, int A) {
    if (!mu || !log_std || !action || !adv || !old_lp || !grad_log_std) return 0;
    WideArgs w{};
    w.x = x; w.W = W; w.gx = gx; w.m = m; w.relu_in = relu_in;
    w.mu = mu; w.log_std = log_std; w.action = action; w.adv = adv; w.old_lp = old_lp;
    w.eps = eps; w.ent_coeff = ent_coeff; w.grad_log_std = grad_log_std; w.loss_accum = loss_accum;
    return out_bwd_wide_launch(w, gW, gb, n, A, true);
}

int phip_out_head_supported(int head, int n, int A) {
    if (n != 64 && n != 128 && n != 256 && n != 512 && !(n == 1024 && A == 1)) return 0;
    return head == 0 ? A == 1 : (A == 1 || A == 6);
}

void phip_out_head(int head, int bf16, const void* x, int relu_in, const void* W, const float* b, int m, int n,
                   int A, const float* tgt, const float* log_std, const float* action, const float* adv,
                   const float* old_lp, float eps, float ent_coeff, float* y, void* gx, float* gW, float* gb,
                   float* grad_log_std, float* loss_accum) {
    if (m <= 0) return;
    PPO_REQUIRE(phip_out_head_supported(head, n, A), "phip_out_head: unsupported shape");
    PPO_REQUIRE(x && W && b && y && gx && gW && gb, "phip_out_head: null operand");
    PPO_REQUIRE(head == 0 ? tgt != nullptr : (log_std && action && adv && old_lp && grad_log_std),
                "phip_out_head: missing head inputs");
    PPO_REQUIRE((((uintptr_t)x | (uintptr_t)gx | (uintptr_t)W) & 15u) == 0, "phip_out_head: unaligned operands");
    ppo::ProfScope ps(PPO_K_HEAD, 8.0 * m * n);
    OutArgs a{};
    a.x = x; a.W = W; a.b = b; a.m = m; a.n = n; a.relu_in = relu_in;
    a.tgt = tgt; a.log_std = log_std; a.action = action; a.adv = adv; a.old_lp = old_lp;
    a.eps = eps; a.ent_coeff = ent_coeff;
    a.y = y; a.gx = gx; a.gW = gW; a.gb = gb; a.grad_log_std = grad_log_std; a.loss_accum = loss_accum;
    using b16 = unsigned short;
    bool ok = false;
    if (bf16) {
        PPO_REQUIRE(head == 0, "phip_out_head: bf16 storage for the value head only");
        ok = launch_n<1, 0, b16>(a);
    } else if (head == 0) ok = launch_n<1, 0, float>(a);
    else if (A == 1) ok = launch_n<1, 1, float>(a);
    else ok = launch_n<6, 1, float>(a);
    PPO_REQUIRE(ok, "phip_out_head: no instantiation");
}

}  // extern "C"
