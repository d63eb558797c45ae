// gemm.hip — fp32 MFMA GEMMs for the MLP layers (the dominant FLOPs of the PPO update).
//
// Replaces the reference's cuBLAS calls and the kernels fused around them:
//   forward   y = x·Wᵀ + b (+ReLU)       mat_mul.cu:122-163 (K1 add_bias + K2 sgemm) + K5 ReLU
//   grad_x    gx = g·W (·1[y_prev>0])    mat_mul.cu:175-188 (K3) + activation_function.cu:24-29 (K6)
//   grad_W    gW = gᵀ·x, gb = Σ_m g      mat_mul.cu:195-208 (K4) + neural_network.cu:108-118 (K7)
//
// Design (gfx950):
//  * v_mfma_f32_32x32x2_f32 — exact fp32 (a k-ordered fma chain), 64 FLOP/clk/SIMD, the same
//    numerics class as the reference's fp32 sgemm.  No reduced-precision shortcut.
//  * 256-thread workgroups (4 waves), block tile BM×BN, BK = 32.  Both operands are staged in
//    LDS as [row][k] with a 36-float row pitch: each lane's MFMA fragments for a 32-deep k tile
//    are 16 consecutive floats (k-permutation: lane half h owns k ∈ [16h, 16h+16)), read with
//    ds_read_b128 conflict-free (row·9 mod 16 is a bijection over each 16-lane group).
//  * Operands whose k is not the contiguous dimension (W in grad_x, g and x in grad_W) are
//    transposed on the way into LDS; loads stay 128-B-line coalesced (8 lanes per line).
//  * Register prefetch of tile t+1 overlaps the MFMAs of tile t; one LDS buffer → ≥3 WG/CU.
//  * XCD-aware, bijective blockIdx → tile remap: consecutive tiles (which share the x / g
//    panel) land on the same XCD and its private L2 (MI355X_MICROARCH §Workgroup dispatch).
//  * grad_W reduces over the minibatch (K = B up to 32768): split-K over the grid z-range,
//    f32 atomics into a zeroed output; the bias gradient is the row-sum of the g tile already
//    in LDS, taken by the tn == 0 workgroups (no separate pass over g).
#include "dev.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BK = 32;
constexpr int LDK = BK + 4;       // 36-float row pitch (144 B, 16-B aligned)
constexpr int NT_ = 256;          // threads per workgroup

enum Op { OP_NT = 0, OP_NN = 1, OP_TN = 2 };

struct Args {
    const float* A; const float* B; float* C;
    int M, N, K, lda, ldb, ldc;
    const float* bias; int relu;          // OP_NT epilogue
    const float* mask; int ldmask;        // OP_NN epilogue (post-activation of the previous layer)
    float* gbias;                         // OP_TN: Σ over k of A's rows
    int kchunk, splits;                   // OP_TN split-K
    int tiles_m, tiles_n;
    int vec_a, vec_b;
};

// ---------------------------------------------------------------------------
// Loaders.  "kcont": element (row r, k) at P[r*ld + k]  (x, g in grad_x, W in forward)
//           "mncont": element (row r, k) at P[k*ld + r] (W in grad_x, g and x in grad_W)
// Both fill an LDS image [R][LDK] with zeros outside [0,Rmax) × [kbeg,kend).
// ---------------------------------------------------------------------------
template <int R>
struct Stage {
    static constexpr int ITERS = R * BK / 4 / NT_;
    f32x4 v[ITERS];

    __device__ __forceinline__ void load_kcont(const float* __restrict__ P, int ld, int r0, int Rmax, int k0,
                                               int kend, bool vec, int tid) {
#pragma unroll
        for (int it = 0; it < ITERS; ++it) {
            const int idx = tid + it * NT_;
            const int kq = idx & 7, r = idx >> 3;
            const int gr = r0 + r, gk = k0 + kq * 4;
            f32x4 x = {0.f, 0.f, 0.f, 0.f};
            if (gr < Rmax) {
                const float* p = P + (long)gr * ld + gk;
                if (vec && gk + 3 < kend) {
                    x = *reinterpret_cast<const f32x4*>(p);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (gk + e < kend) x[e] = p[e];
                }
            }
            v[it] = x;
        }
    }
    __device__ __forceinline__ void store_kcont(float* lds, int tid) const {
#pragma unroll
        for (int it = 0; it < ITERS; ++it) {
            const int idx = tid + it * NT_;
            const int kq = idx & 7, r = idx >> 3;
            *reinterpret_cast<f32x4*>(lds + r * LDK + kq * 4) = v[it];
        }
    }

    // lanes: kk_lo = idx&7 (8 k-rows), then R/4 row-quads, then kk_hi → 8 full 128-B lines per wave
    __device__ __forceinline__ static void mn_coords(int idx, int& kk, int& nq) {
        const int kk_lo = idx & 7, rest = idx >> 3;
        nq = rest % (R / 4);
        kk = (rest / (R / 4)) * 8 + kk_lo;
    }
    __device__ __forceinline__ void load_mncont(const float* __restrict__ P, int ld, int r0, int Rmax, int k0,
                                                int kend, bool vec, int tid) {
#pragma unroll
        for (int it = 0; it < ITERS; ++it) {
            int kk, nq;
            mn_coords(tid + it * NT_, kk, nq);
            const int gk = k0 + kk, gr = r0 + nq * 4;
            f32x4 x = {0.f, 0.f, 0.f, 0.f};
            if (gk < kend) {
                const float* p = P + (long)gk * ld + gr;
                if (vec && gr + 3 < Rmax) {
                    x = *reinterpret_cast<const f32x4*>(p);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (gr + e < Rmax) x[e] = p[e];
                }
            }
            v[it] = x;
        }
    }
    __device__ __forceinline__ void store_mncont(float* lds, int tid) const {
#pragma unroll
        for (int it = 0; it < ITERS; ++it) {
            int kk, nq;
            mn_coords(tid + it * NT_, kk, nq);
#pragma unroll
            for (int e = 0; e < 4; ++e) lds[(nq * 4 + e) * LDK + kk] = v[it][e];
        }
    }
};

template <int OP, int BM, int BN, int WARPS_M>
__global__ __launch_bounds__(NT_, 2) void gemm_f32_kernel(Args a) {
    constexpr int WARPS_N = 4 / WARPS_M;
    constexpr int WM = BM / WARPS_M, WN = BN / WARPS_N;
    constexpr int TM = WM / 32, TN = WN / 32;
    static_assert(TM >= 1 && TN >= 1, "wave tile must be a multiple of 32x32");

    __shared__ __attribute__((aligned(16))) float lds[(BM + BN) * LDK];
    float* As = lds;
    float* Bs = lds + BM * LDK;

    // XCD-aware bijective remap of the linear block id (guide §5 "XCD swizzle must be bijective")
    const int nwg = gridDim.x, b = blockIdx.x;
    const int xcd = b & 7, q = nwg >> 3, rr = nwg & 7;
    const int t = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (b >> 3);
    const int tn = t % a.tiles_n;
    const int rest = t / a.tiles_n;
    const int tm = rest % a.tiles_m;
    const int split = rest / a.tiles_m;
    const int m0 = tm * BM, n0 = tn * BN;
    const int kbeg = split * a.kchunk;
    const int kend = min(a.K, kbeg + a.kchunk);

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WARPS_N, wn = w % WARPS_N;
    const int r = lane & 31, h = lane >> 5;

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    // bias-gradient row sums (OP_TN, tn == 0 workgroups only)
    constexpr int TPR = NT_ / BM > 0 ? NT_ / BM : 1;     // threads per A-row
    constexpr int KPT = BK / TPR;                         // k per thread
    const bool do_bsum = OP == OP_TN && a.gbias != nullptr && tn == 0 && (NT_ % BM == 0);
    float bsum = 0.f;

    Stage<BM> sa;
    Stage<BN> sb;
    const bool va = a.vec_a, vb = a.vec_b;

    auto load = [&](int k0) {
        if (OP == OP_TN) sa.load_mncont(a.A, a.lda, m0, a.M, k0, kend, va, tid);
        else             sa.load_kcont(a.A, a.lda, m0, a.M, k0, kend, va, tid);
        if (OP == OP_NT) sb.load_kcont(a.B, a.ldb, n0, a.N, k0, kend, vb, tid);
        else             sb.load_mncont(a.B, a.ldb, n0, a.N, k0, kend, vb, tid);
    };

    if (kbeg < kend) load(kbeg);
    for (int k0 = kbeg; k0 < kend; k0 += BK) {
        if (OP == OP_TN) sa.store_mncont(As, tid); else sa.store_kcont(As, tid);
        if (OP == OP_NT) sb.store_kcont(Bs, tid);  else sb.store_mncont(Bs, tid);
        __syncthreads();
        if (k0 + BK < kend) load(k0 + BK);        // in flight during this tile's MFMAs

        if (do_bsum) {
            const int row = tid / TPR, seg = tid % TPR;
#pragma unroll
            for (int kk = 0; kk < KPT; ++kk) bsum += As[row * LDK + seg * KPT + kk];
        }

#pragma unroll
        for (int half = 0; half < 2; ++half) {
            f32x4 fa[TM][2], fb[TN][2];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const float* p = As + (wm * WM + i * 32 + r) * LDK + h * 16 + half * 8;
                fa[i][0] = *reinterpret_cast<const f32x4*>(p);
                fa[i][1] = *reinterpret_cast<const f32x4*>(p + 4);
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const float* p = Bs + (wn * WN + j * 32 + r) * LDK + h * 16 + half * 8;
                fb[j][0] = *reinterpret_cast<const f32x4*>(p);
                fb[j][1] = *reinterpret_cast<const f32x4*>(p + 4);
            }
#pragma unroll
            for (int s = 0; s < 8; ++s)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][s >> 2][s & 3], fb[j][s >> 2][s & 3],
                                                                         acc[i][j], 0, 0, 0);
        }
        __syncthreads();
    }

    if (do_bsum) {
#pragma unroll
        for (int o = TPR / 2; o > 0; o >>= 1) bsum += __shfl_xor(bsum, o, 64);
        const int row = tid / TPR, seg = tid % TPR;
        if (seg == 0 && m0 + row < a.M) {
            if (a.splits > 1) atomicAdd(a.gbias + m0 + row, bsum);
            else a.gbias[m0 + row] = bsum;
        }
    }

    // epilogue: 32x32 C/D map — col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int col = n0 + wn * WN + j * 32 + r;
            if (col >= a.N) continue;
            float bcol = 0.f;
            if (OP == OP_NT && a.bias) bcol = a.bias[col];
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int row = m0 + wm * WM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
                if (row >= a.M) continue;
                float v = acc[i][j][e];
                float* dst = a.C + (long)row * a.ldc + col;
                if (OP == OP_NT) {
                    v += bcol;
                    if (a.relu) v = v > 0.f ? v : 0.f;
                    *dst = v;
                } else if (OP == OP_NN) {
                    if (a.mask && !(a.mask[(long)row * a.ldmask + col] > 0.f)) v = 0.f;
                    *dst = v;
                } else {
                    if (a.splits > 1) atomicAdd(dst, v);
                    else *dst = v;
                }
            }
        }
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

template <int OP, int BM, int BN, int WARPS_M>
void launch(Args a) {
    a.tiles_m = ppo_divup(a.M, BM);
    a.tiles_n = ppo_divup(a.N, BN);
    if (a.splits < 1) a.splits = 1;
    const long grid = (long)a.tiles_m * a.tiles_n * a.splits;
    PPO_REQUIRE(grid > 0 && grid < (1L << 31), "gemm: grid out of range");
    hipLaunchKernelGGL((gemm_f32_kernel<OP, BM, BN, WARPS_M>), dim3((unsigned)grid), dim3(NT_), 0,
                       ppo::stream(), a);
    PPO_LAUNCH_CHECK();
}

// Tile selection: skinny-N (layer outputs 1 / A, Pendulum input 3), skinny-M, or 128x128.
template <int OP>
void dispatch(Args& a) {
    if (a.N <= 32 && a.M > 32)       launch<OP, 256, 32, 4>(a);
    else if (a.M <= 32 && a.N > 32)  launch<OP, 32, 256, 1>(a);
    else if (a.M <= 64 || a.N <= 64) launch<OP, 64, 64, 2>(a);
    else                             launch<OP, 128, 128, 2>(a);
}

int tile_m_for(int M, int N) { return (N <= 32 && M > 32) ? 256 : (M <= 32 && N > 32) ? 32 : (M <= 64 || N <= 64) ? 64 : 128; }
int tile_n_for(int M, int N) { return (N <= 32 && M > 32) ? 32 : (M <= 32 && N > 32) ? 256 : (M <= 64 || N <= 64) ? 64 : 128; }

}  // namespace

extern "C" {

void phip_linear_fwd(float* y, const float* x, const float* W, const float* b, int m, int n, int l, int relu) {
    if (m <= 0 || l <= 0) return;
    PPO_REQUIRE(y && x && W && n > 0, "phip_linear_fwd: null operand");
    Args a{};
    a.A = x; a.lda = n; a.B = W; a.ldb = n; a.C = y; a.ldc = l;
    a.M = m; a.N = l; a.K = n; a.kchunk = n; a.splits = 1;
    a.bias = b; a.relu = relu;
    a.vec_a = (n % 4 == 0) && aligned16(x);
    a.vec_b = (n % 4 == 0) && aligned16(W);
    ppo::ProfScope ps(PPO_K_GEMM, 2.0 * m * n * l);
    dispatch<OP_NT>(a);
}

void phip_linear_bwd_x(float* gx, const float* g, const float* W, const float* mask, int m, int n, int l) {
    if (m <= 0 || n <= 0) return;
    PPO_REQUIRE(gx && g && W && l > 0, "phip_linear_bwd_x: null operand");
    Args a{};
    a.A = g; a.lda = l; a.B = W; a.ldb = n; a.C = gx; a.ldc = n;
    a.M = m; a.N = n; a.K = l; a.kchunk = l; a.splits = 1;
    a.mask = mask; a.ldmask = n;
    a.vec_a = (l % 4 == 0) && aligned16(g);
    a.vec_b = (n % 4 == 0) && aligned16(W);
    ppo::ProfScope ps(PPO_K_GEMM, 2.0 * m * n * l);
    dispatch<OP_NN>(a);
}

void phip_linear_bwd_w(float* gW, float* gb, const float* g, const float* x, int m, int n, int l) {
    if (l <= 0 || n <= 0) return;
    PPO_REQUIRE(gW && g && x, "phip_linear_bwd_w: null operand");
    Args a{};
    a.A = g; a.lda = l; a.B = x; a.ldb = n; a.C = gW; a.ldc = n;
    a.M = l; a.N = n; a.K = m;
    a.gbias = gb;
    a.vec_a = (l % 4 == 0) && aligned16(g);
    a.vec_b = (n % 4 == 0) && aligned16(x);
    // split-K over the minibatch: aim for ~2 workgroups per CU, ≥ 8 k-tiles per split
    const long tiles = (long)ppo_divup(l, tile_m_for(l, n)) * ppo_divup(n, tile_n_for(l, n));
    int splits = (int)((512 + tiles - 1) / tiles);
    const int max_splits = m / (8 * BK) > 0 ? m / (8 * BK) : 1;
    if (splits > max_splits) splits = max_splits;
    if (splits < 1) splits = 1;
    int kchunk = ppo_divup(m, splits);
    kchunk = ppo_divup(kchunk, BK) * BK;
    splits = ppo_divup(m, kchunk);
    a.kchunk = kchunk; a.splits = splits;
    if (m <= 0) {   // empty batch: gradients are zero
        phip_memset(gW, 0, sizeof(float) * (size_t)l * n);
        if (gb) phip_memset(gb, 0, sizeof(float) * (size_t)l);
        return;
    }
    if (splits > 1) {
        phip_memset(gW, 0, sizeof(float) * (size_t)l * n);
        if (gb) phip_memset(gb, 0, sizeof(float) * (size_t)l);
    }
    ppo::ProfScope ps(PPO_K_GEMM, 2.0 * m * n * l);
    dispatch<OP_TN>(a);
}

}  // extern "C"
