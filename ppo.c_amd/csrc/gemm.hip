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

constexpr int NT_ = 256;          // threads per workgroup

enum Op { OP_NT = 0, OP_NN = 1, OP_TN = 2 };

struct Args {
    const float* A; const float* B; float* C;
    int M, N, K, lda, ldb, ldc;
    const float* bias; int relu;          // OP_NT epilogue
    const float* mask; int ldmask;        // OP_NN epilogue (post-activation of the previous layer)
    const int* ridx;                      // OP_NT: A row r is memory row ridx[r] (fused gather)
    float* acopy;                         // OP_NT: tn == 0 workgroups write the gathered A rows here
    unsigned* bits_out;                   // OP_NT + relu: bit (row, col) = y > 0, rows of wpr words
    const unsigned* bits_in;              // OP_NN: the ReLU′ mask as bits (replaces `mask`)
    int wpr;                              // words per row of a bit mask = ⌈N/32⌉
    float* gbias;                         // OP_TN: Σ over k of A's rows
    int kchunk, splits;                   // OP_TN split-K
    int tiles_m, tiles_n;
    int vec_a, vec_b;
    int flags;                            // experiment bits (ppo_gemm_flags): 1 = s_setprio around MFMAs
};

// ---------------------------------------------------------------------------
// Operand staging.  An operand tile covers R rows (of the output's M or N) × BK of k.
//  "kcont"  (MN = false): element (row r, k) at P[r*ld + k]   (x and W in forward, g in grad_x).
//           LDS image [R][BK+4]; each lane's fragments for one k-tile are KH = BK/2 consecutive k
//           (lane half h owns k ∈ [h·KH, h·KH + KH)), read 4 at a time with ds_read_b128 —
//           conflict-free because row·(BK+4)/4 mod 16 is a bijection over each 16-lane group.
//  "mncont" (MN = true):  element (row r, k) at P[k*ld + r]   (W in grad_x, g and x in grad_W).
//           LDS image [BK][R]: the loaded float4 (4 consecutive rows of one k) is stored as-is
//           with ds_write_b128, and a fragment is one ds_read_b32 per k (32 consecutive rows per
//           lane half: conflict-free).  No transpose through registers.
//
// VEC: the contiguous extent (kend for kcont, Rmax for mncont) and the leading dimension are
// multiples of 4 and the base is 16-B aligned, so every float4 lies wholly inside or wholly outside
// the operand.  The load address is then clamped into the operand: the k-loop has no branches (the
// guarded scalar form compiles to ~20 exec-mask branches per k-tile).  Rows past Rmax only feed
// output rows/columns that are never stored, so they need no masking; k past kend must be zero and
// is masked by a select at LDS-store time — never right after the load, where it would make the
// wave wait for its prefetch before the current tile's MFMAs.  !VEC keeps the guarded scalar form
// for odd shapes (S = 3, A = 17).
// ---------------------------------------------------------------------------
template <int R, int BK, bool MN>
struct Stage {
    static constexpr int LDK = BK + 4;                     // kcont row pitch (floats)
    static constexpr int IMG = MN ? BK * R : R * LDK;      // floats per LDS image
    static constexpr int TOTAL = R * BK / 4;               // float4s per tile
    static constexpr int ITERS = (TOTAL + NT_ - 1) / NT_;
    static constexpr int KQ = BK / 4;                      // float4s per kcont row
    static constexpr int RQ = R / 4;                       // float4s per mncont k-row
    static_assert(R % 4 == 0, "tile rows");
    f32x4 v[ITERS];
    bool kok[ITERS];                                       // element's k inside [k0, kend)
    int src[ITERS];                                        // kcont: memory row of tile row (gather)

    // kcont rows are fixed for the whole k-loop: resolve them (clamp, optional row indirection
    // `ridx` — the minibatch gather fused into layer 0) once, before it.
    __device__ __forceinline__ void prep(const int* __restrict__ ridx, int r0, int Rmax, int tid) {
#pragma unroll
        for (int it = 0; it < ITERS; ++it) {
            int row, k;
            coords(tid + it * NT_, row, k);
            const int gr = min(r0 + row, Rmax - 1);
            src[it] = ridx ? ridx[gr] : gr;
        }
    }

    __device__ __forceinline__ static void coords(int idx, int& row, int& k) {
        if (MN) { row = (idx % RQ) * 4; k = idx / RQ; }    // lanes sweep a k-row: full 128-B lines
        else    { row = idx / KQ; k = (idx % KQ) * 4; }
    }

    template <bool VEC>
    __device__ __forceinline__ void load(const float* __restrict__ P, int ld, int r0, int Rmax, int k0, int kend,
                                         int tid) {
#pragma unroll
        for (int it = 0; it < ITERS; ++it) {
            const int idx = tid + it * NT_;
            f32x4 x = {0.f, 0.f, 0.f, 0.f};
            kok[it] = true;
            if (TOTAL % NT_ == 0 || idx < TOTAL) {
                int row, k;
                coords(idx, row, k);
                const int gr = r0 + row, gk = k0 + k;
                if (VEC) {
                    kok[it] = gk < kend;
                    const float* p = MN ? P + (long)(gk < kend ? gk : kend - 1) * ld + (gr < Rmax ? gr : Rmax - 4)
                                        : P + (long)src[it] * ld + (gk < kend ? gk : kend - 4);
                    x = *reinterpret_cast<const f32x4*>(p);
                } else if (MN) {
                    if (gk < kend) {
                        const float* p = P + (long)gk * ld + gr;
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            if (gr + e < Rmax) x[e] = p[e];
                    }
                } else if (gr < Rmax) {
                    const float* p = P + (long)src[it] * ld + gk;
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (gk + e < kend) x[e] = p[e];
                }
            }
            v[it] = x;
        }
    }

    // kcont: write the staged tile (rows < Rmax, k < kend) to dst[row*ldd + k] — the gathered
    // minibatch that layer 0's grad_W reads back.  Called at LDS-store time (data already waited for).
    __device__ __forceinline__ void copy_out(float* __restrict__ dst, int ldd, int r0, int Rmax, int k0, int kend,
                                             int tid) const {
#pragma unroll
        for (int it = 0; it < ITERS; ++it) {
            const int idx = tid + it * NT_;
            if (TOTAL % NT_ == 0 || idx < TOTAL) {
                int row, k;
                coords(idx, row, k);
                const int gr = r0 + row, gk = k0 + k;
                if (gr >= Rmax) continue;
                float* q = dst + (long)gr * ldd + gk;
                if (gk + 3 < kend && ((ldd & 3) == 0)) {
                    *reinterpret_cast<f32x4*>(q) = v[it];
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (gk + e < kend) q[e] = v[it][e];
                }
            }
        }
    }

    __device__ __forceinline__ void store(float* img, int tid) const {
#pragma unroll
        for (int it = 0; it < ITERS; ++it) {
            const int idx = tid + it * NT_;
            if (TOTAL % NT_ == 0 || idx < TOTAL) {
                int row, k;
                coords(idx, row, k);
                const f32x4 z = {0.f, 0.f, 0.f, 0.f};
                const f32x4 x = kok[it] ? v[it] : z;
                *reinterpret_cast<f32x4*>(img + (MN ? k * R + row : row * LDK + k)) = x;
            }
        }
    }

    // fragments of k-group q4 (k = kb + s, s = 0..3, kb = h·KH + 4·q4) for image row `row`
    __device__ __forceinline__ static f32x4 frag(const float* img, int row, int kb) {
        if (MN) {
            f32x4 f;
#pragma unroll
            for (int s = 0; s < 4; ++s) f[s] = img[(kb + s) * R + row];
            return f;
        }
        return *reinterpret_cast<const f32x4*>(img + row * LDK + kb);
    }

    // Σ over the tile's k of image row `row`, k ∈ [k_lo, k_lo + n)
    __device__ __forceinline__ static float rowsum(const float* img, int row, int k_lo, int n) {
        float t = 0.f;
        for (int kk = 0; kk < n; ++kk) t += MN ? img[(k_lo + kk) * R + row] : img[row * LDK + k_lo + kk];
        return t;
    }
};

// Workgroups per CU the tile is built for: BK=16 128x128 fits ≤128 VGPRs → 4 (16 waves), BK=32
// needs 3, 256x128 needs 2.  With DBUF the LDS image doubles (4 × 40 KiB = the whole 160 KiB).
constexpr int min_waves(int area, int bk) { return area >= 256 * 128 ? 2 : (bk >= 32 ? 3 : 4); }

// DBUF: two LDS images; the staged tile t+1 is written into the idle image behind tile t's MFMAs,
// so each k-tile needs one barrier instead of two.
template <int OP, int BM, int BN, int BK, bool DBUF>
constexpr int lds_floats() {
    return (DBUF ? 2 : 1) * (Stage<BM, BK, OP == OP_TN>::IMG + Stage<BN, BK, OP != OP_NT>::IMG);
}

// One workgroup's output tile: block b of an nwg-block grid (the kernels below pass their own
// block id, or an offset one when two GEMMs share a launch).
template <int OP, int BM, int BN, int WARPS_M, int BK, bool VEC, bool DBUF>
__device__ __forceinline__ void gemm_tile(const Args& a, const int b, const int nwg, float* __restrict__ lds) {
    constexpr int WARPS_N = 4 / WARPS_M;
    constexpr int WM = BM / WARPS_M, WN = BN / WARPS_N;
    constexpr int TM = WM / 32, TN = WN / 32;
    constexpr int KH = BK / 2;         // k per lane-half per tile (k-permutation)
    constexpr bool A_MN = OP == OP_TN, B_MN = OP != OP_NT;
    using SA = Stage<BM, BK, A_MN>;
    using SB = Stage<BN, BK, B_MN>;
    constexpr int IMG = SA::IMG + SB::IMG;
    static_assert(TM >= 1 && TN >= 1, "wave tile must be a multiple of 32x32");
    static_assert(BK == 16 || BK == 32, "BK");

    // XCD-aware bijective remap of the linear block id (guide §5 "XCD swizzle must be bijective")
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
    constexpr int KPT = BK / TPR > 0 ? BK / TPR : 1;      // k per thread
    const bool do_bsum = OP == OP_TN && a.gbias != nullptr && tn == 0 && (NT_ % BM == 0) && BK >= TPR;
    float bsum = 0.f;

    SA sa;
    SB sb;

    if (!A_MN) sa.prep(OP == OP_NT ? a.ridx : nullptr, m0, a.M, tid);
    if (!B_MN) sb.prep(nullptr, n0, a.N, tid);
    const bool do_copy = OP == OP_NT && a.acopy != nullptr && tn == 0;

    auto load = [&](int k0) {
        sa.template load<VEC>(a.A, a.lda, m0, a.M, k0, kend, tid);
        sb.template load<VEC>(a.B, a.ldb, n0, a.N, k0, kend, tid);
    };
    auto store = [&](float* img, int k0) {
        if (do_copy) sa.copy_out(a.acopy, a.K, m0, a.M, k0, kend, tid);
        sa.store(img, tid);
        sb.store(img + SA::IMG, tid);
    };
    auto compute = [&](const float* img) {
        const float* As = img;
        const float* Bs = img + SA::IMG;
        if (do_bsum) bsum += SA::rowsum(As, tid / TPR, (tid % TPR) * KPT, KPT);
        // s_setprio 1 around the MFMA block: +1.5–4 % on forward, grad_x and the 64×64 grad_W tiles,
        // −1…3 % on 128×128 grad_W tiles (tools/gemm_sweep.py --flags 0,1, profiles/r01_gemm_sweep_prio.txt);
        // flag bit 0 inverts the default for experiments
        constexpr bool PRIO = !(OP == OP_TN && BM * BN >= 128 * 128);
        const bool prio = PRIO != ((a.flags & 1) != 0);
        if (prio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int q4 = 0; q4 < KH / 4; ++q4) {
            f32x4 fa[TM], fb[TN];
            const int kb = h * KH + q4 * 4;
#pragma unroll
            for (int i = 0; i < TM; ++i) fa[i] = SA::frag(As, wm * WM + i * 32 + r, kb);
#pragma unroll
            for (int j = 0; j < TN; ++j) fb[j] = SB::frag(Bs, wn * WN + j * 32 + r, kb);
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
        }
        if (prio) __builtin_amdgcn_s_setprio(0);
    };

    if (DBUF) {
        int cur = 0;
        if (kbeg < kend) {
            load(kbeg);
            store(lds, kbeg);
        }
        __syncthreads();
        for (int k0 = kbeg; k0 < kend; k0 += BK) {
            const bool more = k0 + BK < kend;
            if (more) load(k0 + BK);               // in flight during this tile's MFMAs
            compute(lds + cur * IMG);
            if (more) store(lds + (cur ^ 1) * IMG, k0 + BK);  // idle image: its last readers passed the barrier
            __syncthreads();
            cur ^= 1;
        }
    } else {
        if (kbeg < kend) load(kbeg);
        for (int k0 = kbeg; k0 < kend; k0 += BK) {
            store(lds, k0);
            __syncthreads();
            if (k0 + BK < kend) load(k0 + BK);        // in flight during this tile's MFMAs
            compute(lds);
            __syncthreads();
        }
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

    // epilogue: 32x32 C/D map — col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5).
    // Every global load an output block needs (bias, ReLU′ mask) is issued as one batch before the
    // block's first store: interleaved with the stores, the compiler cannot prove they do not alias
    // and serialises one load→wait→store round trip per element.
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int c0 = n0 + wn * WN + j * 32;            // 32-aligned: one bit-mask word per row
            const int col = c0 + r;
            const int r0 = m0 + wm * WM + i * 32 + 4 * h;
            const bool col_ok = col < a.N;
            const int colc = col_ok ? col : a.N - 1;
            float bcol = 0.f;
            if (OP == OP_NT && a.bias) bcol = a.bias[colc];
            bool keep[16];
            if (OP == OP_NN) {                                // mode is wave-uniform: loads unconditional
                if (a.bits_in) {
                    unsigned wv[16];
#pragma unroll
                    for (int e = 0; e < 16; ++e)
                        wv[e] = a.bits_in[(long)min(r0 + (e & 3) + 8 * (e >> 2), a.M - 1) * a.wpr + (c0 >> 5)];
#pragma unroll
                    for (int e = 0; e < 16; ++e) keep[e] = (wv[e] >> r) & 1u;
                } else if (a.mask) {
                    float mv[16];
#pragma unroll
                    for (int e = 0; e < 16; ++e)
                        mv[e] = a.mask[(long)min(r0 + (e & 3) + 8 * (e >> 2), a.M - 1) * a.ldmask + colc];
#pragma unroll
                    for (int e = 0; e < 16; ++e) keep[e] = mv[e] > 0.f;
                } else {
#pragma unroll
                    for (int e = 0; e < 16; ++e) keep[e] = true;
                }
            }
            unsigned word = 0;                                 // OP_NT bits: lane e (+32) keeps row e's word
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int row = r0 + (e & 3) + 8 * (e >> 2);
                const bool ok = col_ok && row < a.M;
                float v = acc[i][j][e];
                float* dst = a.C + (long)row * a.ldc + col;
                if (OP == OP_NT) {
                    v += bcol;
                    if (a.relu) v = v > 0.f ? v : 0.f;
                    if (ok) *dst = v;
                    if (a.bits_out) {                          // wave-uniform branch: ballot stays converged
                        const unsigned long long b = __ballot(ok && v > 0.f);
                        if (r == e) word = h ? (unsigned)(b >> 32) : (unsigned)b;
                    }
                } else if (OP == OP_NN) {
                    if (ok) *dst = keep[e] ? v : 0.f;
                } else if (ok) {
                    if (a.splits > 1) atomicAdd(dst, v);
                    else *dst = v;
                }
            }
            if (OP == OP_NT && a.bits_out && r < 16) {
                const int row = r0 + (r & 3) + 8 * (r >> 2);
                if (row < a.M && c0 < a.N) a.bits_out[(long)row * a.wpr + (c0 >> 5)] = word;
            }
        }
}

template <int OP, int BM, int BN, int WARPS_M, int BK, bool VEC, bool DBUF>
__global__ __launch_bounds__(NT_, min_waves(BM * BN, BK)) void gemm_f32_kernel(Args a) {
    __shared__ __attribute__((aligned(16))) float lds[lds_floats<OP, BM, BN, BK, DBUF>()];
    gemm_tile<OP, BM, BN, WARPS_M, BK, VEC, DBUF>(a, blockIdx.x, gridDim.x, lds);
}

// grad_W and grad_x of one layer in one launch (both 128x128/BK16, vector loads): blocks
// [0, g1) are grad_W tiles, the rest grad_x tiles.  The two products are independent, so grad_x
// tiles fill the CUs that grad_W tiles leave while their split-K atomics drain — the lock-step
// tail of two back-to-back one-round grids becomes one.
// Instantiated for the hidden layers (both 128x128, vector loads) and the output layer (grad_W on
// 32x128 tiles, grad_x on 128x128; K = A is not a multiple of 4: guarded loads).
template <int BMW, int BNW, int WMW, bool VW, int BMX, int BNX, int WMX, bool VX>
__global__ __launch_bounds__(NT_, 4) void gemm_pair_kernel(Args aw, Args ax, int g1) {
    constexpr int LW = lds_floats<OP_TN, BMW, BNW, 16, false>(), LX = lds_floats<OP_NN, BMX, BNX, 16, false>();
    __shared__ __attribute__((aligned(16))) float lds[LW > LX ? LW : LX];
    if ((int)blockIdx.x < g1) gemm_tile<OP_TN, BMW, BNW, WMW, 16, VW, false>(aw, blockIdx.x, g1, lds);
    else gemm_tile<OP_NN, BMX, BNX, WMX, 16, VX, false>(ax, blockIdx.x - g1, gridDim.x - g1, lds);
}

// ---------------------------------------------------------------------------
// Small-M products (rollout steps over E environments, the reference's B = 64 minibatches).  The
// 128-row tiles of gemm_f32_kernel would put a 64 × 512 product on 8–16 workgroups that each walk
// the whole K serially (17 µs for a 64×512×512 grad_x).  Here a 512-thread workgroup owns a 32 × 32
// output block and splits K over its 8 waves; each wave streams its K-slice straight from global
// memory into MFMA operands (lane half h takes 32 consecutive k of each 64-deep chunk: float4 loads
// along a k-contiguous operand, one coalesced scalar per k across the 32 lanes of a row-contiguous
// one; no LDS staging), and the 8 partial 32×32 accumulators are summed through LDS before the
// fused epilogue.  Same fp32 MFMA numerics.
//   NT forward  A(r, k) = x[ridx(r)·lda + k]   B(c, k) = W[c·ldb + k]   + bias, ReLU, bits, gathered copy
//   NN grad_x   A(r, k) = g[r·lda + k]         B(c, k) = W[k·ldb + c]   ⊙ ReLU′ (bits or mask)
//   TN grad_W   A(r, k) = g[k·lda + r]         B(c, k) = x[k·ldb + c]   whole K per workgroup (plain
//               stores, no split-K) + the bias gradient Σ_k A(r, k) from the tn == 0 column of blocks
// ---------------------------------------------------------------------------
constexpr int SM_WAVES = 8;

template <int OP, bool VEC>
__global__ __launch_bounds__(64 * SM_WAVES) void gemm_smallm_kernel(Args a) {
    __shared__ float red[SM_WAVES][32 * 33];
    __shared__ float bred[SM_WAVES][64];
    const int tiles_n = a.tiles_n;
    const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
    const int m0 = tm * 32, n0 = tn * 32;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int K = a.K;
    const int kslice = ((K + SM_WAVES - 1) / SM_WAVES + 63) / 64 * 64;   // per-wave K range, 64-aligned
    const int kb = w * kslice, ke = min(K, kb + kslice);
    const float* __restrict__ PA = a.A;
    const float* __restrict__ PB = a.B;
    const int arow = min(m0 + r, a.M - 1), bcol = min(n0 + r, a.N - 1);
    const long abase = OP == OP_TN ? (long)arow : (long)(OP == OP_NT && a.ridx ? a.ridx[arow] : arow) * a.lda;
    const long bbase = OP == OP_NT ? (long)bcol * a.ldb : (long)bcol;
    const bool copy = OP == OP_NT && a.acopy != nullptr && tn == 0 && m0 + r < a.M;
    const bool bsum = OP == OP_TN && a.gbias != nullptr && tn == 0;
    float bpart = 0.f;

    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    for (int k0 = kb; k0 < ke; k0 += 64) {
        const int kl = k0 + 32 * h;                      // this lane's 32 k values
        float av[32], bv[32];
        if (OP != OP_TN && VEC) {                        // A k-contiguous: float4 loads
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int kq = kl + 4 * q;
                const bool ok = kq < ke;
                const f32x4 ta = *reinterpret_cast<const f32x4*>(PA + abase + (ok ? kq : 0));
                if (copy && ok) *reinterpret_cast<f32x4*>(a.acopy + (long)(m0 + r) * K + kq) = ta;
#pragma unroll
                for (int e = 0; e < 4; ++e) av[4 * q + e] = ok ? ta[e] : 0.f;
            }
        } else if (OP != OP_TN) {
#pragma unroll
            for (int q = 0; q < 32; ++q) {
                const bool ok = kl + q < ke;
                av[q] = ok ? PA[abase + kl + q] : 0.f;
                if (copy && ok) a.acopy[(long)(m0 + r) * K + kl + q] = av[q];
            }
        } else {                                         // A row-contiguous: one scalar per k
#pragma unroll
            for (int q = 0; q < 32; ++q) {
                const bool ok = kl + q < ke;
                av[q] = ok ? PA[abase + (long)(ok ? kl + q : 0) * a.lda] : 0.f;
            }
        }
        if (OP == OP_NT && VEC) {                        // B k-contiguous
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int kq = kl + 4 * q;
                const bool ok = kq < ke;
                const f32x4 tb = *reinterpret_cast<const f32x4*>(PB + bbase + (ok ? kq : 0));
#pragma unroll
                for (int e = 0; e < 4; ++e) bv[4 * q + e] = ok ? tb[e] : 0.f;
            }
        } else if (OP == OP_NT) {
#pragma unroll
            for (int q = 0; q < 32; ++q) bv[q] = kl + q < ke ? PB[bbase + kl + q] : 0.f;
        } else {                                         // B row-contiguous
#pragma unroll
            for (int q = 0; q < 32; ++q) {
                const bool ok = kl + q < ke;
                bv[q] = ok ? PB[bbase + (long)(ok ? kl + q : 0) * a.ldb] : 0.f;
            }
        }
        if (bsum) {
#pragma unroll
            for (int q = 0; q < 32; ++q) bpart += av[q];
        }
#pragma unroll
        for (int q = 0; q < 32; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[q], bv[q], acc, 0, 0, 0);
    }
    // C/D map: col = r, row = (e&3) + 8(e>>2) + 4h
#pragma unroll
    for (int e = 0; e < 16; ++e) red[w][((e & 3) + 8 * (e >> 2) + 4 * h) * 33 + r] = acc[e];
    if (bsum) bred[w][h * 32 + r] = bpart;
    __syncthreads();
    if (bsum && threadIdx.x < 32) {                      // bias gradient of row m0 + r: Σ over all k
        float t = 0.f;
        for (int q = 0; q < SM_WAVES; ++q) t += bred[q][threadIdx.x] + bred[q][32 + threadIdx.x];
        if (m0 + (int)threadIdx.x < a.M) a.gbias[m0 + threadIdx.x] = t;
    }
    if (w == 0) {
        const int col = n0 + r;
        const bool col_ok = col < a.N;
        const float bc = (OP == OP_NT && a.bias && col_ok) ? a.bias[col] : 0.f;
        unsigned word = 0;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int rr = (e & 3) + 8 * (e >> 2) + 4 * h;
            float v = 0.f;
#pragma unroll
            for (int q = 0; q < SM_WAVES; ++q) v += red[q][rr * 33 + r];
            const int row = m0 + rr;
            const bool ok = col_ok && row < a.M;
            if (OP == OP_NT) {
                v += bc;
                if (a.relu) v = v > 0.f ? v : 0.f;
                if (ok) a.C[(long)row * a.ldc + col] = v;
                if (a.bits_out) {
                    const unsigned long long bb = __ballot(ok && v > 0.f);
                    if (r == e) word = h ? (unsigned)(bb >> 32) : (unsigned)bb;
                }
            } else if (OP == OP_NN) {
                if (ok) {
                    bool keep = true;
                    if (a.bits_in) keep = (a.bits_in[(long)row * a.wpr + (n0 >> 5)] >> r) & 1u;
                    else if (a.mask) keep = a.mask[(long)row * a.ldmask + col] > 0.f;
                    a.C[(long)row * a.ldc + col] = keep ? v : 0.f;
                }
            } else if (ok) {
                a.C[(long)row * a.ldc + col] = v;
            }
        }
        if (OP == OP_NT && a.bits_out && r < 16) {
            const int row = m0 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (row < a.M && n0 < a.N) a.bits_out[(long)row * a.wpr + (n0 >> 5)] = word;
        }
    }
}

template <int OP>
void launch_smallm(Args a, bool vec) {
    a.tiles_n = ppo_divup(a.N, 32);
    const long grid = (long)ppo_divup(a.M, 32) * a.tiles_n;
    PPO_REQUIRE(grid > 0 && grid < (1L << 31), "gemm (small M): grid out of range");
    if (vec) PPO_TIMED_LAUNCH((gemm_smallm_kernel<OP, true>), dim3((unsigned)grid), dim3(64 * SM_WAVES), 0, ppo::stream(), a);
    else PPO_TIMED_LAUNCH((gemm_smallm_kernel<OP, false>), dim3((unsigned)grid), dim3(64 * SM_WAVES), 0, ppo::stream(), a);
    PPO_LAUNCH_CHECK();
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

int g_flags = 0;               // experiment bits passed to every tiled launch (ppo_gemm_flags)

template <int OP, int BM, int BN, int WARPS_M, int BK, bool DBUF>
void launch(Args a) {
    a.tiles_m = ppo_divup(a.M, BM);
    a.tiles_n = ppo_divup(a.N, BN);
    if (a.splits < 1) a.splits = 1;
    a.flags = g_flags;
    const long grid = (long)a.tiles_m * a.tiles_n * a.splits;
    PPO_REQUIRE(grid > 0 && grid < (1L << 31), "gemm: grid out of range");
    if (a.vec_a && a.vec_b)
        PPO_TIMED_LAUNCH((gemm_f32_kernel<OP, BM, BN, WARPS_M, BK, true, DBUF>), dim3((unsigned)grid), dim3(NT_),
                           0, ppo::stream(), a);
    else
        PPO_TIMED_LAUNCH((gemm_f32_kernel<OP, BM, BN, WARPS_M, BK, false, DBUF>), dim3((unsigned)grid), dim3(NT_),
                           0, ppo::stream(), a);
    PPO_LAUNCH_CHECK();
}

// Tile configurations: {BM, BN, WARPS_M, BK, DBUF}
struct TileCfg { int bm, bn, wm, bk, dbuf; };
constexpr TileCfg kCfgs[] = {
    {128, 128, 2, 16, 0},    // 0: main tile, 4 waves of 64x64, ≤128 VGPRs → 4 WG/CU
    {128, 128, 2, 32, 0},    // 1: main tile, deeper k-step
    {128, 32, 4, 16, 0},     // 2: skinny N (layer outputs 1 / A, tiny inputs)
    {32, 128, 1, 16, 0},     // 3: skinny M (grad_W of the output layer)
    {64, 64, 2, 16, 0},      // 4: small problems (Pendulum-sized layers)
    {128, 64, 2, 16, 0},     // 5: 4 waves of 64x32
    {256, 128, 4, 16, 0},    // 6: 4 waves of 64x128
    {128, 128, 2, 16, 1},    // 7: main tile, double-buffered LDS (one barrier per k-tile)
    {128, 64, 2, 16, 1},     // 8: 128x64, double-buffered
    {64, 64, 2, 32, 1},      // 9: 64x64 BK32 double-buffered (grad_W: small partial tiles)
    {128, 32, 4, 32, 0},     // 10: skinny N, BK32: twice the bytes in flight per workgroup (the output
                             //     layer's forward runs one workgroup per CU: latency-bound)
};
constexpr int kNumCfgs = sizeof(kCfgs) / sizeof(kCfgs[0]);
int g_force_cfg = -1;          // tuning override (ppo_gemm_tune)
int g_splitk_override = 0;     // tuning override of the split-K workgroup target (0 = per shape)

template <int OP>
void launch_cfg(int c, const Args& a) {
    switch (c) {
        case 0: launch<OP, 128, 128, 2, 16, false>(a); break;
        case 1: launch<OP, 128, 128, 2, 32, false>(a); break;
        case 2: launch<OP, 128, 32, 4, 16, false>(a); break;
        case 3: launch<OP, 32, 128, 1, 16, false>(a); break;
        case 4: launch<OP, 64, 64, 2, 16, false>(a); break;
        case 5: launch<OP, 128, 64, 2, 16, false>(a); break;
        case 6: launch<OP, 256, 128, 4, 16, false>(a); break;
        case 7: launch<OP, 128, 128, 2, 16, true>(a); break;
        case 8: launch<OP, 128, 64, 2, 16, true>(a); break;
        case 9: launch<OP, 64, 64, 2, 32, true>(a); break;
        default: launch<OP, 128, 32, 4, 32, false>(a); break;
    }
}

// Measured on MI355X (tools/gemm_sweep.py, profiles/r01_gemm_sweep_*): 128x128/BK16 at 4 WG/CU
// for large forward / grad_x grids; 128x64 when a 128x128 grid would not give every CU two
// workgroups; skinny tiles for the 1- and A-wide output layers.  grad_W (split-K, f32 atomics):
// 128x128 tiles at ~512 workgroups when the output has ≥ 16 such tiles and 128 | N, else 64x64
// tiles at ~2048 workgroups (fewer atomic bytes per CU than wider tiles at the same occupancy).
int pick_cfg(int op, int M, int N, int* splitk_target = nullptr) {
    if (splitk_target) *splitk_target = 1024;
    if (g_force_cfg >= 0 && g_force_cfg < kNumCfgs) return g_force_cfg;
    if (N <= 32 && M > 32) return op == OP_NT ? 10 : 2;   // output-layer forward: BK32 (17.3 vs 21.6 µs at C4)
    if (M <= 32 && N > 32) return 3;
    if (M <= 64 || N <= 64) return 4;
    const long tiles = (long)ppo_divup(M, 128) * ppo_divup(N, 128);
    if (op == OP_TN) {
        const bool big = tiles >= 16 && N % 128 == 0;
        if (splitk_target) *splitk_target = big ? 512 : 2048;
        return big ? 0 : 4;
    }
    return tiles < 512 ? 5 : 0;
}

// the tiled kernel leaves most CUs idle when its grid is small and each workgroup walks all of K
// (n = K): below 64 the K split leaves most of the workgroup idle and 64×64 tiles are faster
// (tools/smallm_sweep.py, profiles/r02_smallm_sweep.txt)
bool use_smallm(int m, int n, int l) {
    const long tiled_wgs = (long)ppo_divup(m, 128) * ppo_divup(l, 64);
    return m <= 1024 && n >= 64 && tiled_wgs < 64;
}

void fwd(float* y, const float* x, const float* W, const float* b, int m, int n, int l, int relu, unsigned* bits,
         int cfg, const int* ridx = nullptr, float* acopy = nullptr) {
    Args a{};
    a.ridx = ridx; a.acopy = acopy;
    a.A = x; a.lda = n; a.B = W; a.ldb = n; a.C = y; a.ldc = l;
    a.M = m; a.N = l; a.K = n; a.kchunk = n; a.splits = 1;
    a.bias = b; a.relu = relu;
    a.bits_out = bits; a.wpr = ppo_divup(l, 32);
    a.vec_a = (n % 4 == 0) && aligned16(x);             // kcont, extent K = n
    a.vec_b = (n % 4 == 0) && aligned16(W);
    // small M (rollout over E envs, B = 64 minibatches): split-K inside a workgroup (the fused
    // gather's copy of the rows is written by the first column of blocks)
    if (cfg < 0 && g_force_cfg < 0 && use_smallm(m, n, l)) {
        launch_smallm<OP_NT>(a, a.vec_a && a.vec_b);
        return;
    }
    launch_cfg<OP_NT>(cfg < 0 ? pick_cfg(OP_NT, m, l) : cfg, a);
}

Args bwd_x_args(float* gx, const float* g, const float* W, const float* mask, const unsigned* bits, int m, int n,
                int l) {
    Args a{};
    a.A = g; a.lda = l; a.B = W; a.ldb = n; a.C = gx; a.ldc = n;
    a.M = m; a.N = n; a.K = l; a.kchunk = l; a.splits = 1;
    a.mask = mask; a.ldmask = n;
    a.bits_in = bits; a.wpr = ppo_divup(n, 32);
    a.vec_a = (l % 4 == 0) && aligned16(g);             // kcont, extent K = l
    a.vec_b = (n % 4 == 0) && aligned16(W);             // mncont, extent N = n, ld = n
    return a;
}

void bwd_x(float* gx, const float* g, const float* W, const float* mask, const unsigned* bits, int m, int n, int l,
           int cfg) {
    const Args a = bwd_x_args(gx, g, W, mask, bits, m, n, l);
    if (cfg < 0 && g_force_cfg < 0 && use_smallm(m, l, n)) {
        launch_smallm<OP_NN>(a, a.vec_a);
        return;
    }
    launch_cfg<OP_NN>(cfg < 0 ? pick_cfg(OP_NN, m, n) : cfg, a);
}

// grad_W over a small batch (K = m): one 32×32 block per workgroup with the whole K split over its
// waves beats split-K tiles at 128 < m ≤ 256 (512×512 at m = 256: 6.1 vs 10.5 µs); below that, 64×64
// tiles (no split) are faster than both (5.1 vs 5.9 µs at m = 64) and than 128×128 (10.3 µs)
bool use_smallm_w(int m, int n, int l) { return m > 128 && m <= 256 && (long)ppo_divup(l, 32) * ppo_divup(n, 32) >= 16; }

// grad_W reduces over the minibatch (K = m): split-K so the grid fills the chip; f32 atomics
// into an output that is zero on entry (zeroed != 0) or zeroed here.  Returns the arguments and
// tile configuration (m > 0).
Args bwd_w_args(float* gW, float* gb, const float* g, const float* x, int m, int n, int l, int zeroed, int cfg,
                int* c_out, int target_override = 0) {
    int target = 1024;
    const int c = cfg < 0 ? pick_cfg(OP_TN, l, n, &target) : cfg;
    if (target_override > 0) target = target_override;
    if (g_splitk_override > 0) target = g_splitk_override;
    const TileCfg& tc = kCfgs[c];
    Args a{};
    a.A = g; a.lda = l; a.B = x; a.ldb = n; a.C = gW; a.ldc = n;
    a.M = l; a.N = n; a.K = m;
    a.gbias = gb;
    a.vec_a = (l % 4 == 0) && aligned16(g);             // mncont, extent M = l, ld = l
    a.vec_b = (n % 4 == 0) && aligned16(x);             // mncont, extent N = n, ld = n
    const long tiles = (long)ppo_divup(l, tc.bm) * ppo_divup(n, tc.bn);
    int splits = (int)(target / tiles);                 // the grid stays within the target's rounds
    const int max_splits = m / (8 * tc.bk) > 0 ? m / (8 * tc.bk) : 1;     // ≥ 8 k-tiles per split
    if (splits > max_splits) splits = max_splits;
    if (splits < 1) splits = 1;
    int kchunk = ppo_divup(m, splits);
    kchunk = ppo_divup(kchunk, tc.bk) * tc.bk;
    splits = ppo_divup(m, kchunk);
    a.kchunk = kchunk; a.splits = splits;
    a.tiles_m = ppo_divup(a.M, tc.bm);
    a.tiles_n = ppo_divup(a.N, tc.bn);
    if (splits > 1 && !zeroed) {
        phip_memset(gW, 0, sizeof(float) * (size_t)l * n);
        if (gb) phip_memset(gb, 0, sizeof(float) * (size_t)l);
    }
    *c_out = c;
    return a;
}

void bwd_w(float* gW, float* gb, const float* g, const float* x, int m, int n, int l, int zeroed, int cfg) {
    if (m <= 0) {
        if (!zeroed) {
            phip_memset(gW, 0, sizeof(float) * (size_t)l * n);
            if (gb) phip_memset(gb, 0, sizeof(float) * (size_t)l);
        }
        return;
    }
    if (cfg < 0 && g_force_cfg < 0 && use_smallm_w(m, n, l)) {       // plain stores: zeroed or not
        Args a{};
        a.A = g; a.lda = l; a.B = x; a.ldb = n; a.C = gW; a.ldc = n;
        a.M = l; a.N = n; a.K = m;
        a.gbias = gb;
        launch_smallm<OP_TN>(a, false);
        return;
    }
    int c = 0;
    const Args a = bwd_w_args(gW, gb, g, x, m, n, l, zeroed, cfg < 0 && g_force_cfg < 0 && m <= 128 && l > 32 && n > 32 ? 4 : cfg,
                              &c);
    launch_cfg<OP_TN>(c, a);
}

// grad_W and grad_x of one layer: one gemm_pair_kernel launch when both pick the 128x128/BK16
// vector tile (hidden layers at C4/C5 minibatch sizes), else two launches.  Flag bit 4 (ppo_gemm_flags)
// forces two launches (A/B runs, tests).  Measured at C4: update 544 → 539 ms (serialised loops:
// 580 → 567 ms).
void bwd_pair(float* gW, float* gb, float* gx, const float* g, const float* x, const float* W, const unsigned* bits,
              int m, int n, int l, int zeroed) {
    const int cw = pick_cfg(OP_TN, l, n), cx = pick_cfg(OP_NN, m, n);
    const bool hidden = cw == 0 && cx == 0;
    const bool output = cw == 3 && cx == 0 && (g_flags & 32) == 0;
    if ((g_flags & 4) == 0 && g_force_cfg < 0 && m > 0 && (hidden || output)) {
        int c = 0;
        // grad_W at a 1024-workgroup split target: with a 1024-tile grad_x the launch is two full
        // rounds of 4 workgroups per CU (at the standalone 512 target it would be 1.5 rounds:
        // measured 549 vs 539 ms per C4 update; 2048: 558 ms)
        Args aw = bwd_w_args(gW, gb, g, x, m, n, l, zeroed, -1, &c, 1024);
        Args ax = bwd_x_args(gx, g, W, nullptr, bits, m, n, l);
        aw.flags = ax.flags = g_flags;
        if (aw.splits < 1) aw.splits = 1;
        ax.tiles_m = ppo_divup(ax.M, 128);
        ax.tiles_n = ppo_divup(ax.N, 128);
        const long g1 = (long)aw.tiles_m * aw.tiles_n * aw.splits;
        const long g2 = (long)ax.tiles_m * ax.tiles_n;
        PPO_REQUIRE(g1 > 0 && g2 > 0 && g1 + g2 < (1L << 31), "gemm pair: grid out of range");
        const dim3 grid((unsigned)(g1 + g2));
        const bool vw = aw.vec_a && aw.vec_b, vx = ax.vec_a && ax.vec_b;
        if (hidden && vw && vx) {
            PPO_TIMED_LAUNCH((gemm_pair_kernel<128, 128, 2, true, 128, 128, 2, true>), grid, dim3(NT_), 0,
                               ppo::stream(), aw, ax, (int)g1);
        } else if (output && !vw && !vx) {
            PPO_TIMED_LAUNCH((gemm_pair_kernel<32, 128, 1, false, 128, 128, 2, false>), grid, dim3(NT_), 0,
                               ppo::stream(), aw, ax, (int)g1);
        } else {
            launch_cfg<OP_TN>(c, aw);           // arguments built (and output zeroed) already
            bwd_x(gx, g, W, nullptr, bits, m, n, l, -1);
            return;
        }
        PPO_LAUNCH_CHECK();
        return;
    }
    bwd_w(gW, gb, g, x, m, n, l, zeroed, -1);
    bwd_x(gx, g, W, nullptr, bits, m, n, l, -1);
}

}  // namespace

extern "C" {

void phip_linear_fwd_bits(float* y, const float* x, const float* W, const float* b, int m, int n, int l, int relu,
                          unsigned* bits) {
    if (m <= 0 || l <= 0) return;
    PPO_REQUIRE(y && x && W && n > 0, "phip_linear_fwd: null operand");
    ppo::ProfScope ps(PPO_K_GEMM, 2.0 * m * n * l, ppo::gemm_key(0, 0, m, n, l));
    fwd(y, x, W, b, m, n, l, relu, relu ? bits : nullptr, -1);
}

void phip_linear_fwd(float* y, const float* x, const float* W, const float* b, int m, int n, int l, int relu) {
    phip_linear_fwd_bits(y, x, W, b, m, n, l, relu, nullptr);
}

void phip_linear_fwd_gather(float* y, const float* x, const int* ridx, float* xcopy, const float* W, const float* b,
                            int m, int n, int l, int relu, unsigned* bits) {
    if (m <= 0 || l <= 0) return;
    PPO_REQUIRE(y && x && ridx && W && n > 0, "phip_linear_fwd_gather: null operand");
    ppo::ProfScope ps(PPO_K_GEMM, 2.0 * m * n * l, ppo::gemm_key(0, 0, m, n, l));
    fwd(y, x, W, b, m, n, l, relu, relu ? bits : nullptr, -1, ridx, xcopy);
}

void phip_linear_bwd_x_bits(float* gx, const float* g, const float* W, const float* mask, const unsigned* bits, int m,
                            int n, int l) {
    if (m <= 0 || n <= 0) return;
    PPO_REQUIRE(gx && g && W && l > 0, "phip_linear_bwd_x: null operand");
    ppo::ProfScope ps(PPO_K_GEMM, 2.0 * m * n * l, ppo::gemm_key(1, 0, m, n, l));
    bwd_x(gx, g, W, mask, bits, m, n, l, -1);
}

void phip_linear_bwd_x(float* gx, const float* g, const float* W, const float* mask, int m, int n, int l) {
    phip_linear_bwd_x_bits(gx, g, W, mask, nullptr, m, n, l);
}

void phip_linear_bwd_w_ex(float* gW, float* gb, const float* g, const float* x, int m, int n, int l, int zeroed) {
    if (l <= 0 || n <= 0) return;
    PPO_REQUIRE(gW && g && x, "phip_linear_bwd_w: null operand");
    ppo::ProfScope ps(PPO_K_GEMM, 2.0 * m * n * l, ppo::gemm_key(2, 0, m, n, l));
    bwd_w(gW, gb, g, x, m, n, l, zeroed, -1);
}

void phip_linear_bwd_w(float* gW, float* gb, const float* g, const float* x, int m, int n, int l) {
    phip_linear_bwd_w_ex(gW, gb, g, x, m, n, l, 0);
}

void phip_linear_bwd_pair(float* gW, float* gb, float* gx, const float* g, const float* x, const float* W,
                          const unsigned* bits, int m, int n, int l, int zeroed) {
    if (l <= 0 || n <= 0) return;
    PPO_REQUIRE(gW && gx && g && x && W, "phip_linear_bwd_pair: null operand");
    ppo::ProfScope ps(PPO_K_GEMM, 4.0 * m * n * l, ppo::gemm_key(3, 0, m, n, l));
    bwd_pair(gW, gb, gx, g, x, W, bits, m, n, l, zeroed);
}

int ppo_gemm_flags(int flags) {
    const int old = g_flags;
    if (flags >= 0) g_flags = flags;
    return old;
}

// ppo_gemm_tune(·, 1): split-K off — deterministic (atomic-free) parameter gradients requested
int phip_gemm_deterministic(void) { return g_splitk_override == 1; }

int ppo_gemm_tune(int force_cfg, int splitk_target) {
    g_force_cfg = force_cfg;
    if (splitk_target >= 0) g_splitk_override = splitk_target;
    return kNumCfgs;
}

// Tuning / roofline utility: average device time (µs) of one launch of `op` (0 fwd, 1 grad_x,
// 2 grad_W) at the given shape, measured with HIP events on libppo's stream.
double ppo_bench_gemm(int op, int m, int n, int l, int iters, int cfg) {
    ppo::ensure_device();
    const size_t sx = (size_t)m * n, sw = (size_t)l * n, sy = (size_t)m * l;
    float* x = (float*)phip_malloc(sizeof(float) * sx);
    float* W = (float*)phip_malloc(sizeof(float) * sw);
    float* y = (float*)phip_malloc(sizeof(float) * (sy > sx ? sy : sx));
    float* b = (float*)phip_malloc(sizeof(float) * (size_t)(l > n ? l : n));
    float* gw = (float*)phip_malloc(sizeof(float) * sw);
    phip_fill_uniform(x, (long)sx, 1, -1.f, 1.f);
    phip_fill_uniform(W, (long)sw, 2, -0.1f, 0.1f);
    phip_fill_uniform(y, (long)(sy > sx ? sy : sx), 3, -1.f, 1.f);
    phip_fill_uniform(b, (long)(l > n ? l : n), 4, -0.1f, 0.1f);
    auto run = [&]() {
        if (op == 0) fwd(y, x, W, b, m, n, l, 1, nullptr, cfg);
        else if (op == 3) fwd(y, x, W, b, m, n, l, 0, nullptr, cfg);        // output layer: no activation
        else if (op == 1) bwd_x(x, y, W, nullptr, nullptr, m, n, l, cfg);
        else bwd_w(gw, b, y, x, m, n, l, 0, cfg);
    };
    for (int i = 0; i < 3; ++i) run();
    hipEvent_t e0, e1;
    PPO_CHECK(hipEventCreate(&e0));
    PPO_CHECK(hipEventCreate(&e1));
    PPO_CHECK(hipEventRecord(e0, ppo::stream()));
    for (int i = 0; i < iters; ++i) run();
    PPO_CHECK(hipEventRecord(e1, ppo::stream()));
    PPO_CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    PPO_CHECK(hipEventElapsedTime(&ms, e0, e1));
    PPO_CHECK(hipEventDestroy(e0));
    PPO_CHECK(hipEventDestroy(e1));
    phip_free(x); phip_free(W); phip_free(y); phip_free(b); phip_free(gw);
    return 1000.0 * ms / (iters > 0 ? iters : 1);
}

// Two independent C4-shaped minibatch chains (376 → 512 ×3 → out: forward with bits, then grad_W /
// grad_x per layer), `steps` steps each, issued interleaved either on one stream (two = 0) or on
// two streams (two = 1).  Returns total device µs.  Measures what running the value and policy
// minibatch loops concurrently would gain.
double ppo_bench_streams(int two, int steps, int B, int out) {
    ppo::ensure_device();
    const int S = 376, H = 512;
    const int dims[5] = {S, H, H, H, out};
    struct Chain { float *x, *act[5], *g[5], *W[4], *b[4], *gW[4], *gb[4]; unsigned* bits[4]; } c[2];
    for (auto& ch : c) {
        ch.x = (float*)phip_malloc(sizeof(float) * (size_t)B * S);
        phip_fill_uniform(ch.x, (long)B * S, 1, -1.f, 1.f);
        ch.act[0] = ch.x;
        for (int i = 0; i < 4; ++i) {
            const size_t wn = (size_t)dims[i] * dims[i + 1];
            ch.W[i] = (float*)phip_malloc(sizeof(float) * wn);
            phip_fill_uniform(ch.W[i], (long)wn, 2 + i, -0.05f, 0.05f);
            ch.b[i] = (float*)phip_malloc(sizeof(float) * dims[i + 1]);
            phip_fill_uniform(ch.b[i], dims[i + 1], 9 + i, -0.05f, 0.05f);
            ch.gW[i] = (float*)phip_malloc(sizeof(float) * wn);
            ch.gb[i] = (float*)phip_malloc(sizeof(float) * dims[i + 1]);
            ch.act[i + 1] = (float*)phip_malloc(sizeof(float) * (size_t)B * dims[i + 1]);
            ch.g[i + 1] = (float*)phip_malloc(sizeof(float) * (size_t)B * dims[i + 1]);
            ch.bits[i] = (unsigned*)phip_malloc(sizeof(unsigned) * (size_t)B * ppo_divup(dims[i + 1], 32));
        }
        phip_fill_uniform(ch.g[4], (long)B * out, 17, -1.f, 1.f);
    }
    auto step = [&](Chain& ch) {
        for (int i = 0; i < 4; ++i)
            fwd(ch.act[i + 1], ch.act[i], ch.W[i], ch.b[i], B, dims[i], dims[i + 1], i < 3, i < 3 ? ch.bits[i] : nullptr,
                -1);
        for (int i = 3; i >= 0; --i) {
            bwd_w(ch.gW[i], ch.gb[i], ch.g[i + 1], ch.act[i], B, dims[i], dims[i + 1], 0, -1);
            if (i > 0) bwd_x(ch.g[i], ch.g[i + 1], ch.W[i], nullptr, ch.bits[i - 1], B, dims[i], dims[i + 1], -1);
        }
    };
    hipEvent_t e0, e1;
    PPO_CHECK(hipEventCreate(&e0));
    PPO_CHECK(hipEventCreate(&e1));
    for (int rep = 0; rep < 2; ++rep) {              // rep 0 warms up
        PPO_CHECK(hipEventRecord(e0, ppo::stream()));
        if (two) phip_side_fork();
        for (int k = 0; k < steps; ++k) {
            step(c[0]);
            if (two) phip_side_use(1);
            step(c[1]);
            if (two) phip_side_use(0);
        }
        if (two) phip_side_join();
        PPO_CHECK(hipEventRecord(e1, ppo::stream()));
        PPO_CHECK(hipEventSynchronize(e1));
    }
    float ms = 0.f;
    PPO_CHECK(hipEventElapsedTime(&ms, e0, e1));
    PPO_CHECK(hipEventDestroy(e0));
    PPO_CHECK(hipEventDestroy(e1));
    for (auto& ch : c) {
        phip_free(ch.x);
        for (int i = 0; i < 4; ++i) {
            phip_free(ch.W[i]); phip_free(ch.b[i]); phip_free(ch.gW[i]); phip_free(ch.gb[i]);
            phip_free(ch.act[i + 1]); phip_free(ch.g[i + 1]); phip_free(ch.bits[i]);
        }
    }
    return 1000.0 * ms;
}

}  // extern "C"
