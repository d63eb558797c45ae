// gemm16.hip — bf16-MFMA GEMMs for the bf16 compute mode (BASELINE config C5: "4×1024 MLP bf16").
//
// The same three linear-layer products as gemm.hip (reference mat_mul.cu:122-217, the fused
// bias/ReLU of activation_function.cu and the bias-gradient sum of neural_network.cu:108-118), on
// v_mfma_f32_32x32x16_bf16: bf16 operands, fp32 accumulation, 16× the fp32-MFMA rate.
//   forward   y = x·Wᵀ + b (+ReLU, +ReLU′ bits)     NT
//   grad_x    gx = (g·W) ⊙ 1[y_prev > 0]              NN
//   grad_W    gW += gᵀ·x, gb += Σ g   (split-K, f32 atomics)  TN
// Operands may be stored fp32 (network input, the heads' output gradient) or bf16 (hidden
// activations and their gradients, the bf16 weight shadow); they are rounded to bf16 on the way
// into LDS.  Outputs are fp32 or bf16 (hidden activations / gradients), accumulation always fp32.
// (fp32 mode's products run on the same MFMA through the exact three-plane split of gemm_x3.hip.)
//
// Design (gfx950):
//  * 256-thread workgroups (4 waves), block tile BM×BN, BK = 32 or 64 (two or four MFMA k-steps).
//  * k-contiguous operands ("kcont": x, g in grad_x, W in forward) are staged as [row][BK+8] bf16:
//    a lane's fragment (A[r][8h..8h+7]) is one conflict-free ds_read_b128 (80-B pitch: row·20 mod
//    64 dwords spreads every 16-lane group over distinct banks).
//  * row-contiguous operands ("mncont": W in grad_x, g and x in grad_W) are staged as
//    [BK][R (+32)] bf16 exactly as loaded, and a fragment is two ds_read_b64_tr_b16 hardware
//    transposes (4 k × 16 rows per 16-lane group); the pitch ≡ 16 or 48 dwords (mod 64) keeps the
//    4 rows × 2 groups of each 32-lane half on disjoint banks.
//  * Branch-free clamped loads, the k-mask applied at LDS-store time, register prefetch of the next
//    k-tile behind this tile's MFMAs, XCD-aware block remap — as in gemm.hip.
#include "dev.h"

#include <algorithm>

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int NT_ = 256;

#ifndef PPO_G16_ABLATE
#define PPO_G16_ABLATE 0          // diagnostic builds only (tools/build_variant.sh): 1 no MFMA, 2 no epilogue
#endif                            // stores, 4 no steady-state global loads, 8 no steady-state LDS stores,
                                  // 16 no fragment reads, 32 stamps, 64 no bias / mask loads, 128 grad_W plain stores
#if PPO_G16_ABLATE & 32
// s_memtime of wave 0 of each workgroup: start, after the mainloop, epilogue issued, stores drained;
// s_memrealtime (100 MHz) at start and drained
__device__ unsigned long long g_g16_stamps[8192 * 8];
#endif

enum Op { OP_NT = 0, OP_NN = 1, OP_TN = 2 };

struct Args {
    const void* A; const void* B; void* C;
    int M, N, K, lda, ldb, ldc;
    const float* bias; int relu;
    const int* ridx; void* acopy;         // OP_NT: fused gather of A's rows + the gathered copy (bf16)
    unsigned* bits_out; const unsigned* bits_in; int wpr;
    float* gbias;
    int kchunk, splits, tiles_m, tiles_n;
    int vec;
    int cvec;                             // bf16 C: N and ldc multiples of 8, C 16-B aligned (LDS-staged epilogue)
};

// fp32 → bf16, round to nearest even (NaN stays NaN: v_cvt_pk_bf16_f32)
__device__ __forceinline__ unsigned pack2(float lo, float hi) {
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    bf16x2 p = {(__bf16)lo, (__bf16)hi};
    return __builtin_bit_cast(unsigned, p);
}
__device__ __forceinline__ float bf_lo(unsigned u) { return __builtin_bit_cast(float, u << 16); }

// ---------------------------------------------------------------------------
// Staging of one operand tile (R rows × BK k) into a bf16 LDS image.  T = float or unsigned short
// (bf16 bits).  One 16-B global load per slot: 4 fp32 or 8 bf16 elements.
// ---------------------------------------------------------------------------
template <int R, int BK, bool MN, typename T, int NTS = NT_>
struct Stage16 {
    static constexpr bool F32 = sizeof(T) == 4;
    static constexpr int EPL = F32 ? 4 : 8;                 // elements per 16-B load
    static constexpr int PK = BK + 8;                       // kcont pitch (elements) = 80 B
    static constexpr int PR = ((R / 2) % 64 == 16 || (R / 2) % 64 == 48) ? R : R + 32;   // mncont pitch
    static constexpr int IMG = MN ? BK * PR : R * PK;       // bf16 elements
    static constexpr int PER_ROW = MN ? R / EPL : BK / EPL; // loads along the contiguous dimension
    static constexpr int TOTAL = MN ? BK * PER_ROW : R * PER_ROW;
    static constexpr int ITERS = (TOTAL + NTS - 1) / NTS;
    static_assert(R % EPL == 0 && R >= 32, "tile rows");
    u32x4 v[ITERS];
    bool kok[ITERS];
    int src[ITERS];

    __device__ __forceinline__ static void coords(int idx, int& row, int& k) {
        if (MN) { row = (idx % PER_ROW) * EPL; k = idx / PER_ROW; }
        else    { row = idx / PER_ROW; k = (idx % PER_ROW) * EPL; }
    }

    __device__ __forceinline__ void prep(const int* __restrict__ ridx, int r0, int Rmax, int tid) {
#pragma unroll
        for (int it = 0; it < ITERS; ++it) {
            int row, k;
            coords(tid + it * NTS, row, k);
            const int gr = min(r0 + row, Rmax - 1);
            src[it] = ridx ? ridx[gr] : gr;
        }
    }

    // vec: every contiguous extent and ld are multiples of EPL and the base is 16-B aligned
    __device__ __forceinline__ void load(const T* __restrict__ src_p, int ld, int r0, int Rmax, int k0, int kend,
                                         bool vec, int tid) {
#pragma unroll
        for (int it = 0; it < ITERS; ++it) {
            const int idx = tid + it * NTS;
            u32x4 x = u32x4{0u, 0u, 0u, 0u};
            kok[it] = true;
            if (TOTAL % NTS == 0 || idx < TOTAL) {
                int row, k;
                coords(idx, row, k);
                const int gr = r0 + row, gk = k0 + k;
                if (vec) {
                    kok[it] = gk < kend;
                    const T* p = MN ? src_p + (long)(gk < kend ? gk : kend - 1) * ld + (gr < Rmax ? gr : Rmax - EPL)
                                    : src_p + (long)src[it] * ld + (gk < kend ? gk : kend - EPL);
                    x = *reinterpret_cast<const u32x4*>(p);
                } else {
                    T e[EPL];
#pragma unroll
                    for (int c = 0; c < EPL; ++c) e[c] = T(0);
                    if (MN) {
                        if (gk < kend) {
                            const T* p = src_p + (long)gk * ld + gr;
#pragma unroll
                            for (int c = 0; c < EPL; ++c)
                                if (gr + c < Rmax) e[c] = p[c];
                        }
                    } else if (gr < Rmax) {
                        const T* p = src_p + (long)src[it] * ld + gk;
#pragma unroll
                        for (int c = 0; c < EPL; ++c)
                            if (gk + c < kend) e[c] = p[c];
                    }
                    x = __builtin_bit_cast(u32x4, e);
                }
            }
            v[it] = x;
        }
    }

    __device__ __forceinline__ void store(unsigned short* img, int tid) const {
#pragma unroll
        for (int it = 0; it < ITERS; ++it) {
            const int idx = tid + it * NTS;
            if (TOTAL % NTS == 0 || idx < TOTAL) {
                int row, k;
                coords(idx, row, k);
                unsigned short* d = img + (MN ? k * PR + row : row * PK + k);
                const u32x4 z = {0u, 0u, 0u, 0u};
                const u32x4 x = kok[it] ? v[it] : z;
                if (F32) {
                    const f32x4 f = __builtin_bit_cast(f32x4, x);
                    const u32x2 p = {pack2(f[0], f[1]), pack2(f[2], f[3])};
                    *reinterpret_cast<u32x2*>(d) = p;
                } else {
                    *reinterpret_cast<u32x4*>(d) = x;
                }
            }
        }
    }

    // A-side fused gather: write the staged rows (rows < Rmax, k < kend) to dst[row*ldd + k] as bf16
    __device__ __forceinline__ void copy_out(void* __restrict__ dstv, int ldd, int r0, int Rmax, int k0,
                                             int kend, int tid) const {
        unsigned short* __restrict__ dst = static_cast<unsigned short*>(dstv);
#pragma unroll
        for (int it = 0; it < ITERS; ++it) {
            const int idx = tid + it * NTS;
            if (TOTAL % NTS == 0 || idx < TOTAL) {
                int row, k;
                coords(idx, row, k);
                const int gr = r0 + row, gk = k0 + k;
                if (gr >= Rmax) continue;
                unsigned short* q = dst + (long)gr * ldd + gk;
                if (F32) {
                    const f32x4 f = __builtin_bit_cast(f32x4, v[it]);
                    if (gk + 3 < kend && (ldd & 3) == 0) {             // one 8-B store of 4 bf16
                        const u32x2 p = {pack2(f[0], f[1]), pack2(f[2], f[3])};
                        *reinterpret_cast<u32x2*>(q) = p;
                    } else {
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            if (gk + e < kend) q[e] = (unsigned short)(pack2(f[e], 0.f) & 0xffffu);
                    }
                } else if (gk + 7 < kend && (ldd & 7) == 0) {
                    *reinterpret_cast<u32x4*>(q) = v[it];
                } else {
                    const unsigned short* s = reinterpret_cast<const unsigned short*>(&v[it]);
#pragma unroll
                    for (int e = 0; e < 8; ++e)
                        if (gk + e < kend) q[e] = s[e];
                }
            }
        }
    }

    // MFMA fragment of k-step ks for image row `row`: elements k = 16·ks + 8h + j, j = 0..7
    __device__ __forceinline__ static bf16x8 frag(const unsigned short* img, int row, int ks, int lane) {
        const int h = lane >> 5;
        if (!MN) return __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(img + row * PK + 16 * ks + 8 * h));
        // hardware transpose: in each 16-lane group, lane 4q+p addresses k-row q, rows 4p..4p+3 of the
        // group's 16; lane i receives row i of the 4 k-rows.  Two reads give k = 8h+0..3 and 8h+4..7.
        const int gi = lane & 15, q = gi >> 2, p = gi & 3;
        const int rbase = row - gi;                       // first row of this lane's 16-row group
        typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
        const unsigned short* a0 = img + (16 * ks + 8 * h + q) * PR + rbase + 4 * p;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * PR));
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        const s16x8 f = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return __builtin_bit_cast(bf16x8, f);
    }

    // Σ over this tile's k of image row `row` (fp32), k ∈ [k_lo, k_lo + n)
    __device__ __forceinline__ static float rowsum(const unsigned short* img, int row, int k_lo, int n) {
        float t = 0.f;
        for (int kk = 0; kk < n; ++kk) {
            const int o = MN ? (k_lo + kk) * PR + row : row * PK + k_lo + kk;
            t += __builtin_bit_cast(float, (unsigned)img[o] << 16);
        }
        return t;
    }
};

template <typename T> struct Bits;
template <> struct Bits<float> { static constexpr int code = 0; };
template <> struct Bits<unsigned short> { static constexpr int code = 1; };

template <int OP, int BM, int BN, int WARPS_M, int BK, typename TA, typename TB, typename TC, int MF = 32>
__global__ __launch_bounds__(NT_, 2) void gemm_bf16_kernel(Args a) {
    static_assert(MF == 32 || (MF == 16 && OP == OP_TN && BK % 32 == 0), "16×16×32 form: grad_W");
    constexpr int WARPS_N = NT_ / 64 / WARPS_M;
    constexpr int WM = BM / WARPS_M, WN = BN / WARPS_N;
    constexpr int TM = WM / 32, TN = WN / 32;
    constexpr bool A_MN = OP == OP_TN, B_MN = OP != OP_NT;
    using SA = Stage16<BM, BK, A_MN, TA>;
    using SB = Stage16<BN, BK, B_MN, TB>;
    static_assert(TM >= 1 && TN >= 1, "wave tile must be a multiple of 32x32");
    static_assert(!(OP == OP_TN) || sizeof(TC) == 4, "grad_W accumulates in fp32");

    extern __shared__ __attribute__((aligned(16))) unsigned short lds[];     // SA::IMG + SB::IMG

    // XCD-aware remap: each XCD gets a contiguous range of linear tiles (n fastest)
    const int nwg = gridDim.x, b = blockIdx.x;
    const int xcd = b & 7, qq = nwg >> 3, rr = nwg & 7;
    const int t = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (b >> 3);
    const int tn = t % a.tiles_n;
    const int rest = t / a.tiles_n;
    const int tm = rest % a.tiles_m;
    const int m0 = tm * BM, n0 = tn * BN;
    const int kbeg = (rest / a.tiles_m) * a.kchunk;
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

    constexpr int TPR = NT_ / BM > 0 ? NT_ / BM : 1;
    constexpr int KPT = BK / TPR > 0 ? BK / TPR : 1;
    const bool do_bsum = OP == OP_TN && a.gbias != nullptr && tn == 0 && (NT_ % BM == 0);
    float bsum = 0.f;

    SA sa;
    SB sb;
    if (!A_MN) sa.prep(OP == OP_NT ? a.ridx : nullptr, m0, a.M, tid);
    if (!B_MN) sb.prep(nullptr, n0, a.N, tid);
    const bool do_copy = OP == OP_NT && a.acopy != nullptr && tn == 0;
    const bool vec = a.vec != 0;
    const TA* __restrict__ PA = static_cast<const TA*>(a.A);
    const TB* __restrict__ PB = static_cast<const TB*>(a.B);

    // 16×16×32 form (grad_W): both operands row-contiguous; transposed reads of 16 columns × 8 k
    typedef float f32x4v __attribute__((ext_vector_type(4)));
    constexpr int TM16 = MF == 16 ? WM / 16 : 1, TN16 = MF == 16 ? WN / 16 : 1;
    f32x4v acc16[TM16][TN16];
    if constexpr (MF == 16) {
#pragma unroll
        for (int i = 0; i < TM16; ++i)
#pragma unroll
            for (int j = 0; j < TN16; ++j) acc16[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};
    }
    auto frag16 = [&](const unsigned short* im, int pitch, int cbase, int s) {
        const int l15 = lane & 15, g4 = lane >> 4, q = l15 >> 2, p = l15 & 3;
        typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
        const unsigned short* a0 = im + (32 * s + 8 * g4 + q) * pitch + cbase + 4 * p;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * pitch));
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        const s16x8 f = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return __builtin_bit_cast(bf16x8, f);
    };
    auto compute = [&]() {
        const unsigned short* As = lds;
        const unsigned short* Bs = lds + SA::IMG;
        if constexpr (MF == 16) {
#pragma unroll
            for (int s = 0; s < BK / 32; ++s) {
                bf16x8 fa[TM16], fb[TN16];
#pragma unroll
                for (int i = 0; i < TM16; ++i) fa[i] = frag16(As, SA::PR, wm * WM + i * 16, s);
#pragma unroll
                for (int j = 0; j < TN16; ++j) fb[j] = frag16(Bs, SB::PR, wn * WN + j * 16, s);
#pragma unroll
                for (int i = 0; i < TM16; ++i)
#pragma unroll
                    for (int j = 0; j < TN16; ++j)
                        acc16[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc16[i][j], 0, 0, 0);
            }
            return;
        }
#pragma unroll
        for (int ks = 0; ks < BK / 16; ++ks) {
            bf16x8 fa[TM], fb[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) fa[i] = SA::frag(As, wm * WM + i * 32 + r, ks, lane);
#pragma unroll
            for (int j = 0; j < TN; ++j) fb[j] = SB::frag(Bs, wn * WN + j * 32 + r, ks, lane);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
    };

    if (kbeg < kend) {
        sa.load(PA, a.lda, m0, a.M, kbeg, kend, vec, tid);
        sb.load(PB, a.ldb, n0, a.N, kbeg, kend, vec, tid);
    }
    for (int k0 = kbeg; k0 < kend; k0 += BK) {
        if (do_copy) sa.copy_out(a.acopy, a.K, m0, a.M, k0, kend, tid);
        sa.store(lds, tid);
        sb.store(lds + SA::IMG, tid);
        __syncthreads();
        if (k0 + BK < kend) {                               // in flight during this tile's MFMAs
            sa.load(PA, a.lda, m0, a.M, k0 + BK, kend, vec, tid);
            sb.load(PB, a.ldb, n0, a.N, k0 + BK, kend, vec, tid);
        }
        if (do_bsum) bsum += SA::rowsum(lds, tid / TPR, (tid % TPR) * KPT, KPT);
        compute();
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

    if constexpr (MF == 16) {                          // 16×16 block: column lane & 15, rows 4(lane >> 4) + e
#pragma unroll
        for (int i = 0; i < TM16; ++i)
#pragma unroll
            for (int j = 0; j < TN16; ++j) {
                const int col = n0 + wn * WN + j * 16 + (lane & 15);
                const int r0 = m0 + wm * WM + i * 16 + 4 * (lane >> 4);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (col < a.N && r0 + e < a.M) {
                        float* dst = static_cast<float*>(a.C) + (long)(r0 + e) * a.ldc + col;
                        if (a.splits > 1) atomicAdd(dst, acc16[i][j][e]);
                        else *dst = acc16[i][j][e];
                    }
                }
            }
        return;
    }
    // epilogue (C/D map as gemm.hip); every load a block needs is issued before its stores
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int c0 = n0 + wn * WN + j * 32;
            const int col = c0 + r;
            const int r0 = m0 + wm * WM + i * 32 + 4 * h;
            const bool col_ok = col < a.N;
            float bcol = 0.f;
            if (OP == OP_NT && a.bias) bcol = a.bias[col_ok ? col : a.N - 1];
            bool keep[16];
            if (OP == OP_NN) {
                if (a.bits_in) {
                    unsigned wv[16];
#pragma unroll
                    for (int e = 0; e < 16; ++e)
                        wv[e] = a.bits_in[(long)min(r0 + (e & 3) + 8 * (e >> 2), a.M - 1) * a.wpr + (c0 >> 5)];
#pragma unroll
                    for (int e = 0; e < 16; ++e) keep[e] = (wv[e] >> r) & 1u;
                } else {
#pragma unroll
                    for (int e = 0; e < 16; ++e) keep[e] = true;
                }
            }
            unsigned word = 0;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int row = r0 + (e & 3) + 8 * (e >> 2);
                const bool ok = col_ok && row < a.M;
                float v = acc[i][j][e];
                const long off = (long)row * a.ldc + col;
                if (OP == OP_NT) {
                    v += bcol;
                    if (a.relu) v = v > 0.f ? v : 0.f;
                    if (Bits<TC>::code == 1) {
                        const unsigned short hv = (unsigned short)(pack2(v, 0.f) & 0xffffu);
                        v = bf_lo(hv);                  // bits describe the stored (rounded) value
                        if (ok) static_cast<unsigned short*>(a.C)[off] = hv;
                    } else if (ok) {
                        static_cast<float*>(a.C)[off] = v;
                    }
                    if (a.bits_out) {
                        const unsigned long long bb = __ballot(ok && v > 0.f);
                        if (r == e) word = h ? (unsigned)(bb >> 32) : (unsigned)bb;
                    }
                } else if (OP == OP_NN) {
                    if (ok) {
                        v = keep[e] ? v : 0.f;
                        if (Bits<TC>::code == 1) static_cast<unsigned short*>(a.C)[off] =
                            (unsigned short)(pack2(v, 0.f) & 0xffffu);
                        else static_cast<float*>(a.C)[off] = v;
                    }
                } else if (ok) {
                    float* dst = static_cast<float*>(a.C) + off;
                    if (PPO_G16_ABLATE & 128) {                 // diagnostic: plain stores
                        *dst = v;
                    } else if (a.splits > 1) {
                        atomicAdd(dst, v);
                    } else {
                        *dst = v;
                    }
                }
            }
            if (OP == OP_NT && a.bits_out && r < 16) {
                const int row = r0 + (r & 3) + 8 * (r >> 2);
                if (row < a.M && c0 < a.N) a.bits_out[(long)row * a.wpr + (c0 >> 5)] = word;
            }
        }
}

// second half of the LDS-staged bf16 epilogue: the BM×BN tile image (pitch BN + 32 bf16, written by
// every wave before this call's barrier) leaves as 16-B row stores; grad_x's incoming mask and the
// forward's ReLU′ bits are applied on this row-major read-back, 8 columns per lane
template <int OP, int BM, int BN, int NTH>
__device__ __forceinline__ void c_image_out(const Args& a, const unsigned short* cimg, int m0, int n0, int tid) {
    constexpr int AB = PPO_G16_ABLATE;
    constexpr int CP = BN + 32;
    __syncthreads();
    constexpr int CH = BN / 8;                        // 16-B chunks per tile row (4 per 32-bit word)
    constexpr int IT = BM * CH / NTH;
    unsigned short* __restrict__ C = static_cast<unsigned short*>(a.C);
    unsigned mword[IT];
    if (OP == OP_NN) {                                // grad_x: the mask words, all loads first
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int idx = tid + it * NTH;
            const int grow = min(m0 + idx / CH, a.M - 1), gcol = n0 + (idx % CH) * 8;
            mword[it] = (a.bits_in && !(AB & 64)) ? a.bits_in[(long)grow * a.wpr + (min(gcol, a.N - 1) >> 5)]
                                                   : ~0u;
        }
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int idx = tid + it * NTH;
        const int row = idx / CH, ch = idx % CH;
        const int grow = m0 + row, gcol = n0 + ch * 8;
        u32x4 v = *reinterpret_cast<const u32x4*>(cimg + row * CP + ch * 8);
        if (OP == OP_NN) {
            const unsigned byte = mword[it] >> (8 * (ch & 3));
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const unsigned keep = (0xffffu * ((byte >> (2 * q)) & 1u)) | (0xffff0000u * ((byte >> (2 * q + 1)) & 1u));
                v[q] &= keep;
            }
        }
        const bool ok = grow < a.M && gcol < a.N;
        if (ok) *reinterpret_cast<u32x4*>(C + (long)grow * a.ldc + gcol) = v;
        if (OP == OP_NT && a.bits_out) {
            // bit c of the byte: column gcol + c stored > 0 (post-ReLU values are ≥ +0)
            unsigned byte = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                byte |= (unsigned)((short)(v[q] & 0xffffu) > 0) << (2 * q);
                byte |= (unsigned)((short)(v[q] >> 16) > 0) << (2 * q + 1);
            }
            if (!ok) byte = 0;                      // columns past N carry no bits
            // the 4 lanes of a quad hold the 4 bytes of one 32-column word (ch & 3 = lane & 3)
            const int b1 = __builtin_amdgcn_mov_dpp((int)byte, 0x55, 0xF, 0xF, true);   // quad lane 1
            const int b2 = __builtin_amdgcn_mov_dpp((int)byte, 0xAA, 0xF, 0xF, true);   // quad lane 2
            const int b3 = __builtin_amdgcn_mov_dpp((int)byte, 0xFF, 0xF, 0xF, true);   // quad lane 3
            const unsigned word = byte | ((unsigned)b1 << 8) | ((unsigned)b2 << 16) | ((unsigned)b3 << 24);
            if ((ch & 3) == 0 && ok) a.bits_out[(long)grow * a.wpr + (gcol >> 5)] = word;
        }
    }
}

// Epilogue of the 256×256 kernels (8 waves of (TM·32)×(TN·32), 32×32 accumulator blocks: lane (r, h)
// holds column r, rows 4h + (e&3) + 8(e>>2)).  LDS (BM × (BN + 32) bf16) must be free on entry.
template <int OP, int BM, int BN, int TM, int TN, int NTH, typename TC, typename S>
__device__ __forceinline__ void epilogue256(const Args& a, f32x16 (&acc)[TM][TN], unsigned short* lds, int m0,
                                            int n0, int wm, int wn, int tid, S&& stamp) {
    constexpr int WM = TM * 32, WN = TN * 32;
    constexpr int AB = PPO_G16_ABLATE;
    const int lane = tid & 63, r = lane & 31, h = lane >> 5;
    (void)stamp;
    // bf16 output: the tile goes through LDS (free after the last barrier) as packed column pairs,
    // then out as 16-B stores, 32 lanes per 512-B row segment; the ReLU′ bits (forward) and the
    // incoming mask (grad_x) are applied on that row-major read-back, 8 columns per lane, so the
    // register phase is branch-free (measured at C5: the per-element ballots, mask loads and 2-B
    // stores of the generic epilogue took 14 of the forward's 53 µs and 8 of grad_x's 48 µs)
    if constexpr (sizeof(TC) == 2) {
        if (a.cvec) {
            constexpr int CP = BN + 32;                       // pitch ≡ 16 dwords (mod 32): rows a, a+1 of
            unsigned short* const cimg = lds;                 // a write on disjoint banks (callers size LDS)
            const bool odd = r & 1;
            float bcol[TN];
#pragma unroll
            for (int jj = 0; jj < TN; ++jj) {
                const int col = n0 + wn * WN + jj * 32 + r;
                bcol[jj] = (OP == OP_NT && a.bias && !(AB & 64)) ? a.bias[col < a.N ? col : a.N - 1] : 0.f;
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int jj = 0; jj < TN; ++jj) {
                    float vv[16];
#pragma unroll
                    for (int e = 0; e < 16; ++e) {
                        float v = acc[i][jj][e];
                        if (OP == OP_NT) {
                            v += bcol[jj];
                            if (a.relu) v = v > 0.f ? v : 0.f;
                        }
                        vv[e] = v;
                    }
                    // lanes r, r^1 swap one value (DPP): the even lane writes row e's pair of columns
                    // (r, r+1), the odd lane row e+1's
#pragma unroll
                    for (int e = 0; e < 16; e += 2) {
                        const float send = odd ? vv[e] : vv[e + 1];
                        const float recv = __builtin_bit_cast(
                            float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, send), 0xB1, 0xF, 0xF, true));
                        const float lo = odd ? recv : vv[e], hi = odd ? vv[e + 1] : recv;
                        const int lrow = wm * WM + i * 32 + 4 * h + (e & 3) + 8 * (e >> 2) + (odd ? 1 : 0);
                        *reinterpret_cast<unsigned*>(cimg + lrow * CP + wn * WN + jj * 32 + (r & ~1)) = pack2(lo, hi);
                    }
                }
            c_image_out<OP, BM, BN, NTH>(a, cimg, m0, n0, tid);
            if constexpr ((AB & 32) != 0) {
                stamp(2);
                __builtin_amdgcn_s_waitcnt(0);
                stamp(3);
            }
            return;
        }
    }
    // epilogue (as gemm_bf16_kernel): every load a block needs is issued before its stores
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int jj = 0; jj < TN; ++jj) {
            const int c0 = n0 + wn * WN + jj * 32;
            const int col = c0 + r;
            const int r0 = m0 + wm * WM + i * 32 + 4 * h;
            const bool col_ok = col < a.N;
            float bcol = 0.f;
            if (OP == OP_NT && a.bias) bcol = a.bias[col_ok ? col : a.N - 1];
            bool keep[16];
            if (OP == OP_NN) {
                if (a.bits_in) {
                    unsigned wv[16];
#pragma unroll
                    for (int e = 0; e < 16; ++e)
                        wv[e] = a.bits_in[(long)min(r0 + (e & 3) + 8 * (e >> 2), a.M - 1) * a.wpr + (c0 >> 5)];
#pragma unroll
                    for (int e = 0; e < 16; ++e) keep[e] = (wv[e] >> r) & 1u;
                } else {
#pragma unroll
                    for (int e = 0; e < 16; ++e) keep[e] = true;
                }
            }
            unsigned word = 0;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int row = r0 + (e & 3) + 8 * (e >> 2);
                const bool ok = col_ok && row < a.M;
                float v = acc[i][jj][e];
                const long off = (long)row * a.ldc + col;
                if (OP == OP_NT) {
                    v += bcol;
                    if (a.relu) v = v > 0.f ? v : 0.f;
                    if (Bits<TC>::code == 1) {
                        const unsigned short hv = (unsigned short)(pack2(v, 0.f) & 0xffffu);
                        v = bf_lo(hv);                  // bits describe the stored (rounded) value
                        if (ok) static_cast<unsigned short*>(a.C)[off] = hv;
                    } else if (ok) {
                        static_cast<float*>(a.C)[off] = v;
                    }
                    if (a.bits_out) {
                        const unsigned long long bb = __ballot(ok && v > 0.f);
                        if (r == e) word = h ? (unsigned)(bb >> 32) : (unsigned)bb;
                    }
                } else if (ok) {
                    v = keep[e] ? v : 0.f;
                    if (Bits<TC>::code == 1) static_cast<unsigned short*>(a.C)[off] =
                        (unsigned short)(pack2(v, 0.f) & 0xffffu);
                    else static_cast<float*>(a.C)[off] = v;
                }
            }
            if (OP == OP_NT && a.bits_out && r < 16) {
                const int row = r0 + (r & 3) + 8 * (r >> 2);
                if (row < a.M && c0 < a.N) a.bits_out[(long)row * a.wpr + (c0 >> 5)] = word;
            }
        }
}

// ---------------------------------------------------------------------------
// Double-buffered 256×256 tile for forward and grad_x at wide shapes (C5: 16384 × 1024 × 1024):
// 512 threads = 8 waves of 64×128, BK = 64 (four MFMA k-steps of 32 products per wave), two LDS
// images (2 × 72 KiB, one workgroup per CU) so each k-tile costs ONE barrier, and the LDS stores
// of tile j+1 and the global loads of tile j+2 are issued between tile j's k-steps (the gemm_x3
// pipeline with a single bf16 plane).  The classic kernel above (one image, two barriers per
// k-tile, 4 waves) stays for grad_W and narrow products.
// ---------------------------------------------------------------------------
template <int OP, int BM, int BN, int WARPS_M, int BK, int NTH, typename TA, typename TB, typename TC>
__global__ __launch_bounds__(NTH, 1) void gemm_bf16_db_kernel(Args a) {
    static_assert(OP != OP_TN, "forward / grad_x only");
    static_assert(BK == 64, "four k-steps per k-tile");
    constexpr int NW = NTH / 64, WARPS_N = NW / WARPS_M;
    constexpr int WM = BM / WARPS_M, WN = BN / WARPS_N;
    constexpr int TM = WM / 32, TN = WN / 32;
    static_assert(TM >= 1 && TN >= 1 && WARPS_M * WARPS_N == NW, "wave tiling");
    constexpr bool B_MN = OP == OP_NN;
    using SA = Stage16<BM, BK, false, TA, NTH>;
    using SB = Stage16<BN, BK, B_MN, TB, NTH>;
    constexpr int BUF = SA::IMG + SB::IMG;

    extern __shared__ __attribute__((aligned(16))) unsigned short lds[];     // 2 × BUF

    const int nwg = gridDim.x, b = blockIdx.x;
    const int xcd = b & 7, qq = nwg >> 3, rr = nwg & 7;
    const int t = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (b >> 3);
    const int tn = t % a.tiles_n;
    const int tm = (t / a.tiles_n) % a.tiles_m;
    const int m0 = tm * BM, n0 = tn * BN;
    const int K = a.K;

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WARPS_N, wn = w % WARPS_N;
    const int r = lane & 31;

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    SA sa;
    SB sb;
    sa.prep(OP == OP_NT ? a.ridx : nullptr, m0, a.M, tid);
    if (!B_MN) sb.prep(nullptr, n0, a.N, tid);
    const bool vec = a.vec != 0;
    const TA* __restrict__ PA = static_cast<const TA*>(a.A);
    const TB* __restrict__ PB = static_cast<const TB*>(a.B);
    unsigned short* const buf0 = lds;
    unsigned short* const buf1 = lds + BUF;

    auto load = [&](int j) {
        sa.load(PA, a.lda, m0, a.M, j * BK, K, vec, tid);
        sb.load(PB, a.ldb, n0, a.N, j * BK, K, vec, tid);
    };
    constexpr int AB = PPO_G16_ABLATE;
    auto stamp = [&](int slot) {
#if PPO_G16_ABLATE & 32
        if (tid == 0 && b < 8192) {
            g_g16_stamps[b * 8 + slot] = __builtin_amdgcn_s_memtime();
            if (slot == 0 || slot == 3) g_g16_stamps[b * 8 + 4 + slot / 3] = __builtin_amdgcn_s_memrealtime();
        }
#endif
        (void)slot;
    };
    stamp(0);
    auto kstep = [&](const unsigned short* img, int ks) {
        bf16x8 fa[TM], fb[TN];
        if constexpr (AB & 16) {
#pragma unroll
            for (int i = 0; i < TM; ++i) fa[i] = __builtin_bit_cast(bf16x8, u32x4{(unsigned)ks, 1u, 2u, 3u});
#pragma unroll
            for (int j = 0; j < TN; ++j) fb[j] = __builtin_bit_cast(bf16x8, u32x4{(unsigned)lane, 1u, 2u, 3u});
        } else {
#pragma unroll
            for (int i = 0; i < TM; ++i) fa[i] = SA::frag(img, wm * WM + i * 32 + r, ks, lane);
#pragma unroll
            for (int j = 0; j < TN; ++j) fb[j] = SB::frag(img + SA::IMG, wn * WN + j * 32 + r, ks, lane);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                if constexpr (AB & 1) {
                    acc[i][j][0] += __builtin_bit_cast(u32x4, fa[i])[0] ^ __builtin_bit_cast(u32x4, fb[j])[1];
                } else {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
                }
            }
    };

    const int nk = (K + BK - 1) / BK;
    if (nk > 0) {
        load(0);
        sa.store(buf0, tid);
        sb.store(buf0 + SA::IMG, tid);
    }
    if (nk > 1) load(1);
    __syncthreads();
    int j = 0;
    // steady state: tile j's k-steps from one image; tile j+1's LDS stores into the other between
    // them; tile j+2's loads behind; one barrier
    for (; j < nk - 2; ++j) {
        const unsigned short* cur = (j & 1) ? buf1 : buf0;
        unsigned short* nxt = (j & 1) ? buf0 : buf1;
        kstep(cur, 0);
        __builtin_amdgcn_sched_barrier(0);
        kstep(cur, 1);
        if constexpr (!(AB & 8)) sa.store(nxt, tid);
        __builtin_amdgcn_sched_barrier(0);
        kstep(cur, 2);
        if constexpr (!(AB & 8)) sb.store(nxt + SA::IMG, tid);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!(AB & 4)) load(j + 2);
        kstep(cur, 3);
        __syncthreads();
    }
    for (; j < nk; ++j) {                                     // the last one or two tiles
        const unsigned short* cur = (j & 1) ? buf1 : buf0;
        unsigned short* nxt = (j & 1) ? buf0 : buf1;
#pragma unroll
        for (int ks = 0; ks < BK / 16; ++ks) kstep(cur, ks);
        if (j + 1 < nk) {
            sa.store(nxt, tid);
            sb.store(nxt + SA::IMG, tid);
        }
        __syncthreads();
    }

    stamp(1);
    if constexpr (AB & 2) {                                   // keep the accumulators live
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int jj = 0; jj < TN; ++jj)
#pragma unroll
                for (int e = 0; e < 16; ++e) t += acc[i][jj][e];
        if (t == 1234.5f) static_cast<float*>(a.C)[tid] = t;
        return;
    }
    static_assert((size_t)BM * (BN + 32) <= 2 * (size_t)BUF, "gemm16 (db): C image exceeds LDS");
    epilogue256<OP, BM, BN, TM, TN, NTH, TC>(a, acc, lds, m0, n0, wm, wn, tid, stamp);
}

// s_waitcnt vmcnt(N) with N a compile-time count of this wave's outstanding vector-memory operations
// (the prologue waits below: "all but the pieces of the second image have landed", so N = the 1-KiB
// pieces one wave issues per k-tile — derived from the tile constants, never a literal)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N <= 63, "vmcnt immediate");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// One LDS-DMA piece: 16 B per lane from `g` into the wave's 1 KiB at `l` (global_load_lds_dwordx4).
// Issued from asm: the compiler's waitcnt pass treats __builtin_amdgcn_global_load_lds as an LDS
// store of unknown extent and puts `s_waitcnt vmcnt(0)` in front of the next ds_read of ANY image —
// in the double-buffered loops below the DMA of tile j+2, issued right after the barrier, then had
// to land before tile j+1's first fragment read, exposing the whole DMA latency once per k-tile.
// Hidden from that pass, each image is published only by the loops' own `s_waitcnt vmcnt` +
// barrier (the "memory" clobber keeps the compiler's LDS accesses in program order around it).
// PPO_G16_BUILTIN_DMA=1 restores the builtin (A/B).
typedef __attribute__((address_space(3))) void* lds_vptr;
typedef __attribute__((address_space(1))) void* glb_vptr;
__device__ __forceinline__ void dma16(glb_vptr g, lds_vptr l) {
#if defined(PPO_G16_BUILTIN_DMA) && PPO_G16_BUILTIN_DMA
    __builtin_amdgcn_global_load_lds(g, l, 16, 0, 0);
#else
    const unsigned base = __builtin_amdgcn_readfirstlane((unsigned)(unsigned long)l);
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(base) : "memory");
#endif
}

// ---------------------------------------------------------------------------
// LDS-DMA 256×256 tile (forward and grad_x with bf16 operands, K a multiple of 64): each k-tile's A
// and B images arrive by global_load_lds_dwordx4 (1 KiB per wave-instruction, no VGPR staging, no
// ds_write pass), two images, one barrier per k-tile; the next k-step's fragments are read while
// this k-step's MFMAs run.  Images are unpadded with XOR-swizzled 16-B chunks, the swizzle applied
// on the per-lane global SOURCE address (the DMA destination is lane-linear):
//   k-contiguous [R][64]:  row R's chunk c (k 8c..8c+7) at position c ^ ((R >> 1) & 7) — the 16
//                          rows of a ds_read_b128 lane group land on 16 distinct 16-B bank slots
//   n-contiguous [64][256] (grad_x's W): k-row q's chunk c (n 8c..8c+7) at c ^ ((q & 3) << 2) —
//                          the 4 k-rows of a ds_read_b64_tr_b16 group on distinct 64-B bank ranges
// Measured at C5 16384×1024×1024 (profiles/r02_gemm16_dma.txt): forward 47.5 -> 41.3 µs, grad_x
// 44.8 -> 43.1 µs against the register-staged kernel above.  Not adopted: a ring of 4 or 5 stages
// of 32 k (one barrier per stage; forward 42.4 / 43.2, grad_x 49.2 / 51.4 µs) and a tile-dependent
// rotation of the k order (forward 44.4 µs: tiles sharing an A panel stop sharing its L2 lines).
// The MFMA-free loop alone (DMA + fragment reads + barriers) takes 45k of the forward's 56k
// mainloop cycles: the per-CU operand intake (≈ 50 GB/s per CU), not the MFMA, bounds it.
// ---------------------------------------------------------------------------
template <int OP, typename TC>
__global__ __launch_bounds__(512, 1) void gemm_bf16_dma_kernel(Args a) {
    static_assert(OP != OP_TN, "forward / grad_x only");
    constexpr int BM = 256, BN = 256, BK = 64, NTH = 512, WARPS_N = 2;
    constexpr int WM = 64, WN = 128, TM = 2, TN = 4;
    constexpr bool B_MN = OP == OP_NN;
    constexpr int IMG = BM * BK;                       // elements per operand image (32 KiB)
    static_assert(IMG / 512 / 8 == 4, "dma(): 4 + 4 one-KiB pieces per wave per k-tile (the prologue wait)");
    constexpr int BUF = 2 * IMG;
    extern __shared__ __attribute__((aligned(16))) unsigned short lds[];     // max(2·BUF, C image)
    typedef __attribute__((address_space(3))) void* lds_ptr;
    typedef __attribute__((address_space(1))) void* g_ptr;

    const int nwg = gridDim.x, b = blockIdx.x;
    const int xcd = b & 7, qq = nwg >> 3, rr = nwg & 7;
    const int t = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (b >> 3);
    const int tn = t % a.tiles_n;
    const int tm = (t / a.tiles_n) % a.tiles_m;
    const int m0 = tm * BM, n0 = tn * BN;

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WARPS_N, wn = w % WARPS_N;
    const int r = lane & 31, h = lane >> 5;
    constexpr int AB = PPO_G16_ABLATE;
    auto stamp = [&](int slot) {
#if PPO_G16_ABLATE & 32
        if (tid == 0 && b < 8192) {
            g_g16_stamps[b * 8 + slot] = __builtin_amdgcn_s_memtime();
            if (slot == 0 || slot == 3) g_g16_stamps[b * 8 + 4 + slot / 3] = __builtin_amdgcn_s_memrealtime();
        }
#endif
        (void)slot;
    };
    stamp(0);

    // DMA sources: wave w fills the images' 1-KiB pieces 4w..4w+3 (piece q: rows 8q..8q+7 of a
    // k-contiguous image, k-rows 2q, 2q+1 of the n-contiguous one); element offsets without k0
    const unsigned short* __restrict__ PA = static_cast<const unsigned short*>(a.A);
    const unsigned short* __restrict__ PB = static_cast<const unsigned short*>(a.B);
    int offa[4], offb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int q = 4 * w + i;
        {
            const int row = 8 * q + (lane >> 3), p = lane & 7, c = p ^ ((row >> 1) & 7);
            const int gr = min(m0 + row, a.M - 1);
            offa[i] = (a.ridx ? a.ridx[gr] : gr) * a.lda + 8 * c;
        }
        if (!B_MN) {
            const int row = 8 * q + (lane >> 3), p = lane & 7, c = p ^ ((row >> 1) & 7);
            offb[i] = min(n0 + row, a.N - 1) * a.ldb + 8 * c;
        } else {
            const int kr = 2 * q + (lane >> 5), p = lane & 31, c = p ^ ((kr & 3) << 2);
            offb[i] = kr * a.ldb + n0 + 8 * c;
        }
    }
    const int kstride_b = B_MN ? BK * a.ldb : BK;     // element step of B's source per k-tile
    const int nk = a.K / BK;
    auto dma = [&](int j, unsigned short* img) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            dma16((g_ptr)(PA + offa[i] + j * BK), (lds_ptr)(img + (4 * w + i) * 512));
#pragma unroll
        for (int i = 0; i < 4; ++i)
            dma16((g_ptr)(PB + offb[i] + (long)j * kstride_b),
                  (lds_ptr)(img + IMG + (4 * w + i) * 512));
    };
    // fragment of k-step ks (elements k = 16ks + 8h .. +7) for image row R
    auto frag_k = [&](const unsigned short* img, int R, int ks) {
        const int c = (2 * ks + h) ^ ((R >> 1) & 7);
        return __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(img + R * BK + 8 * c));
    };
    auto frag_n = [&](const unsigned short* img, int col, int ks) {   // transposed read, n-contiguous
        const int gi = lane & 15, q = gi >> 2, p = gi & 3;
        const int cb = col - gi + 4 * p;                               // first of this lane's 4 columns
        typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
        const int kr = 16 * ks + 8 * h + q;                            // kr & 3 = q for both reads
        const int pos = ((cb >> 3) ^ (q << 2)) * 8 + (cb & 7);
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + kr * BN + pos));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + (kr + 4) * BN + pos));
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        const s16x8 f = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return __builtin_bit_cast(bf16x8, f);
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    struct Fr { bf16x8 a[TM], b[TN]; };
    auto read = [&](const unsigned short* img, int ks, Fr& f) {
#pragma unroll
        for (int i = 0; i < TM; ++i) f.a[i] = frag_k(img, wm * WM + i * 32 + r, ks);
#pragma unroll
        for (int j = 0; j < TN; ++j)
            f.b[j] = B_MN ? frag_n(img + IMG, wn * WN + j * 32 + r, ks) : frag_k(img + IMG, wn * WN + j * 32 + r, ks);
    };
    auto mma = [&](const Fr& f) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                if constexpr (AB & 1) {
                    acc[i][j][0] += __builtin_bit_cast(u32x4, f.a[i])[0] ^ __builtin_bit_cast(u32x4, f.b[j])[1];
                } else {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[i], f.b[j], acc[i][j], 0, 0, 0);
                }
            }
    };

    unsigned short* const buf0 = lds;
    unsigned short* const buf1 = lds + BUF;
    dma(0, buf0);
    if (nk > 1) {
        dma(1, buf1);
        wait_vmcnt<4 + 4>();                                  // tile 0's 4 + 4 pieces (this wave's) landed
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    for (int j = 0; j < nk; ++j) {
        unsigned short* cur = (j & 1) ? buf1 : buf0;
        Fr f0, f1;
        read(cur, 0, f0);
        read(cur, 1, f1);
        mma(f0);
        read(cur, 2, f0);
        mma(f1);
        read(cur, 3, f1);
        mma(f0);
        mma(f1);
        // every wave is done reading `cur`, and tile j+1 has landed: refill `cur` with tile j+2
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (j + 2 < nk && !(AB & 4)) dma(j + 2, cur);
    }
    stamp(1);
    epilogue256<OP, BM, BN, TM, TN, NTH, TC>(a, acc, lds, m0, n0, wm, wn, tid, stamp);
}

// ---------------------------------------------------------------------------
// The same LDS-DMA tile on v_mfma_f32_16x16x32_bf16 (bf16 output with the LDS-staged epilogue): per
// 32-k step a wave's 64×128 tile is 4×8 blocks of 16×16, read as 4 A + 8 B fragments — the LDS
// traffic of the 32×32×16 form — while the MFMA measured ≈ 1.12–1.14× the 32×32×16 FLOP rate with
// operands re-read from LDS (MI355X_MICROARCH.md).  The k-contiguous swizzle is unchanged (its 16
// rows per lane group stay on distinct bank slots); grad_x's transposed W reads take chunk
// c ^ (((q & 3) << 2) | (((q >> 3) & 1) << 1)) for k-row q (the 16×16×32 B operand puts k-rows q
// and q + 8 in one 32-lane group).
// ---------------------------------------------------------------------------
template <int OP>
__global__ __launch_bounds__(512, 1) void gemm_bf16_dma16_kernel(Args a) {
    static_assert(OP != OP_TN, "forward / grad_x only");
    typedef float f32x4v __attribute__((ext_vector_type(4)));
    constexpr int BM = 256, BN = 256, BK = 64, NTH = 512, WARPS_N = 2;
    constexpr int WM = 64, WN = 128, TM = 4, TN = 8;           // 16×16 blocks per wave
    constexpr bool B_MN = OP == OP_NN;
    constexpr int IMG = BM * BK;
    static_assert(IMG / 512 / 8 == 4, "dma(): 4 + 4 one-KiB pieces per wave per k-tile (the prologue wait)");
    constexpr int BUF = 2 * IMG;
    extern __shared__ __attribute__((aligned(16))) unsigned short lds[];     // max(2·BUF, C image)
    typedef __attribute__((address_space(3))) void* lds_ptr;
    typedef __attribute__((address_space(1))) void* g_ptr;

    const int nwg = gridDim.x, b = blockIdx.x;
    const int xcd = b & 7, qq = nwg >> 3, rr = nwg & 7;
    const int t = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (b >> 3);
    const int tn = t % a.tiles_n;
    const int tm = (t / a.tiles_n) % a.tiles_m;
    const int m0 = tm * BM, n0 = tn * BN;

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WARPS_N, wn = w % WARPS_N;
    const int l15 = lane & 15, g4 = lane >> 4;
    auto swz_n = [](int kr) { return ((kr & 3) << 2) | (((kr >> 3) & 1) << 1); };

    const unsigned short* __restrict__ PA = static_cast<const unsigned short*>(a.A);
    const unsigned short* __restrict__ PB = static_cast<const unsigned short*>(a.B);
    int offa[4], offb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int q = 4 * w + i;
        {
            const int row = 8 * q + (lane >> 3), c = (lane & 7) ^ ((row >> 1) & 7);
            const int gr = min(m0 + row, a.M - 1);
            offa[i] = (a.ridx ? a.ridx[gr] : gr) * a.lda + 8 * c;
        }
        if (!B_MN) {
            const int row = 8 * q + (lane >> 3), c = (lane & 7) ^ ((row >> 1) & 7);
            offb[i] = min(n0 + row, a.N - 1) * a.ldb + 8 * c;
        } else {
            const int kr = 2 * q + (lane >> 5), c = (lane & 31) ^ swz_n(kr);
            offb[i] = kr * a.ldb + n0 + 8 * c;
        }
    }
    const int kstride_b = B_MN ? BK * a.ldb : BK;
    auto dma = [&](int j, unsigned short* img) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            dma16((g_ptr)(PA + offa[i] + j * BK), (lds_ptr)(img + (4 * w + i) * 512));
#pragma unroll
        for (int i = 0; i < 4; ++i)
            dma16((g_ptr)(PB + offb[i] + (long)j * kstride_b),
                  (lds_ptr)(img + IMG + (4 * w + i) * 512));
    };
    // 16×32 fragment of 32-k step s: row R = block base + (lane & 15), k = 32s + 8(lane >> 4) .. +7
    auto frag_k = [&](const unsigned short* img, int R, int s) {
        const int c = (4 * s + g4) ^ ((R >> 1) & 7);
        return __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(img + R * BK + 8 * c));
    };
    auto frag_n = [&](const unsigned short* img, int cbase, int s) {   // transposed read, n-contiguous
        const int q = l15 >> 2, p = l15 & 3;
        const int cb = cbase + 4 * p;
        typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
        const int kr = 32 * s + 8 * g4 + q;                            // kr + 4: same swizzle
        const int pos = ((cb >> 3) ^ swz_n(kr)) * 8 + (cb & 7);
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + kr * BN + pos));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + (kr + 4) * BN + pos));
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        const s16x8 f = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return __builtin_bit_cast(bf16x8, f);
    };

    f32x4v acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};

    auto step = [&](const unsigned short* img, int s) {
        bf16x8 fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = frag_k(img, wm * WM + i * 16 + l15, s);
#pragma unroll
        for (int j = 0; j < TN; ++j)
            fb[j] = B_MN ? frag_n(img + IMG, wn * WN + j * 16, s) : frag_k(img + IMG, wn * WN + j * 16 + l15, s);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    };

    const int nk = a.K / BK;
    unsigned short* const buf0 = lds;
    unsigned short* const buf1 = lds + BUF;
    dma(0, buf0);
    if (nk > 1) {
        dma(1, buf1);
        wait_vmcnt<4 + 4>();                                  // the 4 + 4 pieces per wave of dma() above
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    for (int j = 0; j < nk; ++j) {
        unsigned short* cur = (j & 1) ? buf1 : buf0;
        step(cur, 0);
        step(cur, 1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (j + 2 < nk) dma(j + 2, cur);
    }

    // epilogue: 16×16 block (i, j): lane holds column (lane & 15), rows 4(lane >> 4) + e; bias /
    // ReLU, then DPP-paired columns into the LDS C image (images free after the last barrier)
    constexpr int CP = BN + 32;
    unsigned short* const cimg = lds;
    const bool odd = lane & 1;
    float bcol[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int col = n0 + wn * WN + j * 16 + l15;
        bcol[j] = (OP == OP_NT && a.bias) ? a.bias[col < a.N ? col : a.N - 1] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            float vv[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float v = acc[i][j][e];
                if (OP == OP_NT) {
                    v += bcol[j];
                    if (a.relu) v = v > 0.f ? v : 0.f;
                }
                vv[e] = v;
            }
#pragma unroll
            for (int e = 0; e < 4; e += 2) {
                const float send = odd ? vv[e] : vv[e + 1];
                const float recv = __builtin_bit_cast(
                    float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, send), 0xB1, 0xF, 0xF, true));
                const float lo = odd ? recv : vv[e], hi = odd ? vv[e + 1] : recv;
                const int lrow = wm * WM + i * 16 + 4 * g4 + e + (odd ? 1 : 0);
                *reinterpret_cast<unsigned*>(cimg + lrow * CP + wn * WN + j * 16 + (l15 & ~1)) = pack2(lo, hi);
            }
        }
    c_image_out<OP, BM, BN, NTH>(a, cimg, m0, n0, tid);
}

// ---------------------------------------------------------------------------
// grad_W on the LDS-DMA tile (bf16 g and x, fp32 partials): gW[l, n] = gᵀ·x over one split of the
// batch.  Both operands are row-contiguous along the output's dimensions, so both images are
// [64 k][R] n-contiguous ones (the swizzle of gemm_bf16_dma16_kernel's grad_x W), every fragment a
// pair of hardware transposes; 256×BN tiles over 8 waves of 64×(BN/2) as 16×16×32 blocks, two
// images, one barrier per k-tile.  A split's partial tile leaves with plain stores into its slab
// (ppo::slab_reduce sums the slabs in a fixed order; 16 MB of f32 atomics per launch had set the
// register-staged kernel's time) or straight into gW for one split.  The bias gradient (Σ_k g) of
// the tiles in column 0 is summed from the g image: thread t adds 8 columns of 4 k-rows per k-tile
// (one ds_read_b128 each), the 16 k-row groups meet in LDS after the mainloop.
// ---------------------------------------------------------------------------
template <int BN>
__global__ __launch_bounds__(512, 1) void gemm_bf16_dma_tn_kernel(Args a, float* __restrict__ slab) {
    typedef float f32x4v __attribute__((ext_vector_type(4)));
    constexpr int BM = 256, BK = 64, WARPS_N = 2;
    constexpr int WM = 64, WN = BN / 2, TM = WM / 16, TN = WN / 16;
    constexpr int IMGA = BK * BM, IMGB = BK * BN, BUF = IMGA + IMGB;
    constexpr int PA_ = IMGA / 512 / 8, PB_ = IMGB / 512 / 8;      // 1-KiB pieces per wave
    static_assert(BN == 256 || BN == 128, "tile width");
    extern __shared__ __attribute__((aligned(16))) unsigned short lds[];
    typedef __attribute__((address_space(3))) void* lds_ptr;
    typedef __attribute__((address_space(1))) void* g_ptr;

    // XCD-aware remap (n fastest, then m, then split: one split's tiles share an XCD's L2)
    const int nwg = gridDim.x, b = blockIdx.x;
    const int xcd = b & 7, qq = nwg >> 3, rr = nwg & 7;
    const int t = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (b >> 3);
    const int tn = t % a.tiles_n;
    const int rest = t / a.tiles_n;
    const int tm = rest % a.tiles_m;
    const int split = rest / a.tiles_m;
    const int m0 = tm * BM, n0 = tn * BN;
    const int kbeg = split * a.kchunk;
    const int nk = (min(a.K, kbeg + a.kchunk) - kbeg) / BK;

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / WARPS_N, wn = w % WARPS_N;
    const int l15 = lane & 15, g4 = lane >> 4;
    auto swz = [](int kr) { return ((kr & 3) << 2) | (((kr >> 3) & 1) << 1); };

    const unsigned short* __restrict__ PA = static_cast<const unsigned short*>(a.A);
    const unsigned short* __restrict__ PB = static_cast<const unsigned short*>(a.B);
    int offa[PA_], offb[PB_];
#pragma unroll
    for (int i = 0; i < PA_; ++i) {                  // piece q: k-rows 2q, 2q+1 of the [64][256] image
        const int q = PA_ * w + i, kr = 2 * q + (lane >> 5), c = (lane & 31) ^ swz(kr);
        offa[i] = (kbeg + kr) * a.lda + m0 + 8 * c;
    }
#pragma unroll
    for (int i = 0; i < PB_; ++i) {
        const int q = PB_ * w + i;
        if constexpr (BN == 256) {
            const int kr = 2 * q + (lane >> 5), c = (lane & 31) ^ swz(kr);
            offb[i] = (kbeg + kr) * a.ldb + n0 + 8 * c;
        } else {                                     // [64][128]: k-rows 4q .. 4q+3 per piece
            const int kr = 4 * q + (lane >> 4), c = (lane & 15) ^ swz(kr);
            offb[i] = (kbeg + kr) * a.ldb + n0 + 8 * c;
        }
    }
    const long sa = (long)BK * a.lda, sb = (long)BK * a.ldb;
    auto dma = [&](int j, unsigned short* img) {
#pragma unroll
        for (int i = 0; i < PA_; ++i)
            dma16((g_ptr)(PA + offa[i] + j * sa), (lds_ptr)(img + (PA_ * w + i) * 512));
#pragma unroll
        for (int i = 0; i < PB_; ++i)
            dma16((g_ptr)(PB + offb[i] + j * sb),
                  (lds_ptr)(img + IMGA + (PB_ * w + i) * 512));
    };
    // transposed read of an n-contiguous image of pitch P: lane gets column cbase + (lane & 15),
    // k = 32s + 8(lane >> 4) .. +7
    auto frag = [&](const unsigned short* img, int P, int cbase, int s) {
        const int q = l15 >> 2, p = l15 & 3;
        const int cb = cbase + 4 * p;
        typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
        const int kr = 32 * s + 8 * g4 + q;                            // kr + 4: same swizzle
        const int pos = ((cb >> 3) ^ swz(kr)) * 8 + (cb & 7);
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + kr * P + pos));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + (kr + 4) * P + pos));
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        const s16x8 f = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return __builtin_bit_cast(bf16x8, f);
    };

    f32x4v acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};

    auto step = [&](const unsigned short* img, int s) {
        bf16x8 fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = frag(img, BM, wm * WM + i * 16, s);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = frag(img + IMGA, BN, wn * WN + j * 16, s);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                if constexpr (PPO_G16_ABLATE & 1)
                    acc[i][j][0] += __builtin_bit_cast(u32x4, fa[i])[0] ^ __builtin_bit_cast(u32x4, fb[j])[1];
                else
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
            }
    };

    const bool do_bias = a.gbias != nullptr && tn == 0;
    const int bcg = tid & 31, bkq = tid >> 5;           // bias: columns 8·bcg .. +7, k-rows 4·bkq .. +3
    float bs[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) bs[e] = 0.f;
    auto bias_tile = [&](const unsigned short* img) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int kr = 4 * bkq + r;
            const u32x4 v = *reinterpret_cast<const u32x4*>(img + kr * BM + 8 * (bcg ^ swz(kr)));
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                bs[2 * e] += bf_lo(v[e]);
                bs[2 * e + 1] += __builtin_bit_cast(float, v[e] & 0xffff0000u);
            }
        }
    };

    unsigned short* const buf0 = lds;
    unsigned short* const buf1 = lds + BUF;
    dma(0, buf0);
    if (nk > 1) {
        dma(1, buf1);
        wait_vmcnt<PA_ + PB_>();                              // tile 0's pieces (this wave's) landed
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    for (int j = 0; j < nk; ++j) {
        unsigned short* cur = (j & 1) ? buf1 : buf0;
        step(cur, 0);
        if (do_bias) bias_tile(cur);
        step(cur, 1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (j + 2 < nk && !(PPO_G16_ABLATE & 4)) dma(j + 2, cur);
    }
    if constexpr (PPO_G16_ABLATE & 2) {                       // keep the accumulators live
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int jj = 0; jj < TN; ++jj)
#pragma unroll
                for (int e = 0; e < 4; ++e) t += acc[i][jj][e];
        if (t == 1234.5f) static_cast<float*>(a.C)[tid] = t;
        return;
    }

    // a.cvec (split-K with gb = gW + l·n, the flat gradient layout): each split's bias partial goes
    // to its slab behind the gW partial and the slab reduce sums both — no atomics, no memset
    const long sstride = (long)a.M * a.N + (a.cvec ? a.M : 0);
    float* const out = a.splits > 1 ? slab + (long)split * sstride : static_cast<float*>(a.C);
    if (do_bias) {                                       // images free after the last barrier
        float* red = reinterpret_cast<float*>(lds);      // [16][256]
#pragma unroll
        for (int e = 0; e < 8; ++e) red[bkq * 256 + 8 * bcg + e] = bs[e];
        __syncthreads();
        if (tid < 256) {
            float s = 0.f;
#pragma unroll
            for (int q = 0; q < 16; ++q) s += red[q * 256 + tid];
            if (a.splits == 1) a.gbias[m0 + tid] = s;
            else if (a.cvec) out[(long)a.M * a.N + m0 + tid] = s;
            else atomicAdd(a.gbias + m0 + tid, s);
        }
    }
    // partial tile stores straight from the accumulators (16 lanes = 64 contiguous bytes per row;
    // staging through LDS for whole-row float4 stores measured 1.3 µs slower at C5)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int col = n0 + wn * WN + j * 16 + l15;
            const int r0 = m0 + wm * WM + i * 16 + 4 * g4;
#pragma unroll
            for (int e = 0; e < 4; ++e) out[(long)(r0 + e) * a.N + col] = acc[i][j][e];
        }
}

using f32 = float;
using b16 = unsigned short;

template <int OP, int BM, int BN, int WM_, int BK, typename TA, typename TB, typename TC, int MF = 32>
void launch(Args a) {
    a.tiles_m = ppo_divup(a.M, BM);
    a.tiles_n = ppo_divup(a.N, BN);
    if (a.splits < 1) a.splits = 1;
    const long grid = (long)a.tiles_m * a.tiles_n * a.splits;
    PPO_REQUIRE(grid > 0 && grid < (1L << 31), "gemm16: grid out of range");
    constexpr bool A_MN = OP == OP_TN, B_MN = OP != OP_NT;
    constexpr size_t lds = sizeof(unsigned short) * (Stage16<BM, BK, A_MN, TA>::IMG + Stage16<BN, BK, B_MN, TB>::IMG);
    static_assert(lds <= 160 * 1024, "gemm16: LDS image exceeds 160 KiB");
    auto kern = gemm_bf16_kernel<OP, BM, BN, WM_, BK, TA, TB, TC, MF>;
    if (lds > 64 * 1024) {
        static bool attr = false;                      // once per instantiation
        if (!attr) {
            PPO_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            attr = true;
        }
    }
    PPO_TIMED_LAUNCH(kern, dim3((unsigned)grid), dim3(NT_), lds, ppo::stream(), a);
    PPO_LAUNCH_CHECK();
}

template <int OP, typename TA, typename TB, typename TC, int NTH = 512, int WM_ = 4>
void launch_db(Args a) {
    constexpr int BM = 256, BN = 256, BK = 64;
    a.tiles_m = ppo_divup(a.M, BM);
    a.tiles_n = ppo_divup(a.N, BN);
    a.splits = 1;
    const long grid = (long)a.tiles_m * a.tiles_n;
    PPO_REQUIRE(grid > 0 && grid < (1L << 31), "gemm16 (db): grid out of range");
    PPO_REQUIRE(a.acopy == nullptr, "gemm16 (db): no gathered copy");
    constexpr size_t lds = 2 * sizeof(unsigned short) *
                           (Stage16<BM, BK, false, TA, NTH>::IMG + Stage16<BN, BK, OP == OP_NN, TB, NTH>::IMG);
    static_assert(lds <= 160 * 1024, "gemm16 (db): LDS images exceed 160 KiB");
    a.cvec = a.N % 8 == 0 && a.ldc % 8 == 0 && ((uintptr_t)a.C & 15u) == 0;
    auto kern = gemm_bf16_db_kernel<OP, BM, BN, WM_, BK, NTH, TA, TB, TC>;
    static bool attr = false;                          // once per instantiation
    if (!attr) {
        PPO_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        attr = true;
    }
    PPO_TIMED_LAUNCH(kern, dim3((unsigned)grid), dim3(NTH), lds, ppo::stream(), a);
    PPO_LAUNCH_CHECK();
}

int g_dma16 = -1;           // LDS-DMA 256×256 kernel: -1 = read PPO_G16_DMA (default 1 = on), 0 off

int dma16_setting() {
    if (g_dma16 < 0) {
        const char* e = getenv("PPO_G16_DMA");
        g_dma16 = e ? atoi(e) : 1;
    }
    return g_dma16;
}
// the 16×16×32 MFMA form for bf16-output DMA products and for grad_W (the round-2 PPO_G16_MF16 switch
// is gone: the 32×32×16 form remains only where this one does not apply).  Measured at C5 16384×1024×1024: forward 41.5 -> 37.3 µs,
// grad_x 42.1 -> 40.7 µs (C5 update 276.4 -> 271.9 ms); grad_W 82.6 -> 80.3 µs (273.7 -> 271.8 ms)
constexpr int g_mf16 = 1;

template <int OP, typename TC>
bool launch_dma(Args a) {
    dma16_setting();
    const bool ok = g_dma16 >= 1 && a.vec && a.acopy == nullptr && a.K % 64 == 0 && a.lda % 8 == 0 &&
                    a.ldb % 8 == 0 && (OP == OP_NT || a.N % 256 == 0) &&
                    (long)a.M * a.lda < (1L << 31) && (long)(OP == OP_NT ? a.N : a.K) * a.ldb < (1L << 31) &&
                    (((uintptr_t)a.A | (uintptr_t)a.B) & 15u) == 0;
    if (!ok) return false;
    a.tiles_m = ppo_divup(a.M, 256);
    a.tiles_n = ppo_divup(a.N, 256);
    a.splits = 1;
    a.cvec = a.N % 8 == 0 && a.ldc % 8 == 0 && ((uintptr_t)a.C & 15u) == 0;
    constexpr size_t lds = std::max<size_t>(2 * 2 * 2 * 256 * 64, 2 * 256 * (256 + 32));
    static_assert(lds <= 160 * 1024, "gemm16 (dma): LDS");
    const long grid = (long)a.tiles_m * a.tiles_n;
    if constexpr (sizeof(TC) == 2) {
        if (a.cvec && g_mf16 != 0) {                   // 16×16×32 MFMA form (bf16 output)
            auto kern = gemm_bf16_dma16_kernel<OP>;
            static bool attr = false;
            if (!attr) {
                PPO_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
                attr = true;
            }
            PPO_TIMED_LAUNCH(kern, dim3((unsigned)grid), dim3(512), lds, ppo::stream(), a);
            PPO_LAUNCH_CHECK();
            return true;
        }
    }
    auto kern = gemm_bf16_dma_kernel<OP, TC>;
    static bool attr = false;                          // once per instantiation
    if (!attr) {
        PPO_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        attr = true;
    }
    PPO_TIMED_LAUNCH(kern, dim3((unsigned)grid), dim3(512), lds, ppo::stream(), a);
    PPO_LAUNCH_CHECK();
    return true;
}

// tile configurations {BM, BN, BK}: 0 = 128x128 (4 waves of 64x64), 1 = 128x32 (skinny N),
// 2 = 32x128 (skinny M), 3 = 64x64, 4 = 128x128 with BK = 64, 5 = 256x128/64, 6 = 128x256/64,
// 7 = 256x128/32, 8 = 128x32 with BK = 64 (output-layer forward), 9 = 256x256/64 double-buffered
// over 8 waves of 64x128 (forward / grad_x; grad_W takes cfg 6).  Measured at C5 16384x1024x1024
// (profiles/r02_gemm16_db.txt): forward 54.1 -> 52.8 µs, grad_x 49.9 -> 46.4 µs against cfg 6; the
// same tile over 4 waves of 128x128 (one wave per SIMD) 73.6 / 59.7 µs (not adopted)
struct Cfg { int bm, bn, bk; };
constexpr Cfg kCfgs[] = {{128, 128, 32}, {128, 32, 32}, {32, 128, 32}, {64, 64, 32}, {128, 128, 64},
                         {256, 128, 64}, {128, 256, 64}, {256, 128, 32}, {128, 32, 64}, {128, 256, 64}};
int g_force16 = -1;
int g_split16 = 0;          // split-K workgroup target override for grad_W (0 = automatic)

template <int OP, typename TA, typename TB, typename TC>
void launch_cfg(int c, const Args& a) {
    switch (c) {
        case 0: launch<OP, 128, 128, 2, 32, TA, TB, TC>(a); break;
        case 1: launch<OP, 128, 32, 4, 32, TA, TB, TC>(a); break;
        case 2: launch<OP, 32, 128, 1, 32, TA, TB, TC>(a); break;
        case 3: launch<OP, 64, 64, 2, 32, TA, TB, TC>(a); break;
        case 4: launch<OP, 128, 128, 2, 64, TA, TB, TC>(a); break;
        case 5: launch<OP, 256, 128, 2, 64, TA, TB, TC>(a); break;       // waves of 128x64
        case 6:                                                          // waves of 64x128
            if constexpr (OP == OP_TN) {
                if (g_mf16 != 0 && g_mf16 != 2) { launch<OP, 128, 256, 2, 64, TA, TB, TC, 16>(a); break; }
            }
            launch<OP, 128, 256, 2, 64, TA, TB, TC>(a);
            break;
        case 7: launch<OP, 256, 128, 2, 32, TA, TB, TC>(a); break;
        case 9:
            if constexpr (OP != OP_TN) {
                if constexpr (sizeof(TA) == 2 && sizeof(TB) == 2) {
                    if (launch_dma<OP, TC>(a)) break;
                }
                if (a.vec && a.acopy == nullptr) { launch_db<OP, TA, TB, TC>(a); break; }
            }
            launch<OP, 128, 256, 2, 64, TA, TB, TC>(a);
            break;
        default: launch<OP, 128, 32, 4, 64, TA, TB, TC>(a); break;      // skinny N, BK64
    }
}

// measured (tools/gemm16_sweep.py, profiles/r01_gemm16_sweep*.txt): 128x256/BK64 (waves of 64x128)
// for all three products at the C5 shapes (grad_W with split-K at ~256 workgroups); 128x128/BK32
// where N is not a multiple of 256
int pick16(int M, int N, int op = OP_NT) {
    if (g_force16 >= 0) return g_force16;
    if (N <= 32 && M > 32) return op == OP_NT ? 8 : 1;   // output-layer forward: BK64 (13.8 vs 17.0 µs at C5)
    if (M <= 32 && N > 32) return 2;
    if (M <= 64 || N <= 64) return 3;
    // forward / grad_x with a grid of ≥ 256 double-buffered 256×256 tiles (one per CU)
    if (op != OP_TN && (long)ppo_divup(M, 256) * ppo_divup(N, 256) >= 256) return 9;
    if (N % 256 == 0 && M >= 256) return 6;
    return op == OP_NN ? 4 : 0;
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15u) == 0; }
inline int epl(int t) { return t ? 8 : 4; }

// grad_W on the LDS-DMA TN tile (bf16 g and x): l a multiple of 256, n of 128, the batch of 64;
// PPO_G16_TN=0 keeps the register-staged kernel, PPO_G16_TN_BN=128|256 (or ppo_gemm16_tn_width)
// sets the tile width — 256 × 128 by default: at C5 (1024-wide layers, 16384 rows) its 32 tiles × 8
// splits beat 16 tiles of 256 × 256 × 16 splits in the update, 235.5 vs 244.0 ms
// (profiles/r04_c5_gradw_tile_ab.txt): half the split-partial bytes for the slab reduce
// (C5's hidden layers, 16384 × 1024 × 1024, are the only production bf16 × bf16 grad_W shape: the
// 128 default is the measured choice there; other shapes take it too — they only occur in tests)
constexpr int g_tn_dma = 1;
int g_tn_bn = 128;                                 // ppo_gemm16_tn_width changes it (A/B)
constexpr int g_tn_target = 256;                   // workgroup target of the DMA TN split-K grid: one per CU

bool launch_dma_tn(float* gW, float* gb, const void* g, const void* x, int m, int n, int l, int zeroed) {
    if (g_tn_dma == 0 || dma16_setting() == 0 || g_force16 >= 0) return false;
    if (l % 256 != 0 || n % 128 != 0 || m % 64 != 0 || !al16(g) || !al16(x) || !al16(gW)) return false;
    if ((long)m * l >= (1L << 31) || (long)m * n >= (1L << 31)) return false;
    const int BN = g_tn_bn == 256 && n % 256 == 0 ? 256 : 128;
    if (n % BN != 0) return false;
    Args a{};
    a.A = g; a.lda = l; a.B = x; a.ldb = n; a.C = gW; a.ldc = n;
    a.M = l; a.N = n; a.K = m; a.gbias = gb;
    a.tiles_m = l / 256;
    a.tiles_n = n / BN;
    const long tiles = (long)a.tiles_m * a.tiles_n;
    const int target = g_split16 > 0 ? g_split16 : g_tn_target;
    int splits = (int)std::max<long>(1, target / tiles);
    splits = std::min(splits, std::max(1, m / (4 * 64)));              // ≥ 4 k-tiles per split
    a.kchunk = ppo_divup(ppo_divup(m, splits), 64) * 64;
    a.splits = splits = ppo_divup(m, a.kchunk);
    PPO_REQUIRE(tiles * splits < (1L << 31), "gemm16 (dma tn): grid out of range");
    a.cvec = gb && splits > 1 && gb == gW + (long)l * n;            // bias partials through the slabs
    if (gb && splits > 1 && !a.cvec && !zeroed) phip_memset(gb, 0, sizeof(float) * (size_t)l);
    const long sstride = (long)l * n + (a.cvec ? l : 0);
    float* slab = splits > 1 ? ppo::slab_scratch((size_t)splits * sstride) : nullptr;
    constexpr size_t lds256 = 2 * 2 * (64 * 256 + 64 * 256), lds128 = 2 * 2 * (64 * 256 + 64 * 128);
    static_assert(lds256 <= 160 * 1024 && lds128 <= 160 * 1024, "gemm16 (dma tn): LDS");
    static bool attr[2] = {false, false};
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const bool timed = ppo::take_kernel_events(&e0, &e1);      // one duration: GEMM start → reduce end
    hipEvent_t stop_k = timed && splits == 1 ? e1 : nullptr;
    const dim3 grid((unsigned)(tiles * splits));
    if (BN == 256) {
        auto kern = gemm_bf16_dma_tn_kernel<256>;
        if (!attr[0]) {
            PPO_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds256));
            attr[0] = true;
        }
        if (timed) hipExtLaunchKernelGGL(kern, grid, dim3(512), lds256, ppo::stream(), e0, stop_k, 0, a, slab);
        else hipLaunchKernelGGL(kern, grid, dim3(512), lds256, ppo::stream(), a, slab);
    } else {
        auto kern = gemm_bf16_dma_tn_kernel<128>;
        if (!attr[1]) {
            PPO_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds128));
            attr[1] = true;
        }
        if (timed) hipExtLaunchKernelGGL(kern, grid, dim3(512), lds128, ppo::stream(), e0, stop_k, 0, a, slab);
        else hipLaunchKernelGGL(kern, grid, dim3(512), lds128, ppo::stream(), a, slab);
    }
    PPO_LAUNCH_CHECK();
    if (splits > 1) ppo::slab_reduce(slab, gW, sstride, sstride, splits, timed ? e1 : nullptr);
    return true;
}

}  // namespace

extern "C" {

// dtype codes: 0 = fp32, 1 = bf16 (storage).  W16 is the bf16 shadow of W [l, n].
void phip_linear16_fwd(void* y, int ty, const void* x, int tx, const int* ridx, void* xcopy16, const void* W16,
                       const float* b, int m, int n, int l, int relu, unsigned* bits) {
    if (m <= 0 || l <= 0) return;
    PPO_REQUIRE(y && x && W16 && n > 0, "phip_linear16_fwd: null operand");
    ppo::ProfScope ps(PPO_K_GEMM, 2.0 * m * n * l, ppo::gemm_key(0, 2, m, n, l));
    Args a{};
    a.A = x; a.lda = n; a.B = W16; a.ldb = n; a.C = y; a.ldc = l;
    a.M = m; a.N = l; a.K = n; a.kchunk = n; a.splits = 1;
    a.bias = b; a.relu = relu; a.ridx = ridx; a.acopy = xcopy16;
    a.bits_out = relu ? bits : nullptr; a.wpr = ppo_divup(l, 32);
    a.vec = n % 8 == 0 && al16(x) && al16(W16);
    const int c = pick16(m, l);
    if (tx == 0 && ty == 0) launch_cfg<OP_NT, f32, b16, f32>(c, a);
    else if (tx == 0) launch_cfg<OP_NT, f32, b16, b16>(c, a);
    else if (ty == 0) launch_cfg<OP_NT, b16, b16, f32>(c, a);
    else launch_cfg<OP_NT, b16, b16, b16>(c, a);
}

void phip_linear16_bwd_x(void* gx, int tgx, const void* g, int tg, const void* W16, const unsigned* bits, int m,
                         int n, int l) {
    if (m <= 0 || n <= 0) return;
    PPO_REQUIRE(gx && g && W16 && l > 0, "phip_linear16_bwd_x: null operand");
    ppo::ProfScope ps(PPO_K_GEMM, 2.0 * m * n * l, ppo::gemm_key(1, 2, m, n, l));
    Args a{};
    a.A = g; a.lda = l; a.B = W16; a.ldb = n; a.C = gx; a.ldc = n;
    a.M = m; a.N = n; a.K = l; a.kchunk = l; a.splits = 1;
    a.bits_in = bits; a.wpr = ppo_divup(n, 32);
    a.vec = l % epl(tg) == 0 && n % 8 == 0 && al16(g) && al16(W16);
    const int c = pick16(m, n, OP_NN);
    if (tg == 0 && tgx == 0) launch_cfg<OP_NN, f32, b16, f32>(c, a);
    else if (tg == 0) launch_cfg<OP_NN, f32, b16, b16>(c, a);
    else if (tgx == 0) launch_cfg<OP_NN, b16, b16, f32>(c, a);
    else launch_cfg<OP_NN, b16, b16, b16>(c, a);
}

void phip_linear16_bwd_w(float* gW, float* gb, const void* g, int tg, const void* x, int tx, int m, int n, int l,
                         int zeroed) {
    if (l <= 0 || n <= 0) return;
    PPO_REQUIRE(gW && g && x, "phip_linear16_bwd_w: null operand");
    ppo::ProfScope ps(PPO_K_GEMM, 2.0 * m * n * l, ppo::gemm_key(2, 2, m, n, l));
    if (m <= 0) {
        if (!zeroed) {
            phip_memset(gW, 0, sizeof(float) * (size_t)l * n);
            if (gb) phip_memset(gb, 0, sizeof(float) * (size_t)l);
        }
        return;
    }
    if (tg == 1 && tx == 1 && launch_dma_tn(gW, gb, g, x, m, n, l, zeroed)) return;
    const int c = pick16(l, n, OP_TN);
    const int BK = kCfgs[c].bk;
    const long tiles = (long)ppo_divup(l, kCfgs[c].bm) * ppo_divup(n, kCfgs[c].bn);
    // split-K: the grid stays at or below one round of workgroup slots (rounding the split count up
    // would put the last few workgroups into a second round)
    const int target = g_split16 > 0 ? g_split16 : (c == 6 ? 256 : 512);
    int splits = (int)(target / tiles);
    const int max_splits = m / (4 * BK) > 0 ? m / (4 * BK) : 1;          // ≥ 4 k-tiles per split
    if (splits > max_splits) splits = max_splits;
    if (splits < 1) splits = 1;
    int kchunk = ppo_divup(ppo_divup(m, splits), BK) * BK;
    splits = ppo_divup(m, kchunk);
    Args a{};
    a.A = g; a.lda = l; a.B = x; a.ldb = n; a.C = gW; a.ldc = n;
    a.M = l; a.N = n; a.K = m; a.kchunk = kchunk; a.splits = splits;
    a.gbias = gb;
    a.vec = l % epl(tg) == 0 && n % epl(tx) == 0 && al16(g) && al16(x);
    if (splits > 1 && !zeroed) {
        phip_memset(gW, 0, sizeof(float) * (size_t)l * n);
        if (gb) phip_memset(gb, 0, sizeof(float) * (size_t)l);
    }
    if (tg == 0 && tx == 0) launch_cfg<OP_TN, f32, f32, f32>(c, a);
    else if (tg == 0) launch_cfg<OP_TN, f32, b16, f32>(c, a);
    else if (tx == 0) launch_cfg<OP_TN, b16, f32, f32>(c, a);
    else launch_cfg<OP_TN, b16, b16, f32>(c, a);
}

int ppo_gemm16_tune(int force_cfg) {
    g_force16 = force_cfg;
    return (int)(sizeof(kCfgs) / sizeof(kCfgs[0]));
}

// Tuning utility: average device µs of one bf16 launch — op 0 forward (bf16 in/out, +ReLU/bits),
// 1 grad_x (bf16), 2 grad_W (bf16 operands, fp32 out), 3 output-layer forward (fp32 out) — at
// m = batch, n = in, l = out.
double ppo_bench_gemm16(int op, int m, int n, int l, int iters, int cfg, int splitk_target) {
    ppo::ensure_device();
    const size_t sx = (size_t)m * n, sw = (size_t)l * n, sy = (size_t)m * l;
    unsigned short* x = (unsigned short*)phip_malloc(2 * sx);
    unsigned short* W = (unsigned short*)phip_malloc(2 * sw);
    unsigned short* y = (unsigned short*)phip_malloc(2 * (sy > sx ? sy : sx));
    float* tmp = (float*)phip_malloc(4 * (sx > sw ? (sx > sy ? sx : sy) : (sw > sy ? sw : sy)));
    float* b = (float*)phip_malloc(4 * (size_t)(l > n ? l : n));
    float* gw = (float*)phip_malloc(4 * sw);
    unsigned* bits = (unsigned*)phip_malloc(4 * (size_t)m * ppo_divup(l > n ? l : n, 32));
    phip_fill_uniform(tmp, (long)sx, 1, -1.f, 1.f);
    phip_f32_to_bf16(x, tmp, (long)sx);
    phip_fill_uniform(tmp, (long)sw, 2, -0.05f, 0.05f);
    phip_f32_to_bf16(W, tmp, (long)sw);
    phip_fill_uniform(tmp, (long)(sy > sx ? sy : sx), 3, -1.f, 1.f);
    phip_f32_to_bf16(y, tmp, (long)(sy > sx ? sy : sx));
    const int saved = g_force16, saved_split = g_split16;
    g_force16 = cfg;
    g_split16 = splitk_target;
    auto run = [&]() {
        if (op == 0) phip_linear16_fwd(y, 1, x, 1, nullptr, nullptr, W, b, m, n, l, 1, bits);
        else if (op == 3) phip_linear16_fwd(tmp, 0, x, 1, nullptr, nullptr, W, b, m, n, l, 0, nullptr);   // output layer
        else if (op == 1) phip_linear16_bwd_x(x, 1, y, 1, W, bits, m, n, l);
        else phip_linear16_bwd_w(gw, b, y, 1, x, 1, m, n, l, 0);
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
    g_force16 = saved;
    g_split16 = saved_split;
    phip_free(x); phip_free(W); phip_free(y); phip_free(tmp); phip_free(b); phip_free(gw); phip_free(bits);
    return 1000.0 * ms / (iters > 0 ? iters : 1);
}

int ppo_g16_stamps(unsigned long long* out, int n) {
#if PPO_G16_ABLATE & 32
    phip_sync();
    PPO_CHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_g16_stamps), sizeof(unsigned long long) * (size_t)std::min(n, 8192 * 8)));
    return 8192 * 8;
#else
    (void)out; (void)n;
    return 0;
#endif
}

int ppo_gemm16_dma(int on) {
    const int old = dma16_setting();
    if (on == 0 || on == 1) g_dma16 = on;
    return old;
}

int ppo_gemm16_tn_width(int bn) {
    const int old = g_tn_bn;
    if (bn == 128 || bn == 256) g_tn_bn = bn;
    return old;
}

}  // extern "C"
