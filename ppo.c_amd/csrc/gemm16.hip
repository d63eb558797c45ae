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
//
// Design (gfx950):
//  * 256-thread workgroups (4 waves), block tile BM×BN, BK = 32 (two MFMA k-steps per tile).
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
    long psA, psB, psC;                   // x3 engine: plane strides (elements) of pre-split operands / output
    int flags;                            // x3 experiment bits (PPO_X3_FLAGS): 1 = s_setprio 1 around the MFMAs
};

// fp32 → bf16, round to nearest even (NaN stays NaN: v_cvt_pk_bf16_f32)
__device__ __forceinline__ unsigned pack2(float lo, float hi) {
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    bf16x2 p = {(__bf16)lo, (__bf16)hi};
    return __builtin_bit_cast(unsigned, p);
}
__device__ __forceinline__ float bf_lo(unsigned u) { return __builtin_bit_cast(float, u << 16); }
__device__ __forceinline__ float bf_hi(unsigned u) { return __builtin_bit_cast(float, u & 0xffff0000u); }

// x3 output: v = h0 + h1 + h2 exactly (each bf16, round-to-nearest), plane q at dst + q·ps
__device__ __forceinline__ void store_planes(unsigned short* dst, long ps, float v) {
    const unsigned a = pack2(v, 0.f);
    const float r = v - bf_lo(a);
    const unsigned b = pack2(r, 0.f);
    const unsigned c = pack2(r - bf_lo(b), 0.f);
    dst[0] = (unsigned short)a;
    dst[ps] = (unsigned short)b;
    dst[2 * ps] = (unsigned short)c;
}

// ---------------------------------------------------------------------------
// Staging of one operand tile (R rows × BK k) into a bf16 LDS image.  T = float or unsigned short
// (bf16 bits).  One 16-B global load per slot: 4 fp32 or 8 bf16 elements.
// ---------------------------------------------------------------------------
template <int R, int BK, bool MN, typename T, int P = 1, bool FPI = false, int NTS = NT_>
struct Stage16 {
    static constexpr bool F32 = sizeof(T) == 4;
    static_assert(P == 1 || P == 3, "one bf16 image or three planes");
    static constexpr int EPL = F32 ? 4 : 8;                 // elements per 16-B load
    static constexpr int PK = BK + 8;                       // kcont pitch (elements) = 80 B
    static constexpr int PR = ((R / 2) % 64 == 16 || (R / 2) % 64 == 48) ? R : R + 32;   // mncont pitch
    static constexpr int IMG = MN ? BK * PR : R * PK;       // bf16 elements
    static constexpr int PER_ROW = MN ? R / EPL : BK / EPL; // loads along the contiguous dimension
    static constexpr int TOTAL = MN ? BK * PER_ROW : R * PER_ROW;
    static constexpr int ITERS = (TOTAL + NTS - 1) / NTS;
    static_assert(R % EPL == 0 && R >= 32, "tile rows");
    static constexpr bool PL = P == 3 && !F32;              // operand stored as three bf16 planes
    // FPI (x3, k-contiguous fp32 operand): the LDS image holds the fp32 values ([row][BK+4] floats)
    // and each wave splits its fragments after reading them (split at read, not at store)
    static_assert(!FPI || (F32 && !MN && P == 3), "fp32 image: fp32 k-contiguous x3 operands only");
    static constexpr int PKF = BK + 4;                      // fp32 pitch: 36 dwords at BK 32 (conflict-free b128)
    static constexpr int LDSZ = FPI ? R * PKF * 2 : IMG * P;   // LDS footprint in 16-bit units
    static constexpr int NV = PL ? 3 : 1;                   // 16-B loads per slot
    u32x4 v[ITERS * NV];
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

    // vec: every contiguous extent and ld are multiples of EPL and the base is 16-B aligned.
    // Pre-split planes (P == 3, bf16 storage): the three planes sit at src_p + q·pstride.
    __device__ __forceinline__ void load(const T* __restrict__ src_p, int ld, int r0, int Rmax, int k0, int kend,
                                         bool vec, int tid, long pstride = 0) {
#pragma unroll
        for (int it = 0; it < ITERS; ++it) {
            const int idx = tid + it * NTS;
            u32x4 x[NV];
#pragma unroll
            for (int q = 0; q < NV; ++q) x[q] = u32x4{0u, 0u, 0u, 0u};
            kok[it] = true;
            if (TOTAL % NTS == 0 || idx < TOTAL) {
                int row, k;
                coords(idx, row, k);
                const int gr = r0 + row, gk = k0 + k;
                if (vec) {
                    kok[it] = gk < kend;
                    const T* p = MN ? src_p + (long)(gk < kend ? gk : kend - 1) * ld + (gr < Rmax ? gr : Rmax - EPL)
                                    : src_p + (long)src[it] * ld + (gk < kend ? gk : kend - EPL);
#pragma unroll
                    for (int q = 0; q < NV; ++q) x[q] = *reinterpret_cast<const u32x4*>(p + q * pstride);
                } else {
#pragma unroll
                    for (int q = 0; q < NV; ++q) {
                        T e[EPL];
#pragma unroll
                        for (int c = 0; c < EPL; ++c) e[c] = T(0);
                        if (MN) {
                            if (gk < kend) {
                                const T* p = src_p + q * pstride + (long)gk * ld + gr;
#pragma unroll
                                for (int c = 0; c < EPL; ++c)
                                    if (gr + c < Rmax) e[c] = p[c];
                            }
                        } else if (gr < Rmax) {
                            const T* p = src_p + q * pstride + (long)src[it] * ld + gk;
#pragma unroll
                            for (int c = 0; c < EPL; ++c)
                                if (gk + c < kend) e[c] = p[c];
                        }
                        x[q] = __builtin_bit_cast(u32x4, e);
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < NV; ++q) v[it * NV + q] = x[q];
        }
    }

    __device__ __forceinline__ void store(unsigned short* img, int tid, bool nosplit = false) const {
#pragma unroll
        for (int it = 0; it < ITERS; ++it) {
            const int idx = tid + it * NTS;
            if (TOTAL % NTS == 0 || idx < TOTAL) {
                int row, k;
                coords(idx, row, k);
                unsigned short* d = img + (MN ? k * PR + row : row * PK + k);
                const u32x4 z = {0u, 0u, 0u, 0u};
                const u32x4 x = kok[it] ? v[it * NV] : z;
                if (FPI) {
                    *reinterpret_cast<u32x4*>(reinterpret_cast<float*>(img) + row * PKF + k) = x;
                } else if (PL) {
#pragma unroll
                    for (int q = 0; q < NV; ++q)
                        *reinterpret_cast<u32x4*>(d + q * IMG) = kok[it] ? v[it * NV + q] : z;
                } else if (F32 && P == 3 && nosplit) {          // ablation (PPO_X3_FLAGS & 8): no split
                    const f32x4 f = __builtin_bit_cast(f32x4, x);
                    const u32x2 p = {pack2(f[0], f[1]), pack2(f[2], f[3])};
                    *reinterpret_cast<u32x2*>(d) = p;
                    *reinterpret_cast<u32x2*>(d + IMG) = p;
                    *reinterpret_cast<u32x2*>(d + 2 * IMG) = p;
                } else if (F32 && P == 3) {
                    // exact 3-way split x = x0 + x1 + x2 (each bf16, round-to-nearest): x0 holds the
                    // top 8 significant bits, the residual x − x0 has ≤ 16 and x1 takes 8 of them, so
                    // x − x0 − x1 has ≤ 8 and is exactly a bf16 (fp32 subtractions are exact here)
                    const f32x4 f = __builtin_bit_cast(f32x4, x);
                    const unsigned a0 = pack2(f[0], f[1]), b0 = pack2(f[2], f[3]);
                    const float r0 = f[0] - bf_lo(a0), r1 = f[1] - bf_hi(a0);
                    const float r2 = f[2] - bf_lo(b0), r3 = f[3] - bf_hi(b0);
                    const unsigned a1 = pack2(r0, r1), b1 = pack2(r2, r3);
                    const unsigned a2 = pack2(r0 - bf_lo(a1), r1 - bf_hi(a1));
                    const unsigned b2 = pack2(r2 - bf_lo(b1), r3 - bf_hi(b1));
                    *reinterpret_cast<u32x2*>(d) = u32x2{a0, b0};
                    *reinterpret_cast<u32x2*>(d + IMG) = u32x2{a1, b1};
                    *reinterpret_cast<u32x2*>(d + 2 * IMG) = u32x2{a2, b2};
                } else if (F32) {
                    const f32x4 f = __builtin_bit_cast(f32x4, x);
                    const u32x2 p = {pack2(f[0], f[1]), pack2(f[2], f[3])};
                    *reinterpret_cast<u32x2*>(d) = p;
                } else {
                    *reinterpret_cast<u32x4*>(d) = x;
                }
            }
        }
    }

    // A-side fused gather: write the staged rows (rows < Rmax, k < kend) to dst[row*ldd + k] — as bf16,
    // or (3-plane split mode) as the fp32 values themselves
    __device__ __forceinline__ void copy_out(void* __restrict__ dstv, int ldd, int r0, int Rmax, int k0,
                                             int kend, int tid) const {
        if (PL) return;                      // (host never asks for a copy of pre-split planes)
        if (P == 3) {
            float* __restrict__ dst = static_cast<float*>(dstv);
#pragma unroll
            for (int it = 0; it < ITERS; ++it) {
                const int idx = tid + it * NTS;
                if (TOTAL % NTS == 0 || idx < TOTAL) {
                    int row, k;
                    coords(idx, row, k);
                    const int gr = r0 + row, gk = k0 + k;
                    if (gr >= Rmax) continue;
                    float* q = dst + (long)gr * ldd + gk;
                    const f32x4 f = __builtin_bit_cast(f32x4, v[it]);
                    if (gk + 3 < kend && (ldd & 3) == 0) {
                        *reinterpret_cast<f32x4*>(q) = f;
                    } else {
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            if (gk + e < kend) q[e] = f[e];
                    }
                }
            }
            return;
        }
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

    // FPI: the three bf16 planes of the k-step-ks fragment of image row `row` (k = 16·ks + 8h + j)
    __device__ __forceinline__ static void frag3(const unsigned short* img, int row, int ks, int lane, bf16x8& f0,
                                                 bf16x8& f1, bf16x8& f2) {
        const float* s = reinterpret_cast<const float*>(img) + row * PKF + 16 * ks + 8 * (lane >> 5);
        const f32x4 x = *reinterpret_cast<const f32x4*>(s), y = *reinterpret_cast<const f32x4*>(s + 4);
        const float e[8] = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
        u32x4 p0, p1, p2;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const unsigned a0 = pack2(e[2 * q], e[2 * q + 1]);
            const float r0 = e[2 * q] - bf_lo(a0), r1 = e[2 * q + 1] - bf_hi(a0);
            const unsigned a1 = pack2(r0, r1);
            p0[q] = a0;
            p1[q] = a1;
            p2[q] = pack2(r0 - bf_lo(a1), r1 - bf_hi(a1));
        }
        f0 = __builtin_bit_cast(bf16x8, p0);
        f1 = __builtin_bit_cast(bf16x8, p1);
        f2 = __builtin_bit_cast(bf16x8, p2);
    }

    // Σ over this tile's k of image row `row` (fp32), k ∈ [k_lo, k_lo + n); in 3-plane mode each
    // element is recombined exactly (x0 + x1 + x2) before it is added
    __device__ __forceinline__ static float rowsum(const unsigned short* img, int row, int k_lo, int n) {
        float t = 0.f;
        for (int kk = 0; kk < n; ++kk) {
            const int o = MN ? (k_lo + kk) * PR + row : row * PK + k_lo + kk;
            float e = __builtin_bit_cast(float, (unsigned)img[o] << 16);
            if (P == 3)
                e += __builtin_bit_cast(float, (unsigned)img[o + IMG] << 16) +
                     __builtin_bit_cast(float, (unsigned)img[o + 2 * IMG] << 16);
            t += e;
        }
        return t;
    }
};

template <typename T> struct Bits;
template <> struct Bits<float> { static constexpr int code = 0; };
template <> struct Bits<unsigned short> { static constexpr int code = 1; };

constexpr bool var_fpi(int v) { return v == 1 || v == 2 || v == 4 || v == 6; }   // fp32 images, split at read
constexpr bool var_pp(int v) { return v == 3 || v == 6; }                          // ping-pong tile pair
constexpr bool var_pc(int v) { return v == 7; }                     // producer / consumer waves, one tile
constexpr bool var_w8(int v) { return v == 8; }                     // one tile over all 8 waves
constexpr bool var_wide(int v) { return var_pp(v) || var_pc(v) || var_w8(v); }   // 512-thread workgroups
constexpr bool var_pipe(int v) { return v == 4 || v == 6; }                        // pipelined split at read

// VAR (x3 only): 0 = operands split into plane images at LDS-store time; 1 = k-contiguous fp32
// operands staged as fp32 and split at fragment read; 2 = as 1 with a double-buffered LDS image (one
// barrier per k-tile, the next tile's LDS write after this tile's MFMAs).  EOP = epilogue op (grad_x
// computed as an NT product against Wᵀ uses OP_NT staging with the OP_NN epilogue).
template <int OP, int BM, int BN, int WARPS_M, int BK, typename TA, typename TB, typename TC, int P, int VAR = 0,
          int EOP = OP>
__global__ __launch_bounds__(var_wide(VAR) ? 2 * NT_ : NT_, var_wide(VAR) ? 1 : 2) void gemm_bf16_kernel(Args a) {
    constexpr int NTH = var_w8(VAR) ? 2 * NT_ : NT_;          // threads sharing one tile
    constexpr int WARPS_N = NTH / 64 / WARPS_M;
    constexpr int WM = BM / WARPS_M, WN = BN / WARPS_N;
    constexpr int TM = WM / 32, TN = WN / 32;
    constexpr bool A_MN = OP == OP_TN, B_MN = OP != OP_NT;
    constexpr bool FPA = var_fpi(VAR) && !A_MN && sizeof(TA) == 4, FPB = var_fpi(VAR) && !B_MN && sizeof(TB) == 4;
    constexpr bool DB = VAR == 2;
    using SA = Stage16<BM, BK, A_MN, TA, P, FPA, NTH>;
    using SB = Stage16<BN, BK, B_MN, TB, P, FPB, NTH>;
    constexpr int BUF = SA::LDSZ + SB::LDSZ;                  // one LDS image (16-bit units)
    static_assert(!(DB && OP == OP_TN), "double-buffered image: no bias-gradient row sums");
    static_assert(TM >= 1 && TN >= 1, "wave tile must be a multiple of 32x32");
    static_assert(!(OP == OP_TN) || sizeof(TC) == 4, "grad_W accumulates in fp32");
    constexpr bool OUT_PL = P == 3 && sizeof(TC) == 2;      // x3: output written as three bf16 planes

    extern __shared__ __attribute__((aligned(16))) unsigned short lds[];     // (SA::IMG + SB::IMG) * P
    const bool prio = (a.flags & 1) != 0;

    // VAR 3 (ping-pong): a 512-thread workgroup holds two independent 256-thread groups, each with
    // its own output tile (tiles 2·t' and 2·t' + 1) and LDS image; one group splits and stages
    // while the other runs its MFMAs, then they swap (see the VAR 3 loop below)
    constexpr bool PP = var_pp(VAR);
    const int grp = PP ? (int)(threadIdx.x >> 8) : 0;
    const int nwg = gridDim.x, b = blockIdx.x;
    const int xcd = b & 7, qq = nwg >> 3, rr = nwg & 7;
    const int t1 = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (b >> 3);
    const int total = a.tiles_m * a.tiles_n * a.splits;
    auto tile_k = [&](int tt, int& kb, int& ke) {        // k range of linear tile tt (empty if none)
        if (tt >= total) { kb = ke = 0; return; }
        kb = (tt / (a.tiles_n * a.tiles_m)) * a.kchunk;
        ke = min(a.K, kb + a.kchunk);
    };
    const int t = PP ? 2 * t1 + grp : t1;
    const bool has_tile = !PP || t < total;
    const int tn = t % a.tiles_n;
    const int rest = t / a.tiles_n;
    const int tm = rest % a.tiles_m;
    const int m0 = tm * BM, n0 = tn * BN;
    int kbeg, kend;
    tile_k(PP ? t : 0, kbeg, kend);
    if (!PP) {
        kbeg = (rest / a.tiles_m) * a.kchunk;
        kend = min(a.K, kbeg + a.kchunk);
    }

    const int tid = threadIdx.x & (NTH - 1), lane = tid & 63, w = tid >> 6;
    const int wm = w / WARPS_N, wn = w % WARPS_N;
    const int r = lane & 31, h = lane >> 5;

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    constexpr int TPR = NTH / BM > 0 ? NTH / BM : 1;
    constexpr int KPT = BK / TPR > 0 ? BK / TPR : 1;
    const bool do_bsum = OP == OP_TN && EOP == OP_TN && a.gbias != nullptr && tn == 0 && (NTH % BM == 0) && has_tile;
    float bsum = 0.f;

    SA sa;
    SB sb;
    if (!A_MN) sa.prep(OP == OP_NT ? a.ridx : nullptr, m0, a.M, tid);
    if (!B_MN) sb.prep(nullptr, n0, a.N, tid);
    const bool do_copy = OP == OP_NT && a.acopy != nullptr && tn == 0 && has_tile;
    const bool vec = a.vec != 0;
    const TA* __restrict__ PA = static_cast<const TA*>(a.A);
    const TB* __restrict__ PB = static_cast<const TB*>(a.B);

    auto load = [&](int k0) {
        sa.load(PA, a.lda, m0, a.M, k0, kend, vec, tid, a.psA);
        sb.load(PB, a.ldb, n0, a.N, k0, kend, vec, tid, a.psB);
    };

    // one k-tile of MFMAs on the image at `img`
    auto compute = [&](const unsigned short* img) {
        const unsigned short* As = img;
        const unsigned short* Bs = img + SA::LDSZ;
        if (prio) __builtin_amdgcn_s_setprio(1);
        if constexpr (var_pipe(VAR)) {
            // fp32 images split at read, software-pipelined: k-step 1's fragment reads and splits
            // are interleaved with k-step 0's MFMAs (≈ 6 VALU per MFMA fill the MFMA's issue gap)
            static_assert(BK == 32, "two k-steps per tile");
            bf16x8 fa[2][P][TM], fb[2][P][TN];
            auto frags = [&](int ks, bf16x8 (&xa)[P][TM], bf16x8 (&xb)[P][TN]) {
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    if constexpr (FPA) SA::frag3(As, wm * WM + i * 32 + r, ks, lane, xa[0][i], xa[1][i], xa[2][i]);
                    else
#pragma unroll
                        for (int p = 0; p < P; ++p) xa[p][i] = SA::frag(As + p * SA::IMG, wm * WM + i * 32 + r, ks, lane);
                }
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    if constexpr (FPB) SB::frag3(Bs, wn * WN + j * 32 + r, ks, lane, xb[0][j], xb[1][j], xb[2][j]);
                    else
#pragma unroll
                        for (int p = 0; p < P; ++p) xb[p][j] = SB::frag(Bs + p * SB::IMG, wn * WN + j * 32 + r, ks, lane);
                }
            };
            auto mfmas = [&](const bf16x8 (&xa)[P][TM], const bf16x8 (&xb)[P][TN]) {
#pragma unroll
                for (int q = 0; q < 6; ++q) {
                    constexpr int pa_[6] = {2, 0, 1, 1, 0, 0}, pb_[6] = {0, 2, 1, 0, 1, 0};
#pragma unroll
                    for (int i = 0; i < TM; ++i)
#pragma unroll
                        for (int j = 0; j < TN; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xa[pa_[q]][i], xb[pb_[q]][j], acc[i][j],
                                                                                0, 0, 0);
                }
            };
            frags(0, fa[0], fb[0]);
            frags(1, fa[1], fb[1]);
            mfmas(fa[0], fb[0]);
            mfmas(fa[1], fb[1]);
            constexpr int NM = 6 * TM * TN;                 // MFMAs per k-step
            __builtin_amdgcn_sched_group_barrier(0x100, 4 * (TM + TN), 0);   // k-step 0 reads
            __builtin_amdgcn_sched_group_barrier(0x002, 200, 0);             // k-step 0 splits
            __builtin_amdgcn_sched_group_barrier(0x100, 4 * (TM + TN), 0);   // k-step 1 reads
#pragma unroll
            for (int q = 0; q < NM; ++q) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 7, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);
            if (prio) __builtin_amdgcn_s_setprio(0);
            return;
        }
#pragma unroll
        for (int ks = 0; ks < BK / 16; ++ks) {
            bf16x8 fa[P][TM], fb[P][TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                if constexpr (FPA) {
                    SA::frag3(As, wm * WM + i * 32 + r, ks, lane, fa[0][i], fa[P - 2][i], fa[P - 1][i]);
                } else {
#pragma unroll
                    for (int p = 0; p < P; ++p) fa[p][i] = SA::frag(As + p * SA::IMG, wm * WM + i * 32 + r, ks, lane);
                }
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                if constexpr (FPB) {
                    SB::frag3(Bs, wn * WN + j * 32 + r, ks, lane, fb[0][j], fb[P - 2][j], fb[P - 1][j]);
                } else {
#pragma unroll
                    for (int p = 0; p < P; ++p) fb[p][j] = SB::frag(Bs + p * SB::IMG, wn * WN + j * 32 + r, ks, lane);
                }
            }
            // 3-plane mode: the six products whose planes sum to ≤ 2 (smallest first); the three
            // dropped ones are below 2^-24 relative to the product
#pragma unroll
            for (int q = 0; q < (P == 3 ? 6 : 1); ++q) {
                constexpr int pa_[6] = {2, 0, 1, 1, 0, 0}, pb_[6] = {0, 2, 1, 0, 1, 0};
                const int pa = P == 3 ? pa_[q] : 0, pb = P == 3 ? pb_[q] : 0;
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[pa][i], fb[pb][j], acc[i][j], 0, 0, 0);
            }
        }
        if (prio) __builtin_amdgcn_s_setprio(0);
    };
    // PPO_X3_FLAGS ablations (timing diagnostics only, results wrong): 4 = no reload after the first
    // k-tile, 8 = no split (plane 0 in every plane), 16 = no MFMAs
    const bool nosplit = (a.flags & 8) != 0, noreload = (a.flags & 4) != 0, nomfma = (a.flags & 16) != 0;
    auto stage = [&](unsigned short* img, int k0) {
        if (do_copy) sa.copy_out(a.acopy, a.K, m0, a.M, k0, kend, tid);
        sa.store(img, tid, nosplit);
        sb.store(img + SA::LDSZ, tid, nosplit);
    };

    if constexpr (var_pc(VAR)) {
        // Producer / consumer waves (VAR 7): waves 4–7 only load, split and stage; waves 0–3 only
        // read fragments and run the MFMAs, one wave of each kind per SIMD, so the split VALU and
        // the LDS stores issue in the MFMA pipe's gaps.  Two plane images; one barrier per k-tile:
        // in iteration it the producers write tile it into image it&1 while the consumers multiply
        // tile it−1 from the other image (written before the previous barrier, and read before this
        // one ends, so the next write into it comes after).
        const bool producer = (threadIdx.x >> 8) != 0;
        const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
        if (producer) {
            // two register sets: tile it+2's loads are issued as tile it is staged, so each load
            // has two phases (≈ 2 × 48 MFMAs) to arrive
            SA sa1 = sa;
            SB sb1 = sb;
            auto load_set = [&](SA& xa, SB& xb, int k0) {
                xa.load(PA, a.lda, m0, a.M, k0, kend, vec, tid, a.psA);
                xb.load(PB, a.ldb, n0, a.N, k0, kend, vec, tid, a.psB);
            };
            auto stage_set = [&](SA& xa, SB& xb, unsigned short* img, int k0) {
                if (do_copy) xa.copy_out(a.acopy, a.K, m0, a.M, k0, kend, tid);
                xa.store(img, tid, nosplit);
                xb.store(img + SA::LDSZ, tid, nosplit);
            };
            if (nk > 0) load_set(sa, sb, kbeg);
            if (nk > 1) load_set(sa1, sb1, kbeg + BK);
            for (int it = 0; it < nk; ++it) {
                const int k0 = kbeg + it * BK;
                if (it & 1) {
                    stage_set(sa1, sb1, lds + BUF, k0);
                    if (it + 2 < nk) load_set(sa1, sb1, k0 + 2 * BK);
                } else {
                    stage_set(sa, sb, lds, k0);
                    if (it + 2 < nk) load_set(sa, sb, k0 + 2 * BK);
                }
                __syncthreads();
            }
            return;                                         // consumers run the epilogue
        }
        for (int it = 0; it < nk; ++it) {
            if (it >= 1) {
                const unsigned short* img = lds + ((it - 1) & 1) * BUF;
                if (do_bsum) bsum += SA::rowsum(img, tid / TPR, (tid % TPR) * KPT, KPT);
                if (!nomfma) compute(img);
            }
            __syncthreads();
        }
        if (nk > 0) {
            const unsigned short* img = lds + ((nk - 1) & 1) * BUF;
            if (do_bsum) bsum += SA::rowsum(img, tid / TPR, (tid % TPR) * KPT, KPT);
            compute(img);
        }
    } else if constexpr (PP) {
        // Ping-pong over two groups (one wave of each on every SIMD).  Phase A: group 0 splits and
        // stages its tile it while group 1 multiplies its tile it−1; phase B: group 0 multiplies tile
        // it while group 1 stages tile it.  The barrier between phases orders each group's LDS
        // write before its reads and its reads before its next write (one image per group), and
        // keeps the two groups half a k-tile apart, so one SIMD's MFMA pipe runs one group's
        // products while the other group's split (VALU) and LDS stores issue beside them.
        unsigned short* img = lds + grp * BUF;
        int kb0, ke0, kb1, ke1;
        tile_k(2 * t1, kb0, ke0);
        tile_k(2 * t1 + 1, kb1, ke1);
        const int nk0 = ke0 > kb0 ? (ke0 - kb0 + BK - 1) / BK : 0;
        const int nk1 = ke1 > kb1 ? (ke1 - kb1 + BK - 1) / BK : 0;
        const int nk = grp ? nk1 : nk0, nkmax = max(nk0, nk1);
        if (nk > 0) load(kbeg);
        auto stage_it = [&](int it) {
            const int k0 = kbeg + it * BK;
            stage(img, k0);
            if (it + 1 < nk && !noreload) load(k0 + BK);   // in flight through the partner's phase
        };
        auto compute_it = [&]() {
            if (do_bsum) bsum += SA::rowsum(img, tid / TPR, (tid % TPR) * KPT, KPT);
            if (!nomfma) compute(img);
        };
        for (int it = 0; it < nkmax; ++it) {
            if (grp == 0) {
                if (it < nk) stage_it(it);
            } else if (it >= 1 && it <= nk) {
                compute_it();
            }
            __syncthreads();
            if (grp == 0) {
                if (it < nk) compute_it();
            } else if (it < nk) {
                stage_it(it);
            }
            __syncthreads();
        }
        // group 1's last tile runs beside group 0's epilogue (no barrier after this point)
        if (grp == 1 && nk > 0 && nk == nkmax) compute_it();
        if (!has_tile) return;
    } else if constexpr (DB) {
        // double-buffered image: tile t+1's loads fly during tile t's MFMAs and are written into the
        // other image right after them; one barrier per k-tile
        if (kbeg < kend) {
            load(kbeg);
            stage(lds, kbeg);
        }
        __syncthreads();
        int cur = 0;
        for (int k0 = kbeg; k0 < kend; k0 += BK) {
            const bool more = k0 + BK < kend;
            if (more) load(k0 + BK);
            compute(lds + cur * BUF);
            if (more) stage(lds + (cur ^ 1) * BUF, k0 + BK);
            __syncthreads();
            cur ^= 1;
        }
    } else {
        if (kbeg < kend) load(kbeg);
        for (int k0 = kbeg; k0 < kend; k0 += BK) {
            stage(lds, k0);
            __syncthreads();
            if (k0 + BK < kend && !noreload) load(k0 + BK);   // in flight during this tile's MFMAs
            if (do_bsum) bsum += SA::rowsum(lds, tid / TPR, (tid % TPR) * KPT, KPT);
            if (!nomfma) compute(lds);
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
            if (EOP == OP_NT && a.bias) bcol = a.bias[col_ok ? col : a.N - 1];
            bool keep[16];
            if (EOP == OP_NN) {
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
                if (EOP == OP_NT) {
                    v += bcol;
                    if (a.relu) v = v > 0.f ? v : 0.f;
                    if (OUT_PL) {
                        if (ok) store_planes(static_cast<unsigned short*>(a.C) + off, a.psC, v);
                    } else if (Bits<TC>::code == 1) {
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
                } else if (EOP == OP_NN) {
                    if (ok) {
                        v = keep[e] ? v : 0.f;
                        if (OUT_PL) store_planes(static_cast<unsigned short*>(a.C) + off, a.psC, v);
                        else if (Bits<TC>::code == 1) static_cast<unsigned short*>(a.C)[off] =
                            (unsigned short)(pack2(v, 0.f) & 0xffffu);
                        else static_cast<float*>(a.C)[off] = v;
                    }
                } else if (ok) {
                    float* dst = static_cast<float*>(a.C) + off;
                    if (a.splits > 1) atomicAdd(dst, v);
                    else *dst = v;
                }
            }
            if (EOP == OP_NT && a.bits_out && r < 16) {
                const int row = r0 + (r & 3) + 8 * (r >> 2);
                if (row < a.M && c0 < a.N) a.bits_out[(long)row * a.wpr + (c0 >> 5)] = word;
            }
        }
}

using f32 = float;
using b16 = unsigned short;

template <int OP, int BM, int BN, int WM_, int BK, typename TA, typename TB, typename TC, int P = 1, int VAR = 0,
          int EOP = OP>
void launch(Args a) {
    a.tiles_m = ppo_divup(a.M, BM);
    a.tiles_n = ppo_divup(a.N, BN);
    if (a.splits < 1) a.splits = 1;
    const long tiles = (long)a.tiles_m * a.tiles_n * a.splits;
    const long grid = var_pp(VAR) ? (tiles + 1) / 2 : tiles;
    PPO_REQUIRE(grid > 0 && tiles < (1L << 31), "gemm16: grid out of range");
    constexpr bool A_MN = OP == OP_TN, B_MN = OP != OP_NT;
    constexpr size_t lds = sizeof(unsigned short) * (VAR == 2 || var_pp(VAR) || var_pc(VAR) ? 2 : 1) *
                           (Stage16<BM, BK, A_MN, TA, P, var_fpi(VAR) && !A_MN && sizeof(TA) == 4>::LDSZ +
                            Stage16<BN, BK, B_MN, TB, P, var_fpi(VAR) && !B_MN && sizeof(TB) == 4>::LDSZ);
    static_assert(lds <= 160 * 1024, "gemm16: LDS image exceeds 160 KiB");
    auto kern = gemm_bf16_kernel<OP, BM, BN, WM_, BK, TA, TB, TC, P, VAR, EOP>;
    if (lds > 64 * 1024) {
        static bool attr = false;                      // once per instantiation
        if (!attr) {
            PPO_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            attr = true;
        }
    }
    PPO_TIMED_LAUNCH(kern, dim3((unsigned)grid), dim3(var_wide(VAR) ? 2 * NT_ : NT_), lds, ppo::stream(), a);
    PPO_LAUNCH_CHECK();
}

// tile configurations {BM, BN, BK}: 0 = 128x128 (4 waves of 64x64), 1 = 128x32 (skinny N),
// 2 = 32x128 (skinny M), 3 = 64x64, 4 = 128x128 with BK = 64, 5 = 256x128/64, 6 = 128x256/64,
// 7 = 256x128/32, 8 = 128x32 with BK = 64 (output-layer forward)
struct Cfg { int bm, bn, bk; };
constexpr Cfg kCfgs[] = {{128, 128, 32}, {128, 32, 32}, {32, 128, 32}, {64, 64, 32}, {128, 128, 64},
                         {256, 128, 64}, {128, 256, 64}, {256, 128, 32}, {128, 32, 64}};
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
        case 6: launch<OP, 128, 256, 2, 64, TA, TB, TC>(a); break;       // waves of 64x128
        case 7: launch<OP, 256, 128, 2, 32, TA, TB, TC>(a); break;
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
    if (N % 256 == 0 && M >= 256) return 6;
    return op == OP_NN ? 4 : 0;
}


// ---------------------------------------------------------------------------
// fp32 GEMMs on the bf16 MFMA ("x3" engine): fp32 operands are split exactly into three bf16
// planes on the way into LDS and the six plane products with pa + pb ≤ 2 are accumulated in fp32.
// The dropped products (1,2), (2,1), (2,2) are < 2^-25 of |a·b|, so each product is carried to
// about fp32 rounding — same accuracy class as v_mfma_f32_32x32x2_f32 — at 6/16 of its MFMA cycles.
// LDS: three bf16 images per operand (128x128/BK32: 60 KiB, 2 workgroups per CU).
// tile configurations: 0 = 128x128, 1 = 128x32 (skinny N), 2 = 32x128 (skinny M), 3 = 64x64, all BK 32
// ---------------------------------------------------------------------------
int g_force3 = -1;
int g_split3 = 0;

template <int OP, typename TA, typename TB, typename TC, int EOP = OP>
void launch_cfg3(int c, const Args& a) {
    switch (c) {
        case 1: launch<OP, 128, 32, 4, 32, TA, TB, TC, 3, 0, EOP>(a); break;
        case 2: launch<OP, 32, 128, 1, 32, TA, TB, TC, 3, 0, EOP>(a); break;
        case 3: launch<OP, 64, 64, 2, 32, TA, TB, TC, 3, 0, EOP>(a); break;
        case 4: launch<OP, 128, 128, 2, 64, TA, TB, TC, 3, 0, EOP>(a); break;   // 110 KiB LDS: 1 workgroup per CU
        case 5: launch<OP, 128, 128, 2, 32, TA, TB, TC, 3, 1, EOP>(a); break;   // fp32 images, split at read
        case 6:                                                                  // + double-buffered image
            if constexpr (OP == OP_TN) launch<OP, 128, 128, 2, 32, TA, TB, TC, 3, 0, EOP>(a);
            else launch<OP, 128, 128, 2, 32, TA, TB, TC, 3, 2, EOP>(a);
            break;
        case 7: launch<OP, 128, 128, 2, 32, TA, TB, TC, 3, 3, EOP>(a); break;   // ping-pong pair of tiles
        case 8: launch<OP, 128, 128, 2, 32, TA, TB, TC, 3, 4, EOP>(a); break;   // fp32 images, pipelined split
        case 9: launch<OP, 128, 128, 2, 32, TA, TB, TC, 3, 6, EOP>(a); break;   // ping-pong + cfg 8
        case 10: launch<OP, 128, 128, 2, 32, TA, TB, TC, 3, 7, EOP>(a); break;  // producer / consumer waves
        case 11: launch<OP, 128, 256, 2, 32, TA, TB, TC, 3, 8, EOP>(a); break;  // 8 waves of 64x64
        case 12: launch<OP, 256, 128, 4, 32, TA, TB, TC, 3, 8, EOP>(a); break;  // 8 waves of 64x64
        default: launch<OP, 128, 128, 2, 32, TA, TB, TC, 3, 0, EOP>(a); break;
    }
}
constexpr Cfg kCfgs3[] = {{128, 128, 32}, {128, 32, 32}, {32, 128, 32}, {64, 64, 32}, {128, 128, 64},
                          {128, 128, 32}, {128, 128, 32}, {128, 128, 32}, {128, 128, 32}, {128, 128, 32},
                          {128, 128, 32}, {128, 256, 32}, {256, 128, 32}};
int g_flags3 = -1;          // PPO_X3_FLAGS (read once)
int flags3() {
    if (g_flags3 < 0) {
        const char* e = getenv("PPO_X3_FLAGS");
        g_flags3 = e ? atoi(e) : 0;
    }
    return g_flags3;
}

// Forward and grad_x with wide output (N a multiple of 128, large M): 256x128 tiles over 8 waves
// (cfg 12) stage 25 % fewer elements per output than two 128x128 workgroups (C4 512x512 forward
// 143 -> 120 us, grad_x 121 -> 112 us; profiles/r01_x3_8wave.txt); grad_W keeps the 128x128 tile
// (its split-K grid of 8-wave tiles measured slower).  cfg 8 (fp32 images split at fragment read,
// pipelined; 3-6 % faster per isolated launch than cfg 0, 1 % slower per C4 update) is opt-in via
// PPO_X3_PIPE=1 for the shapes cfg 12 does not take.
int pick3(int M, int N, int op = OP_TN) {
    if (g_force3 >= 0) return g_force3;
    if (N <= 32 && M > 32) return 1;
    if (M <= 32 && N > 32) return 2;
    if (M <= 64 || N <= 64) return 3;
    if (op == OP_TN) return 0;
    static const int wide = getenv("PPO_X3_NOWIDE") ? 0 : 12;      // A/B switch
    if (wide && M >= 2048 && N % 128 == 0) return wide;
    static const int pipe = getenv("PPO_X3_PIPE") ? 8 : 0;
    return pipe;
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// dst planes (stride m·S) of the rows src[rows[i]] (rows == nullptr: row i), 4 elements per thread
__global__ void gather_rows_x3_kernel(unsigned short* __restrict__ dst, const float* __restrict__ src,
                                      const int* __restrict__ rows, int m, int S, int vec) {
    const long ps = (long)m * S;
    const int per_row = vec ? S / 4 : S;
    const long total = (long)m * per_row;
    for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
        const int i = (int)(t / per_row), c = (int)(t % per_row);
        const long srow = rows ? rows[i] : i;
        if (vec) {
            const f32x4 f = *reinterpret_cast<const f32x4*>(src + srow * S + 4 * c);
            const unsigned a0 = pack2(f[0], f[1]), b0 = pack2(f[2], f[3]);
            const float r0 = f[0] - bf_lo(a0), r1 = f[1] - bf_hi(a0), r2 = f[2] - bf_lo(b0), r3 = f[3] - bf_hi(b0);
            const unsigned a1 = pack2(r0, r1), b1 = pack2(r2, r3);
            const unsigned a2 = pack2(r0 - bf_lo(a1), r1 - bf_hi(a1)), b2 = pack2(r2 - bf_lo(b1), r3 - bf_hi(b1));
            unsigned short* d = dst + (long)i * S + 4 * c;
            *reinterpret_cast<u32x2*>(d) = u32x2{a0, b0};
            *reinterpret_cast<u32x2*>(d + ps) = u32x2{a1, b1};
            *reinterpret_cast<u32x2*>(d + 2 * ps) = u32x2{a2, b2};
        } else {
            store_planes(dst + (long)i * S + c, ps, src[srow * S + c]);
        }
    }
}

__global__ void split_x3_kernel(unsigned short* __restrict__ dst, long stride, const float* __restrict__ p, long n) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        store_planes(dst + i, stride, p[i]);
}
inline int epl(int t) { return t ? 8 : 4; }

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
    const int c = pick16(l, n, OP_TN);
    const int BK = kCfgs[c].bk;
    const long tiles = (long)ppo_divup(l, kCfgs[c].bm) * ppo_divup(n, kCfgs[c].bn);
    const int target = g_split16 > 0 ? g_split16 : (c == 6 ? 256 : 512);
    int splits = (int)(target / tiles);                 // at or below one round (see x3 bwd_w)
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

// fp32-accurate products on the bf16 MFMA (x3 engine, above).  Operands are fp32 (split on the way
// into LDS) or pre-split (phip_opnd.planes: three bf16 planes at p + q·pstride); outputs of the
// forward and grad_x likewise (written split in the epilogue).  Supported storage combinations
// (everything else is a host bug): forward x ∈ {fp32, planes} with W planes, or all fp32 (the
// mat_mul API); grad_x g ∈ {fp32, planes} with W planes, or all fp32; grad_W any.
static inline bool al16o(const phip_opnd& o) { return al16(o.p) && (!o.planes || o.pstride % 8 == 0); }
static inline int eplo(const phip_opnd& o) { return o.planes ? 8 : 4; }

void phip_linear_x3_fwd(phip_opnd y, phip_opnd x, const int* ridx, float* xcopy, phip_opnd W, const float* b,
                        int m, int n, int l, int relu, unsigned* bits) {
    if (m <= 0 || l <= 0) return;
    PPO_REQUIRE(y.p && x.p && W.p && n > 0, "phip_linear_x3_fwd: null operand");
    PPO_REQUIRE(!(ridx && x.planes), "phip_linear_x3_fwd: fused gather from pre-split planes");
    PPO_REQUIRE(W.planes || (!x.planes && !y.planes), "phip_linear_x3_fwd: unsupported storage combination");
    ppo::ProfScope ps(PPO_K_GEMM, 2.0 * m * n * l, ppo::gemm_key(0, 1, m, n, l));
    Args a{};
    a.flags = flags3();
    a.A = x.p; a.lda = n; a.B = W.p; a.ldb = n; a.C = y.p; a.ldc = l;
    a.psA = x.pstride; a.psB = W.pstride; a.psC = y.pstride;
    a.M = m; a.N = l; a.K = n; a.kchunk = n; a.splits = 1;
    a.bias = b; a.relu = relu; a.ridx = ridx; a.acopy = ridx ? xcopy : nullptr;
    a.bits_out = relu ? bits : nullptr; a.wpr = ppo_divup(l, 32);
    a.vec = n % eplo(x) == 0 && n % eplo(W) == 0 && al16o(x) && al16o(W);
    const int c = pick3(m, l, OP_NT);
    if (!W.planes) launch_cfg3<OP_NT, f32, f32, f32>(c, a);
    else if (!x.planes && !y.planes) launch_cfg3<OP_NT, f32, b16, f32>(c, a);
    else if (!x.planes) launch_cfg3<OP_NT, f32, b16, b16>(c, a);
    else if (!y.planes) launch_cfg3<OP_NT, b16, b16, f32>(c, a);
    else launch_cfg3<OP_NT, b16, b16, b16>(c, a);
}

void phip_linear_x3_bwd_x(phip_opnd gx, phip_opnd g, phip_opnd W, const float* Wt, const unsigned* bits, int m,
                          int n, int l) {
    if (m <= 0 || n <= 0) return;
    PPO_REQUIRE(gx.p && g.p && W.p && l > 0, "phip_linear_x3_bwd_x: null operand");
    if (Wt && !g.planes && !gx.planes) {
        // gx = g·W as an NT product against Wᵀ [n, l]: both operands k-contiguous fp32
        ppo::ProfScope ps(PPO_K_GEMM, 2.0 * m * n * l);
        Args a{};
        a.flags = flags3();
        a.A = g.p; a.lda = l; a.B = Wt; a.ldb = l; a.C = gx.p; a.ldc = n;
        a.M = m; a.N = n; a.K = l; a.kchunk = l; a.splits = 1;
        a.bits_in = bits; a.wpr = ppo_divup(n, 32);
        a.vec = l % 4 == 0 && al16(g.p) && al16(Wt);
        launch_cfg3<OP_NT, f32, f32, f32, OP_NN>(pick3(m, n, OP_NT), a);
        return;
    }
    PPO_REQUIRE(W.planes || (!g.planes && !gx.planes), "phip_linear_x3_bwd_x: unsupported storage combination");
    ppo::ProfScope ps(PPO_K_GEMM, 2.0 * m * n * l, ppo::gemm_key(1, 1, m, n, l));
    Args a{};
    a.flags = flags3();
    a.A = g.p; a.lda = l; a.B = W.p; a.ldb = n; a.C = gx.p; a.ldc = n;
    a.psA = g.pstride; a.psB = W.pstride; a.psC = gx.pstride;
    a.M = m; a.N = n; a.K = l; a.kchunk = l; a.splits = 1;
    a.bits_in = bits; a.wpr = ppo_divup(n, 32);
    a.vec = l % eplo(g) == 0 && n % eplo(W) == 0 && al16o(g) && al16o(W);
    const int c = pick3(m, n, OP_NN);
    if (!W.planes) launch_cfg3<OP_NN, f32, f32, f32>(c, a);
    else if (!g.planes && !gx.planes) launch_cfg3<OP_NN, f32, b16, f32>(c, a);
    else if (!g.planes) launch_cfg3<OP_NN, f32, b16, b16>(c, a);
    else if (!gx.planes) launch_cfg3<OP_NN, b16, b16, f32>(c, a);
    else launch_cfg3<OP_NN, b16, b16, b16>(c, a);
}

void phip_linear_x3_bwd_w(float* gW, float* gb, phip_opnd g, phip_opnd x, int m, int n, int l, int zeroed) {
    if (l <= 0 || n <= 0) return;
    PPO_REQUIRE(gW && g.p && x.p, "phip_linear_x3_bwd_w: null operand");
    ppo::ProfScope ps(PPO_K_GEMM, 2.0 * m * n * l, ppo::gemm_key(2, 1, m, n, l));
    if (m <= 0) {
        if (!zeroed) {
            phip_memset(gW, 0, sizeof(float) * (size_t)l * n);
            if (gb) phip_memset(gb, 0, sizeof(float) * (size_t)l);
        }
        return;
    }
    const int c = pick3(l, n);
    const int BK = kCfgs3[c].bk;
    const long tiles = (long)ppo_divup(l, kCfgs3[c].bm) * ppo_divup(n, kCfgs3[c].bn);
    // target = workgroup slots of one round (2 per CU): the grid stays at or below it (rounding
    // the split count up would put the last few workgroups into a second round — 516 workgroups
    // for the 512 x 376 layer-0 gradient, 142 us instead of ~100)
    const int target = g_split3 > 0 ? g_split3 : 512;
    int splits = (int)(target / tiles);
    const int max_splits = m / (4 * BK) > 0 ? m / (4 * BK) : 1;          // ≥ 4 k-tiles per split
    if (splits > max_splits) splits = max_splits;
    if (splits < 1) splits = 1;
    int kchunk = ppo_divup(ppo_divup(m, splits), BK) * BK;
    splits = ppo_divup(m, kchunk);
    Args a{};
    a.flags = flags3();
    a.A = g.p; a.lda = l; a.B = x.p; a.ldb = n; a.C = gW; a.ldc = n;
    a.psA = g.pstride; a.psB = x.pstride;
    a.M = l; a.N = n; a.K = m; a.kchunk = kchunk; a.splits = splits;
    a.gbias = gb;
    a.vec = l % eplo(g) == 0 && n % eplo(x) == 0 && al16o(g) && al16o(x);
    if (splits > 1 && !zeroed) {
        phip_memset(gW, 0, sizeof(float) * (size_t)l * n);
        if (gb) phip_memset(gb, 0, sizeof(float) * (size_t)l);
    }
    if (!g.planes && !x.planes) launch_cfg3<OP_TN, f32, f32, f32>(c, a);
    else if (!g.planes) launch_cfg3<OP_TN, f32, b16, f32>(c, a);
    else if (!x.planes) launch_cfg3<OP_TN, b16, f32, f32>(c, a);
    else launch_cfg3<OP_TN, b16, b16, f32>(c, a);
}

void phip_gather_rows_x3(unsigned short* dst, const float* src, const int* rows, int m, int S) {
    if (m <= 0 || S <= 0) return;
    ppo::ProfScope ps(PPO_K_GATHER, 10.0 * m * S);
    const int vec = S % 4 == 0 && al16(src) && ((uintptr_t)dst & 7u) == 0 && ((long)m * S) % 4 == 0;
    const long total = (long)m * (vec ? S / 4 : S);
    const int grid = (int)std::min<long>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(gather_rows_x3_kernel, dim3(grid), dim3(256), 0, ppo::stream(), dst, src, rows, m, S, vec);
    PPO_LAUNCH_CHECK();
}

void phip_split_x3(unsigned short* dst, long stride, const float* p, long n) {
    if (n <= 0) return;
    const int grid = (int)std::min<long>((n + 255) / 256, 2048);
    hipLaunchKernelGGL(split_x3_kernel, dim3(grid), dim3(256), 0, ppo::stream(), dst, stride, p, n);
    PPO_LAUNCH_CHECK();
}

int ppo_gemm16_tune(int force_cfg) {
    g_force16 = force_cfg;
    return (int)(sizeof(kCfgs) / sizeof(kCfgs[0]));
}

// Tuning utility: average device µs of one bf16 launch — op 0 forward (bf16 in/out, +ReLU/bits),
// 1 grad_x (bf16), 2 grad_W (bf16 operands, fp32 out) — at m = batch, n = in, l = out.
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

}  // extern "C"
