// gemm_x3.hip — fp32 linear-layer GEMMs on the bf16 MFMA (the "x3" engine of fp32 mode).
//
// Reference products (mat_mul.cu:122-217 with the fused bias / ReLU of activation_function.cu:17-29
// and the bias-gradient sum of neural_network.cu:108-118):
//   forward   y  = x·Wᵀ + b (+ReLU, +ReLU′ bit mask, + the minibatch gather of x's rows)   NT
//   grad_x    gx = (g·W) ⊙ 1[y_prev > 0]                                                   NN
//   grad_W    gW = gᵀ·x, gb = Σ_rows g      (split-K over the batch, f32 atomics)          TN
//
// Arithmetic.  Every fp32 operand value splits exactly into three bf16 planes x = x0 + x1 + x2
// (round-to-nearest v_cvt_pk_bf16_f32 of x, of the residual, of the second residual: x0 carries 8
// significant bits, x − x0 ≤ 16 of which x1 takes 8, so x − x0 − x1 is itself a bf16).  A product
// a·b is Σ_{p+q≤2} a_p·b_q: six v_mfma_f32_32x32x16_bf16 with fp32 accumulation per fp32 product;
// the dropped terms (1,2), (2,1), (2,2) are below 2^-24 of |a·b|, so the engine is as accurate as
// the exact fp32 MFMA (tests/test_gpu_x3.py).  Ceiling: 2.5 PF/s ÷ 6 = 417 TF/s fp32-equivalent.
//
// Pipeline (one workgroup per CU):
//   * BK = 16 k-tiles; the three planes of both operand tiles live in a TRIPLE-buffered LDS ring,
//     one barrier per k-tile: while tile t's MFMAs run, the split + LDS stores of tile t+2 and the
//     global loads of tile t+3 are issued, and tile t+1's fragments (complete since the previous
//     barrier) are read into the fragment registers as tile t's plane products retire them — so
//     the MFMAs after a barrier start on fragments already in registers (no LDS-latency bubble per
//     k-tile, no extra registers: the plane-product order frees each fragment plane early);
//   * the split happens once per staged element (at LDS-store time), not once per wave reading it;
//   * images are unpadded and XOR-swizzled (the ring fits in 144 KiB): k-contiguous operands (x and
//     W of the forward) are staged [row][16] bf16 per plane with the two 16-B k-chunks of a row
//     swapped on odd 8-row groups — a fragment is one conflict-free ds_read_b128; row-contiguous
//     operands (W in grad_x, g and x in grad_W) are staged [k][R] with 32-B row segments XOR-permuted
//     per k-row and read with two ds_read_b64_tr_b16 hardware transposes per fragment, conflict-free;
//   * grad_W (split-K, f32 atomics) runs two k-groups per workgroup that sum through LDS, halving
//     the atomics per output element;
//   * XCD-aware block remap: tiles that share an operand panel run on one XCD's L2.
#include "dev.h"

#include <algorithm>
#include <type_traits>

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int BK = 16;
enum { OP_NT = 0, OP_NN = 1, OP_TN = 2 };

// diagnostic stamps (ABL & 32): s_memtime of wave 0 of each workgroup at kernel start, after the
// prologue, after the mainloop, at the end
__device__ unsigned long long g_x3_stamps[8192 * 8];

struct X3Args {
    const float* A; const float* B; float* C;
    int M, N, K, lda, ldb, ldc;
    const float* bias; int relu;
    const int* ridx; float* acopy;        // forward: fused gather of A's rows + the gathered copy
    unsigned* bits_out; const unsigned* bits_in; int wpr;
    float* gbias;                         // grad_W: bias gradient (Σ over the batch of g)
    int kchunk, splits, tiles_m, tiles_n;
    float* slab;                          // grad_W split-K: per-split partial tiles [splits][M][N] (plain
                                          // stores, summed by slab_reduce_kernel) instead of f32 atomics
    // value-head fold (the 1-wide output layer y = h·w + b of a value network folded into the last
    // hidden layer's kernels; neural_network.c nn_value_fold_step):
    const float* ydot;                    // forward: w — each wave's Σ_cols relu(z)·w per row into ypart
    float* ypart;                         //   [tiles_n · WARPS_N][M] (slot = column tile · WARPS_N + wave col)
    // backward: the upper gradient is G(i, c) = g_i·w_c·1[h(i, c) > 0] (g = ∂L/∂y), so with the 0/1 mask
    // as the operand — exact in one bf16 plane: three plane products instead of six — g and w become row /
    // column scales: grad_x = diag(g)·(mask·diag(w)·W) (W scaled per k-row by w as it is staged),
    // grad_W = diag(w)·(maskᵀ·diag(g)·x), grad_b = diag(w)·maskᵀ·g
    const float* fold_g;                  // g [M batch rows]
    const float* fold_w;                  // w [units] (grad_x: W's row scale — B = diag(w)·W staged from W)
    const unsigned* fold_bits;            // grad_x: the mask words of h [M][fold_wpr]
    int fold_wpr;
    float* fold_gw;                       // grad_W (A = h, fp32): + Σ_rows g·h per unit — the output layer's gW
    // grad_W fold carrying the value head (vh_ypart set): each workgroup forms g = 2(y − t)/m of its split's
    // batch rows from the forward's partial dots (y = Σ_slots ypart + b, slot order as the head kernel) in
    // LDS before its mainloop; tile (0, 0) of each split also writes y and g and adds the loss / m and the
    // output bias gradient Σ g (kernels.hip value_head_kernel, which runs instead when LDS is short)
    const float* vh_ypart; const float* vh_b; const float* vh_t;
    float* vh_y; float* vh_gb; float* vh_loss;
    int vh_slots;
    // grad_x carrying the previous grad_W's split-K reduction (phip_x3_defer_reduce): workgroups
    // gemm_wgs … gemm_wgs + red_wgs − 1 sum red_splits slabs of red_n floats (stride red_stride) into red_out
    const float* red_slab; float* red_out;
    long red_n, red_stride;
    int red_splits, red_wgs, gemm_wgs;
    hipEvent_t ev_start, ev_stop;         // explicit dispatch-stamped events (ppo_prof kernel timing)
};

// the split-K slab sum of ONE reduce workgroup of NTH threads, in slab_reduce_kernel<4>'s order (four split
// groups, each summing its splits in order, the groups' partials added in order): NTH/4 float4 columns per
// workgroup, so the result is bitwise that of the standalone reduce
template <int NTH>
__device__ __forceinline__ void x3_slab_reduce_block(const X3Args& a, int blk, float* part) {
    typedef float f32x4_ __attribute__((ext_vector_type(4)));
    constexpr int Q = 4, C = NTH / Q;
    const int c = threadIdx.x % C, q = threadIdx.x / C;
    const long n4 = (a.red_n + 3) >> 2, s4 = a.red_stride >> 2;
    const long i = (long)blk * C + c;
    const int per = (a.red_splits + Q - 1) / Q;
    const int s0 = q * per, s1 = min(a.red_splits, s0 + per);
    const f32x4_* __restrict__ sv = reinterpret_cast<const f32x4_*>(a.red_slab);
    f32x4_ acc = {0.f, 0.f, 0.f, 0.f};
    if (i < n4) {
#pragma unroll 8
        for (int sp = s0; sp < s1; ++sp) acc += sv[(long)sp * s4 + i];
    }
    f32x4_* pv = reinterpret_cast<f32x4_*>(part);
    if (q) pv[(q - 1) * C + c] = acc;
    __syncthreads();
    if (q == 0 && i < n4) {
#pragma unroll
        for (int v = 0; v < Q - 1; ++v) acc += pv[v * C + c];
        if (4 * i + 4 <= a.red_n) {
            reinterpret_cast<f32x4_*>(a.red_out)[i] = acc;
        } else {
            for (int e = 0; e < 4; ++e)
                if (4 * i + e < a.red_n) a.red_out[4 * i + e] = acc[e];
        }
    }
}

// fp32 → bf16 round to nearest even (NaN stays NaN): v_cvt_pk_bf16_f32
__device__ __forceinline__ unsigned pack2(float lo, float hi) {
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    bf16x2 p = {(__bf16)lo, (__bf16)hi};
    return __builtin_bit_cast(unsigned, p);
}
__device__ __forceinline__ float bf_lo(unsigned u) { return __builtin_bit_cast(float, u << 16); }
__device__ __forceinline__ float bf_hi(unsigned u) { return __builtin_bit_cast(float, u & 0xffff0000u); }

// the packed conversion, opaque: otherwise the compiler rebuilds bf_lo(pack2(lo, hi)) as a second
// single-value v_cvt_pk_bf16_f32 + shift (16 extra VALU per k-tile per wave in the x3 mainloop)
__device__ __forceinline__ unsigned pack2_opaque(float lo, float hi) {
    unsigned u = pack2(lo, hi);
    asm("" : "+v"(u));
    return u;
}

// exact three-plane split of 4 values: plane q gets 4 bf16 (2 dwords)
__device__ __forceinline__ void split4(f32x4 f, u32x2& p0, u32x2& p1, u32x2& p2) {
    const unsigned a0 = pack2_opaque(f[0], f[1]), b0 = pack2_opaque(f[2], f[3]);
    const float r0 = f[0] - bf_lo(a0), r1 = f[1] - bf_hi(a0);
    const float r2 = f[2] - bf_lo(b0), r3 = f[3] - bf_hi(b0);
    const unsigned a1 = pack2_opaque(r0, r1), b1 = pack2_opaque(r2, r3);
    p0 = u32x2{a0, b0};
    p1 = u32x2{a1, b1};
    p2 = u32x2{pack2(r0 - bf_lo(a1), r1 - bf_hi(a1)), pack2(r2 - bf_lo(b1), r3 - bf_hi(b1))};
}

// ---------------------------------------------------------------------------------------------
// One operand tile: R rows × BK k, fp32 in HBM → three bf16 planes in LDS.  NTH threads (one
// k-group), each owning NV float4 loads per k-tile.
// MN = the operand is contiguous along its rows (its k is the HBM row).
// ---------------------------------------------------------------------------------------------
template <int R, bool MN, int NTH, int KB = BK>
struct StageX3 {
    static_assert(KB == 16 || KB == 32, "x3 k-tile depth");
    static constexpr int NV = R * KB / (4 * NTH);            // float4 loads per thread
    static_assert(NV >= 1 && R * KB == 4 * NTH * NV, "tile / thread count");
    static_assert(R == 64 || R == 128 || R == 256, "x3 operand tile rows");
    static constexpr int PLANE = R * KB;                     // bf16 elements per plane (unpadded)
    static constexpr int SIZE = 3 * PLANE;
    // k-contiguous [row][KB]: element (row, k) — the 16-B chunks of a row XOR-permuted by its 8-row group
    // (KB 16: the two chunks swapped on odd groups; KB 32: four chunks permuted by the group mod 4)
    __device__ __forceinline__ static int kc_off(int row, int k) {
        return row * KB + 8 * ((k >> 3) ^ ((row >> 3) & (KB / 8 - 1))) + (k & 7);
    }
    // row-contiguous [k][R]: element (k, row) — 32-B segment s of k-row k sits at s ^ sw(k), so the
    // 4 k-rows × 2 segments a 32-lane group of ds_read_b64_tr_b16 touches cover the 8 bank groups
    __device__ __forceinline__ static int sw(int k) { return R >= 128 ? 2 * (k & 3) : 2 * ((k >> 1) & 1); }
    __device__ __forceinline__ static int mn_off(int k, int row) {
        return k * R + 16 * ((row >> 4) ^ sw(k)) + (row & 15);
    }
    static constexpr int TPR = KB / (4 * NV);                // k-contiguous: threads per row
    static constexpr int KSTEP = 4 * NTH / R;                // row-contiguous: k distance of the q-th load
    static_assert(MN || (TPR >= 1 && NTH * 4 * NV == R * KB), "k-contiguous mapping");

    f32x4 v[NV];
    const float* base;                                       // this thread's element (row, k) at k0 = 0
    int row, k;                                              // this thread's first element in the tile
    int ld;
    // value-head fold (FM, kernel FOLD): a row-contiguous operand's per-row scale — g of the k-tile's
    // batch rows, one per float4 load (FM 1) — or a k-contiguous operand taken from the 0/1 ReLU′ mask
    // words of its rows instead of fp32 values (FM 2)
    const float* sg;
    float gq[NV];
    const unsigned* bw_row;
    unsigned bword;

    // src row (k-contiguous: after the gather, clamped into the operand); rows past the end read row
    // Rmax − 1 (their products land in output rows that are never stored)
    __device__ __forceinline__ void init(const float* __restrict__ p, int ld_, const int* __restrict__ ridx, int r0,
                                         int Rmax, int tid) {
        ld = ld_;
        if (MN) {
            row = (tid % (R / 4)) * 4;
            k = tid / (R / 4);
            base = p + (long)k * ld + min(r0 + row, Rmax - 4);
        } else {
            // TPR consecutive lanes take one row's 16 k, the next TPR the next row: 8 lanes (a
            // ds_write_b128 lane group; 16 for ds_write_b64) then cover 4 rows × 32 B = 128 B, every
            // write bank ((a/4) mod 32) once; the global loads stay whole 64-B row segments
            row = tid / TPR;
            k = (tid % TPR) * 4 * NV;
            const int gr = min(r0 + row, Rmax - 1);
            base = p + (long)(ridx ? ridx[gr] : gr) * ld + k;
        }
    }
    __device__ __forceinline__ void init_fold(const float* __restrict__ g, const unsigned* __restrict__ bits, int wpr,
                                              int r0, int Rmax) {
        sg = g;
        if (!MN && bits) bw_row = bits + (long)min(r0 + row, Rmax - 1) * wpr;
    }
    // FULL: the whole k-tile lies inside [kbeg, kend) — no clamping
    template <bool FULL, int FM = 0>
    __device__ __forceinline__ void load(int k0, int kend) {
        if (MN) {
#pragma unroll
            for (int q = 0; q < NV; ++q) {
                const int dk = FULL ? k0 + q * KSTEP : min(k0 + k + q * KSTEP, kend - 1) - k;
                v[q] = *reinterpret_cast<const f32x4*>(base + (long)dk * ld);
                if (FM == 1) gq[q] = sg[k + dk];
            }
        } else if (FM == 2) {
            // the thread's 4·NV consecutive k lie in one 32-bit word (k-tiles start at multiples of 16)
            const int kk = FULL ? k0 + k : min(k0 + k, kend - 1);
            bword = bw_row[kk >> 5];
        } else {
#pragma unroll
            for (int q = 0; q < NV; ++q) {
                const int dk = FULL ? k0 + 4 * q : min(k0 + k + 4 * q, kend - 4) - k;
                v[q] = *reinterpret_cast<const f32x4*>(base + dk);
            }
        }
    }
    // FM 2: the mask bits as 0/1 values (exact in one bf16 plane)
    __device__ __forceinline__ void bits_to_values(int k0) {
        const unsigned w = bword >> ((k0 + k) & 31);
#pragma unroll
        for (int q = 0; q < NV; ++q)
#pragma unroll
            for (int e = 0; e < 4; ++e) v[q][e] = ((w >> (4 * q + e)) & 1u) ? 1.f : 0.f;
    }
    __device__ __forceinline__ bool kvalid(int q, int k0, int kend) const {
        return MN ? k0 + k + q * KSTEP < kend : k0 + k + 4 * q < kend;
    }
    // ONE: the values are exact in one bf16 plane (0/1 masks): plane 0 only, planes 1 and 2 never read
    template <bool FULL, bool NOSPLIT = false, bool ONE = false>
    __device__ __forceinline__ void store(unsigned short* img, int k0, int kend) {
        f32x4* vv = v;
        if (!FULL) {
#pragma unroll
            for (int q = 0; q < NV; ++q)
                if (!kvalid(q, k0, kend)) vv[q] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        // NOSPLIT (timing ablation only): raw bits into the planes, no split VALU
        auto split = [](f32x4 f, u32x2& p0, u32x2& p1, u32x2& p2) {
            if (NOSPLIT) { p0 = p1 = p2 = u32x2{__builtin_bit_cast(unsigned, f[0]), __builtin_bit_cast(unsigned, f[3])}; }
            else if (ONE) { p0 = u32x2{pack2(f[0], f[1]), pack2(f[2], f[3])}; p1 = p2 = p0; }
            else split4(f, p0, p1, p2);
        };
        if (MN) {
#pragma unroll
            for (int q = 0; q < NV; ++q) {
                u32x2 p0, p1, p2;
                split(vv[q], p0, p1, p2);
                unsigned short* d = img + mn_off(k + q * KSTEP, row);
                *reinterpret_cast<u32x2*>(d) = p0;
                if (!ONE) {
                    *reinterpret_cast<u32x2*>(d + PLANE) = p1;
                    *reinterpret_cast<u32x2*>(d + 2 * PLANE) = p2;
                }
            }
        } else if (NV == 2) {                                 // 8 consecutive k: one ds_write_b128 per plane
            u32x2 a0, a1, a2, b0, b1, b2;
            split(vv[0], a0, a1, a2);
            split(vv[NV - 1], b0, b1, b2);
            unsigned short* d = img + kc_off(row, k);
            *reinterpret_cast<u32x4*>(d) = u32x4{a0[0], a0[1], b0[0], b0[1]};
            if (!ONE) {
                *reinterpret_cast<u32x4*>(d + PLANE) = u32x4{a1[0], a1[1], b1[0], b1[1]};
                *reinterpret_cast<u32x4*>(d + 2 * PLANE) = u32x4{a2[0], a2[1], b2[0], b2[1]};
            }
        } else {
#pragma unroll
            for (int q = 0; q < NV; ++q) {
                u32x2 p0, p1, p2;
                split(vv[q], p0, p1, p2);
                unsigned short* d = img + kc_off(row, k + 4 * q);
                *reinterpret_cast<u32x2*>(d) = p0;
                if (!ONE) {
                    *reinterpret_cast<u32x2*>(d + PLANE) = p1;
                    *reinterpret_cast<u32x2*>(d + 2 * PLANE) = p2;
                }
            }
        }
    }
    // forward's fused gather: the staged rows written to dst (rows < Rmax, k < kend)
    __device__ __forceinline__ void copy_out(float* __restrict__ dst, int ldd, int r0, int Rmax, int k0,
                                             int kend) const {
        if (MN || r0 + row >= Rmax) return;
#pragma unroll
        for (int q = 0; q < NV; ++q)
            if (kvalid(q, k0, kend)) {
                f32x4* p = reinterpret_cast<f32x4*>(dst + (long)(r0 + row) * ldd + k0 + k + 4 * q);
// (a non-temporal store here measured slower: the layer-0 forward that reads the copy back from L2
                // took 99.6-100.2 vs 82.7-82.9 µs, C4 310.3 vs 306.6 ms; profiles/r06_x3_copy_nt_rejected.txt)
                *p = v[q];
            }
    }
    // MFMA fragment (32 rows × 16 k of k-half kh, bf16x8 per lane: row `rr`, k = 16kh + 8h..+7) of one plane
    __device__ __forceinline__ static bf16x8 frag(const unsigned short* plane, int rr, int lane, int kh = 0) {
        const int h = lane >> 5;
        if (!MN) return __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(plane + kc_off(rr, 16 * kh + 8 * h)));
        // hardware transpose: in each 16-lane group lane 4q+p addresses k-row q, rows 4p..4p+3 of
        // the group's 16; lane i receives row i of the 4 k-rows (two reads: k 8h+0..3, 8h+4..7;
        // sw(k + 4) = sw(k), so the second read is 4 k-rows further)
        const int gi = lane & 15, q = gi >> 2, p = gi & 3;
        typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
        const unsigned short* a0 = plane + mn_off(16 * kh + 8 * h + q, rr - gi) + 4 * p;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * R));
        const s16x8 f = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return __builtin_bit_cast(bf16x8, f);
    }
};

// ---------------------------------------------------------------------------------------------
// The kernel.  BM×BN output tile per workgroup of NTH threads in KG k-groups; each k-group
// (NTH/KG threads = WARPS_M × WARPS_N waves) runs its own pipeline over every KG-th k-tile of the
// workgroup's split [kbeg, kend) and the groups' accumulators are summed through LDS at the end
// (grad_W: fewer split-K workgroups per output tile, so fewer f32 atomics — they execute at the
// memory side at ≈1.3 TB/s chip-wide, MI355X_MICROARCH.md § Global float atomics).
// ---------------------------------------------------------------------------------------------
// ABL (timing ablations, results wrong; PPO_X3_ABLATE, -DPPO_X3_DIAG builds, cfgs 0 and 3): 1 = no
// MFMAs, 2 = no split / LDS stores, 4 = no epilogue stores, 8 = no global loads after the prologue,
// 32 = stamps, 64 = no split (raw bits stored to the planes), 128 = every other k-tile barrier skipped,
// 256 / 512 = no B / A fragment reads after the prologue (stale fragments: the LDS read cost)
// forward / grad_x epilogue: 32×32 accumulator block (i, j): lane (r, h) holds column r, rows
// 4h + (e&3) + 8(e>>2).  Branch-free per element: the bias loads hoisted, the ReLU′-bit ballots in a
// loop version of their own, grad_x's mask words brought into LDS (BM·BN/32 words, free on entry) by
// one coalesced pass (they were 16 dependent loads per block).  Element stores in the accumulator
// layout (each wave store: two 128-B row segments).
template <int OP, int BM, int BN, int TM, int TN, int NTH, bool YD = false, bool FG = false>
__device__ __forceinline__ void x3_epilogue_out(const X3Args& a, f32x16 (&acc)[TM][TN], unsigned short* lds, int m0,
                                                int n0, int wm, int wn, int tid) {
    constexpr int WM = TM * 32, WN = TN * 32;
    const int lane = tid & 63, r = lane & 31, h = lane >> 5;
    float bcol[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int col = n0 + wn * WN + j * 32 + r;
        bcol[j] = (OP == OP_NT && a.bias) ? a.bias[col < a.N ? col : a.N - 1] : 0.f;
    }
    constexpr int WPT = BN / 32;                            // mask words per tile row
    unsigned* const mk = reinterpret_cast<unsigned*>(lds);  // images no longer read (last barrier)
    const bool masked = OP == OP_NN && a.bits_in != nullptr;
    // grad_x fold (FG): the rows' g, a row scale of the product (grad_x = diag(g)·(mask·diag(w)·W))
    float* const gsh = reinterpret_cast<float*>(mk + BM * WPT);
    if (FG) {
        for (int idx = tid; idx < BM; idx += NTH) gsh[idx] = a.fold_g[min(m0 + idx, a.M - 1)];
    }
    if (masked) {
        for (int idx = tid; idx < BM * WPT; idx += NTH) {
            const int grow = min(m0 + idx / WPT, a.M - 1);
            const int gw = min((n0 >> 5) + idx % WPT, a.wpr - 1);
            mk[idx] = a.bits_in[(long)grow * a.wpr + gw];
        }
    }
    if (masked || FG) __syncthreads();
    // value-head fold (YD): each wave's partial y = Σ over its columns of relu(z)·w, per row — the
    // wave's 32 rows of block row i summed over its TN column blocks, then over the 32 lanes of each
    // half-wave, reduce-scattered so that lane r < 16 ends with row e = r of its half
    constexpr int WARPS_N = BN / WN;
    float wcol[TN];
    if constexpr (YD) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int col = n0 + wn * WN + j * 32 + r;
            wcol[j] = col < a.N ? a.ydot[col] : 0.f;
        }
    }
    auto ydot_block = [&](float (&yp)[16], int i) {
        // the two 16-lane rows of each half-wave add (lane i ↔ i ^ 16), then a reduce-scatter within each
        // row on DPP moves (pairs i ↔ 15 − i, 7 − i, i ^ 2, i ^ 1: each pair keeps the half its higher
        // member's bit selects), so lane i ends with value index i & 15
#pragma unroll
        for (int u = 0; u < 16; ++u) yp[u] += __shfl_xor(yp[u], 16, 64);
        const int li = lane & 15;
        auto level = [&](auto CTRLc, auto Oc) {
            constexpr int CTRL = decltype(CTRLc)::value, O = decltype(Oc)::value;
            const bool up = (li & O) != 0;
#pragma unroll
            for (int u = 0; u < O; ++u) {
                const float send = up ? yp[u] : yp[u + O];
                const float keep = up ? yp[u + O] : yp[u];
                yp[u] = keep + ppo::dpp_mov<CTRL>(send);
            }
        };
        level(std::integral_constant<int, 0x140>{}, std::integral_constant<int, 8>{});   // row_mirror
        level(std::integral_constant<int, 0x141>{}, std::integral_constant<int, 4>{});   // row_half_mirror
        level(std::integral_constant<int, 0x4E>{}, std::integral_constant<int, 2>{});    // quad_perm [2,3,0,1]
        level(std::integral_constant<int, 0xB1>{}, std::integral_constant<int, 1>{});    // quad_perm [1,0,3,2]
        const int e = li;
        const int row = m0 + wm * WM + i * 32 + 4 * h + (e & 3) + 8 * (e >> 2);
        const int slot = (n0 / BN) * WARPS_N + wn;
        if (r < 16 && row < a.M) a.ypart[(long)slot * a.M + row] = yp[0];
    };
    auto body = [&](auto BITSc) {
        constexpr bool BITS = decltype(BITSc)::value;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            float yp[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) yp[u] = 0.f;
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int c0 = n0 + wn * WN + j * 32;
                const int col = c0 + r;
                const int lr0 = wm * WM + i * 32 + 4 * h;      // tile row of element 0
                const int r0 = m0 + lr0;
                const bool col_ok = col < a.N;
                unsigned word = 0;
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int dr = (e & 3) + 8 * (e >> 2);
                    const int row = r0 + dr;
                    const bool ok = col_ok && row < a.M;
                    float v = acc[i][j][e];
                    float* dst = a.C + (long)row * a.ldc + col;
                    if (OP == OP_NT) {
                        v += bcol[j];
                        if (a.relu) v = v > 0.f ? v : 0.f;
#ifdef PPO_X3_NTSTORE
                        if (ok) __builtin_nontemporal_store(v, dst);
#else
                        if (ok) *dst = v;
#endif
                        if constexpr (YD) yp[e] += v * wcol[j];
                        if constexpr (BITS) {
                            const unsigned long long bb = __ballot(ok && v > 0.f);
                            const unsigned half = h ? (unsigned)(bb >> 32) : (unsigned)bb;
                            word = r == e ? half : word;
                        }
                    } else {
                        if (FG) v *= gsh[lr0 + dr];
                        if (masked && !((mk[(lr0 + dr) * WPT + ((c0 - n0) >> 5)] >> r) & 1u)) v = 0.f;
#ifdef PPO_X3_NTSTORE
                        if (ok) __builtin_nontemporal_store(v, dst);
#else
                        if (ok) *dst = v;
#endif
                    }
                }
                if (BITS && r < 16) {
                    const int row = r0 + (r & 3) + 8 * (r >> 2);
                    if (row < a.M && c0 < a.N) a.bits_out[(long)row * a.wpr + (c0 >> 5)] = word;
                }
            }
            if constexpr (YD) ydot_block(yp, i);
        }
    };
    if (OP == OP_NT && a.bits_out) body(std::true_type{});
    else body(std::false_type{});
}

// FOLD: the value-head fold variant (forward: ydot / ypart; grad_x / grad_W: A synthesised from h).
// The body of one workgroup (block b of a grid of `grid` blocks), a device function so that one launch
// could run several products' tiles (a grad_W + grad_x pair was measured and not kept, see phip_x3_bwd_w)
template <int OP, int BM, int BN, int WARPS_M, int NTH, int OCC, int KG, int ABL = 0, int FOLD = 0, int KB = BK>
__device__ __forceinline__ void x3_body(const X3Args& a, int b, int grid) {
    constexpr int NTG = NTH / KG;                                  // threads per k-group
    constexpr int NW = NTG / 64, WARPS_N = NW / WARPS_M;
    constexpr int WM = BM / WARPS_M, WN = BN / WARPS_N;
    constexpr int TM = WM / 32, TN = WN / 32;
    static_assert(TM >= 1 && TN >= 1 && WARPS_M * WARPS_N == NW, "wave tiling");
    static_assert(KG == 1 || OP == OP_TN, "k-groups: grad_W only");
    constexpr bool A_MN = OP == OP_TN, B_MN = OP != OP_NT;
    using SA = StageX3<BM, A_MN, NTG, KB>;
    using SB = StageX3<BN, B_MN, NTG, KB>;
    constexpr int BUF = SA::SIZE + SB::SIZE;
    constexpr int KH = KB / 16;                                    // MFMA k-steps (16 k) per k-tile

    constexpr int NS = 3;                                          // LDS ring stages
    extern __shared__ __attribute__((aligned(16))) unsigned short lds[];     // KG × NS × BUF

    // grad_x launches may carry the previous grad_W's slab reduce in extra workgroups past the tiles
    if constexpr (OP == OP_NN) {
        if (a.red_wgs && b >= a.gemm_wgs) {
            x3_slab_reduce_block<NTH>(a, b - a.gemm_wgs, reinterpret_cast<float*>(lds));
            return;
        }
    }

    // XCD-aware remap: hardware deals blocks round-robin over the 8 XCDs; give each XCD a
    // contiguous range of linear tiles (n fastest), so tiles sharing an A panel share an L2
    const int nwg = (OP == OP_NN && a.red_wgs) ? a.gemm_wgs : grid;
    const int xcd = b & 7, qq = nwg >> 3, rr = nwg & 7;
    const int t = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (b >> 3);
    const int tn = t % a.tiles_n;
    const int rest = t / a.tiles_n;
    const int tm = rest % a.tiles_m;
    const int m0 = tm * BM, n0 = tn * BN;
    const int kbeg = (rest / a.tiles_m) * a.kchunk;
    const int kend = min(a.K, kbeg + a.kchunk);

    const int tid = threadIdx.x, lane = tid & 63;
    // wave-uniform, and the compiler must know it: otherwise the k-tile count, the k offsets and the
    // ring slot of a k-group are per-lane values — VGPR loop control (exec-masked back edge), 64-bit
    // v_mad per global load and VALU ring-slot addresses in every grad_W iteration
    const int grp = KG > 1 ? __builtin_amdgcn_readfirstlane(tid / NTG) : 0;
    const int lt = KG > 1 ? tid % NTG : tid;
    const int w = lt >> 6;
    const int wm = w / WARPS_N, wn = w % WARPS_N;
    auto stamp = [&](int slot) {
        if (tid == 0 && b < 8192) {
            g_x3_stamps[b * 8 + slot] = __builtin_amdgcn_s_memtime();
            if (slot == 0 || slot == 3) g_x3_stamps[b * 8 + 4 + slot / 3] = __builtin_amdgcn_s_memrealtime();
        }
    };
    if (ABL & 32) stamp(0);
    const int r = lane & 31, h = lane >> 5;

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    SA sa;
    SB sb;
    sa.init(a.A, a.lda, OP == OP_NT ? a.ridx : nullptr, m0, a.M, lt);
    sb.init(a.B, a.ldb, nullptr, n0, a.N, lt);
    // value-head fold (grad_x: A from the mask words, B = W scaled by w per k-row; grad_W: A = h → mask,
    // B = x scaled by g per k-row)
    constexpr bool syn = OP != OP_NT && FOLD != 0;
    constexpr int FMA_ = !syn ? 0 : OP == OP_NN ? 2 : 1;          // A's fold load mode
    constexpr int FMB_ = syn ? 1 : 0;                             // B's
    const float* fold_g = a.fold_g;
    if constexpr (OP == OP_TN && FOLD != 0) {
        if (a.vh_ypart) {                                         // the value head, carried (X3Args vh_*)
            float* gl = reinterpret_cast<float*>(lds + KG * NS * BUF);
            const bool head = tm == 0 && tn == 0;
            const float bias = a.vh_b[0];
            float ls = 0.f, sgs = 0.f;
            for (int rr = tid; rr < kend - kbeg; rr += NTH) {
                const int row = kbeg + rr;
                float yv = 0.f;
                for (int q = 0; q < a.vh_slots; ++q) yv += a.vh_ypart[(long)q * a.K + row];
                yv += bias;
                const float tv = a.vh_t[row];
                const float d = tv - yv;
                const float gv = 2 * (yv - tv) / (float)a.K;
                gl[rr] = gv;
                if (head) {
                    a.vh_y[row] = yv;
                    const_cast<float*>(a.fold_g)[row] = gv;
                    ls += d * d;
                    sgs += gv;
                }
            }
            if (head) {
                ls = ppo::wave_sum64(ls);
                sgs = ppo::wave_sum64(sgs);
                if (lane == 0) {
                    atomicAdd(a.vh_gb, sgs);
                    if (a.vh_loss) atomicAdd(a.vh_loss, ls * (1.0f / (float)a.K));
                }
            }
            __syncthreads();
            fold_g = gl - kbeg;
        }
    }
    if (syn) {
        sa.init_fold(fold_g, OP == OP_NN ? a.fold_bits : nullptr, a.fold_wpr, m0, a.M);
        sb.init_fold(OP == OP_NN ? a.fold_w : fold_g, nullptr, 0, n0, a.N);
    }
    // the fused gather's copy of A's rows: every column tile of a row block stages the same rows, so
    // they share the copy — column tile tn writes the k-tiles with index ≡ tn (mod tiles_n) (one
    // workgroup writing all of it finished its tile ≈ a copy later than the others in a one-round grid)
    const bool do_copy = OP == OP_NT && a.acopy != nullptr;
    // grad_W bias: Σ over this split's k of the A (= g) tile, from the staging registers
    const bool do_bsum = OP == OP_TN && a.gbias != nullptr && tn == 0;
    f32x4 bs[SA::NV], bs3[SA::NV];                     // bs3: the folded output layer's Σ g·h (grad_W fold)
#pragma unroll
    for (int q = 0; q < SA::NV; ++q) bs[q] = bs3[q] = f32x4{0.f, 0.f, 0.f, 0.f};

    // fragment registers: plane p of the A (fa) and B (fb) operand tiles of the current k-tile
    bf16x8 fa[3][TM][KH], fb[3][TN][KH];
    // (fold: A is a 0/1 mask in plane 0 only — its planes 1, 2 and their three products are skipped)
    bool first_rd = true;                                          // (ABL 256 / 512: the prologue's reads only)
    auto rd_a = [&](const unsigned short* img, int p) {
        if (syn && p != 0) return;
        if ((ABL & 512) && !first_rd) return;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int kh = 0; kh < KH; ++kh) fa[p][i][kh] = SA::frag(img + p * SA::PLANE, wm * WM + i * 32 + r, lane, kh);
    };
    auto rd_b = [&](const unsigned short* img, int p) {
        if ((ABL & 256) && !first_rd) return;
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int kh = 0; kh < KH; ++kh)
                fb[p][j][kh] = SB::frag(img + SA::SIZE + p * SB::PLANE, wn * WN + j * 32 + r, lane, kh);
    };
    // plane product A_pa·B_pb of the current k-tile (the six with pa + pb ≤ 2)
    auto mm = [&](int pa, int pb) {
        if (syn && pa != 0) return;
        if (ABL & 1) {               // keep the fragment reads live
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[i][j][0] += (float)fa[pa][i][0][0] + (float)fb[pb][j][0][1];
            return;
        }
#pragma unroll
        for (int kh = 0; kh < KH; ++kh)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[pa][i][kh], fb[pb][j][kh], acc[i][j], 0, 0, 0);
    };

    // this group's k-tiles: j = 0 … NK−1 at k0 = kbeg + (KG·j + grp)·BK; only the last one can be
    // partial (or, for a k-group past the end, empty: every element masked to zero)
    const int nkt = kend > kbeg ? (kend - kbeg + KB - 1) / KB : 0;
    const int NK = (nkt + KG - 1) / KG;
    auto k0_of = [&](int j) { return kbeg + (KG * j + grp) * KB; };
    auto is_full = [&](int j) { return k0_of(j) + KB <= kend; };
    const int tail = NK > 0 && !is_full(NK - 1) ? 1 : 0;
    unsigned short* const ring = lds + (KG > 1 ? grp * NS * BUF : 0);

    // split + LDS store of the staged tile at k0 (FULL: no k tail); COPY: also the gathered rows
    // COPY (forward, fused gather): also the gathered rows; BSUM (grad_W of a bias): also Σ g — both
    // compile-time, so the mainloop of the workgroups that do neither carries no dead VALU
    auto stage_a = [&](auto FULLc, auto COPYc, auto SYNc, unsigned short* img, int k0) {
        constexpr bool FULL = decltype(FULLc)::value, COPY = OP == OP_NT && decltype(COPYc)::value;
        constexpr bool BSUM = OP == OP_TN && decltype(COPYc)::value;
        constexpr bool SYN = OP != OP_NT && decltype(SYNc)::value;
        if ((ABL & 2) && k0 != kbeg) return;
        if constexpr (COPY) {
            if (((k0 - kbeg) / KB) % a.tiles_n == tn) sa.copy_out(a.acopy, a.K, m0, a.M, k0, kend);
        }
        if constexpr (SYN && OP == OP_NN) sa.bits_to_values(k0);
        if constexpr (SYN && OP == OP_TN) {
            // A = h: the output layer's Σ g·h and the bias's Σ 1[h > 0]·g (valid batch rows), then the mask
#pragma unroll
            for (int q = 0; q < SA::NV; ++q) {
                const bool ok = FULL || sa.kvalid(q, k0, kend);
                const float g = sa.gq[q];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float hv = sa.v[q][e];
                    const bool on = hv > 0.f;
                    if (BSUM && ok) {
                        bs3[q][e] += g * hv;
                        bs[q][e] += on ? g : 0.f;
                    }
                    sa.v[q][e] = on ? 1.f : 0.f;
                }
            }
        }
        sa.template store<FULL, (ABL & 64) != 0, SYN>(img, k0, kend);
        if constexpr (BSUM && !SYN) {
#pragma unroll
            for (int q = 0; q < SA::NV; ++q) bs[q] += sa.v[q];
        }
    };
    auto stage_b = [&](auto FULLc, unsigned short* img, int k0) {
        constexpr bool FULL = decltype(FULLc)::value;
        if ((ABL & 2) && k0 != kbeg) return;
        if constexpr (FMB_ == 1) {                       // fold: x rows scaled by g (grad_W), W rows by w (grad_x)
#pragma unroll
            for (int q = 0; q < SB::NV; ++q) sb.v[q] *= sb.gq[q];
        }
        sb.template store<FULL, (ABL & 64) != 0>(img + SA::SIZE, k0, kend);
    };
    auto load = [&](auto FULLc, auto SYNc, int k0) {
        constexpr bool FULL = decltype(FULLc)::value;
        constexpr bool SYN = OP != OP_NT && decltype(SYNc)::value;
        if ((ABL & 8) && k0 != kbeg) return;
        sa.template load<FULL, SYN ? FMA_ : 0>(k0, kend);
        sb.template load<FULL, SYN ? FMB_ : 0>(k0, kend);
    };
    using T = std::true_type;
    using F = std::false_type;
    auto load_t = [&](auto SYNc, int j) {
        if (is_full(j)) load(T{}, SYNc, k0_of(j)); else load(F{}, SYNc, k0_of(j));
    };
    auto stage_a_t = [&](auto COPYc, auto SYNc, unsigned short* img, int j) {
        if (is_full(j)) stage_a(T{}, COPYc, SYNc, img, k0_of(j)); else stage_a(F{}, COPYc, SYNc, img, k0_of(j));
    };
    auto stage_b_t = [&](unsigned short* img, int j) {
        if (is_full(j)) stage_b(T{}, img, k0_of(j)); else stage_b(F{}, img, k0_of(j));
    };

    // Pipeline, iteration j over the ring (cur = tile j, n1 = tile j+1, n2 ← tile j+2):
    //   a1, b1 of tile j (needed from the third product on) ← cur
    //   A2·B0 | fa2 ← n1      A0·B0 | split + store A of tile j+2 → n2
    //   A1·B0 | fb0 ← n1, split + store B of tile j+2     A0·B2 | fb2 ← n1, loads of tile j+3
    //   A0·B1 | fa0 ← n1      A1·B1
    //   barrier
    // Each fragment plane of tile j+1 is read right after tile j's last product that uses it (into
    // the same registers), at least one product group ahead of its first use; tile j+1's image was
    // completed by the previous iteration's barrier, tile j+2's by this one.  WAR: the ring slot
    // restaged in iteration j+1 (tile j+3 → cur) was last read in iteration j's first block.
    // region boundary: a full scheduling barrier, preceded (forward / grad_x) by an interleave request
    // — each of the region's MFMAs followed by NV VALU, one DS and one VMEM instruction.  Without it
    // the compiler front-loads a region's split VALU (≈30 in a row) ahead of its MFMAs, and the two
    // lock-stepped waves of a SIMD leave the matrix pipe idle together: 3761 → 3400 cycles per k-tile
    // at C4 (profiles/r03_x3_stamps.txt).  grad_W measured no gain (PPO_X3_SGB=0/1 builds).
    auto region_end = [&](auto NVc) {
#if defined(PPO_X3_SGB) || !defined(PPO_X3_NO_SGB)
        constexpr int NVV = decltype(NVc)::value;
#ifdef PPO_X3_SGB
        constexpr bool SGB = true;
#else
        constexpr bool SGB = OP != OP_TN;
#endif
        if constexpr (SGB) {
#pragma unroll
            for (int q = 0; q < TM * TN * KH; ++q) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                if (NVV) __builtin_amdgcn_sched_group_barrier(0x002, NVV, 0);
                __builtin_amdgcn_sched_group_barrier(0x080, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
            }
        }
#endif
        __builtin_amdgcn_sched_barrier(0);
    };
    using I0 = std::integral_constant<int, 0>;
    using I2 = std::integral_constant<int, 2>;
    using I6 = std::integral_constant<int, 6>;
    auto iter = [&](auto STEADYc, auto COPYc, auto SYNc, int j, unsigned short* cur, unsigned short* n1,
                    unsigned short* n2) {
        constexpr bool STEADY = decltype(STEADYc)::value;
        const bool has1 = STEADY || j + 1 < NK, has2 = STEADY || j + 2 < NK, has3 = STEADY || j + 3 < NK;
        rd_a(cur, 1);
        rd_b(cur, 1);
#ifdef PPO_X3_PRIO
        __builtin_amdgcn_s_setprio(1);
#endif
        mm(2, 0);
        if (has1) rd_a(n1, 2);
        region_end(I0{});
        mm(0, 0);
        if (STEADY) stage_a(T{}, COPYc, SYNc, n2, k0_of(j + 2));
        else if (has2) stage_a_t(COPYc, SYNc, n2, j + 2);
        region_end(I6{});
        mm(1, 0);
        if (has1) rd_b(n1, 0);
        if (STEADY) stage_b(T{}, n2, k0_of(j + 2));
        else if (has2) stage_b_t(n2, j + 2);
        region_end(I6{});
        mm(0, 2);
        if (has1) rd_b(n1, 2);
        if (STEADY) load(T{}, SYNc, k0_of(j + 3));
        else if (has3) load_t(SYNc, j + 3);
        region_end(I2{});
        mm(0, 1);
        if (has1) rd_a(n1, 0);
        region_end(I0{});
        mm(1, 1);
#ifdef PPO_X3_PRIO
        __builtin_amdgcn_s_setprio(0);
#endif
        if (!((ABL & 128) && (j & 1))) __syncthreads();      // (ABL 128, timing only: every other barrier)
    };
    auto mainloop = [&](auto COPYc, auto SYNc) {
        unsigned short* cur = ring;
        unsigned short* n1 = ring + BUF;
        unsigned short* n2 = ring + 2 * BUF;
        if (NK > 0) { load_t(SYNc, 0); stage_a_t(COPYc, SYNc, cur, 0); stage_b_t(cur, 0); }
        if (NK > 1) { load_t(SYNc, 1); stage_a_t(COPYc, SYNc, n1, 1); stage_b_t(n1, 1); }
        if (NK > 2) load_t(SYNc, 2);
        __syncthreads();
        if (NK > 0) { rd_a(cur, 2); rd_b(cur, 0); rd_b(cur, 2); rd_a(cur, 0); }
        if ((ABL & 768) && NK > 0) { rd_a(cur, 1); rd_b(cur, 1); }
        first_rd = false;
        if (ABL & 32) stamp(1);
        // steady state: tiles j+2 and j+3 exist and are full.  grad_W's loop is unrolled by the ring
        // length, so every ring slot's fragment / staging addresses are loop-invariant registers (no
        // per-iteration slot arithmetic: 130 → 92 VALU per k-tile); the 256×256 kernels have no
        // registers for three slots' addresses (the unrolled form spills)
        const int steady = NK - 3 - tail;
        int j = 0;
        if constexpr (KG > 1) {
            unsigned short* const s0 = cur;
            unsigned short* const s1 = n1;
            unsigned short* const s2 = n2;
            for (; j + 3 <= steady; j += 3) {
                iter(T{}, COPYc, SYNc, j, s0, s1, s2);
                iter(T{}, COPYc, SYNc, j + 1, s1, s2, s0);
                iter(T{}, COPYc, SYNc, j + 2, s2, s0, s1);
            }
        }
        for (; j < steady; ++j) {
            iter(T{}, COPYc, SYNc, j, cur, n1, n2);
            unsigned short* t = cur; cur = n1; n1 = n2; n2 = t;
        }
        for (; j < NK; ++j) {                                  // the last two or three tiles
            iter(F{}, COPYc, SYNc, j, cur, n1, n2);
            unsigned short* t = cur; cur = n1; n1 = n2; n2 = t;
        }
    };
#ifdef PPO_X3_PRIO2
    if ((tid >> 6) >= NTH / 128) __builtin_amdgcn_s_setprio(1);   // the second-dispatched half wins VALU arbitration
#endif
    // (COPYc: the gather copy / Σ g; SYNc: the folded value head's synthesised A)
    auto run = [&](auto COPYc) {
        if constexpr (syn) mainloop(COPYc, T{});
        else mainloop(COPYc, F{});
    };
    if (do_copy || do_bsum) run(T{});
    else run(F{});
#ifdef PPO_X3_PRIO2
    __builtin_amdgcn_s_setprio(0);
#endif

    // LDS scratch after the mainloop (the images are no longer read): bias-gradient partial sums,
    // then the k-groups' accumulator exchange
    constexpr int RED_FLOATS = OP == OP_TN ? (NTH / (BM / 4)) * BM : 0;
    if (do_bsum) {
        // rows of this thread's float4s: row .. row+3; reduce over the threads sharing them
        // (tid ≡ tid' mod BM/4), through LDS
        __syncthreads();
        float* red = reinterpret_cast<float*>(lds);
        constexpr int G = BM / 4;                       // float4 row groups
        constexpr int S = NTH / G;                      // threads per group (one per k-row slot)
        static_assert(NTG % G == 0, "bias-sum row mapping");
#pragma unroll
        for (int q = 1; q < SA::NV; ++q) bs[0] += bs[q];
        *reinterpret_cast<f32x4*>(red + (tid / G) * BM + (tid % G) * 4) = bs[0];
        __syncthreads();
        if (tid < BM) {
            float s = 0.f;
            for (int j = 0; j < S; ++j) s += red[j * BM + tid];
            if (m0 + tid < a.M) {
                if (syn) s *= a.fold_w[m0 + tid];            // grad_b = diag(w)·maskᵀ·g
                if (a.splits > 1) atomicAdd(a.gbias + m0 + tid, s);
                else a.gbias[m0 + tid] = s;
            }
        }
        if constexpr (OP == OP_TN && syn) {           // the folded output layer's gW: the same reduction
            __syncthreads();
#pragma unroll
            for (int q = 1; q < SA::NV; ++q) bs3[0] += bs3[q];
            *reinterpret_cast<f32x4*>(red + (tid / G) * BM + (tid % G) * 4) = bs3[0];
            __syncthreads();
            if (tid < BM) {
                float s = 0.f;
                for (int j = 0; j < S; ++j) s += red[j * BM + tid];
                if (m0 + tid < a.M) atomicAdd(a.fold_gw + m0 + tid, s);
            }
        }
    }
    // k-groups: block (i, j) of a wave's tile is finished by the group (i·TN + j) mod KG; every
    // other group's wave at the same position hands its partial block over through LDS
    auto mine = [&](int i, int j) { return KG == 1 || ((i * TN + j) % KG) == grp; };
    if constexpr (KG > 1) {
        static_assert(KG == 2, "k-group exchange: two groups");
        static_assert((RED_FLOATS * 4 + NW * TM * TN * 4096) <= KG * NS * BUF * 2, "k-group exchange: LDS");
        f32x4* xch = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(lds) + RED_FLOATS);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                if (mine(i, j)) continue;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    xch[((w * TM * TN + i * TN + j) * 4 + q) * 64 + lane] =
                        f32x4{acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
            }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                if (!mine(i, j)) continue;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const f32x4 o = xch[((w * TM * TN + i * TN + j) * 4 + q) * 64 + lane];
#pragma unroll
                    for (int e = 0; e < 4; ++e) acc[i][j][4 * q + e] += o[e];
                }
            }
    }

    if (ABL & 32) stamp(2);
    if (ABL & 4) {
        float t = 0.f;                                          // keep every accumulator live
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) t += acc[i][j][e];
        if (t == 12345.678f) a.C[tid] = 1.f;
        return;
    }
    if constexpr (OP != OP_TN) {
        static_assert(BM * (BN / 32 + 1) * 4 <= KG * NS * BUF * 2, "x3 epilogue: mask words exceed LDS");
        x3_epilogue_out<OP, BM, BN, TM, TN, NTH, OP == OP_NT && FOLD != 0, OP == OP_NN && FOLD != 0>(a, acc, lds, m0,
                                                                                                  n0, wm, wn, tid);
        if (ABL & 32) stamp(3);
        return;
    }
    // grad_W epilogue: every load a block needs is issued before its stores
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            if (!mine(i, j)) continue;
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
            // element stores in the accumulator layout (each wave store: two 128-B row segments);
            // a DPP quad transpose to 16-B stores measured slower: the store tail is HBM-write-bound
            // (64 MB in ≈14 µs), not store-issue-bound
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int row = r0 + (e & 3) + 8 * (e >> 2);
                const bool ok = col_ok && row < a.M;
                float v = acc[i][j][e];
                if (OP == OP_TN && syn) v *= a.fold_w[row < a.M ? row : a.M - 1];     // grad_W = diag(w)·(…)
                float* dst = a.C + (long)row * a.ldc + col;
                if (OP == OP_NT) {
                    v += bcol;
                    if (a.relu) v = v > 0.f ? v : 0.f;
#ifdef PPO_X3_NTSTORE
                    if (ok) __builtin_nontemporal_store(v, dst);
#else
                    if (ok) *dst = v;
#endif
                    if (a.bits_out) {
                        const unsigned long long bb = __ballot(ok && v > 0.f);
                        if (r == e) word = h ? (unsigned)(bb >> 32) : (unsigned)bb;
                    }
                } else if (OP == OP_NN) {
#ifdef PPO_X3_NTSTORE
                    if (ok) __builtin_nontemporal_store(keep[e] ? v : 0.f, dst);
#else
                    if (ok) *dst = keep[e] ? v : 0.f;
#endif
                } else if (ok) {
                    if (a.slab) a.slab[(long)(kbeg / a.kchunk) * a.M * a.N + (long)row * a.N + col] = v;
                    else if (a.splits > 1) atomicAdd(dst, v);
                    else *dst = v;
                }
            }
            if (OP == OP_NT && a.bits_out && r < 16) {
                const int row = r0 + (r & 3) + 8 * (r >> 2);
                if (row < a.M && c0 < a.N) a.bits_out[(long)row * a.wpr + (c0 >> 5)] = word;
            }
        }
    if (ABL & 32) stamp(3);
}

template <int OP, int BM, int BN, int WARPS_M, int NTH, int OCC, int KG, int ABL = 0, int FOLD = 0, int KB = BK>
__global__ __launch_bounds__(NTH, OCC) void gemm_x3_kernel(X3Args a) {
    x3_body<OP, BM, BN, WARPS_M, NTH, OCC, KG, ABL, FOLD, KB>(a, (int)blockIdx.x, (int)gridDim.x);
}

#ifdef PPO_X3_DIAG
int g_x3_ablate = -1;
#endif

int g_x3_last_slots = 0;                 // the last launch's ypart slots (tiles_n × waves along N)

template <int OP, int BM, int BN, int WARPS_M, int NTH, int OCC, int KG, int ABL = 0, int FOLD = 0, int KB = BK>
void launch_x3(X3Args a) {
    a.tiles_m = ppo_divup(a.M, BM);
    a.tiles_n = ppo_divup(a.N, BN);
    g_x3_last_slots = a.tiles_n * (NTH / KG / 64 / WARPS_M);
    if (a.splits < 1) a.splits = 1;
    long grid = (long)a.tiles_m * a.tiles_n * a.splits;
    PPO_REQUIRE(grid > 0 && grid < (1L << 31), "gemm_x3: grid out of range");
    if (a.red_wgs) {
        a.red_wgs = (int)ppo_divup((a.red_n + 3) / 4, NTH / 4);    // NTH/4 float4 columns per reduce workgroup
        PPO_REQUIRE(OP == OP_NN && NTH >= 256 && grid + a.red_wgs < (1L << 31), "gemm_x3: carried reduce");
        a.gemm_wgs = (int)grid;
        grid += a.red_wgs;
    }
    PPO_REQUIRE(a.kchunk % (KG * KB) == 0 || a.splits == 1, "gemm_x3: split-K chunk vs k-groups");
    using SA = StageX3<BM, OP == OP_TN, NTH / KG, KB>;
    using SB = StageX3<BN, OP != OP_NT, NTH / KG, KB>;
    constexpr size_t lds0 = (size_t)KG * 3 * sizeof(unsigned short) * (SA::SIZE + SB::SIZE);   // 3-stage ring
    static_assert(lds0 <= 160 * 1024, "gemm_x3: LDS images exceed 160 KiB");
    size_t lds = lds0;
    if (OP == OP_TN && FOLD && a.vh_ypart) {           // the carried value head's g of the split's rows
        if (lds + 4 * (size_t)a.kchunk <= 160 * 1024) {
            lds += 4 * (size_t)a.kchunk;
        } else {                                       // no room: the head kernel first, g from HBM
            phip_value_head(a.vh_ypart, a.vh_slots, a.vh_b, a.vh_t, a.K, a.vh_y, const_cast<float*>(a.fold_g), a.vh_gb,
                            a.vh_loss);
            a.vh_ypart = nullptr;
        }
    }
    auto kern = gemm_x3_kernel<OP, BM, BN, WARPS_M, NTH, OCC, KG, ABL, FOLD, KB>;
    if (lds > 64 * 1024) {
        static bool attr = false;                      // once per instantiation (the whole LDS)
        if (!attr) {
            PPO_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
            attr = true;
        }
    }
    if (a.ev_start || a.ev_stop)
        hipExtLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NTH), lds, ppo::stream(), a.ev_start, a.ev_stop, 0, a);
    else
        PPO_TIMED_LAUNCH(kern, dim3((unsigned)grid), dim3(NTH), lds, ppo::stream(), a);
    PPO_LAUNCH_CHECK();
}

// grad_W split-K partials: out[i] = Σ_s slab[s][i] in a fixed order (run-to-run deterministic).
// 256/Q float4 columns per workgroup × Q split groups: group q sums its splits in order, then the
// group partials are added in order through LDS (Q = 4; Q = 16 for many splits of few columns, the
// per-workgroup partials of the wide output layer).  (One thread per column over all splits kept 256
// workgroups with a serial chain of loads: 25.6 µs for 32 × 1 MB slabs, ≈1.3 TB/s.)
template <int Q>
__global__ __launch_bounds__(256) void slab_reduce_kernel(const float* __restrict__ slab, float* __restrict__ out,
                                                          long n, long stride, int splits) {
    constexpr int C = 256 / Q;
    __shared__ f32x4 part[Q - 1][C];
    const int c = threadIdx.x % C, q = threadIdx.x / C;
    const long n4 = (n + 3) >> 2, s4 = stride >> 2;      // the last quad may be partial (stride pads it)
    const long i = (long)blockIdx.x * C + c;
    const int per = (splits + Q - 1) / Q;
    const int s0 = q * per, s1 = min(splits, s0 + per);
    const f32x4* __restrict__ sv = reinterpret_cast<const f32x4*>(slab);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (i < n4) {
#pragma unroll 8
        for (int s = s0; s < s1; ++s) acc += sv[(long)s * s4 + i];
    }
    if (q) part[q - 1][c] = acc;
    __syncthreads();
    if (q == 0 && i < n4) {
#pragma unroll
        for (int v = 0; v < Q - 1; ++v) acc += part[v][c];
        if (4 * i + 4 <= n) {
            reinterpret_cast<f32x4*>(out)[i] = acc;
        } else {
            for (int e = 0; e < 4; ++e)
                if (4 * i + e < n) out[4 * i + e] = acc[e];
        }
    }
}

// tile configurations: 0 = 256×256 over 8 waves of 64×128 (forward, grad_x; one workgroup per CU),
// 1 = 128×128 over 4 waves of 64×64, two workgroups per CU (narrow products), 2 = 128×128 over 8
// waves of 32×64, 3 = 128×128 over two k-groups of 4 waves of 64×64, one workgroup per CU (grad_W),
// 4 = 64×64 over 4 waves of 32×32, four workgroups per CU (small outputs: C3's 8192×256 minibatch
// products have 32 tiles of 256×256 — an eighth of the CUs — but 512 of 64×64)
// 5 = 256×128 over 8 waves of 64×64, one workgroup per CU (two rounds at C4: the first round's store
// tail drains under the second round's mainloop)
// 6 = 64×64 over 4 waves of 32×32 with 32-k tiles (two MFMA k-steps per barrier), two workgroups per CU
// (the small products' grids: half the k-tile iterations, barriers and staging round trips of cfg 4)
struct CfgX3 { int bm, bn, kg, slots_per_cu, kb; };
constexpr CfgX3 kCfgX3[] = {{256, 256, 1, 1, 16}, {128, 128, 1, 2, 16}, {128, 128, 1, 1, 16}, {128, 128, 2, 1, 16},
                            {64, 64, 1, 4, 16},   {256, 128, 1, 1, 16}, {64, 64, 1, 2, 32}};
int g_force_x3 = -1;
int g_split_x3 = 0;

template <int OP>
void launch_cfg_x3(int c, const X3Args& a) {
    if (a.ydot || a.fold_g) {                      // the value-head fold variants
        switch (c) {
            case 0: launch_x3<OP, 256, 256, 4, 512, 2, 1, 0, 1>(a); return;
            case 2: launch_x3<OP, 128, 128, 4, 512, 2, 1, 0, 1>(a); return;
            case 4: launch_x3<OP, 64, 64, 2, 256, 4, 1, 0, 1>(a); return;
            case 5: launch_x3<OP, 256, 128, 4, 512, 2, 1, 0, 1>(a); return;
            case 6: launch_x3<OP, 64, 64, 2, 256, 2, 1, 0, 1, 32>(a); return;
            case 3:
                if constexpr (OP == OP_TN) { launch_x3<OP, 128, 128, 2, 512, 2, 2, 0, 1>(a); return; }
                [[fallthrough]];
            default: launch_x3<OP, 128, 128, 2, 256, 2, 1, 0, 1>(a); return;
        }
    }
#ifdef PPO_X3_DIAG
    if (g_x3_ablate < 0) {
        const char* e = getenv("PPO_X3_ABLATE");
        g_x3_ablate = e ? atoi(e) : 0;
    }
    if (g_x3_ablate && (c == 0 || c == 4 || (c == 3 && OP == OP_TN))) {
        auto run = [&](auto ABLc) {
            constexpr int A = decltype(ABLc)::value;
            if (c == 4) launch_x3<OP, 64, 64, 2, 256, 4, 1, A>(a);
            else if constexpr (OP == OP_TN) launch_x3<OP, 128, 128, 2, 512, 2, 2, A>(a);
            else launch_x3<OP, 256, 256, 4, 512, 2, 1, A>(a);
        };
        switch (g_x3_ablate) {
            case 1: run(std::integral_constant<int, 1>{}); return;
            case 2: run(std::integral_constant<int, 2>{}); return;
            case 4: run(std::integral_constant<int, 4>{}); return;
            case 8: run(std::integral_constant<int, 8>{}); return;
            case 32: run(std::integral_constant<int, 32>{}); return;
            case 64: run(std::integral_constant<int, 64>{}); return;
            case 128: run(std::integral_constant<int, 128>{}); return;
            case 256: run(std::integral_constant<int, 256>{}); return;
            case 512: run(std::integral_constant<int, 512>{}); return;
            case 768: run(std::integral_constant<int, 768>{}); return;
            default: break;
        }
    }
#endif
    switch (c) {
        case 0: launch_x3<OP, 256, 256, 4, 512, 2, 1>(a); break;
        case 2: launch_x3<OP, 128, 128, 4, 512, 2, 1>(a); break;
        case 4: launch_x3<OP, 64, 64, 2, 256, 4, 1>(a); break;
        case 5: launch_x3<OP, 256, 128, 4, 512, 2, 1>(a); break;
        case 6: launch_x3<OP, 64, 64, 2, 256, 2, 1, 0, 0, 32>(a); break;
        case 3:
            if constexpr (OP == OP_TN) { launch_x3<OP, 128, 128, 2, 512, 2, 2>(a); break; }
            [[fallthrough]];
        default: launch_x3<OP, 128, 128, 2, 256, 2, 1>(a); break;
    }
}

// forward / grad_x: the largest tile whose grid still gives every CU a workgroup (one round of
// 256×256 tiles, else 128×128 over 8 waves, one per CU, else 64×64 at up to four per CU).  At the
// data-parallel shard shapes (profiles/r03_x3_small_shapes.txt): 8192×512×512 forward 32.1 µs on
// 128×128 at two per CU (4 waves of 64×64) vs 28.0 µs on 8 waves of 32×64; 16384 rows 50.4 vs 47.9
int pick_x3(int M, int N, int op) {
    if (g_force_x3 >= 0) return g_force_x3;
    // (256×128 tiles in two rounds for C4's forward or grad_x, the second round's mainloop under the
    // first round's store tail: 322.3 / 313.3 vs 305.4 ms, profiles/r05_x3_cfg5_rounds_rejected.txt)
    // (cfg 5, 256×128 with slabs, measured slower: r04_x3_tn_cfg5_update_ab.txt; cfg 2, one k-group in 72 KiB
    // so the other loop's kernels fit beside it, fails the accuracy parity — twice as long fp32 chains:
    // profiles/r06_x3_tn_cfg2_accuracy_rejected.txt)
    if (op == OP_TN) return 3;
    auto tiles = [&](int c) { return (long)ppo_divup(M, kCfgX3[c].bm) * ppo_divup(N, kCfgX3[c].bn); };
    if (tiles(0) >= 256) return 0;
    if (tiles(2) >= 256) return 2;
    // 32-k small tiles (cfg 6): each launch alone is faster (shard forward 21.1 -> 20.0 µs, C3 14.4 -> 13.5),
    // but at 72 KiB of LDS per workgroup the other loop's kernels and the carried reduces no longer fit
    // beside them — the shard update 71.6 -> 73.1 ms, C3 26.8 -> 27.2 with every small product on it
    // (profiles/r06_x3_bk32_ab.txt); PPO_X3_BK32 = 1 (every small product) / nt (forwards only) / 0 (default)
    const char* e = getenv("PPO_X3_BK32");
    if (e && e[0] == '1') return 6;
    if (e && e[0] == 'n' && op == OP_NT) return 6;
    return 4;
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

}  // namespace

namespace ppo {


// per-stream slab buffers (the value and policy loops run their grad_W launches on two streams)
static float* g_slab[2] = {nullptr, nullptr};
static size_t g_slab_cap[2] = {0, 0};
float* slab_scratch(size_t floats) {
    const int s = phip_side_active() ? 1 : 0;
    if (floats > g_slab_cap[s]) {
        phip_free(g_slab[s]);
        g_slab[s] = (float*)phip_malloc(sizeof(float) * floats);
        g_slab_cap[s] = floats;
    }
    return g_slab[s];
}

void slab_reduce(const float* slab, float* out, long n, long stride, int splits, hipEvent_t stop) {
    PPO_REQUIRE(stride % 4 == 0 && stride >= n && al16(slab) && al16(out) && splits >= 1, "slab_reduce: operands");
    const long n4 = (n + 3) / 4;
    const bool many = splits >= 64;
    const int C = many ? 16 : 64;
    PPO_REQUIRE(n4 / C + 1 < (1L << 31), "slab_reduce: grid");
    const int grid = (int)std::max<long>(1, (n4 + C - 1) / C);
    auto kern = many ? slab_reduce_kernel<16> : slab_reduce_kernel<4>;
    if (stop)
        hipExtLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, stream(), nullptr, stop, 0, slab, out, n, stride, splits);
    else
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, stream(), slab, out, n, stride, splits);
    PPO_LAUNCH_CHECK();
}

// a grad_W's split-K slab reduce deferred into the grad_x launch that follows it on the same stream
// (phip_x3_defer_reduce): per stream, as the slab scratch
struct PendingReduce { const float* slab; float* out; long n, stride; int splits; bool on; };
static PendingReduce g_pending[2] = {};
static int g_defer_next = 0;

}  // namespace ppo

extern "C" {

// The next phip_x3_bwd_w(_fold) call on this thread leaves its split-K slab reduce (if it uses slabs) to
// the next phip_x3_bwd_x(_fold) launch on the same stream, which runs it in extra workgroups beside its
// tiles: one launch fewer per layer (the caller guarantees that grad_x follows; the next grad_W on the
// stream refuses to start while a deferred reduce is pending)
void phip_x3_defer_reduce(int on) { ppo::g_defer_next = on; }

// Shapes the engine takes (neural_network.c routes the rest to the exact fp32 kernels): the k
// extent and every leading dimension a multiple of 4 floats, 16-B aligned operands, and for
// row-contiguous operands a row extent that is a multiple of 4.
int phip_x3_supported(int op, int m, int n, int l) {
    if (m <= 0 || n <= 0 || l <= 0) return 0;
    if (op == OP_NT) return n % 4 == 0 && l % 4 == 0;          // K = n; W rows l (k-contiguous)
    if (op == OP_NN) return l % 4 == 0 && n % 4 == 0;          // K = l; W row-contiguous along n
    return n % 4 == 0 && l % 4 == 0;                           // K = m; g rows l, x rows n
}

// ydot / ypart (value-head fold): each wave's partial y = Σ relu(z)·ydot over its columns, per row, into
// ypart [slots][m]; returns slots (0 without the fold)
int phip_x3_fwd_vhead(float* y, const float* x, const int* ridx, float* xcopy, const float* W, const float* b, int m,
                      int n, int l, int relu, unsigned* bits, const float* ydot, float* ypart) {
    if (m <= 0 || l <= 0) return 0;
    PPO_REQUIRE(y && x && W && n > 0 && n % 4 == 0 && al16(x) && al16(W), "phip_x3_fwd: unsupported operands");
    PPO_REQUIRE(!ydot || ypart, "phip_x3_fwd: value-head fold without its partial buffer");
    ppo::ProfScope ps(PPO_K_GEMM, 2.0 * m * n * l, ppo::gemm_key(0, 1, m, n, l));
    X3Args a{};
    a.A = x; a.lda = n; a.B = W; a.ldb = n; a.C = y; a.ldc = l;
    a.M = m; a.N = l; a.K = n; a.kchunk = n; a.splits = 1;
    a.bias = b; a.relu = relu; a.ridx = ridx; a.acopy = ridx ? xcopy : nullptr;
    a.bits_out = relu ? bits : nullptr; a.wpr = ppo_divup(l, 32);
    a.ydot = ydot; a.ypart = ypart;
    launch_cfg_x3<OP_NT>(pick_x3(m, l, OP_NT), a);
    return ydot ? g_x3_last_slots : 0;
}

void phip_x3_fwd(float* y, const float* x, const int* ridx, float* xcopy, const float* W, const float* b, int m,
                 int n, int l, int relu, unsigned* bits) {
    (void)phip_x3_fwd_vhead(y, x, ridx, xcopy, W, b, m, n, l, relu, bits, nullptr, nullptr);
}

// the upper layer's gradient A = g [m, l]; value-head fold (fold_g): A = the 0/1 mask words of h
// (fold_bits [m][⌈l/32⌉]), W scaled per k-row by the output weights fold_w as it is staged (diag(w)·W), the
// product scaled by fold_g per row — grad_x = diag(g)·(mask·diag(w)·W) ⊙ the input mask
void phip_x3_bwd_x_fold(float* gx, const float* g, const unsigned* fold_bits, const float* fold_g, const float* fold_w,
                        const float* W, const unsigned* bits, int m, int n, int l) {
    if (m <= 0 || n <= 0) return;
    PPO_REQUIRE(gx && (g || fold_bits) && W && l > 0 && l % 4 == 0 && n % 4 == 0 && (!g || al16(g)) && al16(W),
                "phip_x3_bwd_x: unsupported operands");
    PPO_REQUIRE(!fold_bits || (fold_g && fold_w), "phip_x3_bwd_x: value-head fold operands");
    ppo::ProfScope ps(PPO_K_GEMM, 2.0 * m * n * l, ppo::gemm_key(1, 1, m, n, l));
    X3Args a{};
    a.A = fold_bits ? W : g; a.lda = l; a.B = W; a.ldb = n; a.C = gx; a.ldc = n;
    a.M = m; a.N = n; a.K = l; a.kchunk = l; a.splits = 1;
    a.bits_in = bits; a.wpr = ppo_divup(n, 32);
    a.fold_bits = fold_bits; a.fold_wpr = ppo_divup(l, 32); a.fold_g = fold_g; a.fold_w = fold_w;
    ppo::PendingReduce& pr = ppo::g_pending[phip_side_active() ? 1 : 0];
    if (pr.on) {
        a.red_slab = pr.slab; a.red_out = pr.out; a.red_n = pr.n; a.red_stride = pr.stride;
        a.red_splits = pr.splits; a.red_wgs = 1;              // (sized in launch_x3)
        pr.on = false;
    }
    launch_cfg_x3<OP_NN>(pick_x3(m, n, OP_NN), a);
}

void phip_x3_bwd_x(float* gx, const float* g, const float* W, const unsigned* bits, int m, int n, int l) {
    phip_x3_bwd_x_fold(gx, g, nullptr, nullptr, nullptr, W, bits, m, n, l);
}

void phip_x3_bwd_w_vhead(float* gW, float* gb, const float* g, float* fold_g, const float* fold_w, float* fold_gw,
                         const float* x, int m, int n, int l, int zeroed, const float* ypart, int slots, const float* b,
                         const float* tgt, float* y, float* gb_out, float* loss_accum);

// zeroed: gW / gb already hold zeros (one memset per backward); otherwise they are cleared here
void phip_x3_bwd_w(float* gW, float* gb, const float* g, const float* x, int m, int n, int l, int zeroed) {
    phip_x3_bwd_w_vhead(gW, gb, g, nullptr, nullptr, nullptr, x, m, n, l, zeroed, nullptr, 0, nullptr, nullptr, nullptr,
                        nullptr, nullptr);
}

// value-head fold (fold_g): g = h [m, l] (fp32, its mask is the operand), x scaled by fold_g per row, the
// product and the bias gradient scaled by fold_w per unit — grad_W = diag(w)·(maskᵀ·diag(g)·x), grad_b =
// diag(w)·maskᵀ·g — and fold_gw [l] (zero on entry) += Σ_rows fold_g·h, the output layer's gW
void phip_x3_bwd_w_fold(float* gW, float* gb, const float* g, const float* fold_g, const float* fold_w,
                        float* fold_gw, const float* x, int m, int n, int l, int zeroed) {
    phip_x3_bwd_w_vhead(gW, gb, g, const_cast<float*>(fold_g), fold_w, fold_gw, x, m, n, l, zeroed, nullptr, 0, nullptr,
                        nullptr, nullptr, nullptr, nullptr);
}

// + the carried value head (ypart set): g (fold_g, written) from the forward's partial dots, y, the output
// bias gradient gb_out and the loss, in this launch (X3Args vh_*)
void phip_x3_bwd_w_vhead(float* gW, float* gb, const float* g, float* fold_g, const float* fold_w, float* fold_gw,
                         const float* x, int m, int n, int l, int zeroed, const float* ypart, int slots, const float* b,
                         const float* tgt, float* y, float* gb_out, float* loss_accum) {
    if (l <= 0 || n <= 0) return;
    PPO_REQUIRE(!ypart || (fold_g && slots > 0 && b && tgt && y && gb_out), "phip_x3_bwd_w: carried value head operands");
    PPO_REQUIRE(gW && g && x && n % 4 == 0 && l % 4 == 0 && al16(g) && al16(x), "phip_x3_bwd_w: unsupported operands");
    PPO_REQUIRE(!fold_g || (fold_w && fold_gw && gb), "phip_x3_bwd_w: value-head fold operands");
    const int defer = ppo::g_defer_next;
    ppo::g_defer_next = 0;
    ppo::PendingReduce& pr = ppo::g_pending[phip_side_active() ? 1 : 0];
    PPO_REQUIRE(!pr.on, "phip_x3_bwd_w: a deferred split-K reduce was never run (phip_x3_defer_reduce without grad_x)");
    const int c = pick_x3(l, n, OP_TN);
    const long tiles = (long)ppo_divup(l, kCfgX3[c].bm) * ppo_divup(n, kCfgX3[c].bn);
    // split-K over the batch: the grid stays within one round of workgroup slots (256 CUs × the
    // configuration's workgroups per CU), each split ≥ 8 k-tiles per k-group.  (64×64 tiles for
    // C3's 256×256 gradient measured 23.5 -> 20.7 µs but sum each output over longer fp32 chains:
    // not adopted)
    const int kq = kCfgX3[c].kb * kCfgX3[c].kg;             // a split's k range: whole k-tiles per group
    const int target = g_split_x3 > 0 ? g_split_x3 : 256 * kCfgX3[c].slots_per_cu;
    int splits = (int)(target / tiles);
    const int max_splits = m / (8 * kq) > 0 ? m / (8 * kq) : 1;
    splits = std::max(1, std::min(splits, max_splits));
    int kchunk = m > 0 ? ppo_divup(ppo_divup(m, splits), kq) * kq : kq;
    splits = m > 0 ? ppo_divup(m, kchunk) : 1;
    const bool use_slab = splits > 1 && kchunk <= 1024 && al16(gW);
    // (round 6: grad_W and the grad_x that follows as ONE launch, grad_x tiles starting on the CUs grad_W
    // tiles leave, measured slower at C4 — the pair 178–183 µs vs 91.8 + 79.1 µs apart, the update 315.4 vs
    // 312.3 ms: profiles/r06_x3_pair_and_x0_ab.txt; not kept)
    ppo::ProfScope ps(PPO_K_GEMM, 2.0 * m * n * l, ppo::gemm_key(2, 1, m, n, l));
    if (m <= 0) {
        if (!zeroed) {
            phip_memset(gW, 0, sizeof(float) * (size_t)l * n);
            if (gb) phip_memset(gb, 0, sizeof(float) * (size_t)l);
        }
        return;
    }
    X3Args a{};
    a.A = g; a.lda = l; a.B = x; a.ldb = n; a.C = gW; a.ldc = n;
    a.M = l; a.N = n; a.K = m; a.kchunk = kchunk; a.splits = splits;
    a.gbias = gb;
    a.fold_g = fold_g; a.fold_w = fold_w; a.fold_gw = fold_gw;
    a.vh_ypart = ypart; a.vh_slots = slots; a.vh_b = b; a.vh_t = tgt; a.vh_y = y; a.vh_gb = gb_out; a.vh_loss = loss_accum;
    // split-K partials: per-split slabs written with plain stores and summed by one reduce launch
    // (16 MB of f32 atomics at ≈1.3 TB/s set the grad_W time of small batches; the slab path moves
    // the same bytes at store / load rate, and its sum is deterministic); the bias gradient keeps
    // its per-workgroup atomics (l floats per split)
    // (when each split is short: at C4's 32768 rows, 2048 per split, the atomics hide behind the
    // mainloop and the extra launch costs more — 326.1 vs 323.3 ms per update; at the G = 8 shard's
    // 4096 rows, 256 per split, the slabs win — 89.4 vs 93.4 ms, profiles/r03i_*)
    // (C4 re-measured in round 5 with the reduce carried by grad_x: slabs 306.4 vs atomics 302.4 ms,
    // profiles/r05_c4_gradw_slab_rejected.txt)
    // (the shard's input-layer grad_W, whose reduce has no grad_x to ride on, with 16-adder atomics instead:
    // 75.3 vs 73.2 ms, profiles/r05_shard_input_gradw_atomics_rejected.txt)
    if (splits > 1 && !zeroed) {
        if (!use_slab) phip_memset(gW, 0, sizeof(float) * (size_t)l * n);
        if (gb) phip_memset(gb, 0, sizeof(float) * (size_t)l);
    }
    if (!use_slab) {
        launch_cfg_x3<OP_TN>(c, a);
        return;
    }
    a.slab = ppo::slab_scratch((size_t)splits * l * n);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const bool timed = ppo::take_kernel_events(&e0, &e1);     // one duration: GEMM start → reduce end
    a.ev_start = timed ? e0 : nullptr;
    if (defer && splits < 64) {                               // the reduce rides on the next grad_x launch
        a.ev_stop = timed ? e1 : nullptr;
        launch_cfg_x3<OP_TN>(c, a);
        pr = ppo::PendingReduce{a.slab, gW, (long)l * n, (long)l * n, splits, true};
        return;
    }
    a.ev_stop = nullptr;
    launch_cfg_x3<OP_TN>(c, a);
    ppo::slab_reduce(a.slab, gW, (long)l * n, (long)l * n, splits, timed ? e1 : nullptr);
}

int ppo_gemm_x3_tune(int force_cfg, int splitk_target) {
    g_force_x3 = force_cfg;
    if (splitk_target >= 0) g_split_x3 = splitk_target;
    return (int)(sizeof(kCfgX3) / sizeof(kCfgX3[0]));
}

// average device µs of one launch (op 0 forward + bias + ReLU + bits, 1 grad_x with bits, 2 grad_W
// + bias grad (split-K from zero), 3 forward without activation, 4 – 6 the value-head fold variants of
// 0 – 2); cfg −1 = automatic
double ppo_bench_gemm_x3(int op, int m, int n, int l, int iters, int cfg, int splitk_target) {
    ppo::ensure_device();
    const size_t sx = (size_t)m * n, sw = (size_t)l * n, sy = (size_t)m * l;
    float* x = (float*)phip_malloc(4 * sx);
    float* W = (float*)phip_malloc(4 * sw);
    float* y = (float*)phip_malloc(4 * sy);
    float* b = (float*)phip_malloc(4 * (size_t)std::max(l, n));
    float* gw = (float*)phip_malloc(4 * sw);
    unsigned* bits = (unsigned*)phip_malloc(4 * (size_t)m * ppo_divup(std::max(l, n), 32));
    phip_fill_uniform(x, (long)sx, 1, -1.f, 1.f);
    phip_fill_uniform(W, (long)sw, 2, -0.1f, 0.1f);
    phip_fill_uniform(y, (long)sy, 3, -1.f, 1.f);
    phip_fill_uniform(b, (long)std::max(l, n), 4, -0.1f, 0.1f);
    phip_memset(bits, 0xff, 4 * (size_t)m * ppo_divup(std::max(l, n), 32));
    const int saved = g_force_x3, saved_split = g_split_x3;
    g_force_x3 = cfg;
    g_split_x3 = splitk_target;
    // ops 4 – 6: the value-head fold variants (forward with the partial dots; grad_x from the mask words
    // with the g row scale; grad_W from h with g / w scales and the output layer's gW)
    float* fold = (op >= 4) ? (float*)phip_malloc(4 * ((size_t)m * (2 * ppo_divup(l, 64) + 1) + (size_t)l)) : nullptr;
    if (fold) phip_fill_uniform(fold, (long)m * (2 * ppo_divup(l, 64) + 1) + l, 5, -0.1f, 0.1f);
    auto run = [&]() {
        if (op == 0) phip_x3_fwd(y, x, nullptr, nullptr, W, b, m, n, l, 1, bits);
        else if (op == 3) phip_x3_fwd(y, x, nullptr, nullptr, W, b, m, n, l, 0, nullptr);
        else if (op == 1) phip_x3_bwd_x(x, y, W, bits, m, n, l);
        else if (op == 4) phip_x3_fwd_vhead(y, x, nullptr, nullptr, W, b, m, n, l, 1, bits, fold, fold + l);
        else if (op == 5) phip_x3_bwd_x_fold(x, nullptr, bits, fold, fold + m, W, bits, m, n, l);
        else if (op == 6) phip_x3_bwd_w_fold(gw, b, y, fold, fold + m, fold + m + l, x, m, n, l, 0);
        else phip_x3_bwd_w(gw, b, y, x, m, n, l, 0);
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
    g_force_x3 = saved;
    g_split_x3 = saved_split;
    phip_free(x); phip_free(W); phip_free(y); phip_free(b); phip_free(gw); phip_free(bits); phip_free(fold);
    return 1000.0 * ms / (iters > 0 ? iters : 1);
}

// diagnostic: the stamps of the last PPO_X3_ABLATE=32 launch (4 per workgroup; libppo built with
// -DPPO_X3_DIAG, tools/build_variant.sh)
int ppo_x3_stamps(unsigned long long* out, int n) {
    phip_sync();
    PPO_CHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_x3_stamps), sizeof(unsigned long long) * (size_t)std::min(n, 8192 * 8)));
    return 8192 * 8;
}

}  // extern "C"
