// narrow.hip — the input layer of networks with few inputs (S ≤ 32, e.g. C3's 17 → 256), on the VALU.
//
// Reference products (mat_mul.cu:122-163 forward + bias with activation_function.cu:17-22's ReLU;
// mat_mul.cu:165-217 / neural_network.cu:108-118 weight and bias gradients):
//   forward  y = relu(x[rows]·Wᵀ + b) (+ the ReLU′ bit words, + the gathered copy of x's rows)
//   grad_W   gW = gᵀ·x, gb = Σ_rows g      (the input layer needs no grad_x)
// At K = S ≤ 32 these are 2·m·S·N FLOP against m·(S + N) operand floats: ≈ 17 FMAs per loaded or stored
// float at C3, so the GEMM engines' k-tile machinery (a 16- or 32-wide k-tile, mostly padding) and their
// ≈ 10 µs of fixed latency per launch are the cost, not the arithmetic (profiles/r04_c3_serial_update_
// breakdown.txt: 10.0 µs forward, 12.4 µs grad_W at 8192 rows).  Here one workgroup takes RB minibatch
// rows: their inputs go to LDS once (gathered through the row indices, the copy for grad_W written on
// the way), and thread t computes output columns t, t + 256, … as a K-term fp32 FMA chain per row (then
// + b), the rows' ReLU′ bits by wave ballots.  grad_W: thread t accumulates column t's K + 1 sums over
// the workgroup's rows in registers, then one f32 atomic per element per workgroup (zero on entry, as
// the split-K grad_W GEMMs), through LDS so each atomic wave instruction covers consecutive addresses.
#include "dev.h"

namespace {

constexpr int NTH = 256;
constexpr int KMAX = 32;                   // inputs (padded to KP = ⌈K/4⌉·4 ≤ 32)
constexpr int RB_F = 32;                   // forward: rows per workgroup
constexpr int RB_W = 64;                   // grad_W: rows per workgroup

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct NarrowArgs {
    const float* x; const int* ridx; float* xcopy;   // x [·, K] (rows through ridx when set), copy [m, K]
    const float* W; const float* b;                  // W [N, K], b [N]
    float* y; unsigned* bits; int relu;              // y [m, N], bits [m, N/32]
    const float* g; float* gW; float* gb;            // grad_W: g [m, N], gW [N, K], gb [N]
    int m, K, N;
};

// the workgroup's rows of x into LDS [RB][KP] (zero-padded k ≥ K and rows ≥ m); consecutive threads take
// consecutive floats of the (gathered) rows, so the copy's stores are contiguous
template <int RB>
__device__ __forceinline__ void stage_rows(const NarrowArgs& a, float* xs, int KP, int r0) {
    const int tid = threadIdx.x;
    for (int idx = tid; idx < RB * KP; idx += NTH) {
        const int r = idx / KP, k = idx % KP;
        const int row = r0 + r;
        float v = 0.f;
        if (row < a.m && k < a.K) {
            const long src = a.ridx ? (long)a.ridx[row] : (long)row;
            v = a.x[src * a.K + k];
            if (a.xcopy) a.xcopy[(long)row * a.K + k] = v;
        }
        xs[idx] = v;
    }
}

template <int KP>
__global__ __launch_bounds__(NTH) void narrow_fwd_kernel(NarrowArgs a) {
    __shared__ __attribute__((aligned(16))) float xs[RB_F * KP];
    const int r0 = blockIdx.x * RB_F;
    stage_rows<RB_F>(a, xs, KP, r0);
    __syncthreads();
    const int tid = threadIdx.x, lane = tid & 63;
    const int nrow = min(RB_F, a.m - r0);
    const int wpr = a.N >> 5;
    for (int c0 = 0; c0 < a.N; c0 += NTH) {
        const int col = c0 + tid;
        if (c0 + (tid & ~63) >= a.N) break;                   // whole waves past the last column (N % 64 == 0)
        float w[KP];
#pragma unroll
        for (int k = 0; k < KP; ++k) w[k] = k < a.K ? a.W[(long)col * a.K + k] : 0.f;
        const float bias = a.b ? a.b[col] : 0.f;
        for (int r = 0; r < nrow; ++r) {
            const f32x4* xr = reinterpret_cast<const f32x4*>(xs + r * KP);
            float acc = 0.f;
#pragma unroll
            for (int q = 0; q < KP / 4; ++q) {
                const f32x4 xv = xr[q];                      // one broadcast ds_read_b128
                acc = fmaf(xv[0], w[4 * q], acc);
                acc = fmaf(xv[1], w[4 * q + 1], acc);
                acc = fmaf(xv[2], w[4 * q + 2], acc);
                acc = fmaf(xv[3], w[4 * q + 3], acc);
            }
            float v = acc + bias;
            if (a.relu) v = v > 0.f ? v : 0.f;
            const long row = r0 + r;
            a.y[row * a.N + col] = v;
            if (a.bits) {
                const unsigned long long bb = __ballot(v > 0.f);
                if (lane == 0) a.bits[row * wpr + (col >> 5)] = (unsigned)bb;
                if (lane == 32) a.bits[row * wpr + (col >> 5)] = (unsigned)(bb >> 32);
            }
        }
    }
}

template <int KP>
__global__ __launch_bounds__(NTH) void narrow_bwd_w_kernel(NarrowArgs a) {
    __shared__ __attribute__((aligned(16))) float xs[RB_W * KP];
    __shared__ float part[NTH * (KP + 1)];
    const int r0 = blockIdx.x * RB_W;
    stage_rows<RB_W>(a, xs, KP, r0);                          // (x = the gathered copy: ridx unset)
    __syncthreads();
    const int tid = threadIdx.x;
    const int nrow = min(RB_W, a.m - r0);
    for (int c0 = 0; c0 < a.N; c0 += NTH) {
        const int col = c0 + tid;
        const bool on = col < a.N;
        float acc[KP], accb = 0.f;
#pragma unroll
        for (int k = 0; k < KP; ++k) acc[k] = 0.f;
        for (int r = 0; r < nrow; ++r) {
            const float gv = on ? a.g[(long)(r0 + r) * a.N + col] : 0.f;
            accb += gv;
            const f32x4* xr = reinterpret_cast<const f32x4*>(xs + r * KP);
#pragma unroll
            for (int q = 0; q < KP / 4; ++q) {
                const f32x4 xv = xr[q];
                acc[4 * q] = fmaf(gv, xv[0], acc[4 * q]);
                acc[4 * q + 1] = fmaf(gv, xv[1], acc[4 * q + 1]);
                acc[4 * q + 2] = fmaf(gv, xv[2], acc[4 * q + 2]);
                acc[4 * q + 3] = fmaf(gv, xv[3], acc[4 * q + 3]);
            }
        }
        // column t's K sums + its bias sum → LDS [256][K + 1] in gW's order, then the chunk's
        // (N − c0)·K consecutive gW elements (and gb) by consecutive threads
        __syncthreads();                                      // part reused across column chunks
#pragma unroll
        for (int k = 0; k < KP; ++k)
            if (k < a.K) part[tid * a.K + k] = acc[k];
        part[NTH * a.K + tid] = accb;
        __syncthreads();
        const int ncol = min(NTH, a.N - c0);
        for (int idx = tid; idx < ncol * a.K; idx += NTH) atomicAdd(a.gW + (long)c0 * a.K + idx, part[idx]);
        if (a.gb && tid < ncol) atomicAdd(a.gb + c0 + tid, part[NTH * a.K + tid]);
    }
}

}  // namespace

extern "C" {

int phip_narrow_supported(int m, int n, int l) { return m > 0 && n >= 1 && n <= KMAX && l >= 64 && l % 64 == 0; }

void phip_narrow_fwd(float* y, const float* x, const int* ridx, float* xcopy, const float* W, const float* b, int m,
                     int n, int l, int relu, unsigned* bits) {
    if (m <= 0) return;
    PPO_REQUIRE(y && x && W && phip_narrow_supported(m, n, l), "phip_narrow_fwd: unsupported operands");
    ppo::ProfScope ps(PPO_K_GEMM, 2.0 * m * n * l, ppo::gemm_key(0, 0, m, n, l));
    NarrowArgs a{};
    a.x = x; a.ridx = ridx; a.xcopy = ridx ? xcopy : nullptr; a.W = W; a.b = b;
    a.y = y; a.bits = relu ? bits : nullptr; a.relu = relu;
    a.m = m; a.K = n; a.N = l;
    const dim3 grid(ppo_divup(m, RB_F));
    const int KP = (n + 3) / 4 * 4;
    switch (KP) {
        case 4: PPO_TIMED_LAUNCH(narrow_fwd_kernel<4>, grid, dim3(NTH), 0, ppo::stream(), a); break;
        case 8: PPO_TIMED_LAUNCH(narrow_fwd_kernel<8>, grid, dim3(NTH), 0, ppo::stream(), a); break;
        case 12: PPO_TIMED_LAUNCH(narrow_fwd_kernel<12>, grid, dim3(NTH), 0, ppo::stream(), a); break;
        case 16: PPO_TIMED_LAUNCH(narrow_fwd_kernel<16>, grid, dim3(NTH), 0, ppo::stream(), a); break;
        case 20: PPO_TIMED_LAUNCH(narrow_fwd_kernel<20>, grid, dim3(NTH), 0, ppo::stream(), a); break;
        case 24: PPO_TIMED_LAUNCH(narrow_fwd_kernel<24>, grid, dim3(NTH), 0, ppo::stream(), a); break;
        case 28: PPO_TIMED_LAUNCH(narrow_fwd_kernel<28>, grid, dim3(NTH), 0, ppo::stream(), a); break;
        default: PPO_TIMED_LAUNCH(narrow_fwd_kernel<32>, grid, dim3(NTH), 0, ppo::stream(), a); break;
    }
    PPO_LAUNCH_CHECK();
}

// gW [l, n] += gᵀ·x and gb [l] += Σ_rows g (zero on entry unless `zeroed` is 0: then cleared here)
void phip_narrow_bwd_w(float* gW, float* gb, const float* g, const float* x, int m, int n, int l, int zeroed) {
    PPO_REQUIRE(gW && g && x && phip_narrow_supported(m > 0 ? m : 1, n, l), "phip_narrow_bwd_w: unsupported operands");
    if (!zeroed) {
        phip_memset(gW, 0, sizeof(float) * (size_t)l * n);
        if (gb) phip_memset(gb, 0, sizeof(float) * (size_t)l);
    }
    if (m <= 0) return;
    ppo::ProfScope ps(PPO_K_GEMM, 2.0 * m * n * l, ppo::gemm_key(2, 0, m, n, l));
    NarrowArgs a{};
    a.x = x; a.g = g; a.gW = gW; a.gb = gb;
    a.m = m; a.K = n; a.N = l;
    const dim3 grid(ppo_divup(m, RB_W));
    const int KP = (n + 3) / 4 * 4;
    switch (KP) {
        case 4: PPO_TIMED_LAUNCH(narrow_bwd_w_kernel<4>, grid, dim3(NTH), 0, ppo::stream(), a); break;
        case 8: PPO_TIMED_LAUNCH(narrow_bwd_w_kernel<8>, grid, dim3(NTH), 0, ppo::stream(), a); break;
        case 12: PPO_TIMED_LAUNCH(narrow_bwd_w_kernel<12>, grid, dim3(NTH), 0, ppo::stream(), a); break;
        case 16: PPO_TIMED_LAUNCH(narrow_bwd_w_kernel<16>, grid, dim3(NTH), 0, ppo::stream(), a); break;
        case 20: PPO_TIMED_LAUNCH(narrow_bwd_w_kernel<20>, grid, dim3(NTH), 0, ppo::stream(), a); break;
        case 24: PPO_TIMED_LAUNCH(narrow_bwd_w_kernel<24>, grid, dim3(NTH), 0, ppo::stream(), a); break;
        case 28: PPO_TIMED_LAUNCH(narrow_bwd_w_kernel<28>, grid, dim3(NTH), 0, ppo::stream(), a); break;
        default: PPO_TIMED_LAUNCH(narrow_bwd_w_kernel<32>, grid, dim3(NTH), 0, ppo::stream(), a); break;
    }
    PPO_LAUNCH_CHECK();
}

}  // extern "C"
