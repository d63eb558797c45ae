// cluster_deep.hip — a whole phase of minibatch steps at the reference's B = 64 for S → 512 → 512 →
// 512 → O networks (config C4: S = 376, O = 1 for V, 17 for μ), in ONE launch of NWG = 32
// cooperating workgroups.
//
// Workgroup c owns the 16 hidden units [16c, 16c+16) of all three hidden layers: its rows of W0, W1,
// W2 and their biases stay in LDS for the whole phase (≈ 90 KiB), their Adam moments in HBM (read
// and written around each gradient tile), and the matching input columns of the output layer W3 with the small parameters.  The activations do
// not fit a CU (three 64 × 512 fp32 blocks), so the full-width operands are read from HBM / L2 where
// they were published: the state rows (gathered by index, never copied), h1 and h2.  Per step
// (reference ppo.cu:395-443, arithmetic as in cluster.hip):
//   h1[:, own] = relu(x·W0[own]ᵀ + b0)                         → X1            barrier A
//   h2[:, own] = relu(h1·W1[own]ᵀ + b1)                        → X2            barrier B
//   h3[:, own] = relu(h2·W2[own]ᵀ + b2);  y partial = h3[:, own]·W3[:, own]ᵀ → Y   barrier C
//   policy: rows 2c, 2c+1: y = Σ partials (fixed order) + b3, the head → G3 (∂L/∂y, log σ terms, loss) D
//   value (O = 1): every workgroup reduces all 64 rows' partials and runs the head itself (no D)
//   gW3[:, own], gb3, g3 = (∂L/∂y·W3[:, own]) ⊙ 1[h3 > 0];  P2 = g3·W2[own, :] → Pa               E
//     (gW2[own] = g3ᵀ·h2 with Adam fused, inside E's wait)
//   g2[:, own] = Σ P2 partials ⊙ 1[h2 > 0];  P1 = g2·W1[own, :] → Pb                              F
//     (gW1[own] = g2ᵀ·h1 with Adam fused, inside F's wait)
//   g1[:, own] = Σ P1 partials ⊙ 1[h1 > 0];  gW0[own] = g1ᵀ·x with Adam fused;  Adam of the rest
// Six barriers per policy step, five per value step (cluster_common.h: sc1 hand-offs, split arrive / wait).  b3 and log σ are
// replicated: every workgroup reads the same ∂L/∂y rows and reduces them in the same order.  Buffer
// reuse across steps is safe by the barrier order, except X1, which the F gap of step s reads while a
// workgroup past F may already publish step s + 1's h1: X1 is double-buffered by step parity.
#include "cluster_common.h"

#include <cstdlib>

namespace {
using namespace clu;

constexpr int H = 512, HC = 16, NWG = H / HC;        // 32 workgroups of 16 hidden units
constexpr int HP = H + 4;                            // LDS pitch of [HC][H] weight rows (4·odd)
constexpr int HCP = HC + 4;                          // pitch of [64][HC] arrays (4·odd)
constexpr int SPMAX = 380;                           // W0 row pitch (4·odd): S ≤ 380, S % 4 == 0
constexpr int OMAX = 32;                             // output tiles: two 16-wide
constexpr int OP = 20;                               // output pitch of the hand-offs and actions (O ≤ 20)
constexpr int GOP = 36;                              // LDS pitch of [64][OMAX] arrays
constexpr int GP = 2 * OP + 4;                       // G3 row: ∂L/∂y (OP) | log σ row terms (OP) | loss (4)
constexpr int T12 = (H / 16) / NWAVE;                // gW1 / gW2 tiles per wave (4)
constexpr int T0 = (SPMAX + 15) / 16 / NWAVE;        // gW0 tiles per wave (3)
constexpr int RPW = BB / NWG;                        // head rows per workgroup (2)
constexpr int NSTAMP = 18;
#ifndef CLU_PPAD
#define CLU_PPAD 0                                   // floats of padding per row of the Pa / Pb partial slabs
#endif
constexpr int PH = H + CLU_PPAD;                     // Pa / Pb row pitch
#ifndef CLU_PSLICE
#define CLU_PSLICE 1                                 // Pa / Pb slice-major ([slice][p][b][HC]); 0: row-major [p][b][H]
#endif
// Slice-major: a workgroup's reduction of its own 16 columns over the 32 partials is one contiguous
// 128 KB block. Row-major, it read 64 B from every 2-KB row (2,048 loads at one address offset mod 2 KB),
// and the four slices at offsets 384-511 mod 1024 B (6, 7, 22, 23) were 1.5-1.8 µs slower at barriers A
// and F in every placement (PPO_CLUSTER_ROT moved the slow workgroups with their slices): the step
// waits for them. Slice-major: every slice 13.1 / 5.9 µs (was 14.0 / 7.5, slow 15.5 / 9.3); C4 B = 64
// 9.51-9.69 s per update vs 10.44-10.51 row-major, same box (profiles/r06_c4b64_partial_layout.txt).
// float offset of partial p's row b, hidden unit slice·HC + j, in a Pa / Pb slab
__device__ __forceinline__ int pidx(int slice, int p, int b, int j) {
#if CLU_PSLICE
    return ((slice * NWG + p) * BB + b) * HC + j;
#else
    return (p * BB + b) * PH + slice * HC + j;
#endif
}
#ifndef CLU_GW_PRE
#define CLU_GW_PRE 1                                 // weight-gradient tiles whose operands load under the P partial
#endif
#ifndef CLU_FWD_NG
#define CLU_FWD_NG 4                                 // forward k-groups of 16 in flight per lane (16 — a whole
                                                     // K half — measured slower: 5.7 vs 4.9 µs per layer)
#endif
static_assert(T12 * NWAVE * 16 == H && T0 * NWAVE * 16 >= SPMAX && RPW * NWG == BB, "tile counts");

struct DArgs {
    int S, O, policy;
    float *params, *grads, *m, *v;                   // the network's flat buffers and Adam moments
    long woff[4], boff[4];
    float *log_std, *log_std_grad, *m_ls, *v_ls;
    const float *state, *action, *logprob, *adv, *adv_target;
    int limit, num_batches, n_epochs, total_steps;
    const int* perms;
    Feistel fk[16];
    const float *steps, *steps_ls;                   // per step {lr/bc1, bc2}
    float b1, b2, eps, ent_coeff;
    float* stats;
    float *X1, *X2, *Y, *G3, *Pa, *Pb;               // hand-offs (X1 [2][64][H], X2 [64][H], Y [NWG][64][OP],
                                                     // G3 [64][GP], Pa / Pb [NWG slices][NWG][64][HC])
    unsigned *ctr, *err;
    unsigned long long timeout;                      // barrier wait bound (realtime ticks)
    int active_stride, active_offset;                // workgroup b works iff b % stride == offset
    int rot;                                         // PPO_CLUSTER_ROT (diagnostic): workgroup cw owns hidden
                                                     // slice (cw + rot) mod NWG — separates slice from placement
    unsigned long long* stamps;                      // PPO_CLUSTER_STAMPS: workgroup 0, steps 0..63
    unsigned long long* arr;                         // PPO_CLUSTER_STAMPS=2: every workgroup's arrival and exit
                                                     // time at every barrier, steps 0..63 [64][6][2][NWG]
};

// LDS layout (floats)
struct L {
    static constexpr int W0 = 0;                     // [HC][SPMAX] own rows (pad columns zero)
    static constexpr int W1 = W0 + HC * SPMAX;       // [HC][HP]
    static constexpr int W2 = W1 + HC * HP;          // [HC][HP]
    static constexpr int W3 = W2 + HC * HP;          // [OMAX][HCP] own input columns (rows o ≥ O zero)
    static constexpr int b0 = W3 + OMAX * HCP;       // [HC]
    static constexpr int b1 = b0 + HC;
    static constexpr int b2 = b1 + HC;
    static constexpr int b3 = b2 + HC;               // [OMAX] replicated
    static constexpr int ls = b3 + OMAX;             // [OMAX] log σ, replicated
    static constexpr int h1 = ls + OMAX;             // [64][HCP] own columns of h1, h2, h3
    static constexpr int h2 = h1 + BB * HCP;
    static constexpr int h3 = h2 + BB * HCP;
    static constexpr int g3 = h3 + BB * HCP;         // [64][GOP] ∂L/∂y (columns ≥ O zero)
    static constexpr int glr = g3 + BB * GOP;        // [64][GOP] log σ row terms
    static constexpr int gh = glr + BB * GOP;        // [64][HCP] ∂L/∂h (own columns) of the layer at hand
    static constexpr int gW3 = gh + BB * HCP;        // [OMAX][HCP]
    static constexpr int gb0 = gW3 + OMAX * HCP;
    static constexpr int gb1 = gb0 + HC;
    static constexpr int gb2 = gb1 + HC;
    static constexpr int gb3 = gb2 + HC;             // [OMAX]
    static constexpr int gls = gb3 + OMAX;           // [OMAX]
    static constexpr int rows = gls + OMAX;          // int [2][64] (double-buffered minibatch)
    static constexpr int tgt = rows + 2 * BB;        // [2][64]
    static constexpr int olp = tgt + 2 * BB;         // [2][64]
    static constexpr int act = olp + 2 * BB;         // [2][64][OP]
    static constexpr int hrow = act + 2 * BB * OP;   // [RPW][GP] the head's rows before publishing
    static constexpr int lossr = hrow + RPW * GP;    // [64] per-row loss terms
    static constexpr int scr = lossr + BB;           // [2048] K-split / half-sum hand-over
    static constexpr int flag = scr + 2048;
    static constexpr int TOTAL = flag + 4;
};

struct Small { int lds_p, lds_g; long gflat; int kind; };   // kind 0 network, 1 log σ, 2 replicated net

// the small parameters of a workgroup: W3 columns [O][HC], b0, b1, b2 [HC], b3 [O] (replicated), log σ [O]
__device__ __forceinline__ Small small_elem(const DArgs& a, int e, int c0) {
    const int O = a.O;
    if (e < O * HC) { const int o = e / HC, j = e % HC;
        return {L::W3 + o * HCP + j, L::gW3 + o * HCP + j, a.woff[3] + (long)o * H + c0 + j, 0}; }
    e -= O * HC;
    if (e < 3 * HC) { const int l = e / HC, j = e % HC;
        return {L::b0 + l * HC + j, L::gb0 + l * HC + j, a.boff[l] + c0 + j, 0}; }
    e -= 3 * HC;
    if (e < O) return {L::b3 + e, L::gb3 + e, a.boff[3] + e, 2};
    e -= O;
    return {L::ls + e, L::gls + e, e, 1};
}

__device__ __forceinline__ int gather_src(const DArgs& a, int ep, int kb, int i) {
    const int list = (int)(((long)kb * BB + i) % a.limit);
    return a.perms ? a.perms[(long)ep * a.limit + list] : (int)feistel_index((uint32_t)list, a.fk[ep & 15]);
}
// the minibatch of step (ep, kb) (trajectory_buffer.cu:168-200): row indices and per-row scalars, by
// wave 1 (wave 0's first lane polls the barriers this runs beside)
__device__ __forceinline__ void gather_rows(const DArgs& a, float* lds, int ep, int kb, int buf) {
    const int i = (int)threadIdx.x - 64;
    if (i >= 0 && i < BB) {
        const int src = gather_src(a, ep, kb, i);
        reinterpret_cast<int*>(lds + L::rows)[buf * BB + i] = src;
        if (a.policy) {
            const float ad = a.adv[src], lp = a.logprob[src];
            lds[L::tgt + buf * BB + i] = ad;
            lds[L::olp + buf * BB + i] = lp;
        } else {
            lds[L::tgt + buf * BB + i] = a.adv_target[src];
        }
    }
}
// the policy's action rows (behind a workgroup barrier after gather_rows), by waves 1-7
__device__ __forceinline__ void gather_act(const DArgs& a, float* lds, int buf) {
    if (!a.policy || threadIdx.x < 64) return;
    const int* rows = reinterpret_cast<const int*>(lds + L::rows) + buf * BB;
    const int A = a.O, t = (int)threadIdx.x - 64;
    constexpr int NT = TPB - 64, U = (BB * OP + NT - 1) / NT;
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int e = t + u * NT;
        v[u] = e < BB * A ? a.action[(long)rows[e / A] * A + e % A] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int e = t + u * NT;
        if (e < BB * A) lds[L::act + buf * BB * OP + (e / A) * OP + e % A] = v[u];
    }
}

// Forward tile: acc(j, b) = Σ_{k ∈ [k0, k1)} W[j][k]·X[b][k] for one 16 × 16 block, lane (c, q) holding
// the weight row c (LDS, Wr) and the activation row c (HBM, ldx(k) = 4 values at k).  k runs in groups
// of 16: lane q takes k = 16u + 4q + i for the group's MFMA i — both operands alike, so the sum covers
// every k once (in a different association order than mm_tile's).  k0, k1 multiples of 4.  NG groups'
// activation loads are in flight before their MFMAs (NG = 16: a whole K half, one memory latency per
// tile); the weights are read from LDS group by group.
template <int NG, class LoadX>
__device__ __forceinline__ f32x4 fwd_tile(int tid, const float* Wr, int k0, int k1, LoadX ldx) {
    const int q = (tid & 63) >> 4;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int g0 = k0; g0 < k1; g0 += 16 * NG) {
        f32x4 xv[NG];
#pragma unroll
        for (int u = 0; u < NG; ++u) {
            const int k = g0 + 16 * u + 4 * q;
            xv[u] = k < k1 ? ldx(k) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < NG; ++u) {
            if (g0 + 16 * u < k1) {
                const int k = g0 + 16 * u + 4 * q;
                const f32x4 wv = k < k1 ? *reinterpret_cast<const f32x4*>(Wr + k) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int i = 0; i < 4; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[i], xv[u][i], acc, 0, 0, 0);
            }
        }
    }
    return acc;
}

// Weight-gradient tiles with Adam fused.  The lane's wave owns tiles t = 0 … T−1 at columns
// col = 16(w + 8t) + c (< ncols), rows j = 4q + e: gW[j][col] = Σ_b G[b][j]·X[b][col] over the 64 rows
// (lane (c, q) holds G[b][c] from LDS and X[b][col] = ldb(b, col) for b = 4u + q).  load(): every X
// operand of the T tiles and the moments (HBM, row j at g0 + j·ld) in flight at once; apply(): the
// MFMAs, Adam on the LDS parameters (row j at W + j·pp), the moments written back, and on the last
// step of the phase the gradient too (callers may read it, as after the multi-launch loop).
template <int T>
struct GwTiles {
    float bv[T][16], mm[T][4], vv[T][4];
    template <class LoadB>
    __device__ __forceinline__ void load(int tid, const DArgs& a, long g0, long ld, int ncols, LoadB ldb, int t0 = 0) {
        const int lane = tid & 63, c = lane & 15, q = lane >> 4, w = tid >> 6;
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const int col = 16 * (w + NWAVE * (t0 + t)) + c;
            const bool in = col < ncols;
#pragma unroll
            for (int u = 0; u < 16; ++u) bv[t][u] = in ? ldb(4 * u + q, col) : 0.f;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                mm[t][e] = in ? a.m[g0 + (4 * q + e) * ld + col] : 0.f;
                vv[t][e] = in ? a.v[g0 + (4 * q + e) * ld + col] : 0.f;
            }
        }
    }
    __device__ __forceinline__ void apply(int tid, const DArgs& a, const float* G, float* W, int pp, long g0, long ld,
                                          int ncols, float st, float bc2, bool last, int t0 = 0) {
        const int lane = tid & 63, c = lane & 15, q = lane >> 4, w = tid >> 6;
#pragma unroll
        for (int t = 0; t < T; ++t) {
            if (16 * (w + NWAVE * (t0 + t)) >= ncols) continue;             // wave-uniform
            const int col = 16 * (w + NWAVE * (t0 + t)) + c;
            float av[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) av[u] = G[(4 * u + q) * HCP + c];
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int u = 0; u < 16; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[t][u], acc, 0, 0, 0);
            if (col < ncols) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float* p = W + (4 * q + e) * pp + col;
                    float pv = *p;
                    adam_elem(pv, acc[e], mm[t][e], vv[t][e], st, a.b1, a.b2, bc2);
                    *p = pv;
                    const long gi = g0 + (4 * q + e) * ld + col;
                    a.m[gi] = mm[t][e];
                    a.v[gi] = vv[t][e];
                    if (last) a.grads[gi] = acc[e];
                }
            }
        }
    }
};

// Adam of the thread's small parameter (log σ with the entropy step sizes, ppo.cu:440-442): the b0
// elements when b0 is set, the others otherwise
__device__ __forceinline__ void small_adam(const DArgs& a, float* lds, int tid, int c0, int nsmall, float& sm, float& sv,
                                           int step, float st, float bc2, bool b0) {
    if (tid >= nsmall) return;
    const Small s = small_elem(a, tid, c0);
    if ((s.lds_p >= L::b0 && s.lds_p < L::b0 + HC) != b0) return;
    float pv = lds[s.lds_p];
    const float g = lds[s.lds_g];
    if (s.kind == 1) adam_elem(pv, g, sm, sv, a.steps_ls[2 * step], a.b1, a.b2, a.steps_ls[2 * step + 1]);
    else adam_elem(pv, g, sm, sv, st, a.b1, a.b2, bc2);
    lds[s.lds_p] = pv;
}

// K-split epilogue: waves 4-7 hand their partial to waves 0-3 (tile w & 3) through LDS, then the
// owners return the sum.  Every thread reaches the barrier.
__device__ __forceinline__ f32x4 ksplit_sum(int tid, f32x4 acc, float* lds) {
    const int w = tid >> 6, lane = tid & 63;
    if (w >= 4) *reinterpret_cast<f32x4*>(lds + L::scr + ((w & 3) * 64 + lane) * 4) = acc;
    __syncthreads();
    if (w < 4) acc += *reinterpret_cast<const f32x4*>(lds + L::scr + (w * 64 + lane) * 4);
    return acc;
}

// ∂L/∂h (own columns) = Σ_p P_p[b][c0 + j] (fixed order) ⊙ 1[h[b][j] > 0]: 256 float4 sums, threads
// 256-511 add partials 16…31 and hand them over.  load() issues the thread's 16 loads (so that loads
// issued after it — the next tiles' operands — do not delay its wait); finish() sums and masks.
struct PartialSum {
    f32x4 v[NWG / 2];
    __device__ __forceinline__ void load(int tid, __amdgpu_buffer_rsrc_t rP, int c0) {
        const int it = tid & 255, half = tid >> 8, b = it >> 2, jq = 4 * (it & 3);
#pragma unroll
        for (int p = 0; p < NWG / 2; ++p) v[p] = ld16_sc1(rP, pidx(c0 / HC, half * (NWG / 2) + p, b, jq));
    }
    __device__ __forceinline__ void finish(int tid, const float* hown, float* lds) {
        const int it = tid & 255, half = tid >> 8, b = it >> 2, jq = 4 * (it & 3);
        f32x4 s = v[0];
#pragma unroll
        for (int p = 1; p < NWG / 2; ++p) s += v[p];
        if (half) *reinterpret_cast<f32x4*>(lds + L::scr + 4 * it) = s;
        __syncthreads();
        if (!half) {
            s += *reinterpret_cast<const f32x4*>(lds + L::scr + 4 * it);
#pragma unroll
            for (int e = 0; e < 4; ++e) lds[L::gh + b * HCP + jq + e] = hown[b * HCP + jq + e] > 0.f ? s[e] : 0.f;
        }
    }
};
__device__ __forceinline__ void reduce_partials(int tid, __amdgpu_buffer_rsrc_t rP, int c0, const float* hown,
                                                float* lds) {
    PartialSum ps;
    ps.load(tid, rP, c0);
    ps.finish(tid, hown, lds);
}

// Pᵀ[k][b] = Σ_j W[j][k]·gh[b][j] over the own units (reduction over 16 j): 32 × 4 tiles, published
// (16-B sc1 stores, 4 consecutive k per lane)
__device__ __forceinline__ void publish_partial(int tid, __amdgpu_buffer_rsrc_t rP, int cw, const float* W,
                                                const float* lds) {
    const int w = tid >> 6, lane = tid & 63, c = lane & 15, q = lane >> 4;
    for (int t = w; t < (H / 16) * (BB / 16); t += NWAVE) {
        const int tk = t >> 2, tb = t & 3;
        const f32x4 acc = mm_tile(W + 16 * tk, 1, HP, lds + L::gh + 16 * tb * HCP, 1, HCP, HC, tid);
        st16_sc1(rP, pidx(tk, cw, 16 * tb + c, 4 * q), acc);
    }
}

#define CD_STAMP(slot)                                                                                   \
    do {                                                                                                 \
        if (a.stamps && cw == 0 && tid == 0 && step < 64) {                                             \
            a.stamps[step * NSTAMP + (slot)] = wall_clock64();                                           \
            a.stamps[CLU_STAMP_CLK + step * NSTAMP + (slot)] = __builtin_amdgcn_s_memtime();             \
        }                                                                                                \
    } while (0)

// per-workgroup barrier stamps (PPO_CLUSTER_STAMPS=2): arrival (after the counter adds) and exit (the
// wait returned) of barrier bi (A … F = 0 … 5) at step `step`
#define CD_BAR_STAMP(bi, ex)                                                                              \
    do {                                                                                                  \
        if (a.arr && tid == 0 && step < 64) a.arr[((step * 6 + (bi)) * 2 + (ex)) * NWG + cw] = wall_clock64(); \
    } while (0)

__global__ __launch_bounds__(TPB) void cluster_deep_kernel(DArgs a) {
    if ((int)blockIdx.x % a.active_stride != a.active_offset) return;
    const int cw = (int)blockIdx.x / a.active_stride;
    // diagnostics (PPO_CLUSTER_STAMPS): where this workgroup runs — XCC id, HW_ID (CU / SH / SE fields)
    if (a.stamps && threadIdx.x == 0)
        a.stamps[64 * 32 + cw] = ((unsigned long long)__builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11)) << 32) |
                                 __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
    const int c0 = ((cw + a.rot) % NWG) * HC;
    extern __shared__ float lds[];
    int* flag = reinterpret_cast<int*>(lds + L::flag);
    const int tid = threadIdx.x;
    const int S = a.S, O = a.O, A = a.O;
    const int nsmall = O * HC + 3 * HC + O + (a.policy ? A : 0);
    const auto rX1 = rsrc(a.X1, 2L * BB * H), rX2 = rsrc(a.X2, (long)BB * H);
    const auto rY = rsrc(a.Y, (long)NWG * BB * OP), rG3 = rsrc(a.G3, (long)BB * GP);
    const auto rPa = rsrc(a.Pa, (long)NWG * BB * PH), rPb = rsrc(a.Pb, (long)NWG * BB * PH);

    // ---- phase start: own parameters → LDS, Adam moments → VGPRs ----
    for (int e = tid; e < HC * SPMAX; e += TPB) {
        const int j = e / SPMAX, k = e % SPMAX;
        lds[L::W0 + e] = k < S ? a.params[a.woff[0] + (long)(c0 + j) * S + k] : 0.f;
    }
    for (int e = tid; e < HC * H; e += TPB) {
        const int j = e / H, k = e % H;
        lds[L::W1 + j * HP + k] = a.params[a.woff[1] + (long)(c0 + j) * H + k];
        lds[L::W2 + j * HP + k] = a.params[a.woff[2] + (long)(c0 + j) * H + k];
    }
    for (int e = tid; e < OMAX * HCP; e += TPB) lds[L::W3 + e] = 0.f;
    for (int e = tid; e < OMAX; e += TPB) { lds[L::b3 + e] = 0.f; lds[L::ls + e] = 0.f; }
    for (int e = tid; e < BB * GOP; e += TPB) { lds[L::g3 + e] = 0.f; lds[L::glr + e] = 0.f; }
    __syncthreads();
    float sm = 0.f, sv = 0.f;                                    // one small parameter per thread
    if (tid < nsmall) {
        const Small s = small_elem(a, tid, c0);
        if (s.kind == 1) { lds[s.lds_p] = a.log_std[s.gflat]; sm = a.m_ls[s.gflat]; sv = a.v_ls[s.gflat]; }
        else { lds[s.lds_p] = a.params[s.gflat]; sm = a.m[s.gflat]; sv = a.v[s.gflat]; }
    }
    gather_rows(a, lds, 0, 0, 0);
    __syncthreads();
    gather_act(a, lds, 0);
    __syncthreads();

    unsigned nbar = 0;
    f32x4 pf = {0.f, 0.f, 0.f, 0.f};                             // the next minibatch's state rows, prefetched
    int step = 0;
    bool ok = true;
    for (int ep = 0; ep < a.n_epochs && ok; ++ep) {
        for (int kb = 0; kb < a.num_batches && step < a.total_steps && ok; ++kb, ++step) {
            // lane ids from an opaque copy each step: the compiler cannot hoist the (many) lane-derived
            // addresses out of the step loop and keep them live — they would spill
            int tid = (int)threadIdx.x;
            asm volatile("" : "+v"(tid));
            const int lane = tid & 63, w = tid >> 6, c = lane & 15, q = lane >> 4;
            CD_STAMP(0);
#ifndef CLU_NO_PREFETCH
            asm volatile("" ::"v"(pf));                                  // (the prefetch has landed)
#endif
            const int cur = step & 1;
            const int* rows = reinterpret_cast<const int*>(lds + L::rows) + cur * BB;
            const int tc = L::tgt + cur * BB, oc = L::olp + cur * BB, acb = L::act + cur * BB * OP;
            const int x1o = cur * BB * H;
            const bool has_next = step + 1 < a.total_steps, last = !has_next;
            const int kb_n = kb + 1 < a.num_batches ? kb + 1 : 0, ep_n = kb + 1 < a.num_batches ? ep : ep + 1;
            const float st = a.steps[2 * step], bc2 = a.steps[2 * step + 1];

            // ---- layer 0 (own units): h1ᵀ[j][b] = Σ_s W0[j][s]·x[b][s], the state rows read in place;
            // tile w & 3 of the batch, K split in halves (waves 4-7 the upper) ----
            {
                const int tb = w & 3, ks = w >> 2, kh = ((S / 4 + 1) / 2) * 4;
                const float* xr = a.state + (long)rows[16 * tb + c] * S;
                f32x4 acc = fwd_tile<CLU_FWD_NG>(tid, lds + L::W0 + c * SPMAX, ks ? kh : 0, ks ? S : kh,
                                     [&](int k) { return *reinterpret_cast<const f32x4*>(xr + k); });
                acc = ksplit_sum(tid, acc, lds);
                if (w < 4) {
                    const int b = 16 * tb + c;
                    f32x4 hv;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float v = acc[e] + lds[L::b0 + 4 * q + e];
                        hv[e] = v > 0.f ? v : 0.f;                            // neural_network.cu:74-105
                    }
                    *reinterpret_cast<f32x4*>(lds + L::h1 + b * HCP + 4 * q) = hv;
                    st16_sc1(rX1, x1o + b * H + c0 + 4 * q, hv);
                }
            }
            CD_STAMP(1);
            cluster_arrive(a.ctr);
            CD_BAR_STAMP(0, 0);
            if (has_next) gather_rows(a, lds, ep_n, kb_n, cur ^ 1);     // the next minibatch, part 1
            ok = cluster_wait(a.ctr, a.err, nbar++, NWG, flag, cw, a.timeout);          // A: h1 published
            if (!ok) break;
            CD_BAR_STAMP(0, 1);
            CD_STAMP(2);
            // ---- layer 1: h2ᵀ[j][b] = Σ_k W1[j][k]·h1[b][k] ----
            {
                const int tb = w & 3, ks = w >> 2, b = 16 * tb + c;
                f32x4 acc = fwd_tile<CLU_FWD_NG>(tid, lds + L::W1 + c * HP, ks * (H / 2), (ks + 1) * (H / 2),
                                     [&](int k) { return ld16_sc1(rX1, x1o + b * H + k); });
                acc = ksplit_sum(tid, acc, lds);
                if (w < 4) {
                    f32x4 hv;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float v = acc[e] + lds[L::b1 + 4 * q + e];
                        hv[e] = v > 0.f ? v : 0.f;
                    }
                    *reinterpret_cast<f32x4*>(lds + L::h2 + b * HCP + 4 * q) = hv;
                    st16_sc1(rX2, b * H + c0 + 4 * q, hv);
                }
            }
            CD_STAMP(3);
            cluster_arrive(a.ctr);
            CD_BAR_STAMP(1, 0);
            if (has_next) gather_act(a, lds, cur ^ 1);                   // the next minibatch, part 2
#ifndef CLU_NO_PREFETCH
            // rows 2cw, 2cw + 1 of the next minibatch from HBM into the caches (each workgroup two, so
            // every row is fetched once before the 32 workgroups read all of them at the next layer 0)
            if (has_next && tid < 2 * (S / 4)) {
                const int* rn = reinterpret_cast<const int*>(lds + L::rows) + (cur ^ 1) * BB;
                const int r = tid / (S / 4), k = 4 * (tid % (S / 4));
                pf = *reinterpret_cast<const f32x4*>(a.state + (long)rn[RPW * cw + r] * S + k);
            }
#endif
            ok = cluster_wait(a.ctr, a.err, nbar++, NWG, flag, cw, a.timeout);          // B: h2 published
            if (!ok) break;
            CD_BAR_STAMP(1, 1);
            CD_STAMP(4);
            // ---- layer 2: h3ᵀ[j][b] = Σ_k W2[j][k]·h2[b][k] (own columns stay in LDS) ----
            {
                const int tb = w & 3, ks = w >> 2, b = 16 * tb + c;
                f32x4 acc = fwd_tile<CLU_FWD_NG>(tid, lds + L::W2 + c * HP, ks * (H / 2), (ks + 1) * (H / 2),
                                     [&](int k) { return ld16_sc1(rX2, b * H + k); });
                acc = ksplit_sum(tid, acc, lds);
                if (w < 4) {
                    f32x4 hv;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float v = acc[e] + lds[L::b2 + 4 * q + e];
                        hv[e] = v > 0.f ? v : 0.f;
                    }
                    *reinterpret_cast<f32x4*>(lds + L::h3 + b * HCP + 4 * q) = hv;
                }
            }
            __syncthreads();
            // ---- output layer, own input columns: yᵀ[o][b] = Σ_j W3[o][j]·h3[b][j] → Y[cw] ----
            {
                const int to = w >> 2, tb = w & 3;
                if (16 * to < O) {
                    const f32x4 acc = mm_tile(lds + L::W3 + 16 * to * HCP, HCP, 1, lds + L::h3 + 16 * tb * HCP, 1, HCP, HC, tid);
                    if (16 * to + 4 * q < (a.policy ? OP : 4))
                        st16_sc1(rY, (cw * BB + 16 * tb + c) * OP + 16 * to + 4 * q, acc);
                }
            }
            CD_STAMP(5);
            cluster_arrive(a.ctr);
            CD_BAR_STAMP(2, 0);
            ok = cluster_wait(a.ctr, a.err, nbar++, NWG, flag, cw, a.timeout);          // C: y partials published
            if (!ok) break;
            CD_BAR_STAMP(2, 1);
            CD_STAMP(6);
            if (!a.policy) {
                // ---- the value head, replicated: every workgroup reduces all 64 rows' partials (one
                // float4 each) in the same order — no ∂L/∂y hand-off (loss.cu:5-23) ----
                {
                    const int b = tid >> 3, pg = tid & 7;
                    f32x4 v[NWG / 8];
#pragma unroll
                    for (int u = 0; u < NWG / 8; ++u) v[u] = ld16_sc1(rY, ((pg * (NWG / 8) + u) * BB + b) * OP);
                    float s = v[0][0];
#pragma unroll
                    for (int u = 1; u < NWG / 8; ++u) s += v[u][0];
                    lds[L::scr + tid] = s;
                }
                __syncthreads();
                if (tid < BB) {
                    float y = lds[L::scr + 8 * tid];
                    for (int pg = 1; pg < 8; ++pg) y += lds[L::scr + 8 * tid + pg];
                    y += lds[L::b3];
                    const float t = lds[tc + tid], d = t - y;
                    lds[L::lossr + tid] = d * d;
                    lds[L::g3 + tid * GOP] = 2 * (y - t) / (float)BB;
                }
                __syncthreads();
                CD_STAMP(7);
                CD_STAMP(8);
            } else {
            // ---- the head of rows 2cw, 2cw + 1: y = Σ_p partials (fixed order) + b3 ----
            {
                constexpr int QN = OP / 4, IT = RPW * QN;                // 10 float4 sums of 32 partials
                if (tid < IT * NWG) {
                    const int p = tid % NWG, it = tid / NWG, r = it / QN, oq = 4 * (it % QN);
                    *reinterpret_cast<f32x4*>(lds + L::scr + 4 * (it * NWG + p)) =
                        ld16_sc1(rY, (p * BB + RPW * cw + r) * OP + oq);
                }
                __syncthreads();
                if (tid < IT) {
                    const int r = tid / QN, oq = 4 * (tid % QN);
                    f32x4 s = *reinterpret_cast<const f32x4*>(lds + L::scr + 4 * (tid * NWG));
                    for (int p = 1; p < NWG; ++p) s += *reinterpret_cast<const f32x4*>(lds + L::scr + 4 * (tid * NWG + p));
#pragma unroll
                    for (int e = 0; e < 4; ++e) lds[L::hrow + r * GP + oq + e] = s[e] + lds[L::b3 + oq + e];
                }
                __syncthreads();
                if (tid < RPW) {
                    const int i = RPW * cw + tid;
                    float* yr = lds + L::hrow + tid * GP;                 // y, then ∂L/∂y in place
                    float* gl = yr + OP;                                   // log σ row terms
                    float part;
                    if (!a.policy) {                                       // loss.cu:5-23
                        const float y = yr[0], t = lds[tc + i];
                        const float d = t - y;
                        part = d * d;
                        yr[0] = 2 * (y - t) / (float)BB;
                    } else {                                               // ppo.cu:82-107, policy.cu:67-111
                        float g;
                        const float* ls = lds + L::ls;
                        const float* ac = lds + acb + i * OP;
                        const float lp = log_prob_row(yr, ls, ac, A);
                        part = surrogate(lds[tc + i], lp, lds[oc + i], a.eps, BB, &g);
                        for (int j = 0; j < A; ++j) {
                            const float e2 = expf(-2 * ls[j]);
                            const float d = ac[j] - yr[j];
                            gl[j] = (-1 + d * d * e2) * g;
                            yr[j] = d * e2 * g;
                        }
                    }
                    for (int j = O; j < OP; ++j) { yr[j] = 0.f; gl[j] = 0.f; }
                    if (!a.policy) for (int j = 0; j < OP; ++j) gl[j] = 0.f;
                    yr[2 * OP] = part;
                    yr[2 * OP + 1] = yr[2 * OP + 2] = yr[2 * OP + 3] = 0.f;
                }
                __syncthreads();
                if (tid < RPW * (GP / 4)) {
                    const int r = tid / (GP / 4), qd = tid % (GP / 4);
                    st16_sc1(rG3, (RPW * cw + r) * GP + 4 * qd,
                             *reinterpret_cast<const f32x4*>(lds + L::hrow + r * GP + 4 * qd));
                }
            }
            CD_STAMP(7);
            cluster_arrive(a.ctr);
            CD_BAR_STAMP(3, 0);
            ok = cluster_wait(a.ctr, a.err, nbar++, NWG, flag, cw, a.timeout);          // D: every row's ∂L/∂y published
            if (!ok) break;
            CD_BAR_STAMP(3, 1);
            CD_STAMP(8);
            // ---- ∂L/∂y of all rows → LDS ----
            for (int e = tid; e < BB * (GP / 4); e += TPB) {
                const int r = e / (GP / 4), qd = e % (GP / 4);
                const f32x4 v = ld16_sc1(rG3, r * GP + 4 * qd);
                if (qd < OP / 4) *reinterpret_cast<f32x4*>(lds + L::g3 + r * GOP + 4 * qd) = v;
                else if (qd < 2 * (OP / 4)) *reinterpret_cast<f32x4*>(lds + L::glr + r * GOP + 4 * (qd - OP / 4)) = v;
                else lds[L::lossr + r] = v[0];
            }
            __syncthreads();
            }
            // replicated sums in a fixed order: gb3[o] = Σ_b g3[b][o]; log σ: Σ_b row terms − c_ent
            // (ppo.cu:436-438); the loss sum once (workgroup 0)
            if (w == NWAVE - 1) colsum64<32>(lds + L::g3, GOP, O, 0.f, lds + L::gb3, tid);
            if (w == NWAVE - 2 && a.policy) colsum64<32>(lds + L::glr, GOP, A, -a.ent_coeff, lds + L::gls, tid);
            if (w == NWAVE - 3 && lane == 0 && cw == 0) {
                float part = 0.f;
                for (int b = 0; b < BB; ++b) part += lds[L::lossr + b];
                if (!a.policy) {
                    atomicAdd(a.stats + 0, part * (1.0f / (float)BB));
                } else {
                    float ent = (float)(A * 0.5 * (1 + log(2 * M_PI)));
                    for (int j = 0; j < A; ++j) ent += lds[L::ls + j];
                    atomicAdd(a.stats + 1, -part / BB - a.ent_coeff * ent);
                }
            }
            // gW3[o][j] = Σ_b g3[b][o]·h3[b][j] (waves 0-1); g3h[b][j] = (Σ_o g3[b][o]·W3[o][j]) ⊙ 1[h3 > 0]
            // (waves 2-5, one batch tile each)
            if (w < 2 && 16 * w < O) {
                const f32x4 acc = mm_tile(lds + L::g3 + 16 * w, 1, GOP, lds + L::h3, HCP, 1, BB, tid);
#pragma unroll
                for (int e = 0; e < 4; ++e) lds[L::gW3 + (16 * w + 4 * q + e) * HCP + c] = acc[e];
            }
            if (w >= 2 && w < 6) {
                const int tb = w - 2;
                const f32x4 acc = mm_tile(lds + L::g3 + 16 * tb * GOP, GOP, 1, lds + L::W3, HCP, 1, O, tid);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int b = 16 * tb + 4 * q + e;
                    lds[L::gh + b * HCP + c] = lds[L::h3 + b * HCP + c] > 0.f ? acc[e] : 0.f;
                }
            }
            __syncthreads();
            // ---- layer 2 backward: P2 = g3h·W2[own, :] → Pa; gb2; then gW2[j][k] = Σ_b g3h[b][j]·h2[b][k]
            // with Adam fused, inside E's wait — the first CLU_GW_PRE tiles' operands (h2, moments) in
            // flight under P2, the rest one tile's loads at a time (all four tiles' at once measured
            // slower: 7.9 vs 6.7 µs) ----
            {
                const long g0 = a.woff[2] + (long)c0 * H;
                auto ldx2 = [&](int b, int k) { return ld4_sc1(rX2, b * H + k); };
                GwTiles<CLU_GW_PRE> pre;
                pre.load(tid, a, g0, H, H, ldx2, 0);
                publish_partial(tid, rPa, cw, lds + L::W2, lds);
                if (w == NWAVE - 1) colsum64<HC>(lds + L::gh, HCP, HC, 0.f, lds + L::gb2, tid);
                CD_STAMP(9);
                cluster_arrive(a.ctr);                                   // (its barrier: W2 reads done)
                CD_BAR_STAMP(4, 0);
                pre.apply(tid, a, lds + L::gh, lds + L::W2, HP, g0, H, H, st, bc2, last, 0);
#pragma unroll 1
                for (int t = CLU_GW_PRE; t < T12; ++t) {
                    GwTiles<1> gt;
                    gt.load(tid, a, g0, H, H, ldx2, t);
                    gt.apply(tid, a, lds + L::gh, lds + L::W2, HP, g0, H, H, st, bc2, last, t);
                }
            }
            CD_STAMP(10);
            ok = cluster_wait(a.ctr, a.err, nbar++, NWG, flag, cw, a.timeout);          // E: P2 published
            if (!ok) break;
            CD_BAR_STAMP(4, 1);
            CD_STAMP(11);
            // ---- layer 1 backward: g2h = Σ P2 ⊙ 1[h2 > 0]; P1 = g2h·W1[own, :] → Pb; gb1; gW1 as gW2 (its
            // first tiles' operands in flight under the reduction and P1) ----
            {
                const long g0 = a.woff[1] + (long)c0 * H;
                auto ldx1 = [&](int b, int k) { return ld4_sc1(rX1, x1o + b * H + k); };
                GwTiles<CLU_GW_PRE> pre;
                pre.load(tid, a, g0, H, H, ldx1, 0);
                reduce_partials(tid, rPa, c0, lds + L::h2, lds);
                __syncthreads();
                publish_partial(tid, rPb, cw, lds + L::W1, lds);
                if (w == NWAVE - 1) colsum64<HC>(lds + L::gh, HCP, HC, 0.f, lds + L::gb1, tid);
                CD_STAMP(12);
                cluster_arrive(a.ctr);
                CD_BAR_STAMP(5, 0);
                pre.apply(tid, a, lds + L::gh, lds + L::W1, HP, g0, H, H, st, bc2, last, 0);
#pragma unroll 1
                for (int t = CLU_GW_PRE; t < T12; ++t) {
                    GwTiles<1> gt;
                    gt.load(tid, a, g0, H, H, ldx1, t);
                    gt.apply(tid, a, lds + L::gh, lds + L::W1, HP, g0, H, H, st, bc2, last, t);
                }
            }
            // Adam of the small parameters whose gradients are complete (all but b0: W3's columns, b1,
            // b2, the replicated b3 and log σ — none is read again this step)
            small_adam(a, lds, tid, c0, nsmall, sm, sv, step, st, bc2, false);
            CD_STAMP(13);
            ok = cluster_wait(a.ctr, a.err, nbar++, NWG, flag, cw, a.timeout);          // F: P1 published
            if (!ok) break;
            CD_BAR_STAMP(5, 1);
            CD_STAMP(14);
            // ---- layer 0 backward: g1h = Σ P1 ⊙ 1[h1 > 0]; gW0[j][s] = Σ_b g1h[b][j]·x[b][s] with Adam
            // fused; gb0 ----
            {
                // the state operands and W0's moments in flight under the ∂L/∂h1 reduction (issuing
                // the reduction's loads first measured 0.25 µs slower here and in layer 1)
                GwTiles<T0> gt;
                const long g0 = a.woff[0] + (long)c0 * S;
                gt.load(tid, a, g0, S, S, [&](int b, int s) { return a.state[(long)rows[b] * S + s]; });
                reduce_partials(tid, rPb, c0, lds + L::h1, lds);
                __syncthreads();
                CD_STAMP(15);
                gt.apply(tid, a, lds + L::gh, lds + L::W0, SPMAX, g0, S, S, st, bc2, last);
            }
            CD_STAMP(16);
            if (w == NWAVE - 1) colsum64<HC>(lds + L::gh, HCP, HC, 0.f, lds + L::gb0, tid);
            __syncthreads();
            // ---- Adam of b0 (the rest of the small parameters stepped inside F's wait) ----
            small_adam(a, lds, tid, c0, nsmall, sm, sv, step, st, bc2, true);
            __syncthreads();
            CD_STAMP(17);
        }
    }
    if (!ok) return;
    // ---- phase end: parameters and moments back; the last step's small gradients ----
    int tid_e = tid, c0_e = c0;
    asm volatile("" : "+v"(tid_e), "+s"(c0_e));
    for (int e = tid_e; e < HC * S; e += TPB) {
        const int j = e / S, k = e % S;
        a.params[a.woff[0] + (long)(c0_e + j) * S + k] = lds[L::W0 + j * SPMAX + k];
    }
    for (int e = tid_e; e < HC * H; e += TPB) {
        const int j = e / H, k = e % H;
        a.params[a.woff[1] + (long)(c0_e + j) * H + k] = lds[L::W1 + j * HP + k];
        a.params[a.woff[2] + (long)(c0_e + j) * H + k] = lds[L::W2 + j * HP + k];
    }
    if (tid_e < nsmall) {
        const Small s = small_elem(a, tid_e, c0_e);
        if (s.kind == 0 || cw == 0) {
            if (s.kind == 1) {
                a.log_std[s.gflat] = lds[s.lds_p]; a.m_ls[s.gflat] = sm; a.v_ls[s.gflat] = sv;
                if (step > 0) a.log_std_grad[s.gflat] = lds[s.lds_g];
            } else {
                a.params[s.gflat] = lds[s.lds_p]; a.m[s.gflat] = sm; a.v[s.gflat] = sv;
                if (step > 0) a.grads[s.gflat] = lds[s.lds_g];
            }
        }
    }
}

struct Ws { float* base; unsigned* ctr; long cap; };
Ws g_ws[2] = {};

}  // namespace

extern "C" {

// Returns 0 when launched (or, with n_epochs = 0, when the shape fits); −1 when the network or the
// minibatch does not fit this path; −2 after an earlier barrier timeout.
int phip_cluster_deep_update(const PhipTinyNet* net, const PhipTinyPhase* ph) {
    if (net->L != 4 || ph->B != BB || ph->n_epochs > 16) return -1;
    const int S = net->sizes[0], O = net->sizes[4];
    for (int l = 1; l <= 3; ++l)
        if (net->sizes[l] != H) return -1;
    if (S < 4 || S > SPMAX || S % 4 || O < 1 || O > OP) return -1;
    if (!net->relu[0] || !net->relu[1] || !net->relu[2] || net->relu[3]) return -1;
    if (ph->policy && (!net->log_std || !net->m_ls)) return -1;
    constexpr size_t bytes = sizeof(float) * (size_t)L::TOTAL;
    static_assert(bytes <= 160 * 1024, "cluster_deep: LDS");
    // one workgroup in every `active_stride` (cluster.hip): 2 spreads each phase over four XCDs, so the
    // value and policy phases (64 workgroups, one per CU) fit wherever they land
    int stride = 2;
    if (const char* st = getenv("PPO_CLUSTER_STRIDE")) {
        const int v = atoi(st);
        if (v == 1 || v == 2 || v == 4 || v == 8) stride = v;
    }
    static bool attr = false;
    if (!attr) {
        PPO_CHECK(hipFuncSetAttribute((const void*)cluster_deep_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)bytes));
        attr = true;
    }
    if (!host_grid_fits((const void*)cluster_deep_kernel, bytes, NWG * stride)) return -1;   // multi-launch
    if (ph->n_epochs <= 0 || ph->num_batches <= 0) return 0;     // fit check only
    unsigned* d_err = phip_cluster_err_dev();
    if (!d_err) return -2;
    DArgs a{};
    a.S = S; a.O = O; a.policy = ph->policy;
    a.params = net->params; a.grads = net->grads; a.m = net->m; a.v = net->v;
    for (int l = 0; l < 4; ++l) { a.woff[l] = net->woff[l]; a.boff[l] = net->boff[l]; }
    a.log_std = net->log_std; a.log_std_grad = net->log_std_grad; a.m_ls = net->m_ls; a.v_ls = net->v_ls;
    a.state = ph->state; a.action = ph->action; a.logprob = ph->logprob; a.adv = ph->adv; a.adv_target = ph->adv_target;
    a.limit = ph->limit; a.num_batches = ph->num_batches; a.n_epochs = ph->n_epochs;
    a.total_steps = ph->n_epochs * ph->num_batches;
    if (ph->max_steps > 0 && ph->max_steps < a.total_steps) a.total_steps = (int)ph->max_steps;
    a.perms = ph->perms;
    for (int e = 0; e < ph->n_epochs && !ph->perms; ++e) {
        Feistel& f = a.fk[e];
        int bits = 2;
        while ((1ULL << bits) < (unsigned long long)ph->limit) bits++;
        f.half = (uint32_t)((bits + 1) / 2);
        f.mask = (1u << f.half) - 1u;
        f.n = (uint32_t)ph->limit;
        for (int r = 0; r < 4; ++r) f.k[r] = ph->feistel_k[4 * e + r];
    }
    a.steps = ph->steps; a.steps_ls = ph->steps_ls;
    a.b1 = ph->b1; a.b2 = ph->b2; a.eps = ph->eps; a.ent_coeff = ph->ent_coeff;
    a.stats = ph->stats;
    Ws& ws = g_ws[phip_side_active() ? 1 : 0];
    const long nX1 = 2L * BB * H, nX2 = (long)BB * H, nY = (long)NWG * BB * OP, nG3 = (long)BB * GP,
               nP = (long)NWG * BB * PH;
    const long need = nX1 + nX2 + nY + nG3 + 2 * nP;
    if (ws.cap < need) {
        phip_free(ws.base);
        phip_free(ws.ctr);
        ws.base = (float*)phip_malloc(sizeof(float) * (size_t)need);
        ws.ctr = (unsigned*)phip_malloc(CLU_CTR_BYTES);      // counter replicas
        ws.cap = need;
    }
    a.X1 = ws.base; a.X2 = a.X1 + nX1; a.Y = a.X2 + nX2; a.G3 = a.Y + nY; a.Pa = a.G3 + nG3; a.Pb = a.Pa + nP;
    a.ctr = ws.ctr; a.err = d_err;
    a.timeout = host_timeout_ticks();
    a.active_stride = stride;
    // stride 8 puts a phase on one XCD (blocks b, b + 8 share one); the policy phase then takes XCD 4
    // so the two concurrent phases never share CUs
    a.active_offset = stride == 8 && ph->policy ? 4 : 0;
    if (const char* r = getenv("PPO_CLUSTER_ROT")) a.rot = ((atoi(r) % NWG) + NWG) % NWG;
    static const char* names[NSTAMP] = {"L0", "bar A", "L1", "bar B", "L2+Y", "bar C", "head", "bar D",
                                        "g3+P2", "gW2 adam", "bar E", "g2+P1", "gW1 adam", "bar F",
                                        "g1 reduce", "gW0 adam", "gb0+b0", "step->next"};
    if (getenv("PPO_CLUSTER_STAMPS")) {
        a.stamps = host_stamps(NSTAMP, "cluster_deep", names, ph->policy, a.total_steps, NWG);
        if (getenv("PPO_CLUSTER_STAMPS")[0] == '2') a.arr = host_barrier_stamps(NWG);
    }
    PPO_CHECK(hipMemsetAsync(ws.ctr, 0, CLU_CTR_BYTES, ppo::stream()));
    ppo::ProfScope ps(PPO_K_OTHER, 0.0);
    hipLaunchKernelGGL(cluster_deep_kernel, dim3(NWG * a.active_stride), dim3(TPB), bytes, ppo::stream(), a);
    PPO_LAUNCH_CHECK();
    return 0;
}

}  // extern "C"
