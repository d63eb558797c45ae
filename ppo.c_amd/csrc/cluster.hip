// cluster.hip — a whole phase of minibatch steps at the reference's B = 64 for mid-size networks
// (S → H → H → O with H = 256, config C3), in ONE launch of NWG = H/32 cooperating workgroups.
//
// At B = 64 the multi-launch loop is a chain of ≈ 9 dependent small kernels per step (≈ 36 µs per
// step at C3, profiles/r03_graph_replay.txt) and one workgroup (tiny.hip) cannot hold a 256-wide
// network's Adam state or run its ≈ 27 MFLOP per step fast enough.  Here workgroup c owns the 32
// hidden units [32c, 32c+32) of both hidden layers: rows of W0 and W1, their biases, and the
// matching input columns of the output layer W2; its parameters live in LDS and their Adam moments in
// VGPRs for the whole phase.  Per step (reference ppo.cu:395-443, arithmetic as in tiny.hip):
//   gather (every workgroup, the same 64 rows)           → x [64 × S]
//   h1[:, own] = relu(x·W0[own]ᵀ + b0)                   → published (X1)       — barrier A
//   h1 = every workgroup's columns;  h2[:, own] = relu(h1·W1[own]ᵀ + b1)
//   y partial = h2[:, own]·W2[:, own]ᵀ                   → published (Y)        — barrier B
//   y = Σ partials + b2 (fixed order);  head (MSE or clipped surrogate) — every workgroup, identically
//   gW2[:, own], gb2, g2 = (g3·W2[:, own]) ⊙ 1[h2 > 0];  g1 partial = g2·W1[own, :] → published (G1)
//   gW1[own] = g2ᵀ·h1 with Adam fused into its epilogue                        — barrier C
//   g1[:, own] = Σ partials ⊙ 1[h1 > 0];  gW0[own] = g1ᵀ·x;  Adam of the rest
// Three barriers per step.  Hand-offs (MI355X_MICROARCH.md § inter-workgroup visibility, the first
// row of the sc1 table): every published byte is stored write-through (sc1, 16-B buffer stores),
// every storing wave drains (s_waitcnt vmcnt(0)) before the workgroup barrier, ONE lane per workgroup
// adds to one monotonic counter (agent scope), ONE lane polls it with sc1 loads + s_sleep, the other
// waves wait at the workgroup barrier, and every load of published bytes is an sc1 load.  Spins are
// bounded: a timeout sets the host-visible error word and every workgroup leaves.  b2 and log σ are
// replicated: every workgroup computes their gradients from the same values in the same order and
// applies the same Adam step (bit-identical copies).  GEMMs: v_mfma_f32_16x16x4_f32 (exact fp32).
#include "cluster_common.h"

#include <vector>

#include <cmath>
#include <cstdlib>

namespace {
using namespace clu;

constexpr int OMAX = 16;          // output width
constexpr int OPP = 20;           // pitch of [64][OMAX] arrays

struct ClArgs {
    int S, O, policy, SP;                     // SP: pitch of x and W0 rows in LDS (4·odd ≥ S)
    float *params, *grads, *m, *v;            // the network's flat buffers and Adam moments
    long woff[3], boff[3];
    float *log_std, *log_std_grad, *m_ls, *v_ls;
    const float *state, *action, *logprob, *adv, *adv_target;
    int limit, num_batches, n_epochs, total_steps;
    const int* perms;
    Feistel fk[16];
    const float *steps, *steps_ls;            // per step {lr/bc1, bc2}
    float b1, b2, eps, ent_coeff;
    float* stats;
    float *X1, *Y, *G1;                       // published: h1 [64][H], y partials [NWG][64][OMAX], g1 partials [NWG][NWG][64][HC]
    unsigned* ctr;                            // barrier arrivals (zeroed before the launch)
    unsigned* err;                            // host-visible error word (0 = fine)
    unsigned long long timeout;               // barrier wait bound (realtime ticks)
    int active_stride, active_offset;         // workgroup b works iff b % stride == offset (same-XCD bias)
    unsigned long long* stamps;               // diagnostics (PPO_CLUSTER_STAMPS): wall clock per phase,
                                              // workgroup 0, steps 0..63, 12 slots
};

// LDS layout (floats) for hidden width H, HC hidden units per workgroup
template <int H, int HC>
struct Lay {
    static constexpr int HP = H + 4;                  // pitch of [64][H] and [HC][H] (4·odd)
    static constexpr int HCP = HC + 4;                // pitch of [64][HC] arrays (4·odd: conflict-free strided reads)
    static constexpr int NT1 = 4 * (HC / 16);         // layer-1 output tiles; split over K when < NWAVE
    static constexpr int KS1 = NWAVE / NT1;
    static constexpr int SPMAX = 20;                  // S ≤ 20 (SP = 4·odd ≤ 20)
    // the minibatch's rows, double-buffered (step s uses buffer s & 1; step s + 1's gather runs inside
    // step s's barrier waits)
    static constexpr int x = 0;                       // [2][64][SP]
    static constexpr int rows = x + 2 * BB * SPMAX;   // int [64]
    static constexpr int tgt = rows + BB;             // [2][64] value target / policy advantage
    static constexpr int olp = tgt + 2 * BB;          // [2][64] old log-prob
    static constexpr int act = olp + 2 * BB;          // [2][64][OMAX] actions
    static constexpr int W0 = act + 2 * BB * OMAX;    // [HC][SP]
    static constexpr int b0 = W0 + HC * SPMAX;        // [HC]
    static constexpr int W1 = b0 + HC;                // [HC][HP]
    static constexpr int b1 = W1 + HC * HP;           // [HC]
    static constexpr int W2 = b1 + HC;                // [OMAX][HCP] own input columns of the output layer
    static constexpr int b2 = W2 + OMAX * HCP;        // [OMAX] (replicated)
    static constexpr int ls = b2 + OMAX;              // [OMAX] log σ (replicated)
    static constexpr int h1 = ls + OMAX;              // [64][HP]
    static constexpr int h2 = h1 + BB * HP;           // [64][HCP] own columns
    static constexpr int yo = h2 + BB * HCP;          // [64][OPP] y / μ, then (in place) ∂L/∂y
    static constexpr int g2 = yo + BB * OPP;          // [64][HCP]
    static constexpr int g1 = g2 + BB * HCP;          // [64][HCP]
    static constexpr int gW0 = g1 + BB * HCP;         // [HC][SP]
    static constexpr int gb0 = gW0 + HC * SPMAX;      // [HC]
    static constexpr int gb1 = gb0 + HC;              // [HC]
    static constexpr int gW2 = gb1 + HC;              // [OMAX][HCP]
    static constexpr int gb2 = gW2 + OMAX * HCP;      // [OMAX]
    static constexpr int gls = gb2 + OMAX;            // [OMAX]
    static constexpr int glr = gls + OMAX;            // [64][OMAX] per-row log σ terms (ordered sum)
    static constexpr int red = glr + BB * OMAX;       // [NWAVE] loss partials
    static constexpr int flag = red + NWAVE;          // int: barrier result
    static constexpr int l1s = flag + 4;              // [4·256] upper halves: layer-1 K partials (KS1 = 2), Y and
                                                      // G1 partial sums
    static constexpr int TOTAL = l1s + 4 * 256;
};

// the small parameters of a workgroup (everything but its W1 rows), enumerated e = 0 … nsmall−1:
// W0 rows [HC][S], b0 [HC], b1 [HC], W2 columns [O][HC], b2 [O] (replicated), log σ [O] (policy,
// replicated; its Adam uses the entropy step sizes)
struct Small { int lds_p, lds_g; long gflat; int kind; };   // kind 0 network, 1 log σ, 2 replicated net

template <int H, int HC>
__device__ __forceinline__ Small small_elem(const ClArgs& a, int e, int c0) {
    using L = Lay<H, HC>;
    constexpr int HCP = L::HCP;
    const int S = a.S, O = a.O;
    if (e < HC * S) { const int j = e / S, s = e % S;
        return {L::W0 + j * a.SP + s, L::gW0 + j * a.SP + s, a.woff[0] + (long)(c0 + j) * S + s, 0}; }
    e -= HC * S;
    if (e < HC) return {L::b0 + e, L::gb0 + e, a.boff[0] + c0 + e, 0};
    e -= HC;
    if (e < HC) return {L::b1 + e, L::gb1 + e, a.boff[1] + c0 + e, 0};
    e -= HC;
    if (e < O * HC) { const int o = e / HC, j = e % HC;
        return {L::W2 + o * HCP + j, L::gW2 + o * HCP + j, a.woff[2] + (long)o * H + c0 + j, 0}; }
    e -= O * HC;
    if (e < O) return {L::b2 + e, L::gb2 + e, a.boff[2] + e, 2};
    e -= O;
    return {L::ls + e, L::gls + e, e, 1};
}

// row i of step (ep, kb)'s minibatch (trajectory_buffer.cu:168-200): epoch ep's permutation of the
// `limit` stored rows at list position kb·64 + i (mod limit)
__device__ __forceinline__ int gather_src(const ClArgs& a, int ep, int kb, int i) {
    const int list = (int)(((long)kb * BB + i) % a.limit);
    return a.perms ? a.perms[(long)ep * a.limit + list] : (int)feistel_index((uint32_t)list, a.fk[ep & 15]);
}
// gather, part 1 (wave 1 — wave 0's first lane polls the barriers this runs beside): the row indices
// → rows[], the per-row scalars → buffer `buf`
template <class L>
__device__ __forceinline__ void gather_rows(const ClArgs& a, float* lds, int ep, int kb, int buf) {
    const int i = (int)threadIdx.x - 64;
    if (i >= 0 && i < BB) {
        const int src = gather_src(a, ep, kb, i);
        reinterpret_cast<int*>(lds + L::rows)[i] = src;
        if (a.policy) {
            const float ad = a.adv[src], lp = a.logprob[src];
            lds[L::tgt + buf * BB + i] = ad;
            lds[L::olp + buf * BB + i] = lp;
        } else {
            lds[L::tgt + buf * BB + i] = a.adv_target[src];
        }
    }
}
// gather, part 2 (waves 1-7, behind a workgroup barrier after part 1): the rows' states (and
// actions) → buffer `buf`, every load in flight before the LDS writes
template <class L>
__device__ __forceinline__ void gather_cols(const ClArgs& a, float* lds, int buf) {
    if (threadIdx.x < 64) return;
    constexpr int NT = TPB - 64;
    constexpr int XU = (BB * L::SPMAX + NT - 1) / NT, AU = (BB * OMAX + NT - 1) / NT;
    const int* rows = reinterpret_cast<const int*>(lds + L::rows);
    const int tid = (int)threadIdx.x - 64, S = a.S, A = a.O;
    float xv[XU], av[AU];
#pragma unroll
    for (int u = 0; u < XU; ++u) {
        const int e = tid + u * NT;
        xv[u] = e < BB * S ? a.state[(long)rows[e / S] * S + e % S] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < AU; ++u) {
        const int e = tid + u * NT;
        av[u] = a.policy && e < BB * A ? a.action[(long)rows[e / A] * A + e % A] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < XU; ++u) {
        const int e = tid + u * NT;
        if (e < BB * S) lds[L::x + buf * BB * L::SPMAX + (e / S) * a.SP + e % S] = xv[u];
    }
#pragma unroll
    for (int u = 0; u < AU; ++u) {
        const int e = tid + u * NT;
        if (a.policy && e < BB * A) lds[L::act + buf * BB * OMAX + (e / A) * OMAX + e % A] = av[u];
    }
}

// small parameters per workgroup ≤ HC·(S + 2 + O) + 2·O with S ≤ 20, O ≤ 16: slots per thread
template <int HC>
constexpr int small_slots() { return (HC * (20 + 2 + 16) + 32 + TPB - 1) / TPB; }

#define CL_STAMP(slot)                                                                          \
    do {                                                                                        \
        if (a.stamps && cw == 0 && tid == 0 && step < 64) {                                     \
            a.stamps[step * 12 + (slot)] = wall_clock64();                                       \
            a.stamps[CLU_STAMP_CLK + step * 12 + (slot)] = __builtin_amdgcn_s_memtime();         \
        }                                                                                        \
    } while (0)

template <int H, int HC>
__global__ __launch_bounds__(TPB) void cluster_phase_kernel(ClArgs a) {
    constexpr int NWG = H / HC;
    using L = Lay<H, HC>;
    constexpr int HP = L::HP, HCP = L::HCP;
    constexpr int SMALL_SLOTS = small_slots<HC>();
    if ((int)blockIdx.x % a.active_stride != a.active_offset) return;
    const int cw = (int)blockIdx.x / a.active_stride;
    // diagnostics (PPO_CLUSTER_STAMPS): where this workgroup runs — XCC id, HW_ID (CU / SH / SE fields)
    if (a.stamps && threadIdx.x == 0)
        a.stamps[64 * 32 + cw] = ((unsigned long long)__builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11)) << 32) |
                                 __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));            // this workgroup's unit block
    const int c0 = cw * HC;
    extern __shared__ float lds[];
    int* flag = reinterpret_cast<int*>(lds + L::flag);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int c = lane & 15, q = lane >> 4;
    const int S = a.S, O = a.O, SP = a.SP, A = a.O;
    const int nsmall = HC * S + 2 * HC + O * HC + O + (a.policy ? A : 0);
    const auto rX1 = rsrc(a.X1, (long)BB * H);
    const auto rY = rsrc(a.Y, (long)NWG * BB * OMAX);
    const auto rG1 = rsrc(a.G1, (long)NWG * BB * H);

    // ---- phase start: own parameters → LDS, Adam moments → VGPRs ----
    for (int e = tid; e < HC * H; e += TPB) {
        const int j = e / H, k = e % H;
        lds[L::W1 + j * HP + k] = a.params[a.woff[1] + (long)(c0 + j) * H + k];
    }
    for (int e = tid; e < OMAX * HCP; e += TPB) lds[L::W2 + e] = 0.f;       // rows o ≥ O stay zero
    for (int e = tid; e < OMAX; e += TPB) { lds[L::b2 + e] = 0.f; lds[L::ls + e] = 0.f; }
    __syncthreads();
    float sm[SMALL_SLOTS], sv[SMALL_SLOTS];
#pragma unroll
    for (int u = 0; u < SMALL_SLOTS; ++u) {
        const int e = tid + u * TPB;
        sm[u] = sv[u] = 0.f;
        if (e < nsmall) {
            const Small s = small_elem<H, HC>(a, e, c0);
            if (s.kind == 1) { lds[s.lds_p] = a.log_std[s.gflat]; sm[u] = a.m_ls[s.gflat]; sv[u] = a.v_ls[s.gflat]; }
            else { lds[s.lds_p] = a.params[s.gflat]; sm[u] = a.m[s.gflat]; sv[u] = a.v[s.gflat]; }
        }
    }
    // W1 rows' moments: the elements this lane's gW1 tiles hold (tiles t = w + 8u: rows 16(t/16) + 4q + e,
    // column 16(t%16) + c)
    constexpr int T1 = (HC / 16) * (H / 16) / NWAVE;              // gW1 tiles per wave
    float m1[T1][4], v1[T1][4];
#pragma unroll
    for (int u = 0; u < T1; ++u) {
        const int t = w + NWAVE * u, tj = t / (H / 16), tk = t % (H / 16);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const long g = a.woff[1] + (long)(c0 + 16 * tj + 4 * q + e) * H + 16 * tk + c;
            m1[u][e] = a.m[g];
            v1[u][e] = a.v[g];
        }
    }
    // the first step's minibatch
    gather_rows<L>(a, lds, 0, 0, 0);
    __syncthreads();
    gather_cols<L>(a, lds, 0);
    __syncthreads();

    unsigned nbar = 0;
    int step = 0;
    bool ok = true;
    for (int ep = 0; ep < a.n_epochs && ok; ++ep) {
        for (int kb = 0; kb < a.num_batches && step < a.total_steps && ok; ++kb, ++step) {
            CL_STAMP(0);
            const int cur = step & 1;
            const int xc = L::x + cur * BB * L::SPMAX, tc = L::tgt + cur * BB, oc = L::olp + cur * BB,
                      acb = L::act + cur * BB * OMAX;
            const bool has_next = step + 1 < a.total_steps;
            const int kb_n = kb + 1 < a.num_batches ? kb + 1 : 0, ep_n = kb + 1 < a.num_batches ? ep : ep + 1;
            CL_STAMP(1);
            // ---- layer 0, own units: h1ᵀ[j][b] = Σ_s W0[j][s]·x[b][s] + b0[j]  (HC/16 × 4 tiles, one per wave)
            if (w < 4 * (HC / 16)) {
                const int tj = w / 4, tb = w % 4;
                const f32x4 acc = mm_tile(lds + L::W0 + 16 * tj * SP, SP, 1, lds + xc + 16 * tb * SP, 1, SP, S);
                const int b = 16 * tb + c, j = 16 * tj + 4 * q;
                f32x4 hv;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float v = acc[e] + lds[L::b0 + j + e];
                    hv[e] = v > 0.f ? v : 0.f;                           // neural_network.cu:74-105 (ReLU)
                }
                *reinterpret_cast<f32x4*>(lds + L::h1 + b * HP + c0 + j) = hv;
                st16_sc1(rX1, b * H + c0 + j, hv);                       // publish
            }
            CL_STAMP(2);
            cluster_arrive(a.ctr);
            if (has_next) gather_rows<L>(a, lds, ep_n, kb_n, cur ^ 1);   // the next minibatch, part 1
            ok = cluster_wait(a.ctr, a.err, nbar++, NWG, flag, cw, a.timeout);                     // A: every h1 column published
            if (!ok) break;
            CL_STAMP(3);
            // every other workgroup's h1 columns (sc1 loads): lane → column quad 4·lane, rows w + 8u,
            // all eight loads in flight before the LDS writes
            {
                static_assert(H == 4 * 64 && BB == 8 * NWAVE, "h1 gather mapping");
                const int k = 4 * lane;
                if (k < c0 || k >= c0 + HC) {
                    f32x4 hv[BB / NWAVE];
#pragma unroll
                    for (int u = 0; u < BB / NWAVE; ++u) hv[u] = ld16_sc1(rX1, (w + NWAVE * u) * H + k);
#pragma unroll
                    for (int u = 0; u < BB / NWAVE; ++u)
                        *reinterpret_cast<f32x4*>(lds + L::h1 + (w + NWAVE * u) * HP + k) = hv[u];
                }
            }
            __syncthreads();

            CL_STAMP(4);
            // ---- layer 1, own units: h2[b][j] = relu(Σ_k h1[b][k]·W1[j][k] + b1[j])  (4 × HC/16 tiles; with
            // fewer tiles than waves, K is split in two and the upper half's partial added through LDS)
            {
                constexpr int NT = L::NT1, KS = L::KS1, KL = H / KS;
                const int t = w % NT, ks = w / NT;
                const int tb = t / (HC / 16), tj = t % (HC / 16);
                f32x4 acc = mm_tile(lds + L::h1 + 16 * tb * HP + ks * KL, HP, 1, lds + L::W1 + 16 * tj * HP + ks * KL, 1,
                                    HP, KL);
                if constexpr (KS > 1) {
                    static_assert(KS == 2, "layer-1 K split");
                    if (ks == 1) *reinterpret_cast<f32x4*>(lds + L::l1s + (t * 64 + lane) * 4) = acc;
                    __syncthreads();
                    if (ks == 0) acc += *reinterpret_cast<const f32x4*>(lds + L::l1s + (t * 64 + lane) * 4);
                }
                if (ks == 0) {
                    const int j = 16 * tj + c;
                    const float bj = lds[L::b1 + j];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float v = acc[e] + bj;
                        lds[L::h2 + (16 * tb + 4 * q + e) * HCP + j] = v > 0.f ? v : 0.f;
                    }
                }
            }
            __syncthreads();
            // ---- output layer, own input columns: yᵀ[o][b] = Σ_j W2[o][j]·h2[b][j]  (4 tiles, waves 0-3)
            if (w < 4) {
                const f32x4 acc = mm_tile(lds + L::W2, HCP, 1, lds + L::h2 + 16 * w * HCP, 1, HCP, HC);
                st16_sc1(rY, (cw * BB + 16 * w + c) * OMAX + 4 * q, acc);     // publish Y[cw][b][4q..4q+3]
            }
            CL_STAMP(5);
            cluster_arrive(a.ctr);
            if (has_next) gather_cols<L>(a, lds, cur ^ 1);               // the next minibatch, part 2
            ok = cluster_wait(a.ctr, a.err, nbar++, NWG, flag, cw, a.timeout);                     // B: every y partial published
            if (!ok) break;
            CL_STAMP(6);
            // ---- y = Σ_c partials (fixed order) + b2; the head, identically in every workgroup ----
            // (256 float4 sums: threads 256-511 add partials NWG/2 … NWG−1 and hand them over through LDS)
            {
                static_assert(BB * (OMAX / 4) * 2 == TPB && NWG % 2 == 0, "y sum mapping");
                const int it = tid % (BB * (OMAX / 4)), half = tid / (BB * (OMAX / 4));
                const int b = it / (OMAX / 4), oq = 4 * (it % (OMAX / 4));
                f32x4 v[NWG / 2];
#pragma unroll
                for (int cc = 0; cc < NWG / 2; ++cc) v[cc] = ld16_sc1(rY, ((half * (NWG / 2) + cc) * BB + b) * OMAX + oq);
                f32x4 s = v[0];
#pragma unroll
                for (int cc = 1; cc < NWG / 2; ++cc) s += v[cc];
                if (half) *reinterpret_cast<f32x4*>(lds + L::l1s + 4 * it) = s;
                __syncthreads();
                if (!half) {
                    s += *reinterpret_cast<const f32x4*>(lds + L::l1s + 4 * it);
#pragma unroll
                    for (int e = 0; e < 4; ++e) lds[L::yo + b * OPP + oq + e] = s[e] + lds[L::b2 + oq + e];
                }
            }
            __syncthreads();
            float part = 0.f;
            if (tid < BB) {
                const int i = tid;
                float* yo = lds + L::yo + i * OPP;
                if (!a.policy) {                                         // loss.cu:5-23
                    const float y = yo[0], t = lds[tc + i];
                    const float d = t - y;
                    part = d * d;
                    yo[0] = 2 * (y - t) / (float)BB;
                } else {                                                 // ppo.cu:82-107, policy.cu:67-111
                    float g;
                    const float* ls = lds + L::ls;
                    const float* ac = lds + acb + i * OMAX;
                    const float lp = log_prob_row(yo, ls, ac, A);
                    part = surrogate(lds[tc + i], lp, lds[oc + i], a.eps, BB, &g);
                    for (int j = 0; j < A; ++j) {
                        const float e2 = expf(-2 * ls[j]);
                        const float d = ac[j] - yo[j];
                        lds[L::glr + i * OMAX + j] = (-1 + d * d * e2) * g;
                        yo[j] = d * e2 * g;
                    }
                }
                for (int j = O; j < OMAX; ++j) yo[j] = 0.f;              // padded outputs carry no gradient
                for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
            }
            __syncthreads();
            if (tid == 0 && cw == 0) {                                   // the loss sums (once)
                if (!a.policy) {
                    atomicAdd(a.stats + 0, part * (1.0f / (float)BB));
                } else {
                    float ent = (float)(A * 0.5 * (1 + log(2 * M_PI)));
                    for (int j = 0; j < A; ++j) ent += lds[L::ls + j];
                    atomicAdd(a.stats + 1, -part / BB - a.ent_coeff * ent);
                }
            }
            // replicated gradients in a fixed order: gb2[o] = Σ_b g3[b][o]; log σ: Σ_b row terms − c_ent
            // (ppo.cu:436-438); waves 7 and 6 (the tiles below keep waves 0-1 longest)
            if (w == NWAVE - 1) colsum64<OMAX>(lds + L::yo, OPP, O, 0.f, lds + L::gb2);
            if (w == NWAVE - 2 && a.policy) colsum64<OMAX>(lds + L::glr, OMAX, A, -a.ent_coeff, lds + L::gls);
            // ---- output layer backward, own columns: gW2[o][j] = Σ_b g3[b][o]·h2[b][j]  (HC/16 tiles)
            if (w < HC / 16) {
                const f32x4 acc = mm_tile(lds + L::yo, 1, OPP, lds + L::h2 + 16 * w, HCP, 1, BB);
#pragma unroll
                for (int e = 0; e < 4; ++e) lds[L::gW2 + (4 * q + e) * HCP + 16 * w + c] = acc[e];
            }
            // g2[b][j] = (Σ_o g3[b][o]·W2[o][j]) ⊙ 1[h2[b][j] > 0]  (4 × HC/16 tiles)
            if (w < 4 * (HC / 16)) {
                const int tb = w / (HC / 16), tj = w % (HC / 16);
                const f32x4 acc = mm_tile(lds + L::yo + 16 * tb * OPP, OPP, 1, lds + L::W2 + 16 * tj, HCP, 1, O);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int b = 16 * tb + 4 * q + e, j = 16 * tj + c;
                    lds[L::g2 + b * HCP + j] = lds[L::h2 + b * HCP + j] > 0.f ? acc[e] : 0.f;
                }
            }
            __syncthreads();
            CL_STAMP(7);
            // ---- g1 partial: P[b][k] = Σ_j g2[b][j]·W1[j][k], computed as Pᵀ tiles (4 consecutive k per
            // lane → 16-B publishes): Pᵀ[k][b] = Σ_j W1[j][k]·g2[b][j]  (16 × 4 tiles, 8 per wave)
            for (int t = w; t < (H / 16) * (BB / 16); t += NWAVE) {
                const int tk = t / (BB / 16), tb = t % (BB / 16);
                const f32x4 acc = mm_tile(lds + L::W1 + 16 * tk, 1, HP, lds + L::g2 + 16 * tb * HCP, 1, HCP, HC);
                {
                    // slice-major partials [slice][cw][b][HC] (each workgroup's later read of its own slice
                    // is one contiguous block; the row-major [cw][b][H] form read HC columns of every 1-KB row)
                    const int k = 16 * tk + 4 * q;
#ifdef CLU_G1ROWS
                    st16_sc1(rG1, (cw * BB + 16 * tb + c) * H + k, acc);
#else
                    st16_sc1(rG1, (((k / HC) * NWG + cw) * BB + 16 * tb + c) * HC + k % HC, acc);
#endif
                }
            }
            // bias gradient of layer 1 (fixed order)
            if (w == NWAVE - 1) colsum64<HC>(lds + L::g2, HCP, HC, 0.f, lds + L::gb1);
            cluster_arrive(a.ctr);                                           // (its barrier: every wave done reading W1)
            // ---- gW1[j][k] = Σ_b g2[b][j]·h1[b][k] with Adam fused (the lane holds these elements'
            // moments), overlapping the other workgroups' arrivals ----
            {
                const float st = a.steps[2 * step], bc2 = a.steps[2 * step + 1];
#pragma unroll
                for (int u = 0; u < T1; ++u) {
                    const int t = w + NWAVE * u, tj = t / (H / 16), tk = t % (H / 16);
                    const f32x4 acc = mm_tile(lds + L::g2 + 16 * tj, 1, HCP, lds + L::h1 + 16 * tk, HP, 1, BB);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        float* p = lds + L::W1 + (16 * tj + 4 * q + e) * HP + 16 * tk + c;
                        float pv = *p;
                        adam_elem(pv, acc[e], m1[u][e], v1[u][e], st, a.b1, a.b2, bc2);
                        *p = pv;
                    }
                }
            }
            CL_STAMP(8);
            ok = cluster_wait(a.ctr, a.err, nbar++, NWG, flag, cw, a.timeout);                     // C: every g1 partial published
            if (!ok) break;
            CL_STAMP(9);
            // ---- g1[b][j] = Σ_c partials (fixed order) ⊙ 1[h1 > 0], own units ----
            // (64 × HC/4 float4 sums; threads 256-511 add partials NWG/2 … NWG−1 and hand them over)
            {
                static_assert(BB * (HC / 4) * 2 == TPB && NWG % 2 == 0, "g1 sum mapping");
                const int it = tid % (BB * (HC / 4)), half = tid / (BB * (HC / 4));
                const int b = it / (HC / 4), jq = 4 * (it % (HC / 4));
                f32x4 v[NWG / 2];
#pragma unroll
                for (int cc = 0; cc < NWG / 2; ++cc)
#ifdef CLU_G1ROWS
                    v[cc] = ld16_sc1(rG1, ((half * (NWG / 2) + cc) * BB + b) * H + c0 + jq);
#else
                    v[cc] = ld16_sc1(rG1, (((c0 / HC) * NWG + half * (NWG / 2) + cc) * BB + b) * HC + jq);
#endif
                f32x4 s = v[0];
#pragma unroll
                for (int cc = 1; cc < NWG / 2; ++cc) s += v[cc];
                if (half) *reinterpret_cast<f32x4*>(lds + L::l1s + 4 * it) = s;
                __syncthreads();
                if (!half) {
                    s += *reinterpret_cast<const f32x4*>(lds + L::l1s + 4 * it);
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        lds[L::g1 + b * HCP + jq + e] = lds[L::h1 + b * HP + c0 + jq + e] > 0.f ? s[e] : 0.f;
                }
            }
            __syncthreads();
            // ---- layer 0 backward, own rows: gW0[j][s] = Σ_b g1[b][j]·x[b][s] (HC/16 × ⌈S/16⌉ tiles), gb0 ----
            {
                const int ts = (S + 15) / 16;
                for (int t = w; t < (HC / 16) * ts; t += NWAVE) {
                    const int tj = t / ts, tsb = t % ts;
                    const f32x4 acc = mm_tile(lds + L::g1 + 16 * tj, 1, HCP, lds + xc + 16 * tsb, SP, 1, BB);
                    const int s = 16 * tsb + c;
                    if (s < S) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) lds[L::gW0 + (16 * tj + 4 * q + e) * SP + s] = acc[e];
                    }
                }
                if (w == NWAVE - 1) colsum64<HC>(lds + L::g1, HCP, HC, 0.f, lds + L::gb0);
            }
            __syncthreads();
            CL_STAMP(10);
            // ---- Adam of the small parameters: log σ with the entropy step sizes (ppo.cu:440-442), the
            // network's with its own; the last step writes the gradients out ----
            {
                const float st = a.steps[2 * step], bc2 = a.steps[2 * step + 1];
                const float st_ls = a.policy ? a.steps_ls[2 * step] : 0.f;
                const float bc2_ls = a.policy ? a.steps_ls[2 * step + 1] : 1.f;
#pragma unroll
                for (int u = 0; u < SMALL_SLOTS; ++u) {
                    const int e = tid + u * TPB;
                    if (e < nsmall) {
                        const Small s = small_elem<H, HC>(a, e, c0);
                        float pv = lds[s.lds_p];
                        const float g = lds[s.lds_g];
                        if (s.kind == 1) adam_elem(pv, g, sm[u], sv[u], st_ls, a.b1, a.b2, bc2_ls);
                        else adam_elem(pv, g, sm[u], sv[u], st, a.b1, a.b2, bc2);
                        lds[s.lds_p] = pv;
                    }
                }
            }
            __syncthreads();
            CL_STAMP(11);
        }
    }
    if (!ok) return;
    // ---- phase end.  Addresses are recomputed from opaque copies: the compiler would otherwise keep
    // every 64-bit address of the phase-start loads live across the whole step loop (spills) ----
    int tid_e = tid, c0_e = c0;
    asm volatile("" : "+v"(tid_e), "+s"(c0_e));
    // the last step's gradients (callers may read them, as after the multi-launch loop): the small
    // ones are still in LDS; gW1 is recomputed from the last step's g2 and h1, which are too
    if (step > 0) {
        for (int e = tid_e; e < nsmall; e += TPB) {
            const Small s = small_elem<H, HC>(a, e, c0_e);
            if (s.kind != 0 && cw != 0) continue;
            if (s.kind == 1) a.log_std_grad[s.gflat] = lds[s.lds_g];
            else a.grads[s.gflat] = lds[s.lds_g];
        }
        for (int t = (tid_e >> 6); t < (HC / 16) * (H / 16); t += NWAVE) {
            const int tj = t / (H / 16), tk = t % (H / 16);
            const int ln = tid_e & 63, cc = ln & 15, qq = ln >> 4;
            const f32x4 acc = mm_tile(lds + L::g2 + 16 * tj, 1, HCP, lds + L::h1 + 16 * tk, HP, 1, BB);
#pragma unroll
            for (int e = 0; e < 4; ++e)
                a.grads[a.woff[1] + (long)(c0_e + 16 * tj + 4 * qq + e) * H + 16 * tk + cc] = acc[e];
        }
    }
    for (int e = tid_e; e < HC * H; e += TPB) {
        const int j = e / H, k = e % H;
        a.params[a.woff[1] + (long)(c0_e + j) * H + k] = lds[L::W1 + j * HP + k];
    }
    {
        const int we = tid_e >> 6, ln = tid_e & 63, cc = ln & 15, qq = ln >> 4;
#pragma unroll
        for (int u = 0; u < T1; ++u) {
            const int t = we + NWAVE * u, tj = t / (H / 16), tk = t % (H / 16);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const long g = a.woff[1] + (long)(c0_e + 16 * tj + 4 * qq + e) * H + 16 * tk + cc;
                a.m[g] = m1[u][e];
                a.v[g] = v1[u][e];
            }
        }
    }
#pragma unroll
    for (int u = 0; u < SMALL_SLOTS; ++u) {
        const int e = tid_e + u * TPB;
        if (e < nsmall) {
            const Small s = small_elem<H, HC>(a, e, c0_e);
            if (s.kind != 0 && cw != 0) continue;
            if (s.kind == 1) { a.log_std[s.gflat] = lds[s.lds_p]; a.m_ls[s.gflat] = sm[u]; a.v_ls[s.gflat] = sv[u]; }
            else { a.params[s.gflat] = lds[s.lds_p]; a.m[s.gflat] = sm[u]; a.v[s.gflat] = sv[u]; }
        }
    }
}

// per-stream workspace (the value and policy phases run concurrently on two streams)
struct Ws { float *X1, *Y, *G1; unsigned* ctr; long cap; };
Ws g_ws[2] = {};
unsigned* g_err = nullptr;            // host-mapped error word

// PPO_CLUSTER_STAMPS: one stamp buffer per stream (the phases run concurrently) and the report that
// phip_cluster_report prints once the phases have joined
struct StampSlot {
    unsigned long long* arr = nullptr;                // per-workgroup barrier stamps [64][6][2][arr_nwg] (or null)
    int arr_nwg = 0, arr_on = 0;
    unsigned long long* buf = nullptr;                // [64 steps][32 stamps] | [64 workgroups] placement
    int nstamp = 0, policy = 0, total_steps = 0, pending = 0, nwg = 0;
    const char* kind = nullptr;
    const char* const* names = nullptr;
};
StampSlot g_stamps[2];

}  // namespace

namespace clu {

unsigned long long host_timeout_ticks() {
    if (const char* e = getenv("PPO_CLUSTER_TEST_TIMEOUT"))
        if (*e && *e != '0') return 0ULL;
    int dev = 0, khz = 0;
    PPO_CHECK(hipGetDevice(&dev));
    PPO_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
    return (unsigned long long)(khz > 0 ? khz : 100000) * 2000ULL;          // 2 s
}

bool host_grid_fits(const void* kfn, size_t lds, int grid) {
    int dev = 0, cus = 0, per_cu = 0;
    PPO_CHECK(hipGetDevice(&dev));
    PPO_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, TPB, lds) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return (long)per_cu * cus >= 2L * grid;
}

unsigned long long* host_stamps(int nstamp, const char* kind, const char* const* names, int policy, int total_steps,
                                int nwg) {
    StampSlot& s = g_stamps[phip_side_active() ? 1 : 0];
    if (!s.buf) s.buf = (unsigned long long*)phip_malloc(sizeof(unsigned long long) * (CLU_STAMP_CLK + 64 * 32));
    s.nstamp = nstamp; s.kind = kind; s.names = names; s.policy = policy; s.total_steps = total_steps; s.nwg = nwg;
    s.pending = total_steps >= 64;
    s.arr_on = 0;
    return s.buf;
}

unsigned long long* host_barrier_stamps(int nwg) {
    StampSlot& s = g_stamps[phip_side_active() ? 1 : 0];
    if (!s.arr || s.arr_nwg < nwg) {
        phip_free(s.arr);
        s.arr = (unsigned long long*)phip_malloc(sizeof(unsigned long long) * 64 * 6 * 2 * (size_t)nwg);
        s.arr_nwg = nwg;
    }
    PPO_CHECK(hipMemsetAsync(s.arr, 0, sizeof(unsigned long long) * 64 * 6 * 2 * (size_t)nwg, ppo::stream()));
    s.arr_on = 1;
    return s.arr;
}

}  // namespace clu

extern "C" {

// diagnostics: the per-sub-phase means (µs, steps 1 … 62) of the phases launched since the last call
// (PPO_CLUSTER_STAMPS); synchronises, so the host calls it after the phases have joined
void phip_cluster_report(void) {
    int dev = 0, khz = 0;
    for (int i = 0; i < 2; ++i) {
        StampSlot& s = g_stamps[i];
        if (!s.pending) continue;
        s.pending = 0;
        if (!khz) {
            PPO_CHECK(hipGetDevice(&dev));
            PPO_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
        }
        const double mhz = khz > 0 ? khz / 1000.0 : 100.0;
        unsigned long long h[64 * 32];
        phip_d2h(h, s.buf, sizeof(unsigned long long) * 64 * (size_t)s.nstamp);
        // the shader clock beside the wall clock (s_memtime counts core cycles, s_memrealtime 100 MHz ticks):
        // per sub-phase the mean wall time and the clock it ran at, MHz = Δcycles / Δµs
        unsigned long long c[64 * 32];
        phip_d2h(c, s.buf + CLU_STAMP_CLK, sizeof(unsigned long long) * 64 * (size_t)s.nstamp);
        double acc[32] = {0}, cyc[32] = {0}, tot = 0, tcyc = 0;
        for (int st = 1; st < 63; ++st)
            for (int k = 0; k < s.nstamp; ++k) {
                const int i0 = st * s.nstamp + k, i1 = k < s.nstamp - 1 ? i0 + 1 : (st + 1) * s.nstamp;
                acc[k] += (double)(h[i1] - h[i0]) / mhz;
                cyc[k] += (double)(c[i1] - c[i0]);
            }
        fprintf(stderr, "%s %s step (us):", s.kind, s.policy ? "policy" : "value");
        for (int k = 0; k < s.nstamp; ++k) { fprintf(stderr, " %s %.2f", s.names[k], acc[k] / 62); tot += acc[k] / 62; tcyc += cyc[k] / 62; }
        fprintf(stderr, " | total %.2f\n", tot);
        fprintf(stderr, "%s %s shader clock (MHz):", s.kind, s.policy ? "policy" : "value");
        for (int k = 0; k < s.nstamp; ++k) fprintf(stderr, " %s %.0f", s.names[k], acc[k] > 0 ? cyc[k] / acc[k] : 0.0);
        fprintf(stderr, " | step %.0f\n", tot > 0 ? tcyc / tot : 0.0);
        // placement: per workgroup XCC id and HW_ID's CU [11:8] / SH [12] / SE [14:13] fields
        unsigned long long pl[64];
        phip_d2h(pl, s.buf + 64 * 32, sizeof(unsigned long long) * (size_t)s.nwg);
        int per_xcc[16] = {0};
        fprintf(stderr, "%s %s placement (xcc.se.sh.cu):", s.kind, s.policy ? "policy" : "value");
        for (int w = 0; w < s.nwg; ++w) {
            const unsigned xcc = (unsigned)(pl[w] >> 32) & 15u, hw = (unsigned)pl[w];
            per_xcc[xcc]++;
            fprintf(stderr, " %u.%u.%u.%u", xcc, (hw >> 13) & 3u, (hw >> 12) & 1u, (hw >> 8) & 15u);
        }
        fprintf(stderr, " | per XCC:");
        for (int x = 0; x < 8; ++x) fprintf(stderr, " %d", per_xcc[x]);
        fprintf(stderr, "\n");
        if (s.arr_on) {
            // per barrier over steps 1 … 62: arrival skew (last − first arrival), exit latency (first exit − last
            // arrival: the hand-off's own propagation), and the workgroups that arrive last most often
            const int nw = s.arr_nwg;
            std::vector<unsigned long long> ar((size_t)64 * 6 * 2 * nw);
            phip_d2h(ar.data(), s.arr, sizeof(unsigned long long) * ar.size());
            for (int bi = 0; bi < 6; ++bi) {
                double skew = 0, prop = 0, spread = 0;
                int n = 0;
                std::vector<int> last(nw, 0);
                for (int st = 1; st < 63; ++st) {
                    const unsigned long long* A0 = &ar[((size_t)(st * 6 + bi) * 2 + 0) * nw];
                    const unsigned long long* E0 = &ar[((size_t)(st * 6 + bi) * 2 + 1) * nw];
                    unsigned long long amin = ~0ull, amax = 0, emin = ~0ull, emax = 0;
                    int wl = 0;
                    bool any = true;
                    for (int w = 0; w < nw; ++w) {
                        if (!A0[w] || !E0[w]) { any = false; break; }
                        if (A0[w] < amin) amin = A0[w];
                        if (A0[w] > amax) { amax = A0[w]; wl = w; }
                        emin = E0[w] < emin ? E0[w] : emin;
                        emax = E0[w] > emax ? E0[w] : emax;
                    }
                    if (!any) continue;
                    skew += (double)(amax - amin) / mhz;
                    prop += (double)(emin > amax ? emin - amax : 0) / mhz;
                    spread += (double)(emax - emin) / mhz;
                    last[wl]++;
                    n++;
                }
                if (!n) continue;
                fprintf(stderr, "%s %s barrier %c: arrival skew %.2f us, exit after last arrival %.2f us, exit spread %.2f us;"
                        " last to arrive:", s.kind, s.policy ? "policy" : "value", 'A' + bi, skew / n, prop / n, spread / n);
                for (int k = 0; k < 3; ++k) {
                    int best = 0;
                    for (int w = 1; w < nw; ++w) if (last[w] > last[best]) best = w;
                    if (!last[best]) break;
                    const unsigned xcc = best < 64 ? (unsigned)(pl[best] >> 32) & 15u : 0u;
                    fprintf(stderr, " wg %d (xcc %u) %d/%d", best, xcc, last[best], n);
                    last[best] = 0;
                }
                fprintf(stderr, "\n");
            }
            // per workgroup, the mean length of its own work segment before each barrier (its arrival
            // minus its exit from the barrier before; A's segment starts at the previous step's F): which
            // workgroups are slow, in which segment, independent of the other workgroups' hand-off times
            auto stamp = [&](int st, int bi, int ex, int w) { return ar[((size_t)(st * 6 + bi) * 2 + ex) * nw + w]; };
            for (int bi = 0; bi < 6; ++bi) {
                std::vector<double> seg(nw, 0.0);
                int n = 0;
                for (int st = 2; st < 63; ++st) {
                    int ps = st, pb = bi;
                    for (int k = 1; k <= 5; ++k) {                       // the barrier before (value: no D)
                        ps = bi - k < 0 ? st - 1 : st;
                        pb = bi - k < 0 ? bi - k + 6 : bi - k;
                        if (stamp(ps, pb, 1, 0)) break;
                    }
                    bool any = true;
                    for (int w = 0; w < nw && any; ++w) any = stamp(st, bi, 0, w) && stamp(ps, pb, 1, w);
                    if (!any) continue;
                    for (int w = 0; w < nw; ++w) seg[w] += (double)(stamp(st, bi, 0, w) - stamp(ps, pb, 1, w)) / mhz;
                    n++;
                }
                if (!n) continue;
                fprintf(stderr, "%s %s segment before %c (us per wg):", s.kind, s.policy ? "policy" : "value", 'A' + bi);
                for (int w = 0; w < nw; ++w) fprintf(stderr, " %.1f", seg[w] / n);
                fprintf(stderr, "\n");
                // and each workgroup's mean exit after the first exit: who sees the release late
                std::vector<double> lat(nw, 0.0);
                int ne = 0;
                for (int st = 1; st < 63; ++st) {
                    unsigned long long emin = ~0ull;
                    bool any = true;
                    for (int w = 0; w < nw && any; ++w) {
                        any = stamp(st, bi, 1, w) != 0;
                        if (any && stamp(st, bi, 1, w) < emin) emin = stamp(st, bi, 1, w);
                    }
                    if (!any) continue;
                    for (int w = 0; w < nw; ++w) lat[w] += (double)(stamp(st, bi, 1, w) - emin) / mhz;
                    ne++;
                }
                if (!ne) continue;
                fprintf(stderr, "%s %s exit %c after first exit (us per wg):", s.kind, s.policy ? "policy" : "value", 'A' + bi);
                for (int w = 0; w < nw; ++w) fprintf(stderr, " %.1f", lat[w] / ne);
                fprintf(stderr, "\n");
            }
        }
    }
}

// Host-visible error of the cluster phases (nonzero: a barrier timed out — a workgroup of the launch was
// never resident, or a device fault stopped one).  The word stays set: the update that saw it ends the
// process (ppo_update dies), since the phase left its parameters and Adam state half-written.
int phip_cluster_error(void) {
    if (!g_err) return 0;
    const unsigned e = __atomic_load_n(g_err, __ATOMIC_ACQUIRE);
    return e != 0u;
}

// the device pointer of the host-mapped error word shared by the cluster kernels (allocated on first
// use); NULL, with the error recorded, when an earlier launch left it set
unsigned* phip_cluster_err_dev(void) {
    if (!g_err) {
        PPO_CHECK(hipHostMalloc((void**)&g_err, 64, hipHostMallocMapped | hipHostMallocCoherent));
        *g_err = 0u;
    }
    if (*g_err) {
        phip_record_error("cluster phase: a barrier timed out in an earlier launch");
        return nullptr;
    }
    unsigned* d_err = nullptr;
    PPO_CHECK(hipHostGetDevicePointer((void**)&d_err, g_err, 0));
    return d_err;
}

int phip_cluster_update(const PhipTinyNet* net, const PhipTinyPhase* ph) {
    if (getenv("PPO_NO_CLUSTER")) return -1;
    if (net->L == 4) return phip_cluster_deep_update(net, ph);       // S → 512 × 3 → O (cluster_deep.hip)
    if (net->L != 3 || ph->B != BB || ph->n_epochs > 16) return -1;
    const int S = net->sizes[0], H = net->sizes[1], O = net->sizes[3];
    if (H != 256 || net->sizes[2] != H || S < 1 || S > 20 || O < 1 || O > OMAX) return -1;
    if (!net->relu[0] || !net->relu[1] || net->relu[2]) return -1;
    if (ph->policy && (!net->log_std || !net->m_ls)) return -1;
    constexpr int HC = 16, NWG = 256 / HC;                         // 16 workgroups of 16 hidden units
    constexpr size_t bytes = sizeof(float) * (size_t)Lay<256, HC>::TOTAL;
    static_assert(bytes <= 160 * 1024, "cluster: LDS");
    // one workgroup in every `active_stride`: blocks b and b + 8 are dealt to one XCD (observed,
    // MI355X_MICROARCH.md § Workgroup dispatch), so stride 8 puts the phase on one XCD, 4 on two, 1 on
    // all eight; correctness never depends on it (PPO_CLUSTER_STRIDE overrides; 1, 2, 4 or 8)
    // (value phase — the longer — on one XCD, policy on two: 16 + 8 ≤ 32 CUs wherever they land)
    int stride = ph->policy ? 4 : 8;
    if (const char* st = getenv("PPO_CLUSTER_STRIDE")) {
        const int v = atoi(st);
        if (v == 1 || v == 2 || v == 4 || v == 8) stride = v;
    }
    auto kfn = cluster_phase_kernel<256, HC>;
    static bool attr = false;
    if (!attr) {
        PPO_CHECK(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
        attr = true;
    }
    if (!host_grid_fits((const void*)kfn, bytes, NWG * stride)) return -1;   // not co-resident: multi-launch
    if (ph->n_epochs <= 0 || ph->num_batches <= 0) return 0;     // fit check only
    ClArgs a{};
    a.S = S; a.O = O; a.policy = ph->policy;
    a.SP = ((S + 3) / 4) * 4;
    if (((a.SP / 4) & 1) == 0) a.SP += 4;                         // 4·odd (conflict-free strided reads)
    a.params = net->params; a.grads = net->grads; a.m = net->m; a.v = net->v;
    for (int l = 0; l < 3; ++l) { a.woff[l] = net->woff[l]; a.boff[l] = net->boff[l]; }
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
    const long need = (long)BB * 256 + (long)NWG * BB * OMAX + (long)NWG * BB * 256;
    if (ws.cap < need) {
        phip_free(ws.X1);
        phip_free(ws.ctr);
        ws.X1 = (float*)phip_malloc(sizeof(float) * (size_t)need);
        ws.ctr = (unsigned*)phip_malloc(CLU_CTR_BYTES);      // counter replicas
        ws.cap = need;
    }
    ws.Y = ws.X1 + (long)BB * 256;
    ws.G1 = ws.Y + (long)NWG * BB * OMAX;
    unsigned* d_err = phip_cluster_err_dev();
    if (!d_err) return -2;
    a.X1 = ws.X1; a.Y = ws.Y; a.G1 = ws.G1; a.ctr = ws.ctr; a.err = d_err;
    a.timeout = host_timeout_ticks();
    a.active_stride = stride;
    // stride 8 puts a phase on one XCD (blocks b, b + 8 share one); the policy phase then takes XCD 4
    // so the two concurrent phases never share CUs
    a.active_offset = stride == 8 && ph->policy ? 4 : 0;
    static const char* names[12] = {"gather", "L0", "barrier A", "h1 load", "L1+Y", "barrier B", "head+bwd",
                                    "G1+gW1 adam", "barrier C", "g1+gW0", "adam", "step->next"};
    if (getenv("PPO_CLUSTER_STAMPS")) a.stamps = host_stamps(12, "cluster", names, ph->policy, a.total_steps, NWG);
    PPO_CHECK(hipMemsetAsync(ws.ctr, 0, CLU_CTR_BYTES, ppo::stream()));
    ppo::ProfScope ps(PPO_K_OTHER, 0.0);
    hipLaunchKernelGGL(kfn, dim3(NWG * a.active_stride), dim3(TPB), bytes, ppo::stream(), a);
    PPO_LAUNCH_CHECK();
    return 0;
}

}  // extern "C"
