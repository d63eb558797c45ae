// tiny.hip — the whole minibatch loop of a PPO update in ONE workgroup, for small networks.
//
// Configs C1/C2 (Pendulum: 3 → 64 → 64 → 1, B = 64) do 896 minibatch steps per update, each a
// chain of ~12 tiny launches (gather, 3 forward GEMMs, loss, 3 grad_W + 2 grad_x GEMMs, Adam):
// launch- and latency-bound at ≈65 µs per step, slower than one CPU core.  Here one 1024-thread
// workgroup runs all minibatch steps of a phase (the value epochs, or the policy epochs) back to
// back: the minibatch's activations and gradients stay in LDS, the parameters, gradients and Adam
// moments (a few hundred KB at most) stay in L2, and the only synchronisation is __syncthreads().
//
// Per step, exactly the reference's arithmetic (ppo.cu:391-447 / :479-539):
//   rows = perm[(k·B + i) mod limit]               (trajectory_buffer.cu:168-200; host rand()
//                                                   permutations or libppo's device Feistel)
//   forward  y = act(x·Wᵀ + b) per layer           (neural_network.cu:74-105)
//   value:   L = Σ(t−y)²/B, g = 2(y−t)/B           (loss.cu:5-23)
//   policy:  log π, ratio, clipped surrogate, ∂/∂μ, ∂/∂logσ (−c_ent)   (ppo.cu:82-107,
//            policy.cu:67-111, ppo.cu:436-438)
//   backward gW = gᵀ·x, gb = Σ g, gx = (g·W) ⊙ 1[x > 0]   (neural_network.cu:121-161)
//   Adam     (adam.cu:138-169; the entropy Adam before the policy Adam, ppo.cu:440-442), with the
//            bias corrections the host computes for every step (same powf as the multi-launch path)
// GEMMs are v_mfma_f32_16x16x4_f32 (exact fp32; 16×16 tiles keep all 16 waves busy on 64-wide
// layers), one output tile per wave, operands read straight from LDS.  When they fit (C2: 3→64→64→1
// at B = 64 uses 158 KB), the parameters, gradients, Adam moments and a transposed weight copy (so
// the forward's B operand is read along rows) live in LDS for the whole phase; otherwise in L2.
// One CU's fp32 MFMA rate (256 FLOP/clk) bounds a 64-wide step at ≈4 µs; measured ≈26 µs per step
// (PPO_TINY_STAMPS=1 prints the per-phase split), against ≈65 µs for the multi-launch loop.
#include "dev.h"

#include <cmath>
#include <cstdlib>

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

#ifndef PPO_TINY_TPB
#define PPO_TINY_TPB 1024
#endif
constexpr int TPB = PPO_TINY_TPB;
constexpr int NWAVES = TPB / 64;
constexpr int MAXL = 8;            // linear layers

struct Feistel { uint32_t k[4]; uint32_t half, mask, n; };

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

// identical to buffer.hip's feistel_index (restated in oracle/ref_cpu.c: ref_feistel_index)
__device__ __forceinline__ uint32_t feistel_index(uint32_t i, const Feistel& f) {
    uint32_t x = i;
    do {
        uint32_t L = x >> f.half, R = x & f.mask;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t nl = R;
            R = L ^ (mix32(R ^ f.k[r]) & f.mask);
            L = nl;
        }
        x = (L << f.half) | R;
    } while (x >= f.n);
    return x;
}

struct TinyArgs {
    int L;                          // linear layers
    int sizes[MAXL + 1];            // widths, sizes[0] = S, sizes[L] = output width
    int relu[MAXL];                 // activation after layer l
    long woff[MAXL], boff[MAXL];    // offsets of W_l / b_l in the flat parameter / gradient buffers
    float* params; float* grads; float* m; float* v; long span;       // network + its Adam state
    float* wt; long wtoff[MAXL];    // transposed weights Wᵀ[k][j] (kept current by the Adam loop):
                                    // the forward's B operand then loads 16 consecutive floats per row
    // policy only: log_std and its gradient / Adam state
    float* log_std; float* log_std_grad; float* m_ls; float* v_ls; int A;
    int policy;                     // 0: value phase (MSE), 1: policy phase (clipped surrogate)
    // buffer
    const float* state; const float* action; const float* logprob; const float* adv; const float* adv_target;
    int limit, B, num_batches, n_epochs;
    int total_steps;                // n_epochs·num_batches, or the step cap (ppo_set_step_limit)
    const int* perms;               // [n_epochs][limit] host rand() permutations, or nullptr → Feistel
    Feistel fk[16];                 // per-epoch Feistel keys (device shuffle)
    const float* steps;             // per step: {lr/bc1, bc2} of the network's Adam (value / policy)
    const float* steps_ls;          // per step: {lr/bc1, bc2} of the entropy Adam (policy)
    float b1, b2, eps, ent_coeff;
    float* stats;                   // [0] Σ value loss, [1] Σ policy loss
    int ld[MAXL + 1];               // LDS row pitch (floats) of each activation
    int act_off[MAXL + 1];          // LDS offset of each activation [B][ld]
    int g_off[2];                   // LDS offsets of the two gradient buffers [B][gld]
    int gld;
    int misc_off;                   // LDS: rows[B] (int), targets / adv / old_lp [B], actions [B][A]
    unsigned long long* stamps;     // diagnostics (PPO_TINY_STAMPS): s_memrealtime at phase boundaries
    int res_off;                    // RESIDENT: LDS offset of [params | grads | m | v | Wᵀ]
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// C[M×N] = A(M×K)·B(K×N) on 16×16 tiles, one tile per wave per round; A(i, k) = A[i·a_si + k·a_sk],
// B(k, j) = B[k·b_sk + j·b_sj] (LDS or global).  Operand lane maps: A lane l holds
// A[i0 + (l&15)][k0 + (l>>4)], B lane l holds B[k0 + (l>>4)][j0 + (l&15)]; C/D: col = l&15,
// row = 4·(l>>4) + reg.  Loads are unconditional (indices clamped, out-of-range values zeroed by a
// select) and issued 8 MFMAs' worth at a time, so no exec-mask branches or per-MFMA waits.
// EPI 0: C[i][j] = act(v + bias[j]) (forward, LDS); 1: C[i][j] = v (grad_W, global);
// EPI 2: C[i][j] = (X[i][j] > 0 or !mask) ? v : 0 (grad_x with the ReLU′ mask, LDS).
template <int EPI>
__device__ __forceinline__ void tile_gemm(int M, int N, int K, const float* __restrict__ A, int a_si, int a_sk,
                                          const float* __restrict__ B, int b_sk, int b_sj, float* __restrict__ C,
                                          int c_si, const float* __restrict__ bias, int flag,
                                          const float* __restrict__ X, int x_si) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int tm = (M + 15) / 16, tn = (N + 15) / 16;
    const int c = lane & 15, q = lane >> 4;
    for (int t = w; t < tm * tn; t += NWAVES) {
        const int i0 = (t / tn) * 16, j0 = (t % tn) * 16;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        const int ia = i0 + c, jb = j0 + c;
        const bool iok = ia < M, jok = jb < N;
        const float* Ar = A + (long)min(ia, M - 1) * a_si;
        const float* Bc = B + (long)min(jb, N - 1) * b_sj;
        for (int k0 = 0; k0 < K; k0 += 32) {
            float av[8], bv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int kc = min(k0 + 4 * u + q, K - 1);
                av[u] = Ar[(long)kc * a_sk];
                bv[u] = Bc[(long)kc * b_sk];
            }
            // opaque, after all 16 loads are issued: otherwise the compiler sinks each load under
            // its lane condition (an exec-mask branch and a wait per load)
            asm("" : "+v"(av[0]), "+v"(av[1]), "+v"(av[2]), "+v"(av[3]), "+v"(av[4]), "+v"(av[5]), "+v"(av[6]),
                     "+v"(av[7]), "+v"(bv[0]), "+v"(bv[1]), "+v"(bv[2]), "+v"(bv[3]), "+v"(bv[4]), "+v"(bv[5]),
                     "+v"(bv[6]), "+v"(bv[7]));
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int k = k0 + 4 * u + q;
                av[u] = (iok && k < K) ? av[u] : 0.f;
                bv[u] = (jok && k < K) ? bv[u] : 0.f;
            }
            // a short K tail (layer 0's K = S, the A-wide output layer's grad_x K = A): only the
            // MFMAs whose 4-k slice holds real k (wave-uniform count) — the rest would add zeros
            const int nu = K - k0 >= 32 ? 8 : (K - k0 + 3) >> 2;
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (u < nu) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u], acc, 0, 0, 0);
        }
        const int j = j0 + c;
        if (j < N) {
            const float bj = EPI == 0 ? bias[j] : 0.f;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int i = i0 + 4 * q + e;
                if (i >= M) continue;
                float v = acc[e];
                if (EPI == 0) {
                    v += bj;
                    if (flag) v = v > 0.f ? v : 0.f;
                } else if (EPI == 2) {
                    if (flag && !(X[(long)i * x_si + j] > 0.f)) v = 0.f;
                }
                C[(long)i * c_si + j] = v;
            }
        }
    }
}

__device__ __forceinline__ float log_prob_row(const float* mu, const float* log_std, const float* a, int A) {
    const float cst = (float)(-0.5 * A * (double)logf((float)(2 * M_PI)));
    float lp = cst;
    for (int j = 0; j < A; ++j) {
        const float z = (a[j] - mu[j]) / expf(log_std[j]);
        lp = (float)((double)lp - ((double)log_std[j] + 0.5 * (double)(z * z)));
    }
    return lp;
}

__device__ __forceinline__ float surrogate(float adv, float lp, float old_lp, float eps, int m, float* grad) {
    const float ratio = (float)exp((double)(lp - old_lp));
    const int adv_pos = adv > 0;
    const int ratio_pos = ratio > 1 + eps;
    const int ratio_neg = ratio < 1 - eps;
    *grad = -(adv_pos * !ratio_pos + !adv_pos * !ratio_neg) * adv * ratio / m;
    return adv * (adv_pos * (ratio_pos * (1 + eps) + !ratio_pos * ratio) +
                  !adv_pos * (ratio_neg * (1 - eps) + !ratio_neg * ratio));
}

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float step, float b1, float b2,
                                          float bc2) {
    m = b1 * m + (1 - b1) * g;
    v = b2 * v + (1 - b2) * (g * g);
    const float denom = (float)((double)sqrtf(v / bc2) + 1e-8);
    p -= step * m / denom;
}

#define TINY_STAMP(slot)                                                                         \
    do {                                                                                         \
        if (a.stamps && tid == 0 && step < 64) {                                                 \
            a.stamps[step * 8 + (slot)] = wall_clock64();                                        \
            if ((slot) == 0) a.stamps[step * 8 + 6] = __builtin_amdgcn_s_memtime();              \
        }                                                                                        \
    } while (0)

// RESIDENT: parameters, gradients, Adam moments and Wᵀ live in LDS for the whole phase (loaded at
// the start, written back at the end) — every minibatch step then touches global memory only for
// its gather.  Otherwise they stay in L2 (wider networks).
template <bool RESIDENT>
__global__ __launch_bounds__(TPB) void tiny_update_kernel(TinyArgs a) {
    extern __shared__ float lds[];
    float* P = RESIDENT ? lds + a.res_off : a.params;
    const long sp = (a.span + 3) & ~3L;                      // LDS regions stay 16-B aligned
    float* Gd = RESIDENT ? P + sp : a.grads;
    float* Mv = RESIDENT ? Gd + sp : a.m;
    float* Vv = RESIDENT ? Mv + sp : a.v;
    float* WT = RESIDENT ? Vv + sp : a.wt;
    if (RESIDENT) {
        for (long e = threadIdx.x; e < a.span; e += TPB) {
            P[e] = a.params[e];
            Gd[e] = 0.f;
            Mv[e] = a.m[e];
            Vv[e] = a.v[e];
        }
        __syncthreads();
    }
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int B = a.B, L = a.L, S = a.sizes[0];
    int* rows = reinterpret_cast<int*>(lds + a.misc_off);
    float* tgt = lds + a.misc_off + B;            // value: target; policy: advantage
    float* olp = tgt + B;                         // policy: old log-prob
    float* act = olp + B;                         // policy: actions [B][A]
    __shared__ float red[NWAVES];
    __shared__ float gls_acc[32];

    int step = 0;
    for (int l = 0; l < L; ++l) {                             // Wᵀ from the current parameters
        const int n = a.sizes[l], o = a.sizes[l + 1];
        for (int e = tid; e < n * o; e += TPB) {
            const int j = e / n, k = e % n;
            WT[a.wtoff[l] + (long)k * o + j] = P[a.woff[l] + e];
        }
    }
    __threadfence_block();
    __syncthreads();
    for (int ep = 0; ep < a.n_epochs; ++ep) {
        for (int kb = 0; kb < a.num_batches && step < a.total_steps; ++kb, ++step) {
            TINY_STAMP(0);
            // ---- gather (trajectory_buffer.cu:168-200) ----
            for (int i = tid; i < B; i += TPB) {
                const int list = (int)(((long)kb * B + i) % a.limit);
                const int src = a.perms ? a.perms[(long)ep * a.limit + list]
                                        : (int)feistel_index((uint32_t)list, a.fk[ep & 15]);
                rows[i] = src;
                if (a.policy) {
                    tgt[i] = a.adv[src];
                    olp[i] = a.logprob[src];
                } else {
                    tgt[i] = a.adv_target[src];
                }
            }
            __syncthreads();
            {
                float* x0 = lds + a.act_off[0];
                const int ld0 = a.ld[0];
                for (int e = tid; e < B * S; e += TPB) {
                    const int i = e / S, j = e % S;
                    x0[i * ld0 + j] = a.state[(long)rows[i] * S + j];
                }
                if (a.policy)
                    for (int e = tid; e < B * a.A; e += TPB) {
                        const int i = e / a.A, j = e % a.A;
                        act[i * a.A + j] = a.action[(long)rows[i] * a.A + j];
                    }
            }
            __syncthreads();
            TINY_STAMP(1);
            // ---- forward ----
            for (int l = 0; l < L; ++l) {
                const float* X = lds + a.act_off[l];
                float* Y = lds + a.act_off[l + 1];
                const int ldx = a.ld[l], ldy = a.ld[l + 1], n = a.sizes[l], o = a.sizes[l + 1];
                // y[b][j] = Σ_k x[b][k]·W[j][k]:  A = x (LDS), B(k, j) = Wᵀ[k·o + j] (L2, coalesced)
                tile_gemm<0>(B, o, n, X, ldx, 1, WT + a.wtoff[l], o, 1, Y, ldy, P + a.boff[l],
                             a.relu[l], nullptr, 0);
                __syncthreads();
                if (a.stamps && tid == 0 && step < 64 && l < 3) a.stamps[64 * 8 + step * 4 + l] = wall_clock64();
            }
            TINY_STAMP(2);
            // ---- head: output gradient into g buffer 0 ----
            const float* Yo = lds + a.act_off[L];
            const int ldo = a.ld[L];
            float* G = lds + a.g_off[0];
            const int gld = a.gld;
            float part = 0.f;
            if (!a.policy) {                                   // loss.cu:5-23
                for (int i = tid; i < B; i += TPB) {
                    const float y = Yo[i * ldo], t = tgt[i];
                    const float d = t - y;
                    part += d * d;
                    G[i * gld] = 2 * (y - t) / (float)B;
                }
            } else {                                           // ppo.cu:82-107, policy.cu:67-111
                if (tid < a.A) gls_acc[tid] = 0.f;
                __syncthreads();
                for (int i = tid; i < B; i += TPB) {
                    float g;
                    const float lp = log_prob_row(Yo + i * ldo, a.log_std, act + i * a.A, a.A);
                    part += surrogate(tgt[i], lp, olp[i], a.eps, B, &g);
                    for (int j = 0; j < a.A; ++j) {
                        const float e2 = expf(-2 * a.log_std[j]);
                        const float d = act[i * a.A + j] - Yo[i * ldo + j];
                        G[i * gld + j] = d * e2 * g;
                        atomicAdd(&gls_acc[j], (-1 + d * d * e2) * g);
                    }
                }
            }
            part = wave_sum(part);
            if (lane == 0) red[w] = part;
            __syncthreads();
            if (tid == 0) {
                float s = 0.f;
                for (int q = 0; q < NWAVES; ++q) s += red[q];
                if (!a.policy) {
                    atomicAdd(a.stats + 0, s * (1.0f / (float)B));
                } else {
                    float ent = (float)(a.A * 0.5 * (1 + log(2 * M_PI)));
                    for (int j = 0; j < a.A; ++j) ent += a.log_std[j];
                    atomicAdd(a.stats + 1, -s / B - a.ent_coeff * ent);
                }
            }
            if (a.policy && tid < a.A) a.log_std_grad[tid] = gls_acc[tid] + -a.ent_coeff;   // ppo.cu:436-438
            __syncthreads();
            TINY_STAMP(3);
            // ---- backward ----
            int gi = 0;
            for (int l = L - 1; l >= 0; --l) {
                const float* X = lds + a.act_off[l];
                const int ldx = a.ld[l], n = a.sizes[l], o = a.sizes[l + 1];
                const float* Gc = lds + a.g_off[gi];
                float* gb = Gd + a.boff[l];
                // gW[j][k] = Σ_b g[b][j]·x[b][k]:  A(j, b) = g (LDS), B(b, k) = x (LDS)
                tile_gemm<1>(o, n, B, Gc, 1, gld, X, ldx, 1, Gd + a.woff[l], n, nullptr, 0, nullptr, 0);
                // bias gradient Σ over the batch: one thread per column, rows summed in order from
                // LDS (lanes read consecutive columns: conflict-free) — ≈ 64 wave-level LDS reads
                // instead of 4 columns per wave through six-step shuffle reductions
                for (int j = tid; j < o; j += TPB) {
                    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
                    int b = 0;
                    for (; b + 4 <= B; b += 4) {
                        s0 += Gc[b * gld + j];
                        s1 += Gc[(b + 1) * gld + j];
                        s2 += Gc[(b + 2) * gld + j];
                        s3 += Gc[(b + 3) * gld + j];
                    }
                    for (; b < B; ++b) s0 += Gc[b * gld + j];
                    gb[j] = (s0 + s1) + (s2 + s3);
                }
                if (l > 0) {
                    // gx[b][k] = Σ_j g[b][j]·W[j][k], masked by x > 0:  A = g (LDS), B(j, k) = W[j·n + k]
                    tile_gemm<2>(B, n, o, Gc, gld, 1, P + a.woff[l], n, 1, lds + a.g_off[gi ^ 1], gld,
                                 nullptr, a.relu[l - 1], X, ldx);
                }
                __syncthreads();
                gi ^= 1;
            }
            TINY_STAMP(4);
            // make this step's gradient stores visible to every wave's Adam reads
            __threadfence_block();
            __syncthreads();
            // ---- Adam: entropy (log σ) first, then the network (ppo.cu:440-442) ----
            if (a.policy && tid < a.A) {
                float p = a.log_std[tid], mm = a.m_ls[tid], vv = a.v_ls[tid];
                adam_elem(p, a.log_std_grad[tid], mm, vv, a.steps_ls[2 * step], a.b1, a.b2, a.steps_ls[2 * step + 1]);
                a.log_std[tid] = p; a.m_ls[tid] = mm; a.v_ls[tid] = vv;
            }
            const float st = a.steps[2 * step], bc2 = a.steps[2 * step + 1];
            const long span4 = a.span & ~3L;
            for (long e = span4 + tid; e < a.span; e += TPB) {
                float p = P[e], mm = Mv[e], vv = Vv[e];
                adam_elem(p, Gd[e], mm, vv, st, a.b1, a.b2, bc2);
                P[e] = p; Mv[e] = mm; Vv[e] = vv;
            }
            for (long e = 4 * (long)tid; e < span4; e += 4 * (long)TPB) {
                f32x4 p = *reinterpret_cast<const f32x4*>(P + e);
                const f32x4 g = *reinterpret_cast<const f32x4*>(Gd + e);
                f32x4 mm = *reinterpret_cast<const f32x4*>(Mv + e);
                f32x4 vv = *reinterpret_cast<const f32x4*>(Vv + e);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    float pu = p[u], mu = mm[u], vu = vv[u];
                    adam_elem(pu, g[u], mu, vu, st, a.b1, a.b2, bc2);
                    p[u] = pu; mm[u] = mu; vv[u] = vu;
                }
                *reinterpret_cast<f32x4*>(P + e) = p;
                *reinterpret_cast<f32x4*>(Mv + e) = mm;
                *reinterpret_cast<f32x4*>(Vv + e) = vv;
            }
            __syncthreads();
            for (int l = 0; l < L; ++l) {                         // refresh Wᵀ from the new weights
                const int n = a.sizes[l], o = a.sizes[l + 1];
                const float* Wl = P + a.woff[l];
                float* Tl = WT + a.wtoff[l];
                if (n == o) {
                    // square: diagonal r, lane l takes (k = l, j = l + r mod n) — reads and writes on
                    // distinct LDS banks (row-major order writes at stride o: a 64-way conflict)
                    for (int e = tid; e < n * n; e += TPB) {
                        const int r = e / n, k = e - r * n;
                        int j = k + r;
                        j = j >= n ? j - n : j;
                        Tl[k * n + j] = Wl[j * n + k];
                    }
                } else {
                    for (int e = tid; e < n * o; e += TPB) {
                        const int j = e / n, k = e - j * n;
                        Tl[k * o + j] = Wl[e];
                    }
                }
            }
            __threadfence_block();
            __syncthreads();
            TINY_STAMP(5);
        }
    }
    if (RESIDENT) {
        for (long e = threadIdx.x; e < a.span; e += TPB) {
            a.params[e] = P[e];
            a.grads[e] = Gd[e];
            a.m[e] = Mv[e];
            a.v[e] = Vv[e];
        }
    }
}

// ---------------------------------------------------------------------------
// The same phase for the Pendulum-shaped networks of C1/C2 (S → H → H → 1, ReLU, B = BB rows), with
// every width, pitch and LDS offset a compile-time constant: all operand addresses fold into LDS
// instruction offsets (the generic kernel spends most of its step on 64-bit address arithmetic and
// clamps), the 1-wide output layer and the 3-wide input layer's weight gradient run on the VALU
// instead of 1/16-occupied MFMA tiles, and the weights stay in their [out][in] layout (pitch H + 2),
// so no transposed copy is refreshed after each Adam step.  The hidden GEMMs keep the generic
// kernel's k order (MFMA u of a 32-k chunk takes k = k0 + 4u + q from lane group q), so both kernels
// round every hidden pre-activation alike (a different order can flip a ReLU mask at z ≈ 0).
// Pitch H + 2 ≡ 2 (mod 32): a k-contiguous read (rows c, k = .. + q) is conflict-free, a k-strided
// one 2-way.  Parameters, gradients and Adam moments live in LDS in that padded layout (pads stay
// zero: a zero gradient leaves a zero parameter unchanged under Adam) and are mapped from / to the
// flat buffers at the phase's start / end.
template <int S, int H, int BB>
struct C2Lay {
    static constexpr int SP = 4, P = H + 2;
    static_assert(S <= SP && H % 32 == 0 && BB % 32 == 0 && BB * SP <= TPB && H <= 64, "C2 shape");
    // padded parameter image: W0 [H][SP], b0 [H], W1 [H][P], b1 [H], W2 [H], b2 [4]
    static constexpr int oW0 = 0, ob0 = oW0 + H * SP, oW1 = ob0 + H, ob1 = oW1 + H * P, oW2 = ob1 + H,
                         ob2 = oW2 + H, NPAR = ob2 + 4;
    // flat (reference) layout: W0 [H][S], b0, W1 [H][H], b1, W2 [1][H], b2
    static constexpr int fb0 = H * S, fW1 = fb0 + H, fb1 = fW1 + H * H, fW2 = fb1 + H, fb2 = fW2 + H,
                         NFLAT = fb2 + 1;
    // activations / gradients [BB][P] (X0: two [BB][SP] buffers, this step's and the next's), then
    // rows, targets, old log-probs, actions
    static constexpr int aX0 = 0, aY1 = aX0 + 2 * BB * SP, aY2 = aY1 + BB * P, aG2 = aY2 + BB * P, aG1 = aG2 + BB * P,
                         aG3 = aG1 + BB * P, aT = aG3 + BB, aMisc = aT + 4 * H, aRes = (aMisc + 4 * BB + 3) & ~3,
                         TOTAL = aRes + 4 * NPAR;
    __device__ static int pad_index(int f) {
        if (f < fb0) return oW0 + (f / S) * SP + f % S;
        if (f < fW1) return ob0 + (f - fb0);
        if (f < fb1) return oW1 + ((f - fW1) / H) * P + (f - fW1) % H;
        if (f < fW2) return ob1 + (f - fb1);
        if (f < fb2) return oW2 + (f - fW2);
        return ob2;
    }
};

// 16×16 output tile over K (a multiple of 32): A(i, k), B(k, j) — KC: element (r, k) at base[r·PITCH + k]
// (k-contiguous), else at base[k·PITCH + r]; lane group q holds k = k0 + 4u + q for MFMA u
template <bool KC, int PITCH>
__device__ __forceinline__ void c2_fetch(const float* __restrict__ base, int r, int k0, int q, float (&v)[8]) {
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = KC ? base[r * PITCH + k0 + 4 * u + q] : base[(k0 + 4 * u + q) * PITCH + r];
}
template <int K, bool AKC, int PA, bool BKC, int PB>
__device__ __forceinline__ f32x4 c2_tile(const float* __restrict__ A, int i0, const float* __restrict__ B, int j0,
                                         int lane) {
    const int c = lane & 15, q = lane >> 4;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k0 = 0; k0 < K; k0 += 32) {
        float av[8], bv[8];
        c2_fetch<AKC, PA>(A, i0 + c, k0, q, av);
        c2_fetch<BKC, PB>(B, j0 + c, k0, q, bv);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u], acc, 0, 0, 0);
    }
    return acc;
}

#ifndef PPO_C2_ADAM_U
#define PPO_C2_ADAM_U 2   // Adam rounds interleaved per batch
#endif
#ifndef PPO_C2_AB
#define PPO_C2_AB 0       // diagnostic builds only: 1 no Adam arithmetic, 2 no next-minibatch gather,
#endif                    // 4 no layer-0 gradient phase work, 8 no hidden-layer MFMA tiles
using ppo::row_sum16;
__device__ __forceinline__ float sum16(float v) { return ppo::row_sum16(v); }
__device__ __forceinline__ float sum64(float v) { return ppo::wave_sum64(v); }

// Per step: forward layer 0 | layer 1 | output layer + head + the output layer's grad_x | hidden-layer
// gW1 / grad_x tiles with the bias / output-layer column sums | layer-0 weight + bias gradients |
// Adam with the next minibatch's gather in flight — six barriers.  Measured A/B of the alternatives
// (profiles/r03_c2_kernel_ab.txt): the next gather inside the Adam phase −0.3 ms per C2 update, the
// output layer's grad_x inside the head phase −1.2 ms; layer 0 recomputed per wave instead of a
// barrier +0.5 ms; interleaving the two hidden-layer MFMA chains of a wave ±0.
template <int S, int H, int BB>
__global__ __launch_bounds__(TPB) void tiny_c2_kernel(TinyArgs a) {
    using Ly = C2Lay<S, H, BB>;
    constexpr int P = Ly::P, SP = Ly::SP, HT = H / 16;
    static_assert((BB / 16) * HT == NWAVES && BB == H && TPB / BB == 16 && S < SP, "C2 phase split");
    extern __shared__ float lds[];
    float* const X0b = lds + Ly::aX0;                     // 2 × [BB][SP]; column S holds 1 (bias gradient)
    float* const Y1 = lds + Ly::aY1;
    float* const Y2 = lds + Ly::aY2;
    float* const G2 = lds + Ly::aG2;
    float* const G1 = lds + Ly::aG1;
    float* const G3 = lds + Ly::aG3;
    int* const rows = reinterpret_cast<int*>(lds + Ly::aMisc);
    float* const tgt = lds + Ly::aMisc + BB;              // value: target; policy: advantage
    float* const olp = tgt + BB;
    float* const act = olp + BB;                          // policy: actions (A = 1)
    float* const Pp = lds + Ly::aRes;
    float* const Gd = Pp + Ly::NPAR;
    float* const Mv = Gd + Ly::NPAR;
    float* const Vv = Mv + Ly::NPAR;
    __shared__ float red[NWAVES];
    __shared__ float gls_red[NWAVES];
    __shared__ float s_ls, s_lsg, s_mls, s_vls;           // policy: log σ (A = 1), its gradient and moments
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform values in SGPRs
    const int c = lane & 15, q = lane >> 4;
    const int ti0 = (w / HT) * 16, tj0 = (w % HT) * 16;  // this wave's 16×16 tile

    for (int e = tid; e < 4 * Ly::NPAR; e += TPB) Pp[e] = 0.f;     // pads stay zero
    __syncthreads();
    for (int f = tid; f < Ly::NFLAT; f += TPB) {
        const int d = Ly::pad_index(f);
        Pp[d] = a.params[f];
        Mv[d] = a.m[f];
        Vv[d] = a.v[f];
    }
    if (tid == 0 && a.policy) s_ls = a.log_std[0];
    if (tid == 0 && a.policy) { s_mls = a.m_ls[0]; s_vls = a.v_ls[0]; }

    // gather of minibatch (ep, kb) (trajectory_buffer.cu:168-200): SP threads per row; the loads
    // (fetch) are issued before the Adam pass, the LDS stores (put) after it
    struct Row { float x, t, o, ac; int src; };
    constexpr int G0 = TPB - BB * SP;                    // gather threads: the last BB·SP (one Adam
    const int gt = tid - G0;                             // float4 each, the first ones take two)
    auto fetch = [&](int ep, int kb) {
        Row r{0.f, 0.f, 0.f, 0.f, 0};
        const int i = gt / SP, k = gt % SP;
        const int list = (int)(((long)kb * BB + i) % a.limit);
        r.src = a.perms ? a.perms[(long)ep * a.limit + list] : (int)feistel_index((uint32_t)list, a.fk[ep & 15]);
        r.x = k < S ? a.state[(long)r.src * S + k] : (k == S ? 1.f : 0.f);
        if (k == 0) {
            if (a.policy) {
                r.t = a.adv[r.src];
                r.o = a.logprob[r.src];
                r.ac = a.action[r.src];
            } else {
                r.t = a.adv_target[r.src];
            }
        }
        return r;
    };
    auto put = [&](const Row& r, float* X0) {
        const int i = gt / SP, k = gt % SP;
        X0[i * SP + k] = r.x;
        if (k == 0) {
            rows[i] = r.src;
            tgt[i] = r.t;
            if (a.policy) { olp[i] = r.o; act[i] = r.ac; }
        }
    };
    if (gt >= 0 && a.total_steps > 0) put(fetch(0, 0), X0b);
    __syncthreads();

    int step = 0;
    for (int ep = 0; ep < a.n_epochs; ++ep) {
        for (int kb = 0; kb < a.num_batches && step < a.total_steps; ++kb, ++step) {
            TINY_STAMP(0);
            TINY_STAMP(1);
            const float* const X0 = X0b + (step & 1) * (BB * SP);
            // ---- forward (neural_network.cu:74-105) ----
            {                                                  // layer 0: K = S < 4, one MFMA
                const float av = q < S ? X0[(ti0 + c) * SP + q] : 0.f;
                const float bv = q < S ? Pp[Ly::oW0 + (tj0 + c) * SP + q] : 0.f;
                const f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
                const float bj = Pp[Ly::ob0 + tj0 + c];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float v = acc[e] + bj;
                    Y1[(ti0 + 4 * q + e) * P + tj0 + c] = v > 0.f ? v : 0.f;
                }
            }
            __syncthreads();
            if (a.stamps && tid == 0 && step < 64) a.stamps[64 * 8 + step * 4 + 0] = wall_clock64();
            {                                                  // layer 1: Y1 · W1ᵀ
                const f32x4 acc = c2_tile<H, true, P, true, P>(Y1, ti0, Pp + Ly::oW1, tj0, lane);
                const float bj = Pp[Ly::ob1 + tj0 + c];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float v = acc[e] + bj;
                    Y2[(ti0 + 4 * q + e) * P + tj0 + c] = v > 0.f ? v : 0.f;
                }
            }
            __syncthreads();
            if (a.stamps && tid == 0 && step < 64) a.stamps[64 * 8 + step * 4 + 1] = wall_clock64();
            TINY_STAMP(2);
            // ---- output layer (1 wide, VALU: 16 lanes per row), head, and the output layer's grad_x
            // G2[i] = (g_i ⊗ W2) ⊙ 1[Y2 > 0] by the row's own lanes ----
            float part = 0.f, glsp = 0.f;
            {
                constexpr int KPL = H / 16;
                const int i = tid >> 4, pk = tid & 15;
                float2 yv[KPL / 2], wv[KPL / 2];
                float d = 0.f;
#pragma unroll
                for (int h = 0; h < KPL / 2; ++h) {
                    yv[h] = *reinterpret_cast<const float2*>(Y2 + i * P + pk * KPL + 2 * h);
                    wv[h] = *reinterpret_cast<const float2*>(Pp + Ly::oW2 + pk * KPL + 2 * h);
                    d += yv[h].x * wv[h].x + yv[h].y * wv[h].y;
                }
                d = sum16(d);                                  // every lane of the row: y, the head
                float g;
                {
                    const float y = d + Pp[Ly::ob2];
                    if (!a.policy) {                           // loss.cu:5-23
                        const float t = tgt[i], dd = t - y;
                        part = dd * dd;
                        g = 2 * (y - t) / (float)BB;
                    } else {                                   // ppo.cu:82-107, policy.cu:67-111 (A = 1)
                        float gl;
                        const float ls = s_ls;
                        const float lp = log_prob_row(&y, &ls, act + i, 1);
                        part = surrogate(tgt[i], lp, olp[i], a.eps, BB, &gl);
                        const float e2 = expf(-2 * ls);
                        const float dd = act[i] - y;
                        g = dd * e2 * gl;
                        glsp = (-1 + dd * dd * e2) * gl;
                    }
                    if (pk == 0) G3[i] = g;
                    else part = glsp = 0.f;                    // row sums counted once
                }
#pragma unroll
                for (int h = 0; h < KPL / 2; ++h)
                    *reinterpret_cast<float2*>(G2 + i * P + pk * KPL + 2 * h) =
                        float2{yv[h].x > 0.f ? g * wv[h].x : 0.f, yv[h].y > 0.f ? g * wv[h].y : 0.f};
            }
            part = sum64(part);
            if (a.policy) glsp = sum64(glsp);
            if (lane == 0) {
                red[w] = part;
                gls_red[w] = glsp;
            }
            __syncthreads();
            if (a.stamps && tid == 0 && step < 64) a.stamps[64 * 8 + step * 4 + 2] = wall_clock64();
            TINY_STAMP(3);
            // ---- backward (neural_network.cu:121-161), hidden layer 1: this wave's gW1 = G2ᵀ·Y1 and
            // G1 = (G2·W1) ⊙ 1[Y1 > 0] tiles; columns 4w .. 4w+3 of gb1 = Σ_b G2 and gW2 = Σ_b g·Y2
            // (16 row slices of 4 per column, lanes 16s + col); gb2 and the loss sums by wave 15 ----
            {
                f32x4 aw = {0.f, 0.f, 0.f, 0.f}, ax = aw;
                if constexpr (!(PPO_C2_AB & 8)) {
                    aw = c2_tile<BB, false, P, false, P>(G2, ti0, Y1, tj0, lane);
                    ax = c2_tile<H, true, P, false, P>(G2, ti0, Pp + Ly::oW1, tj0, lane);
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int r = ti0 + 4 * q + e, k = tj0 + c;
                    Gd[Ly::oW1 + r * P + k] = aw[e];
                    G1[r * P + k] = Y1[r * P + k] > 0.f ? ax[e] : 0.f;
                }
                static_assert(H == 4 * NWAVES, "four columns per wave");
                const int col = 4 * w + (lane >> 4), rs = lane & 15;    // a DPP row per column, 16 slices
                float sb = 0.f, sw = 0.f;
#pragma unroll
                for (int r = 0; r < BB / 16; ++r) {
                    const int b = rs * (BB / 16) + r;
                    sb += G2[b * P + col];
                    sw += G3[b] * Y2[b * P + col];
                }
                sb = sum16(sb);
                sw = sum16(sw);
                if (rs == 0) {
                    Gd[Ly::ob1 + col] = sb;
                    Gd[Ly::oW2 + col] = sw;
                }
                if (w == NWAVES - 1) {
                    float g = 0.f;
                    for (int b = lane; b < BB; b += 64) g += G3[b];
                    g = sum64(g);
                    if (lane == 0) Gd[Ly::ob2] = g;
                    if (lane == 1) {
                        float sl = 0.f, gl = 0.f;
                        for (int v = 0; v < NWAVES; ++v) { sl += red[v]; gl += gls_red[v]; }
                        if (!a.policy) {
                            atomicAdd(a.stats + 0, sl * (1.0f / (float)BB));
                        } else {
                            const float ent = (float)(0.5 * (1 + log(2 * M_PI))) + s_ls;
                            atomicAdd(a.stats + 1, -sl / BB - a.ent_coeff * ent);
                            s_lsg = gl + -a.ent_coeff;                      // ppo.cu:436-438
                            a.log_std_grad[0] = s_lsg;
                        }
                    }
                }
            }
            __syncthreads();
            if (a.stamps && tid == 0 && step < 64) a.stamps[64 * 8 + step * 4 + 3] = wall_clock64();
            TINY_STAMP(4);
            // ---- layer 0 + Adam (ppo.cu:440-442: entropy first, then the network), one phase: the
            // next minibatch's gather loads go out first; gW0[j][k] = Σ_b G1[b][j]·X0[b][k] and gb0[j]
            // (X0's ones column, k = S) by 16 lanes per j, and the lane holding each of them applies
            // its Adam step at once; every other parameter's gradient is complete since the barrier ----
            int nep = ep, nkb = kb + 1;
            if (nkb >= a.num_batches) { nep = ep + 1; nkb = 0; }
            const bool next = !(PPO_C2_AB & 2) && step + 1 < a.total_steps && nep < a.n_epochs && gt >= 0;
            Row nr{};
            if (next) nr = fetch(nep, nkb);
            const float st = a.steps[2 * step], bc2 = a.steps[2 * step + 1];
            if (!(PPO_C2_AB & 4)) {
                const int j = tid >> 4, rs = tid & 15;
                float s4[SP] = {};
#pragma unroll
                for (int r = 0; r < BB / 16; ++r) {
                    const int b = rs * (BB / 16) + r;
                    const float g = G1[b * P + j];
                    const f32x4 x = *reinterpret_cast<const f32x4*>(X0 + b * SP);
#pragma unroll
                    for (int k = 0; k < SP; ++k) s4[k] += g * x[k];
                }
#pragma unroll
                for (int k = 0; k < SP; ++k) s4[k] = sum16(s4[k]);
                float v = s4[0];
#pragma unroll
                for (int k = 1; k < SP; ++k) v = rs == k ? s4[k] : v;
                if (rs <= S) {
                    const int e = rs < S ? Ly::oW0 + j * SP + rs : Ly::ob0 + j;
                    Gd[e] = v;
                    float pu = Pp[e], mu = Mv[e], vu = Vv[e];
                    adam_elem(pu, v, mu, vu, st, a.b1, a.b2, bc2);
                    Pp[e] = pu; Mv[e] = mu; Vv[e] = vu;
                }
            }
            if (a.policy && tid == TPB / 2) {
                float p = s_ls, mls = s_mls, vls = s_vls;
                adam_elem(p, s_lsg, mls, vls, a.steps_ls[2 * step], a.b1, a.b2, a.steps_ls[2 * step + 1]);
                s_ls = p; s_mls = mls; s_vls = vls;
                a.log_std[0] = p; a.m_ls[0] = mls; a.v_ls[0] = vls;
            }
            // the rest of the image (W1, b1, W2, b2 and their pads), one element per thread per round,
            // the rounds unrolled so their dependent Adam chains interleave
            {
                constexpr int NR = (Ly::NPAR - Ly::oW1 + TPB - 1) / TPB, U = PPO_C2_ADAM_U;
#pragma unroll
                for (int r0 = 0; r0 < NR; r0 += U) {
                    float pu[U], gu[U], mu[U], vu[U];
#pragma unroll
                    for (int r = 0; r < U; ++r) {
                        const int e = min(Ly::oW1 + tid + (r0 + r) * TPB, Ly::NPAR - 1);
                        pu[r] = Pp[e]; gu[r] = Gd[e]; mu[r] = Mv[e]; vu[r] = Vv[e];
                    }
#pragma unroll
                    for (int r = 0; r < U; ++r) {
                        if constexpr (PPO_C2_AB & 1) pu[r] += gu[r] * st;
                        else adam_elem(pu[r], gu[r], mu[r], vu[r], st, a.b1, a.b2, bc2);
                    }
#pragma unroll
                    for (int r = 0; r < U; ++r) {
                        const int e = Ly::oW1 + tid + (r0 + r) * TPB;
                        if (r0 + r < NR && e < Ly::NPAR) { Pp[e] = pu[r]; Mv[e] = mu[r]; Vv[e] = vu[r]; }
                    }
                }
            }
            if (next) put(nr, X0b + ((step + 1) & 1) * (BB * SP));
            __syncthreads();                                   // (LDS only: no global-memory fence)
            TINY_STAMP(5);
        }
    }
    for (int f = tid; f < Ly::NFLAT; f += TPB) {
        const int d = Ly::pad_index(f);
        a.params[f] = Pp[d];
        a.grads[f] = Gd[d];
        a.m[f] = Mv[d];
        a.v[f] = Vv[d];
    }
}

void print_stamps(const TinyArgs& a, const PhipTinyPhase* ph) {
    if (!a.stamps) return;
    {                      // diagnostics: mean µs per phase over steps 1..63
        unsigned long long h[64 * 12];
        phip_d2h(h, a.stamps, sizeof(h));
        int dev = 0, khz = 0;
        PPO_CHECK(hipGetDevice(&dev));
        PPO_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
        const double mhz = khz > 0 ? khz / 1000.0 : 100.0;     // wall_clock64() ticks per µs
        fprintf(stderr, "tiny: wall clock %.1f MHz\n", mhz);
        double acc[5] = {0, 0, 0, 0, 0};
        int n = 0;
        for (int st = 1; st < 64 && st < a.total_steps; ++st, ++n)
            for (int k = 0; k < 5; ++k) acc[k] += (double)(h[st * 8 + k + 1] - h[st * 8 + k]) / mhz;
        const double clk = (double)(h[63 * 8 + 6] - h[1 * 8 + 6]) / ((double)(h[63 * 8] - h[1 * 8]) / mhz);
        if (n) fprintf(stderr, "tiny: shader clock %.0f MHz\n", clk);
        double fl[4] = {0, 0, 0, 0};
        for (int st = 1; st < 64 && st < a.total_steps; ++st) {
            fl[0] += (double)(h[512 + st * 4 + 0] - h[st * 8 + 1]) / mhz;
            fl[1] += (double)(h[512 + st * 4 + 1] - h[512 + st * 4 + 0]) / mhz;
            fl[2] += (double)(h[512 + st * 4 + 2] - h[512 + st * 4 + 1]) / mhz;
            fl[3] += (double)(h[512 + st * 4 + 3] - h[st * 8 + 3]) / mhz;
        }
        if (n) fprintf(stderr, "tiny: sub-phases (us): layer 0 %.2f, layer 1 %.2f, head %.2f, first backward %.2f\n",
                       fl[0] / n, fl[1] / n, fl[2] / n, fl[3] / n);
        if (n)
            fprintf(stderr, "tiny %s step phases (us): gather %.2f fwd %.2f head %.2f bwd %.2f adam %.2f\n",
                    ph->policy ? "policy" : "value", acc[0] / n, acc[1] / n, acc[2] / n, acc[3] / n, acc[4] / n);
    }
}

}  // namespace

extern "C" {

// Returns 0 when launched; −1 if the network does not fit the single-workgroup path (caller falls
// back to the multi-launch loop).
int phip_tiny_update(const PhipTinyNet* net, const PhipTinyPhase* ph) {
    TinyArgs a{};
    if (net->L < 1 || net->L > MAXL || ph->B <= 0 || ph->n_epochs > 16) return -1;
    if (((uintptr_t)net->params | (uintptr_t)net->grads | (uintptr_t)net->m | (uintptr_t)net->v) & 15) return -1;
    a.L = net->L;
    int maxw = 0;
    for (int l = 0; l <= net->L; ++l) {
        a.sizes[l] = net->sizes[l];
        if (net->sizes[l] > 128 || net->sizes[l] <= 0) return -1;
        if (l > 0 && net->sizes[l] > maxw) maxw = net->sizes[l];
    }
    if (net->sizes[net->L] > 32) return -1;
    for (int l = 0; l < net->L; ++l) {
        a.relu[l] = net->relu[l];
        a.woff[l] = net->woff[l];
        a.boff[l] = net->boff[l];
    }
    a.params = net->params; a.grads = net->grads; a.m = net->m; a.v = net->v; a.span = net->span;
    a.wt = net->wt;
    {
        long off = 0;
        for (int l = 0; l < net->L; ++l) {
            a.wtoff[l] = off;
            off += (long)net->sizes[l] * net->sizes[l + 1];
        }
        if (!net->wt || off > net->wt_cap) return -1;
    }
    a.log_std = net->log_std; a.log_std_grad = net->log_std_grad; a.m_ls = net->m_ls; a.v_ls = net->v_ls;
    a.A = net->sizes[net->L];
    a.policy = ph->policy;
    a.state = ph->state; a.action = ph->action; a.logprob = ph->logprob; a.adv = ph->adv;
    a.adv_target = ph->adv_target;
    a.limit = ph->limit; a.B = ph->B; a.num_batches = ph->num_batches; a.n_epochs = ph->n_epochs;
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
    static unsigned long long* stamps = nullptr;
    if (getenv("PPO_TINY_STAMPS")) {
        if (!stamps) stamps = (unsigned long long*)phip_malloc(sizeof(unsigned long long) * 64 * 12);
        a.stamps = stamps;
    }
    // C1/C2 shape (3 → 64 → 64 → 1, ReLU, B = 64, the flat reference layout): the specialised kernel
    {
        using Ly = C2Lay<3, 64, 64>;
        const bool shape = net->L == 3 && net->sizes[0] == 3 && net->sizes[1] == 64 && net->sizes[2] == 64 &&
                           net->sizes[3] == 1 && net->relu[0] && net->relu[1] && !net->relu[2] && ph->B == 64;
        const bool layout = net->woff[0] == 0 && net->boff[0] == Ly::fb0 && net->woff[1] == Ly::fW1 &&
                            net->boff[1] == Ly::fb1 && net->woff[2] == Ly::fW2 && net->boff[2] == Ly::fb2 &&
                            net->span == Ly::NFLAT;
        if (shape && layout && !getenv("PPO_TINY_GENERIC")) {
            const size_t bytes = sizeof(float) * (size_t)Ly::TOTAL;
            static_assert(sizeof(float) * (size_t)Ly::TOTAL <= 160 * 1024 - 1024, "tiny C2: LDS");
            if (ph->n_epochs <= 0 || ph->num_batches <= 0) return 0;     // fit check only
            auto kfn = tiny_c2_kernel<3, 64, 64>;
            static bool attr = false;
            if (!attr) {
                PPO_CHECK(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
                attr = true;
            }
            ppo::ProfScope ps(PPO_K_OTHER, 0.0);
            hipLaunchKernelGGL(kfn, dim3(1), dim3(TPB), bytes, ppo::stream(), a);
            PPO_LAUNCH_CHECK();
            print_stamps(a, ph);
            return 0;
        }
    }
    // LDS: activations [B][w+1] (odd pitch: conflict-free column reads), two gradient buffers, misc
    int off = 0;
    for (int l = 0; l <= net->L; ++l) {
        a.ld[l] = net->sizes[l] | 1;
        a.act_off[l] = off;
        off += ph->B * a.ld[l];
    }
    a.gld = maxw | 1;
    a.g_off[0] = off; off += ph->B * a.gld;
    a.g_off[1] = off; off += ph->B * a.gld;
    a.misc_off = off;
    off += 3 * ph->B + ph->B * a.A;
    off = (off + 3) & ~3;                                    // 16-B alignment for the float4 Adam loop
    long nw = 0;
    for (int l = 0; l < net->L; ++l) nw += (long)net->sizes[l] * net->sizes[l + 1];
    const long res = 4 * ((net->span + 3) & ~3L) + nw;
    const size_t kMaxLds = 160 * 1024 - 1024;              // the CU's 160 KiB less the static arrays
    const bool resident = (size_t)(off + res) * sizeof(float) <= kMaxLds;
    a.res_off = off;
    const size_t bytes = sizeof(float) * (size_t)(resident ? off + res : off);
    if (bytes > kMaxLds) return -1;
    if (ph->n_epochs <= 0 || ph->num_batches <= 0) return 0;     // fit check only
    const void* kfn = resident ? (const void*)tiny_update_kernel<true> : (const void*)tiny_update_kernel<false>;
    PPO_CHECK(hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    ppo::ProfScope ps(PPO_K_OTHER, 0.0);
    if (resident) hipLaunchKernelGGL(tiny_update_kernel<true>, dim3(1), dim3(TPB), bytes, ppo::stream(), a);
    else hipLaunchKernelGGL(tiny_update_kernel<false>, dim3(1), dim3(TPB), bytes, ppo::stream(), a);
    PPO_LAUNCH_CHECK();
    print_stamps(a, ph);
    return 0;
}

}  // extern "C"
