// adam.hip — Adam as one streaming pass over a flat parameter span (HBM-bound, 28 B/param).
//
// Reference: adam_update (adam.cu:53-74) and adam_update_kernel (adam.cu:138-169, K10), which
// finds each element's layer by a linear search over prefix lengths through a device float**.
// libppo networks keep W and b of every layer in one contiguous buffer, so the update is a
// single float4-vectorised kernel; a multi-tensor variant covers arbitrary tensor lists.
//
// Arithmetic is the reference's, operation for operation (compiled without FMA contraction):
//   m = β1·m + (1−β1)·g;  v = β2·v + (1−β2)·g²;
//   denom = (float)(sqrtf(v/bc2) + 1e-8)   (double add, as in C);   p −= step·m/denom
// so that, given identical gradients, parameters match the oracle bit for bit.
#include "dev.h"

namespace {

constexpr int TPB = 256;

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float step, float b1, float b2,
                                          float bc2, float scale) {
    g = g * scale;
    m = b1 * m + (1 - b1) * g;
    v = b2 * v + (1 - b2) * (g * g);
    const float denom = (float)((double)sqrtf(v / bc2) + 1e-8);
    p -= step * m / denom;
}

// n elements: float4 body plus a scalar tail (a network's span ends with its unpadded output bias).
// w16 (bf16 mode): the parameters' bf16 shadow for the first n16 elements, written in the same pass.
// zero_g: the gradient is cleared once read (ppo_update: the next backward's split-K atomics then
// accumulate into zeros without a memset launch per minibatch step).
__device__ __forceinline__ void adam_vec_body(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                              float* __restrict__ v, long n, float step, float b1, float b2,
                                              float bc2, float scale, __bf16* __restrict__ w16, long n16,
                                              int zero_g) {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    const long n4 = n >> 2;
    for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < n4; i += (long)gridDim.x * TPB) {
        float4 pp = reinterpret_cast<float4*>(p)[i], gg = reinterpret_cast<const float4*>(g)[i];
        float4 mm = reinterpret_cast<float4*>(m)[i], vv = reinterpret_cast<float4*>(v)[i];
        adam_elem(pp.x, gg.x, mm.x, vv.x, step, b1, b2, bc2, scale);
        adam_elem(pp.y, gg.y, mm.y, vv.y, step, b1, b2, bc2, scale);
        adam_elem(pp.z, gg.z, mm.z, vv.z, step, b1, b2, bc2, scale);
        adam_elem(pp.w, gg.w, mm.w, vv.w, step, b1, b2, bc2, scale);
        reinterpret_cast<float4*>(p)[i] = pp;
        reinterpret_cast<float4*>(m)[i] = mm;
        reinterpret_cast<float4*>(v)[i] = vv;
        if (zero_g) reinterpret_cast<float4*>(g)[i] = float4{0.f, 0.f, 0.f, 0.f};
        if (w16 && 4 * i < n16) {
            if (4 * i + 4 <= n16) {
                bf16x4 o = {(__bf16)pp.x, (__bf16)pp.y, (__bf16)pp.z, (__bf16)pp.w};
                reinterpret_cast<bf16x4*>(w16)[i] = o;
            } else {
                const float e[4] = {pp.x, pp.y, pp.z, pp.w};
                for (long j = 4 * i; j < n16; ++j) w16[j] = (__bf16)e[j - 4 * i];
            }
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
        const long j = 4 * n4 + threadIdx.x;
        float pp = p[j], mm = m[j], vv = v[j];
        adam_elem(pp, g[j], mm, vv, step, b1, b2, bc2, scale);
        p[j] = pp; m[j] = mm; v[j] = vv;
        if (zero_g) g[j] = 0.f;
        if (w16 && j < n16) w16[j] = (__bf16)pp;
    }
}

__global__ void adam_flat_vec_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                     float* __restrict__ v, long n, float step, float b1, float b2, float bc2,
                                     float scale, __bf16* __restrict__ w16, long n16, int zero_g) {
    adam_vec_body(p, g, m, v, n, step, b1, b2, bc2, scale, w16, n16, zero_g);
}

// a second, small flat span in the same launch (the policy step's entropy Adam beside the network's,
// ppo.cu:440-442 — independent parameters): the last workgroup's first s.n threads, scalar
struct SideSpan {
    float* p; float* g; float* m; float* v; int n; float step, bc2, scale; int zero_g;
};
__global__ void adam_flat_vec_pair_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                          float* __restrict__ v, long n, float step, float b1, float b2, float bc2,
                                          float scale, __bf16* __restrict__ w16, long n16, int zero_g, SideSpan s) {
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x < s.n) {
        const int j = threadIdx.x;
        float pp = s.p[j], mm = s.m[j], vv = s.v[j];
        adam_elem(pp, s.g[j], mm, vv, s.step, b1, b2, s.bc2, s.scale);
        s.p[j] = pp; s.m[j] = mm; s.v[j] = vv;
        if (s.zero_g) s.g[j] = 0.f;
    }
    adam_vec_body(p, g, m, v, n, step, b1, b2, bc2, scale, w16, n16, zero_g);
}

// the flat Adam with its step size / bias correction from the step table (graph replay); which = 0
// (the network's Adam) also advances the step counter: its last workgroup to finish, after every
// workgroup has read the entry (a workgroup takes its ticket only at its end)
__global__ void adam_flat_tab_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                     float* __restrict__ v, long n, const PhipStepArgs* __restrict__ tab, int* ctr,
                                     unsigned* ticket, int which, float b1, float b2, float scale,
                                     __bf16* __restrict__ w16, long n16, int zero_g) {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    const PhipStepArgs& s = tab[*ctr];
    const float step = which ? s.step_ls : s.step, bc2 = which ? s.bc2_ls : s.bc2;
    const long n4 = n >> 2;
    for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < n4; i += (long)gridDim.x * TPB) {
        float4 pp = reinterpret_cast<float4*>(p)[i], gg = reinterpret_cast<const float4*>(g)[i];
        float4 mm = reinterpret_cast<float4*>(m)[i], vv = reinterpret_cast<float4*>(v)[i];
        adam_elem(pp.x, gg.x, mm.x, vv.x, step, b1, b2, bc2, scale);
        adam_elem(pp.y, gg.y, mm.y, vv.y, step, b1, b2, bc2, scale);
        adam_elem(pp.z, gg.z, mm.z, vv.z, step, b1, b2, bc2, scale);
        adam_elem(pp.w, gg.w, mm.w, vv.w, step, b1, b2, bc2, scale);
        reinterpret_cast<float4*>(p)[i] = pp;
        reinterpret_cast<float4*>(m)[i] = mm;
        reinterpret_cast<float4*>(v)[i] = vv;
        if (zero_g) reinterpret_cast<float4*>(g)[i] = float4{0.f, 0.f, 0.f, 0.f};
        if (w16 && 4 * i + 4 <= n16) {
            bf16x4 o = {(__bf16)pp.x, (__bf16)pp.y, (__bf16)pp.z, (__bf16)pp.w};
            reinterpret_cast<bf16x4*>(w16)[i] = o;
        } else if (w16 && 4 * i < n16) {
            const float e[4] = {pp.x, pp.y, pp.z, pp.w};
            for (long j = 4 * i; j < n16; ++j) w16[j] = (__bf16)e[j - 4 * i];
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
        const long j = 4 * n4 + threadIdx.x;
        float pp = p[j], mm = m[j], vv = v[j];
        adam_elem(pp, g[j], mm, vv, step, b1, b2, bc2, scale);
        p[j] = pp; m[j] = mm; v[j] = vv;
        if (zero_g) g[j] = 0.f;
        if (w16 && j < n16) w16[j] = (__bf16)pp;
    }
    if (which == 0) {
        __syncthreads();                                   // every wave of this workgroup read the entry
        if (threadIdx.x == 0) {
            const unsigned t = atomicAdd(ticket, 1u);
            if (t == gridDim.x - 1) {                      // the last workgroup: all have read it
                *ticket = 0u;
                *ctr += 1;
            }
        }
    }
}

__global__ void adam_flat_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                 float* __restrict__ v, long n, float step, float b1, float b2, float bc2,
                                 float scale) {
    for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < n; i += (long)gridDim.x * TPB) {
        float pp = p[i], mm = m[i], vv = v[i];
        adam_elem(pp, g[i], mm, vv, step, b1, b2, bc2, scale);
        p[i] = pp; m[i] = mm; v[i] = vv;
    }
}

constexpr int MAXT = 24;
struct TensorTable {
    float* p[MAXT];
    const float* g[MAXT];
    long start[MAXT + 1];        // prefix offsets into the flat m / v
    int count;
};

__global__ void adam_multi_kernel(TensorTable t, float* __restrict__ m, float* __restrict__ v, float step, float b1,
                                  float b2, float bc2, float scale) {
    const long total = t.start[t.count];
    for (long i = blockIdx.x * (long)TPB + threadIdx.x; i < total; i += (long)gridDim.x * TPB) {
        int k = 0;
        while (i >= t.start[k + 1]) ++k;           // ≤ 24 tensors, uniform-ish
        const long j = i - t.start[k];
        float pp = t.p[k][j], mm = m[i], vv = v[i];
        adam_elem(pp, t.g[k][j], mm, vv, step, b1, b2, bc2, scale);
        t.p[k][j] = pp; m[i] = mm; v[i] = vv;
    }
}

int grid_for(long n) {
    long g = (n + TPB - 1) / TPB;
    if (g < 1) g = 1;
    if (g > 2048) g = 2048;
    return (int)g;
}

}  // namespace

extern "C" {

void phip_adam_flat_w16(float* p, float* g, float* m, float* v, long n, float lr, float beta1, float beta2,
                        float bias_correction1, float bias_correction2, float grad_scale, unsigned short* w16,
                        long n16, int zero_g) {
    if (n <= 0) return;
    const float step = lr / bias_correction1;
    ppo::ProfScope ps(PPO_K_ADAM, 28.0 * n + (w16 ? 2.0 * n16 : 0.0) + (zero_g ? 4.0 * n : 0.0));
    const bool vec = (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15u) == 0 &&
                     ((uintptr_t)w16 & 7u) == 0;
    if (vec) {
        hipLaunchKernelGGL(adam_flat_vec_kernel, dim3(grid_for((n + 3) / 4)), dim3(TPB), 0, ppo::stream(), p, g, m,
                           v, n, step, beta1, beta2, bias_correction2, grad_scale,
                           reinterpret_cast<__bf16*>(w16), n16, zero_g);
    } else {
        PPO_REQUIRE(!w16 && !zero_g, "phip_adam_flat_w16: unaligned span with a bf16 shadow or gradient clear");
        hipLaunchKernelGGL(adam_flat_kernel, dim3(grid_for(n)), dim3(TPB), 0, ppo::stream(), p, g, m, v, n, step,
                           beta1, beta2, bias_correction2, grad_scale);
    }
    PPO_LAUNCH_CHECK();
}

void phip_adam_flat_pair(float* p, float* g, float* m, float* v, long n, float lr, float beta1, float beta2,
                         float bias_correction1, float bias_correction2, float grad_scale, unsigned short* w16,
                         long n16, int zero_g, float* p2, float* g2, float* m2, float* v2, int n2, float lr2,
                         float bias_correction1_2, float bias_correction2_2, float grad_scale2, int zero_g2) {
    PPO_REQUIRE(n > 0 && n2 >= 0 && n2 <= TPB, "phip_adam_flat_pair: spans");
    PPO_REQUIRE((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15u) == 0 && ((uintptr_t)w16 & 7u) == 0,
                "phip_adam_flat_pair: the network span must be 16-B aligned");
    ppo::ProfScope ps(PPO_K_ADAM, 28.0 * (n + n2) + (w16 ? 2.0 * n16 : 0.0) + (zero_g ? 4.0 * n : 0.0));
    SideSpan s{p2, g2, m2, v2, n2, lr2 / bias_correction1_2, bias_correction2_2, grad_scale2, zero_g2};
    hipLaunchKernelGGL(adam_flat_vec_pair_kernel, dim3(grid_for((n + 3) / 4)), dim3(TPB), 0, ppo::stream(), p, g, m,
                       v, n, lr / bias_correction1, beta1, beta2, bias_correction2, grad_scale,
                       reinterpret_cast<__bf16*>(w16), n16, zero_g, s);
    PPO_LAUNCH_CHECK();
}

void phip_adam_flat_tab(float* p, float* g, float* m, float* v, long n, const PhipStepArgs* tab, int* ctr,
                        unsigned* ticket, int which, float beta1, float beta2, float grad_scale, unsigned short* w16,
                        long n16, int zero_g) {
    if (n <= 0) return;
    PPO_REQUIRE((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15u) == 0 && ((uintptr_t)w16 & 7u) == 0,
                "phip_adam_flat_tab: unaligned span");
    hipLaunchKernelGGL(adam_flat_tab_kernel, dim3(grid_for((n + 3) / 4)), dim3(TPB), 0, ppo::stream(), p, g, m, v, n,
                       tab, ctr, ticket, which, beta1, beta2, grad_scale, reinterpret_cast<__bf16*>(w16), n16, zero_g);
    PPO_LAUNCH_CHECK();
}

void phip_adam_flat(float* p, const float* g, float* m, float* v, long n, float lr, float beta1, float beta2,
                    float bias_correction1, float bias_correction2, float grad_scale) {
    phip_adam_flat_w16(p, const_cast<float*>(g), m, v, n, lr, beta1, beta2, bias_correction1, bias_correction2,
                       grad_scale, nullptr, 0, 0);
}

void phip_adam_multi(float* const* params, float* const* grads, const int* lengths, int num_tensors, float* m,
                     float* v, float lr, float beta1, float beta2, float bias_correction1, float bias_correction2,
                     float grad_scale) {
    const float step = lr / bias_correction1;
    long base = 0;
    for (int t0 = 0; t0 < num_tensors; t0 += MAXT) {
        TensorTable t{};
        t.count = num_tensors - t0 < MAXT ? num_tensors - t0 : MAXT;
        t.start[0] = 0;
        for (int k = 0; k < t.count; ++k) {
            t.p[k] = params[t0 + k];
            t.g[k] = grads[t0 + k];
            t.start[k + 1] = t.start[k] + lengths[t0 + k];
        }
        const long total = t.start[t.count];
        if (total > 0) {
            ppo::ProfScope ps(PPO_K_ADAM, 28.0 * total);
            hipLaunchKernelGGL(adam_multi_kernel, dim3(grid_for(total)), dim3(TPB), 0, ppo::stream(), t, m + base,
                               v + base, step, beta1, beta2, bias_correction2, grad_scale);
            PPO_LAUNCH_CHECK();
        }
        base += total;
    }
}

}  // extern "C"
