// mfma_peak.hip — measures the attainable fp32 / bf16 MFMA rate on this MI355X (the `peak`
// cross-check for bench.py's roofline): every CU runs 4 waves (one per SIMD), each issuing
// independent v_mfma_f32_32x32x2_f32 (or v_mfma_f32_32x32x16_bf16) chains on random operands.
//   hipcc --offload-arch=gfx950 -O3 -Wno-unused-result tools/mfma_peak.hip -o bin/mfma_peak && bin/mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int ITERS>
__global__ __launch_bounds__(256) void f32_loop(float* out, float seed) {
    f32x16 acc[4];
    for (int c = 0; c < 4; ++c)
        for (int e = 0; e < 16; ++e) acc[c][e] = 0.f;
    float a = seed * (threadIdx.x + 1), b = seed * (threadIdx.x + 3);
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[c], 0, 0, 0);
    }
    float s = 0.f;
    for (int c = 0; c < 4; ++c)
        for (int e = 0; e < 16; ++e) s += acc[c][e];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int ITERS>
__global__ __launch_bounds__(256) void bf16_loop(float* out, float seed) {
    f32x16 acc[4];
    for (int c = 0; c < 4; ++c)
        for (int e = 0; e < 16; ++e) acc[c][e] = 0.f;
    bf16x8 a, b;
    for (int e = 0; e < 8; ++e) {
        a[e] = (__bf16)(seed * (threadIdx.x + e));
        b[e] = (__bf16)(seed * (threadIdx.x + 2 * e));
    }
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[c], 0, 0, 0);
    }
    float s = 0.f;
    for (int c = 0; c < 4; ++c)
        for (int e = 0; e < 16; ++e) s += acc[c][e];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const int grid = ncu;  // one 4-wave workgroup per CU = one wave per SIMD
    float* out;
    hipMalloc(&out, sizeof(float) * grid * 256);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    constexpr int IT = 20000;
    for (int pass = 0; pass < 2; ++pass) {
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(e0);
            if (pass == 0) f32_loop<IT><<<grid, 256>>>(out, 0.37f);
            else bf16_loop<IT><<<grid, 256>>>(out, 0.37f);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0.f;
            hipEventElapsedTime(&ms, e0, e1);
            const double flop_per_mfma = pass == 0 ? 2.0 * 32 * 32 * 2 : 2.0 * 32 * 32 * 16;
            const double flops = flop_per_mfma * 4.0 * IT * 4.0 * grid;   // 4 chains x 4 waves
            printf("{\"mfma\": \"%s\", \"cus\": %d, \"ms\": %.3f, \"tflops\": %.1f}\n",
                   pass == 0 ? "v_mfma_f32_32x32x2_f32" : "v_mfma_f32_32x32x16_bf16", ncu, ms,
                   flops / (ms * 1e-3) / 1e12);
        }
    }
    hipFree(out);
    return 0;
}
