// dpp_check.hip — on-device check of the cross-lane primitives the x3 value-head fold's reduce-scatter
// uses (v_permlane16_swap, DPP row_mirror / row_half_mirror / quad_perm): prints which lane each one reads
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CTRL>
__device__ float dpp_mov(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}

__global__ void k(float* out) {
    const int l = threadIdx.x;
    const float x = (float)l;
    const unsigned u = __builtin_bit_cast(unsigned, x);
    const auto s = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    out[0 * 64 + l] = __builtin_bit_cast(float, s[0]);
    out[1 * 64 + l] = __builtin_bit_cast(float, s[1]);
    out[2 * 64 + l] = dpp_mov<0x140>(x);
    out[3 * 64 + l] = dpp_mov<0x141>(x);
    out[4 * 64 + l] = dpp_mov<0x4E>(x);
    out[5 * 64 + l] = dpp_mov<0xB1>(x);
    unsigned y;
    asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "v"(u));     // a distinct register holding the same value
    const auto s2 = __builtin_amdgcn_permlane16_swap(u, y, false, false);
    out[6 * 64 + l] = __builtin_bit_cast(float, s2[0]) + __builtin_bit_cast(float, s2[1]);
}

int main() {
    float* d;
    float h[7 * 64];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    const char* names[7] = {"permlane16_swap[0]", "permlane16_swap[1]", "row_mirror", "row_half_mirror", "quad 0x4E",
                            "quad 0xB1", "swap sum (copy)"};
    for (int r = 0; r < 7; ++r) {
        printf("%-20s", names[r]);
        for (int l = 0; l < 64; ++l) printf(" %2d", (int)h[r * 64 + l]);
        printf("\n");
    }
    (void)hipFree(d);
    return 0;
}
