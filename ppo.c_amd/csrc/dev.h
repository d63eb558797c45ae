// dev.h — internal helpers shared by libppo's HIP translation units (gfx950 only).
//
// Everything here is device-runtime plumbing: the single libppo stream, error
// recording ("fail loudly", SURVEY §8b Errors) and the optional per-launch HIP
// event timing used by bench.py's roofline (ppo_prof_*).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdint>
#include <cstdio>

#include "ppo_hip.h"
#include "../../include/ppo_ext.h"

namespace ppo {

hipStream_t stream();                       // libppo's stream (created on first use)
void        ensure_device();                // aborts with a clear message without a HIP device
void        check(hipError_t e, const char* what, const char* file, int line);
void        fail(const char* msg, const char* file, int line);   // records + aborts
// bit 0: libppo's main stream still has work queued, bit 1: the side stream (hipStreamQuery; an
// error other than "not ready" is fatal).  For bounded waits (comm.hip's watchdog).
int         streams_pending();

// Per-launch timing: begin() records a start event when profiling is on; end()
// records the stop event and attributes `work` (FLOPs or bytes) to class k.
struct ProfScope {
    int k; double work; int slot;
    ProfScope(int k_, double work_, long long key = 0);   // key: shape tag (gemm_key) for per-shape stats
    ~ProfScope();
};

// Kernel-attached timing (ppo_prof_kernel_events): a sampled GEMM scope records no events of its own;
// its one kernel is launched through PPO_TIMED_LAUNCH, whose start/stop events are stamped by the
// dispatch itself (hipExtLaunchKernel) — the kernel's own duration, as rocprofv3 reports it.
bool take_kernel_events(hipEvent_t* start, hipEvent_t* stop);

// split-K grad_W partials (gemm_x3.hip): a per-stream scratch of `floats` floats, and
// out[i] = Σ_s slab[s·stride + i] for i < n in a fixed order (stride % 4 == 0, 16-B aligned slab and
// out); `stop`: an event recorded by the reduce's dispatch (or null)
float* slab_scratch(size_t floats);
void slab_reduce(const float* slab, float* out, long n, long stride, int splits, hipEvent_t stop);

// shape tag of a GEMM launch: op (0 fwd, 1 grad_x, 2 grad_W, 3 paired bwd) [60..63] | engine [56..59] |
// m [32..55] | n [16..31] | l [0..15]; fields masked so an out-of-range width cannot alias another shape
inline long long gemm_key(int op, int engine, long m, long n, long l) {
    return ((long long)(op & 0xF) << 60) | ((long long)(engine & 0xF) << 56) | ((long long)(m & 0xFFFFFF) << 32) |
           ((long long)(n & 0xFFFF) << 16) | (long long)(l & 0xFFFF);
}

// Cross-lane sums on DPP moves (no LDS round trips; a __shfl_xor tree compiles to ds_bpermute,
// ≈ 100+ cycles of latency per step): sum over each 16-lane DPP row — the xor-1 / xor-2 / quad-swap /
// half-swap tree — and over the wave (row sums in row order, read as scalars)
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float row_sum16(float v) {
    v += dpp_mov<0xB1>(v);            // quad_perm [1,0,3,2]
    v += dpp_mov<0x4E>(v);            // quad_perm [2,3,0,1]
    v += dpp_mov<0x141>(v);           // row_half_mirror
    v += dpp_mov<0x140>(v);           // row_mirror
    return v;
}
__device__ __forceinline__ float lane_value(float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
__device__ __forceinline__ float wave_sum64(float v) {
    v = row_sum16(v);
    return ((lane_value(v, 0) + lane_value(v, 16)) + lane_value(v, 32)) + lane_value(v, 48);
}

}  // namespace ppo

#define PPO_TIMED_LAUNCH(kernel, grid, block, lds, strm, ...)                                         \
    do {                                                                                           \
        hipEvent_t ppo_e0_, ppo_e1_;                                                               \
        if (::ppo::take_kernel_events(&ppo_e0_, &ppo_e1_))                                         \
            hipExtLaunchKernelGGL(kernel, grid, block, lds, strm, ppo_e0_, ppo_e1_, 0, __VA_ARGS__); \
        else                                                                                       \
            hipLaunchKernelGGL(kernel, grid, block, lds, strm, __VA_ARGS__);                       \
    } while (0)

#define PPO_CHECK(x) ::ppo::check((x), #x, __FILE__, __LINE__)
#define PPO_LAUNCH_CHECK() ::ppo::check(hipGetLastError(), "kernel launch", __FILE__, __LINE__)
#define PPO_REQUIRE(cond, msg) do { if (!(cond)) ::ppo::fail((msg), __FILE__, __LINE__); } while (0)

static inline int ppo_divup(long a, long b) { return (int)((a + b - 1) / b); }
