// dev.h — internal helpers shared by libppo's HIP translation units (gfx950 only).
//
// Everything here is device-runtime plumbing: the single libppo stream, error
// recording ("fail loudly", SURVEY §8b Errors) and the optional per-launch HIP
// event timing used by bench.py's roofline (ppo_prof_*).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#include "ppo_hip.h"
#include "../../include/ppo_ext.h"

namespace ppo {

hipStream_t stream();                       // libppo's stream (created on first use)
void        ensure_device();                // aborts with a clear message without a HIP device
void        check(hipError_t e, const char* what, const char* file, int line);
void        fail(const char* msg, const char* file, int line);   // records + aborts

// Per-launch timing: begin() records a start event when profiling is on; end()
// records the stop event and attributes `work` (FLOPs or bytes) to class k.
struct ProfScope {
    int k; double work; int slot;
    ProfScope(int k_, double work_);
    ~ProfScope();
};

}  // namespace ppo

#define PPO_CHECK(x) ::ppo::check((x), #x, __FILE__, __LINE__)
#define PPO_LAUNCH_CHECK() ::ppo::check(hipGetLastError(), "kernel launch", __FILE__, __LINE__)
#define PPO_REQUIRE(cond, msg) do { if (!(cond)) ::ppo::fail((msg), __FILE__, __LINE__); } while (0)

static inline int ppo_divup(long a, long b) { return (int)((a + b - 1) / b); }
