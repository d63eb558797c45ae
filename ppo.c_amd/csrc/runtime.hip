// runtime.hip — libppo device runtime: device/stream ownership, HBM allocation,
// copies, error recording and per-launch event timing.
//
// One process drives one MI355X (data parallelism is one process per GPU,
// SURVEY §8e).  All work is issued on a single non-blocking stream so the host
// orchestration never blocks except where the reference API returns a value
// that lives on the device (e.g. mean_squared_error_cuda).
#include "dev.h"
#include "../../include/ppo_ext.h"

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>
#include <unistd.h>

namespace ppo {

static int          g_device = -1;
static hipStream_t  g_stream = nullptr;
static hipStream_t  g_side = nullptr;        // second queue for independent work (grad_W beside grad_x)
static int          g_use_side = 0;
static hipEvent_t   g_fork_ev = nullptr, g_join_ev = nullptr;
static char         g_err[512] = "";
static std::once_flag g_init_once;

void fail(const char* msg, const char* file, int line) {
    if (!g_err[0]) snprintf(g_err, sizeof(g_err), "%s (%s:%d)", msg, file, line);
    fprintf(stderr, "libppo: FATAL: %s (%s:%d)\n", msg, file, line);
    fflush(stderr);
    // drain work already queued so the process never dies with kernels in flight
    if (g_stream) (void)hipStreamSynchronize(g_stream);
    if (g_side) (void)hipStreamSynchronize(g_side);
    fflush(stdout);
    _exit(1);                              // the reference's checks exit(1) (cuda_helper.h:4-16)
}

void check(hipError_t e, const char* what, const char* file, int line) {
    if (e == hipSuccess) return;
    char buf[400];
    snprintf(buf, sizeof(buf), "%s failed: %s", what, hipGetErrorString(e));
    fail(buf, file, line);
}

static void init_impl() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        fail("no HIP device visible: libppo runs only on an AMD Instinct MI355X (gfx950)", __FILE__, __LINE__);
    if (g_device < 0) {
        const char* env = getenv("LOCAL_RANK");
        g_device = env ? atoi(env) % n : 0;
    }
    PPO_CHECK(hipSetDevice(g_device));
    hipDeviceProp_t prop;
    PPO_CHECK(hipGetDeviceProperties(&prop, g_device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        char buf[256];
        snprintf(buf, sizeof(buf), "device %d is %s; libppo is built for gfx950 (MI355X) only", g_device,
                 prop.gcnArchName);
        fail(buf, __FILE__, __LINE__);
    }
    PPO_CHECK(hipStreamCreateWithFlags(&g_stream, hipStreamNonBlocking));
    PPO_CHECK(hipStreamCreateWithFlags(&g_side, hipStreamNonBlocking));
    PPO_CHECK(hipEventCreateWithFlags(&g_fork_ev, hipEventDisableTiming));
    PPO_CHECK(hipEventCreateWithFlags(&g_join_ev, hipEventDisableTiming));
}

void ensure_device() { std::call_once(g_init_once, init_impl); }

hipStream_t stream() {
    ensure_device();
    return g_use_side ? g_side : g_stream;
}

int streams_pending() {
    ensure_device();
    int mask = 0;
    const hipStream_t s[2] = {g_stream, g_side};
    for (int i = 0; i < 2; i++) {
        const hipError_t e = hipStreamQuery(s[i]);
        if (e == hipErrorNotReady) mask |= 1 << i;
        else if (e != hipSuccess) check(e, "hipStreamQuery", __FILE__, __LINE__);
    }
    return mask;
}

// ---------------- per-launch event timing ----------------
struct ProfSlot { hipEvent_t a, b; int k; double work; long long key; int ext; };   // ext: 1 awaiting, 2 stamped
static bool                  g_prof_on = false;
static bool                  g_prof_kattach = false;      // GEMM scopes timed by their kernel's dispatch
static int                   g_pending = -1;              // slot awaiting a PPO_TIMED_LAUNCH
struct ShapeStat { long long key; double ms; long launches; double work; };
static std::vector<ShapeStat> g_shapes;
static std::vector<std::pair<long long, long>> g_shape_issued;   // every launch per shape, sampled or not
static int                   g_prof_stride = 1;
static long                  g_issued[PPO_K_COUNT];
static double                g_issued_work[PPO_K_COUNT];   // algorithmic work of every issued launch
static std::vector<ProfSlot> g_slots;       // recorded, not yet harvested
static std::vector<hipEvent_t> g_free_events;
static double g_ms[PPO_K_COUNT], g_work[PPO_K_COUNT];
static long   g_launches[PPO_K_COUNT];

static hipEvent_t take_event() {
    if (!g_free_events.empty()) { hipEvent_t e = g_free_events.back(); g_free_events.pop_back(); return e; }
    hipEvent_t e;
    PPO_CHECK(hipEventCreate(&e));
    return e;
}

static void harvest() {
    if (g_slots.empty()) return;
    PPO_CHECK(hipStreamSynchronize(g_stream));
    PPO_CHECK(hipStreamSynchronize(g_side));
    for (auto& s : g_slots) {
        g_free_events.push_back(s.a);
        g_free_events.push_back(s.b);
        if (s.ext == 1) continue;                 // its scope launched no timed kernel: not measured
        float ms = 0.f;
        PPO_CHECK(hipEventElapsedTime(&ms, s.a, s.b));
        g_ms[s.k] += ms;
        g_work[s.k] += s.work;
        g_launches[s.k] += 1;
        if (s.key) {
            ShapeStat* st = nullptr;
            for (auto& x : g_shapes) if (x.key == s.key) { st = &x; break; }
            if (!st) { g_shapes.push_back(ShapeStat{s.key, 0.0, 0, 0.0}); st = &g_shapes.back(); }
            st->ms += ms;
            st->launches += 1;
            st->work += s.work;
        }
    }
    g_slots.clear();
}

ProfScope::ProfScope(int k_, double work_, long long key) : k(k_), work(work_), slot(-1) {
    slot = phip_prof_begin_key(k, work, key);
}
ProfScope::~ProfScope() { phip_prof_end(slot); }

bool take_kernel_events(hipEvent_t* start, hipEvent_t* stop) {
    if (g_pending < 0 || g_pending >= (int)g_slots.size()) return false;
    ProfSlot& s = g_slots[g_pending];
    g_pending = -1;
    if (s.ext != 1) return false;
    s.ext = 2;
    *start = s.a;
    *stop = s.b;
    return true;
}

}  // namespace ppo

using namespace ppo;

extern "C" {

static int g_capturing = 0;                  // a hipGraph capture is open on libppo's stream

int phip_prof_begin_key(int cls, double work, long long key) {
    if (!g_prof_on || g_capturing) return -1;
    g_issued_work[cls] += work;
    if (key) {
        bool found = false;
        for (auto& x : g_shape_issued)
            if (x.first == key) { x.second++; found = true; break; }
        if (!found) g_shape_issued.emplace_back(key, 1L);
    }
    if (g_issued[cls]++ % g_prof_stride != 0) return -1;
    if (g_slots.size() >= (1u << 16)) harvest();
    const int ext = g_prof_kattach && cls == PPO_K_GEMM ? 1 : 0;
    ProfSlot s{take_event(), take_event(), cls, work, key, ext};
    if (!ext) PPO_CHECK(hipEventRecord(s.a, stream()));
    g_slots.push_back(s);
    const int idx = (int)g_slots.size() - 1;
    if (ext) g_pending = idx;
    return idx;
}

int phip_prof_begin(int cls, double work) { return phip_prof_begin_key(cls, work, 0); }

void phip_prof_end(int slot) {
    if (slot < 0 || !g_prof_on || slot >= (int)g_slots.size()) return;
    if (slot == g_pending) g_pending = -1;
    if (g_slots[slot].ext) return;               // stamped by the kernel's dispatch (or unmeasured)
    PPO_CHECK(hipEventRecord(g_slots[slot].b, stream()));
}

void phip_init(void) { ensure_device(); }

// why the last capture failed (graph replay is an opt-in speed feature: its failure is a warning with
// this text, not a recorded library error)
static char g_graph_err[256] = "";
const char* phip_graph_error(void) { return g_graph_err; }

static void graph_fail(const char* what, hipError_t e) {
    snprintf(g_graph_err, sizeof(g_graph_err), "%s: %s", what, hipGetErrorString(e));
    (void)hipGetLastError();
}

int phip_graph_begin(void) {
    if (g_capturing) {
        snprintf(g_graph_err, sizeof(g_graph_err), "hipStreamBeginCapture: a capture is already open");
        return -1;
    }
    const hipError_t e = hipStreamBeginCapture(stream(), hipStreamCaptureModeRelaxed);
    if (e != hipSuccess) {
        graph_fail("hipStreamBeginCapture", e);
        return -1;
    }
    g_capturing = 1;
    return 0;
}

void* phip_graph_end(void) {
    if (!g_capturing) {
        snprintf(g_graph_err, sizeof(g_graph_err), "hipStreamEndCapture: no capture open");
        return nullptr;
    }
    hipGraph_t graph = nullptr;
    g_capturing = 0;
    hipError_t e = hipStreamEndCapture(stream(), &graph);
    if (e != hipSuccess || !graph) {
        graph_fail("hipStreamEndCapture", e != hipSuccess ? e : hipErrorInvalidValue);
        return nullptr;
    }
    hipGraphExec_t exec = nullptr;
    e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (e != hipSuccess) {
        graph_fail("hipGraphInstantiate", e);
        return nullptr;
    }
    return (void*)exec;
}

void phip_graph_launch(void* exec) { PPO_CHECK(hipGraphLaunch((hipGraphExec_t)exec, stream())); }

void phip_graph_destroy(void* exec) {
    if (exec) PPO_CHECK(hipGraphExecDestroy((hipGraphExec_t)exec));
}

int phip_capturing(void) { return g_capturing; }

void* phip_malloc(size_t bytes) {
    ensure_device();
    void* p = nullptr;
    if (bytes == 0) bytes = 256;
    PPO_CHECK(hipMalloc(&p, bytes));
    PPO_CHECK(hipMemsetAsync(p, 0, bytes, stream()));   // ordered before this stream's first use
    return p;
}

void phip_free(void* p) {
    if (!p) return;
    phip_sync();
    PPO_CHECK(hipFree(p));
}

void phip_h2d(void* dst, const void* src, size_t bytes) {
    if (!bytes) return;
    PPO_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, stream()));
    PPO_CHECK(hipStreamSynchronize(stream()));   // the host buffer may be reused right after
}

void phip_d2h(void* dst, const void* src, size_t bytes) {
    if (!bytes) return;
    PPO_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, stream()));
    PPO_CHECK(hipStreamSynchronize(stream()));
}

void phip_d2d(void* dst, const void* src, size_t bytes) {
    if (!bytes || dst == src) return;
    PPO_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, stream()));
}

void phip_memset(void* dst, int value, size_t bytes) {
    if (!bytes) return;
    PPO_CHECK(hipMemsetAsync(dst, value, bytes, stream()));
}

void phip_sync(void) {
    ensure_device();
    PPO_CHECK(hipStreamSynchronize(g_side));
    PPO_CHECK(hipStreamSynchronize(g_stream));
}

void phip_side_fork(void) {
    ensure_device();
    PPO_CHECK(hipEventRecord(g_fork_ev, g_stream));
    PPO_CHECK(hipStreamWaitEvent(g_side, g_fork_ev, 0));
}

void phip_side_use(int on) { g_use_side = on != 0; }

int phip_side_active(void) { return g_use_side; }

void phip_side_join(void) {
    ensure_device();
    PPO_CHECK(hipEventRecord(g_join_ev, g_side));
    PPO_CHECK(hipStreamWaitEvent(g_stream, g_join_ev, 0));
}

void phip_drain(void) {                   // before a fatal exit: let queued kernels finish, ignore errors
    if (g_stream) (void)hipStreamSynchronize(g_stream);
    if (g_side) (void)hipStreamSynchronize(g_side);
}

void phip_record_error(const char* msg) {
    if (!g_err[0]) snprintf(g_err, sizeof(g_err), "%s", msg);
}

// ---------------- ppo_ext.h: device & errors ----------------
int ppo_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int ppo_set_device(int device) {
    if (g_stream) {   // already initialised: only the same device is allowed
        return device == g_device ? 0 : -1;
    }
    g_device = device;
    ensure_device();
    return 0;
}

const char* ppo_last_error(void) { return g_err; }
void ppo_clear_error(void) { g_err[0] = 0; }
void ppo_synchronize(void) { phip_sync(); }

const char* ppo_build_info(void) {
    return "libppo: hand-written HIP for gfx950 (MI355X); fp32 MFMA v_mfma_f32_32x32x2_f32 GEMMs; "
           "kernels: gemm{NT,NN,TN}, relu, mse, policy_head, log_prob, gae_scan, welford, normalize, "
           "gather, adam_flat/multi, sample, synthetic fill; comm: RCCL";
}

void* ppo_dev_alloc(size_t bytes) { return phip_malloc(bytes); }
void  ppo_dev_free(void* p) { phip_free(p); }
void  ppo_h2d(void* dst, const void* src, size_t bytes) { phip_h2d(dst, src, bytes); }
void  ppo_d2h(void* dst, const void* src, size_t bytes) { phip_d2h(dst, src, bytes); }
void  ppo_d2d(void* dst, const void* src, size_t bytes) { phip_d2d(dst, src, bytes); phip_sync(); }
void  ppo_dev_memset(void* dst, int value, size_t bytes) { phip_memset(dst, value, bytes); phip_sync(); }

// ---------------- ppo_ext.h: kernel timing ----------------
void ppo_prof_enable(int stride) {
    if (stride <= 0 && g_prof_on) harvest();
    g_prof_on = stride > 0;
    if (stride > 0) g_prof_stride = stride;
}

void ppo_prof_counts(long* out_total) {
    for (int k = 0; k < PPO_K_COUNT; k++) out_total[k] = g_issued[k];
}

void ppo_prof_issued_work(double* out_work) {
    for (int k = 0; k < PPO_K_COUNT; k++) out_work[k] = g_issued_work[k];
}

void ppo_prof_kernel_events(int on) { g_prof_kattach = on != 0; }

int ppo_prof_shapes(long long* keys, double* ms, long* launches, double* work, int cap) {
    harvest();
    const int n = (int)g_shapes.size();
    for (int i = 0; i < n && i < cap; i++) {
        keys[i] = g_shapes[i].key;
        ms[i] = g_shapes[i].ms;
        launches[i] = g_shapes[i].launches;
        work[i] = g_shapes[i].work;
    }
    return n;
}

int ppo_prof_shape_issued(const long long* keys, long* issued, int n) {
    int found = 0;
    for (int i = 0; i < n; i++) {
        issued[i] = 0;
        for (auto& x : g_shape_issued)
            if (x.first == keys[i]) { issued[i] = x.second; found++; break; }
    }
    return found;
}

void ppo_prof_reset(void) {
    harvest();
    g_shapes.clear();
    g_shape_issued.clear();
    for (int k = 0; k < PPO_K_COUNT; k++) { g_ms[k] = 0; g_work[k] = 0; g_launches[k] = 0; g_issued[k] = 0; g_issued_work[k] = 0; }
}

void ppo_prof_read(double* out_ms, double* out_work, long* out_launches) {
    harvest();
    for (int k = 0; k < PPO_K_COUNT; k++) {
        if (out_ms) out_ms[k] = g_ms[k];
        if (out_work) out_work[k] = g_work[k];
        if (out_launches) out_launches[k] = g_launches[k];
    }
}

}  // extern "C"
