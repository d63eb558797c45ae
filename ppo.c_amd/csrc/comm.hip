// comm.hip — data-parallel communicator: RCCL over xGMI, one process per MI355X.
//
// The reference has no multi-GPU code.  libppo shards the rollout buffer by whole
// environments: GAE needs no exchange; advantage statistics need one all-gather of
// a 24-byte Welford triple per update; every minibatch step all-reduces the flat gradient buffer
// of the network being trained (one call per network); replicated Adam keeps the parameters equal,
// which a per-update replica check verifies (a 64-bit parameter hash all-gathered and compared).
//
// Gradient all-reduces (default, "inline"): ONE per minibatch step, over the network's whole flat
// gradient, issued on the training loop's own stream — the value loop on libppo's main stream with
// the communicator, the policy loop on its side stream with a second communicator split from it.
// No cross-stream events: each all-reduce waits for the backward in stream order and Adam waits for
// it the same way, while the other loop's kernels run beside it (the event hand-offs of the bucketed
// form cost ≈ 23 µs per step: profiles/r05_comm_inline_ab.txt).  PPO_COMM_ASYNC=1 selects the
// bucketed form: per-layer buckets on ONE comm stream over ONE communicator in host issue order,
// each overlapping the layers below, joined by events before Adam.
//
// Why two communicators on two streams cannot deadlock (DESIGN.md §6 states it in full):
//  * the only kernels that wait for other kernels are RCCL's (the B = 64 grid-barrier phases never
//    run at world > 1: ppo_update_tiny); GEMMs, heads and Adam finish unconditionally;
//  * each communicator's collectives are issued from ONE stream in program order, and the host
//    interleaves the two loops by a fixed rule (iv·np ≤ ip·nv, host/ppo.c) that does not depend on
//    timing, so every rank submits the same total order of collectives — also the order a shared
//    hardware queue would serialise them in;
//  * every communicator is created with ncclConfig_t.maxCTAs = kMaxCTAs (32; PPO_COMM_MAX_CTAS), so
//    the two collectives that can be in flight at once need ≤ 64 workgroups of 256 CUs: once the
//    finite kernels beside them drain, both are resident, whatever else is queued.
//  By induction over that total order the earliest unfinished collective becomes resident on every
//  rank and completes.  The split's success is agreed over ranks (a min all-reduce) before any rank
//  uses it; on any failure every rank falls back to the bucketed single-communicator form.
// Diagnosis: phip_comm_wait() bounds every host wait of the data-parallel path (replica check,
// barrier) by PPO_COMM_TIMEOUT_S (default 600 s) and polls ncclCommGetAsyncError; a stall or an RCCL
// error aborts both communicators and fails loudly naming the rank, the pending streams and the mode.
//
// The per-update collectives (Welford all-gather, limit min, replica hashes) stay on the comm stream
// with an event pair, outside the loops.  PPO_COMM_SELF=1 at world 1 builds a one-rank communicator
// (and its split) so this exact path runs on a single GPU.
//
// PPO_COMM_LOOPBACK=k (k > 1, at world 1): an in-process stand-in for k ranks holding IDENTICAL
// shards.  ppo_comm_world() reports k, so every world > 1 branch of the update runs (grad_scale
// 1/k, the Welford all-gather + Chan combine, the limit agreement, the comm stream); the all-reduce
// is the exact k-fold sum of identical buffers (×k on the comm stream) and the all-gather
// replicates the local block k times.  For k a power of two an update must equal the 1-GPU update.
// Disagreeing ranks (tests): ppo_comm_loopback_peers() supplies ranks 1…k−1's Welford triples and
// buffer limits, ppo_comm_loopback_peer_grads() their gradient buffers, ppo_comm_loopback_peer_hash()
// their parameter hashes — the all-gather then delivers [own, peers…], the min runs over [own, peers…]
// and an all-reduce over a registered span adds the peers' values, so rank 0 of a k-rank job with
// different shards runs in one process.
#include "dev.h"
#include "../../include/ppo_ext.h"

#include <rccl/rccl.h>
#include <chrono>
#include <cstring>
#include <unistd.h>

namespace {
ncclComm_t g_comm = nullptr;
ncclComm_t g_comm_side = nullptr;            // the policy loop's communicator (split from g_comm)
int g_inline = 1;                            // gradient all-reduces in stream order (PPO_COMM_ASYNC=1: 0)
int g_rank = 0, g_world = 1;
int g_loopback = 0;                          // k > 1: PPO_COMM_LOOPBACK stand-in for k identical ranks
int* g_i32 = nullptr;                        // scratch for host-visible integer collectives

__global__ void scale_kernel(float* __restrict__ x, long n, float s) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
        x[i] *= s;
}

// loopback all-gather: block 0 = the local block; blocks 1…k−1 = the registered peers' blocks
// (peer == nullptr: replicas of the local block)
__global__ void gather_loopback_kernel(const double* __restrict__ src, const double* __restrict__ peer,
                                       double* __restrict__ dst, long n, int k) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n * k; i += (long)gridDim.x * 256)
        dst[i] = (i < n || !peer) ? src[i % n] : peer[i - n];
}
// loopback all-reduce over a registered span: x += Σ_{r=1}^{k−1} peer[r−1]  (rank order, as RCCL's
// two-rank sum; for k = 2 one add, commutative: rank 0's result of a real two-rank all-reduce)
__global__ void add_peers_kernel(float* __restrict__ x, const float* __restrict__ peer, long n, long stride,
                                 int peers) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        float s = x[i];
        for (int r = 0; r < peers; ++r) s += peer[r * stride + i];
        x[i] = s;
    }
}
// loopback stand-in of an integer min all-reduce: x[0] = the local value, x[1…k−1] the peers'
// (peers == 0: every rank holds the local value)
__global__ void min_i32_loopback_kernel(int* __restrict__ x, int k, int peers) {
    const int r = threadIdx.x;
    int v = x[0];
    __syncthreads();
    if (!peers && r < k && r < 64) x[r] = v;
    __syncthreads();
    if (r == 0) {
        int m = x[0];
        for (int i = 1; i < k && i < 64; ++i) m = min(m, x[i]);
        x[0] = m;
    }
}
// registered peer contributions (ppo_comm_loopback_peers / _peer_grads)
double* g_peer_welford = nullptr;            // device [(k−1)·3] or null
long g_peer_welford_n = 0;
int g_peer_limits[64];
int g_peer_limits_set = 0;
struct PeerSpan { const float* base; const float* peer; long n; };
PeerSpan g_peer_spans[4];
int g_peer_nspans = 0;
hipStream_t g_comm_stream = nullptr;
constexpr int kEvents = 16;                  // ring: a wait captures the record at enqueue time
hipEvent_t g_ready[kEvents], g_done[kEvents];
int g_ev = 0;

void comm_stream_init() {
    if (g_comm_stream) return;
    PPO_CHECK(hipStreamCreateWithFlags(&g_comm_stream, hipStreamNonBlocking));
    for (int i = 0; i < kEvents; i++) {
        PPO_CHECK(hipEventCreateWithFlags(&g_ready[i], hipEventDisableTiming));
        PPO_CHECK(hipEventCreateWithFlags(&g_done[i], hipEventDisableTiming));
    }
}

// comm stream waits for the issuing stream's queued work
hipStream_t comm_enter(int* slot) {
    *slot = g_ev;
    g_ev = (g_ev + 1) % kEvents;
    PPO_CHECK(hipEventRecord(g_ready[*slot], ppo::stream()));
    PPO_CHECK(hipStreamWaitEvent(g_comm_stream, g_ready[*slot], 0));
    return g_comm_stream;
}

// the issuing stream waits for the collective
void comm_leave(int slot) {
    PPO_CHECK(hipEventRecord(g_done[slot], g_comm_stream));
    PPO_CHECK(hipStreamWaitEvent(ppo::stream(), g_done[slot], 0));
}

// the loopback all-reduce on the comm stream: a span inside a registered peer span adds the peers'
// values at the same offset (disagreeing ranks); anything else is the k-fold sum of identical ranks
void loopback_allreduce(hipStream_t cs, float* d_buf, long n) {
    int grid = ppo_divup(n, 256);
    if (grid > 2048) grid = 2048;
    for (int i = 0; i < g_peer_nspans; ++i) {
        const PeerSpan& p = g_peer_spans[i];
        if (d_buf >= p.base && d_buf + n <= p.base + p.n) {
            hipLaunchKernelGGL(add_peers_kernel, dim3(grid), dim3(256), 0, cs, d_buf, p.peer + (d_buf - p.base), n,
                               p.n, g_loopback - 1);
            PPO_LAUNCH_CHECK();
            return;
        }
    }
    hipLaunchKernelGGL(scale_kernel, dim3(grid), dim3(256), 0, cs, d_buf, n, (float)g_loopback);
    PPO_LAUNCH_CHECK();
}

void nccl_check(ncclResult_t r, const char* what, int line) {
    if (r == ncclSuccess) return;
    char buf[256];
    snprintf(buf, sizeof(buf), "%s failed: %s", what, ncclGetErrorString(r));
    ppo::fail(buf, __FILE__, line);
}

// workgroups per collective (ncclConfig_t.maxCTAs) — the co-residency bound of the deadlock argument
constexpr int kMaxCTAs = 32;
int comm_max_ctas() {
    const char* e = getenv("PPO_COMM_MAX_CTAS");
    const int v = e ? atoi(e) : 0;
    return v >= 1 && v <= 64 ? v : kMaxCTAs;
}

double comm_timeout_s() {
    const char* e = getenv("PPO_COMM_TIMEOUT_S");
    const double v = e ? atof(e) : 0.0;
    return v > 0 ? v : 600.0;
}

// replica check: 64-bit hash of parameter bits, Σ mix(index, bits) mod 2^64 (order-independent, so the
// grid's atomics give the same value on every rank for the same bits)
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__global__ void param_hash_kernel(const unsigned* __restrict__ p, long n, unsigned long long base,
                                  unsigned long long* __restrict__ out) {
    unsigned long long acc = 0;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
        acc += mix64(((base + (unsigned long long)i) << 32) ^ p[i]);
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    __shared__ unsigned long long part[4];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(out, ((part[0] + part[1]) + part[2]) + part[3]);
}
unsigned long long* g_hash = nullptr;          // device [1 + world]: own hash at [0], the all-gather after it
unsigned long long g_peer_hash[64];
int g_peer_hash_set = 0;
}  // namespace

extern "C" {

int ppo_comm_unique_id(unsigned char* out, int cap) {
    ncclUniqueId id;
    nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId", __LINE__);
    const int n = (int)sizeof(id);
    if (!out || cap < n) return -n;
    memcpy(out, &id, n);
    return n;
}

int ppo_comm_init(int rank, int world, const unsigned char* id) {
    ppo::ensure_device();
    const char* self = getenv("PPO_COMM_SELF");
    const bool self_comm = world <= 1 && self && *self && *self != '0';
    const char* lb = getenv("PPO_COMM_LOOPBACK");
    const int k = lb ? atoi(lb) : 0;
    {
        const char* as = getenv("PPO_COMM_ASYNC");
        g_inline = !(as && *as && *as != '0');
    }
    if (world <= 1 && k > 1) {
        if (g_comm || g_loopback) { phip_record_error("ppo_comm_init: communicator already initialised"); return -1; }
        comm_stream_init();
        g_loopback = k;
        g_rank = 0;
        g_world = k;
        return 0;
    }
    if (world <= 1 && !self_comm) { g_rank = 0; g_world = 1; return 0; }
    if (g_comm) { phip_record_error("ppo_comm_init: communicator already initialised"); return -1; }
    ncclUniqueId uid;
    if (id) memcpy(&uid, id, sizeof(uid));
    else if (world <= 1) nccl_check(ncclGetUniqueId(&uid), "ncclGetUniqueId", __LINE__);
    else { phip_record_error("ppo_comm_init: null unique id at world > 1"); return -1; }
    if (world <= 1) { world = 1; rank = 0; }
    comm_stream_init();
    // every communicator capped at maxCTAs workgroups per collective (the co-residency bound of the
    // two-communicator deadlock argument, header comment); blocking calls
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 1;
    cfg.maxCTAs = comm_max_ctas();
    ncclResult_t r = ncclCommInitRankConfig(&g_comm, world, uid, rank, &cfg);
    if (r != ncclSuccess) {
        phip_record_error(ncclGetErrorString(r));
        g_comm = nullptr;
        return -1;
    }
    if (g_inline) {                                     // collective over g_comm: every rank splits
        ncclConfig_t scfg = NCCL_CONFIG_INITIALIZER;
        scfg.blocking = 1;
        scfg.maxCTAs = comm_max_ctas();
        r = ncclCommSplit(g_comm, 0, rank, &g_comm_side, &scfg);
        // the ranks agree on the outcome (min over g_comm) before any of them uses the side
        // communicator: one failing rank sends every rank to the bucketed single-communicator form
        int* ok = (int*)phip_malloc(sizeof(int));
        const int mine = r == ncclSuccess && g_comm_side != nullptr;
        phip_h2d(ok, &mine, sizeof(int));
        nccl_check(ncclAllReduce(ok, ok, 1, ncclInt32, ncclMin, g_comm, ppo::stream()), "ncclAllReduce(split agree)",
                   __LINE__);
        int all = 0;
        phip_d2h(&all, ok, sizeof(int));
        phip_free(ok);
        if (!all) {
            fprintf(stderr, "libppo: rank %d: ncclCommSplit %s on %s; gradient all-reduces on the comm stream\n",
                    rank, mine ? "succeeded here but failed" : ncclGetErrorString(r), mine ? "another rank" : "this rank");
            if (g_comm_side) ncclCommDestroy(g_comm_side);
            g_comm_side = nullptr;
            g_inline = 0;
        }
    }
    if (g_comm_side) {
        // one collective on each communicator here, in the same order on every rank, so that RCCL's
        // runtime peer connections (set up by a communicator's first collective) are all in place
        // before the two training loops start issuing on them from two streams in interleaved order
        float* w = (float*)phip_malloc(sizeof(float));
        nccl_check(ncclAllReduce(w, w, 1, ncclFloat32, ncclSum, g_comm, g_comm_stream), "ncclAllReduce(warm)",
                   __LINE__);
        nccl_check(ncclAllReduce(w, w, 1, ncclFloat32, ncclSum, g_comm_side, g_comm_stream), "ncclAllReduce(warm)",
                   __LINE__);
        PPO_CHECK(hipStreamSynchronize(g_comm_stream));
        phip_free(w);
    }
    g_rank = rank;
    g_world = world;
    return 0;
}

int ppo_comm_rank(void) { return g_rank; }
int ppo_comm_world(void) { return g_world; }

void ppo_comm_finalize(void) {
    if (g_loopback) {
        phip_sync();
        PPO_CHECK(hipStreamSynchronize(g_comm_stream));
        g_loopback = 0;
        ppo_comm_loopback_clear();
    }
    if (g_comm) {
        phip_sync();
        PPO_CHECK(hipStreamSynchronize(g_comm_stream));
        if (g_comm_side) ncclCommDestroy(g_comm_side);
        g_comm_side = nullptr;
        ncclCommDestroy(g_comm);
        g_comm = nullptr;
    }
    if (g_hash) { phip_free(g_hash); g_hash = nullptr; }
    g_inline = 1;
    g_rank = 0;
    g_world = 1;
}

int phip_comm_world(void) { return g_world; }
int phip_comm_active(void) { return g_comm != nullptr || g_loopback > 1; }
int phip_comm_inline(void) { return g_inline; }
int phip_comm_rank(void) { return g_rank; }

void phip_allreduce_sum_f32(float* d_buf, long n) {
    if ((!g_comm && !g_loopback) || n <= 0) return;
    ppo::ProfScope ps(PPO_K_COMM, 4.0 * n);   // issuing stream: ready -> collective done
    int slot;
    hipStream_t cs = comm_enter(&slot);
    if (g_loopback) {                          // k identical ranks: the sum is k·x
        loopback_allreduce(cs, d_buf, n);
        comm_leave(slot);
        return;
    }
    nccl_check(ncclAllReduce(d_buf, d_buf, (size_t)n, ncclFloat32, ncclSum, g_comm, cs), "ncclAllReduce",
               __LINE__);
    comm_leave(slot);
}

void ppo_comm_allreduce_f32(float* d_buf, long n) { phip_allreduce_sum_f32(d_buf, n); }

// Gradient buckets: the collective is queued on the comm stream behind the issuing stream's work
// so far (a layer's grad_W), but the issuing stream does not wait for it — the backward of the
// layers below runs while it travels; phip_allreduce_join() makes the issuing stream wait for
// every collective queued so far (the comm stream runs them in order: waiting for the last one
// suffices).
static int g_pending = -1;

void phip_allreduce_sum_f32_async(float* d_buf, long n) {
    if ((!g_comm && !g_loopback) || n <= 0) return;
    ppo::ProfScope ps(PPO_K_COMM, 4.0 * n);
    if (g_inline) {                                     // in stream order, the loop's own communicator
        if (g_loopback) {
            loopback_allreduce(ppo::stream(), d_buf, n);
        } else {
            nccl_check(ncclAllReduce(d_buf, d_buf, (size_t)n, ncclFloat32, ncclSum,
                                     phip_side_active() ? g_comm_side : g_comm, ppo::stream()),
                       "ncclAllReduce", __LINE__);
        }
        return;
    }
    int slot;
    hipStream_t cs = comm_enter(&slot);
    if (g_loopback) {
        loopback_allreduce(cs, d_buf, n);
    } else {
        nccl_check(ncclAllReduce(d_buf, d_buf, (size_t)n, ncclFloat32, ncclSum, g_comm, cs), "ncclAllReduce",
                   __LINE__);
    }
    PPO_CHECK(hipEventRecord(g_done[slot], g_comm_stream));
    g_pending = slot;
}

void phip_allreduce_join(void) {
    if (g_pending < 0) return;
    PPO_CHECK(hipStreamWaitEvent(ppo::stream(), g_done[g_pending], 0));
    g_pending = -1;
}

void phip_allgather_f64(const double* d_send, double* d_recv, long n_per_rank) {
    if (!g_comm && !g_loopback) {
        phip_d2d(d_recv, d_send, sizeof(double) * (size_t)n_per_rank);
        return;
    }
    ppo::ProfScope ps(PPO_K_COMM, 8.0 * n_per_rank * g_world);
    int slot;
    hipStream_t cs = comm_enter(&slot);
    if (g_loopback) {                          // [own block, peers' blocks] (or k replicas of the own block)
        const double* peer = g_peer_welford && g_peer_welford_n == n_per_rank * (g_loopback - 1) ? g_peer_welford
                                                                                               : nullptr;
        hipLaunchKernelGGL(gather_loopback_kernel, dim3(1), dim3(256), 0, cs, d_send, peer, d_recv, n_per_rank,
                           g_loopback);
        PPO_LAUNCH_CHECK();
        comm_leave(slot);
        return;
    }
    nccl_check(ncclAllGather(d_send, d_recv, (size_t)n_per_rank, ncclFloat64, g_comm, cs), "ncclAllGather",
               __LINE__);
    comm_leave(slot);
}

// host-level helpers for drivers (bench.py) that keep torch out of the process: a barrier and a
// max-over-ranks of a double, both over the RCCL communicator (synchronous)
static double* g_f64 = nullptr;

double ppo_comm_max_f64(double v) {
    if (!g_comm) return v;
    if (!g_f64) g_f64 = (double*)phip_malloc(sizeof(double));
    phip_h2d(g_f64, &v, sizeof(double));
    int slot;
    hipStream_t cs = comm_enter(&slot);
    nccl_check(ncclAllReduce(g_f64, g_f64, 1, ncclFloat64, ncclMax, g_comm, cs), "ncclAllReduce(max)", __LINE__);
    comm_leave(slot);
    double out = v;
    phip_d2h(&out, g_f64, sizeof(double));
    return out;
}

// Bounded host wait for everything libppo queued (main, side and comm streams): polls the streams and
// RCCL's asynchronous error state; a stall past PPO_COMM_TIMEOUT_S or an RCCL error aborts the
// communicators and fails loudly — a hung collective becomes a diagnosable exit, not a silent hang.
void phip_comm_wait(const char* what) {
    const double limit = comm_timeout_s();
    const auto t0 = std::chrono::steady_clock::now();
    unsigned spins = 0;
    for (;;) {
        int pending = ppo::streams_pending();
        if (g_comm_stream) {
            const hipError_t e = hipStreamQuery(g_comm_stream);
            if (e == hipErrorNotReady) pending |= 4;
            else PPO_CHECK(e);
        }
        if (!pending) return;
        ncclResult_t ae = ncclSuccess, as = ncclSuccess;
        if (g_comm) (void)ncclCommGetAsyncError(g_comm, &ae);
        if (g_comm_side) (void)ncclCommGetAsyncError(g_comm_side, &as);
        const bool rccl_err = (ae != ncclSuccess && ae != ncclInProgress) || (as != ncclSuccess && as != ncclInProgress);
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (rccl_err || s > limit) {
            char buf[400];
            snprintf(buf, sizeof(buf),
                     "rank %d/%d: %s: %s after %.0f s (pending:%s%s%s; gradient all-reduces %s; RCCL: %s / %s); "
                     "communicators aborted",
                     g_rank, g_world, what, rccl_err ? "RCCL error" : "no progress", s, pending & 1 ? " main" : "",
                     pending & 2 ? " side" : "", pending & 4 ? " comm" : "",
                     g_inline ? "inline (per-loop communicators)" : "bucketed (comm stream)", ncclGetErrorString(ae),
                     ncclGetErrorString(as));
            if (g_comm_side) ncclCommAbort(g_comm_side);
            if (g_comm) ncclCommAbort(g_comm);
            g_comm_side = g_comm = nullptr;
            ppo::fail(buf, __FILE__, __LINE__);
        }
        if (++spins > 64) usleep(50);
    }
}

void ppo_comm_barrier(void) {
    phip_comm_wait("ppo_comm_barrier (queued work)");
    (void)ppo_comm_max_f64(0.0);
    phip_sync();
}

// replica check (ppo_comm_check_replicas): this rank's parameter hash
void phip_param_hash(const float* const* spans, const long* lens, int nspans) {
    if (!g_hash) g_hash = (unsigned long long*)phip_malloc(sizeof(unsigned long long) * (size_t)(1 + (g_world > 64 ? g_world : 64)));
    phip_memset(g_hash, 0, sizeof(unsigned long long));
    unsigned long long base = 0;
    for (int i = 0; i < nspans; i++) {
        if (!spans[i] || lens[i] <= 0) continue;
        int grid = ppo_divup(lens[i], 256);
        if (grid > 1024) grid = 1024;
        hipLaunchKernelGGL(param_hash_kernel, dim3(grid), dim3(256), 0, ppo::stream(), (const unsigned*)spans[i],
                           lens[i], base, g_hash);
        PPO_LAUNCH_CHECK();
        base += (unsigned long long)lens[i];
    }
    // the value stays on the device (g_hash[0]); phip_comm_check_hash gathers and reads it
}

// all-gather of every rank's hash (in g_hash[0]) over the communicator, a bounded wait, then the
// comparison: 0 if all equal, −1 with a message naming the ranks that differ from rank 0
int phip_comm_check_hash(int gather, unsigned long long* own, char* msg, int cap) {
    if (!g_hash) return 0;
    const int k = !gather ? 1 : g_world > 64 ? 64 : g_world;
    if (gather && g_comm && g_world > 1) {
        int slot;
        hipStream_t cs = comm_enter(&slot);
        nccl_check(ncclAllGather(g_hash, g_hash + 1, 1, ncclUint64, g_comm, cs), "ncclAllGather(replica hash)",
                   __LINE__);
        comm_leave(slot);
    }
    phip_comm_wait(gather ? "replica check" : "parameter hash");
    unsigned long long h[65];
    phip_d2h(h, g_hash, sizeof(unsigned long long) * (size_t)(1 + k));
    if (own) *own = h[0];
    if (!(gather && g_comm && g_world > 1)) {     // loopback / one rank: [own, own…] or the registered peers
        for (int r = 0; r < k; r++) h[1 + r] = r == 0 || !g_peer_hash_set ? h[0] : g_peer_hash[r - 1];
    }
    int bad = 0, len = 0;
    if (msg && cap > 0) msg[0] = 0;
    for (int r = 1; r < k; r++) {
        if (h[1 + r] == h[1]) continue;
        bad++;
        if (msg && len < cap)
            len += snprintf(msg + len, (size_t)(cap - len), "%srank %d hash %016llx != rank 0 hash %016llx",
                            bad > 1 ? "; " : "", r, h[1 + r], h[1]);
    }
    return bad ? -1 : 0;
}

int ppo_comm_loopback_peer_hash(const unsigned long long* hashes, int count) {
    if (g_loopback < 2 || count != g_loopback - 1 || count > 63 || !hashes) {
        phip_record_error("ppo_comm_loopback_peer_hash: needs PPO_COMM_LOOPBACK=k and count = k - 1 (< 64)");
        return -1;
    }
    for (int r = 0; r < count; r++) g_peer_hash[r] = hashes[r];
    g_peer_hash_set = 1;
    return 0;
}

const char* ppo_comm_mode(void) {
    if (g_loopback > 1) return g_inline ? "loopback (in-process ranks), inline" : "loopback (in-process ranks), bucketed";
    if (!g_comm) return "none";
    return g_inline ? "inline: one all-reduce per step in each loop's stream, per-loop communicators"
                    : "bucketed: per-layer all-reduces on one comm stream, one communicator, event-joined";
}

// min over ranks of a host integer (synchronous; a few µs per call).  The update uses it to agree
// on whether any rank has an empty shard, so either every rank trains or none does.
int phip_comm_min_i32(int v) {
    if (!g_comm && !g_loopback) return v;      // world 1
    if (!g_i32) g_i32 = (int*)phip_malloc(sizeof(int) * 64);
    int x[64];
    x[0] = v;
    const int peers = g_loopback && g_peer_limits_set ? g_loopback - 1 : 0;
    for (int r = 0; r < peers && r < 63; ++r) x[r + 1] = g_peer_limits[r];
    phip_h2d(g_i32, x, sizeof(int) * (size_t)(1 + (peers < 63 ? peers : 63)));
    int slot;
    hipStream_t cs = comm_enter(&slot);
    if (g_loopback) {                          // min over [own, peers…] (or over k copies of the own value)
        hipLaunchKernelGGL(min_i32_loopback_kernel, dim3(1), dim3(64), 0, cs, g_i32, g_loopback, peers);
        PPO_LAUNCH_CHECK();
    } else {
        nccl_check(ncclAllReduce(g_i32, g_i32, 1, ncclInt32, ncclMin, g_comm, cs), "ncclAllReduce(min)", __LINE__);
    }
    comm_leave(slot);
    int out = v;
    phip_d2h(&out, g_i32, sizeof(int));
    return out;
}

void ppo_comm_loopback_clear(void) {
    g_peer_hash_set = 0;
    if (g_peer_welford) { phip_sync(); phip_free(g_peer_welford); }
    g_peer_welford = nullptr;
    g_peer_welford_n = 0;
    g_peer_limits_set = 0;
    g_peer_nspans = 0;
}

int ppo_comm_loopback_peers(const double* welford, const int* limits, int count) {
    if (g_loopback < 2 || count != g_loopback - 1 || count > 63) {
        phip_record_error("ppo_comm_loopback_peers: needs PPO_COMM_LOOPBACK=k and count = k - 1 (< 64)");
        return -1;
    }
    if (welford) {
        if (!g_peer_welford || g_peer_welford_n != 3L * count) {
            phip_free(g_peer_welford);
            g_peer_welford = (double*)phip_malloc(sizeof(double) * 3 * (size_t)count);
            g_peer_welford_n = 3L * count;
        }
        phip_h2d(g_peer_welford, welford, sizeof(double) * 3 * (size_t)count);
    }
    if (limits) {
        for (int r = 0; r < count; ++r) g_peer_limits[r] = limits[r];
        g_peer_limits_set = 1;
    }
    return 0;
}

int ppo_comm_loopback_peer_grads(const float* d_local_base, const float* d_peers, long n) {
    if (g_loopback < 2 || !d_local_base || !d_peers || n <= 0 || g_peer_nspans >= 4) {
        phip_record_error("ppo_comm_loopback_peer_grads: needs PPO_COMM_LOOPBACK=k, device spans, at most 4");
        return -1;
    }
    g_peer_spans[g_peer_nspans++] = PeerSpan{d_local_base, d_peers, n};
    return 0;
}

}  // extern "C"
