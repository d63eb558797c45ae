// comm.hip — data-parallel communicator: RCCL over xGMI, one process per MI355X.
//
// The reference has no multi-GPU code.  libppo shards the rollout buffer by whole
// environments: GAE needs no exchange; advantage statistics need one all-gather of
// a 24-byte Welford triple per update; every minibatch step all-reduces the flat gradient buffer
// of the network being trained (one call per network, on libppo's stream, so it is ordered after
// the backward kernels and before Adam with no host synchronisation).
#include "dev.h"
#include "../../include/ppo_ext.h"

#include <rccl/rccl.h>
#include <cstring>

namespace {
ncclComm_t g_comm = nullptr;
int g_rank = 0, g_world = 1;

void nccl_check(ncclResult_t r, const char* what, int line) {
    if (r == ncclSuccess) return;
    char buf[256];
    snprintf(buf, sizeof(buf), "%s failed: %s", what, ncclGetErrorString(r));
    ppo::fail(buf, __FILE__, line);
}
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
    if (world <= 1) { g_rank = 0; g_world = 1; return 0; }
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof(uid));
    ncclResult_t r = ncclCommInitRank(&g_comm, world, uid, rank);
    if (r != ncclSuccess) {
        phip_record_error(ncclGetErrorString(r));
        return -1;
    }
    g_rank = rank;
    g_world = world;
    return 0;
}

int ppo_comm_rank(void) { return g_rank; }
int ppo_comm_world(void) { return g_world; }

void ppo_comm_finalize(void) {
    if (g_comm) {
        phip_sync();
        ncclCommDestroy(g_comm);
        g_comm = nullptr;
    }
    g_rank = 0;
    g_world = 1;
}

int phip_comm_world(void) { return g_world; }
int phip_comm_rank(void) { return g_rank; }

void phip_allreduce_sum_f32(float* d_buf, long n) {
    if (g_world <= 1 || n <= 0) return;
    ppo::ProfScope ps(PPO_K_COMM, 4.0 * n);
    nccl_check(ncclAllReduce(d_buf, d_buf, (size_t)n, ncclFloat32, ncclSum, g_comm, ppo::stream()),
               "ncclAllReduce", __LINE__);
}

void ppo_comm_allreduce_f32(float* d_buf, long n) { phip_allreduce_sum_f32(d_buf, n); }

void phip_allgather_f64(const double* d_send, double* d_recv, long n_per_rank) {
    if (g_world <= 1) {
        phip_d2d(d_recv, d_send, sizeof(double) * (size_t)n_per_rank);
        return;
    }
    ppo::ProfScope ps(PPO_K_COMM, 8.0 * n_per_rank * g_world);
    nccl_check(ncclAllGather(d_send, d_recv, (size_t)n_per_rank, ncclFloat64, g_comm, ppo::stream()),
               "ncclAllGather", __LINE__);
}

}  // extern "C"
