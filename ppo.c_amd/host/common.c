/* common.c — host helpers: allocation, fatal errors, HBM staging slots. */
#include "internal.h"

#include <unistd.h>

/* fatal errors end the process with status 1, as the reference's checks do (cuda_helper.h:4-16,
 * exit(1)); _exit skips atexit teardown of a HIP runtime that may be in a bad state */
void die(const char* msg) {
    phip_record_error(msg);
    fprintf(stderr, "libppo: FATAL: %s\n", msg);
    fflush(stderr);
    phip_drain();                          /* never leave the process with kernels in flight */
    fflush(stdout);
    _exit(1);
}

void* xmalloc(size_t n) {
    void* p = malloc(n ? n : 1);
    if (!p) die("host allocation failed");
    return p;
}

void* xcalloc(size_t n, size_t sz) {
    void* p = calloc(n ? n : 1, sz ? sz : 1);
    if (!p) die("host allocation failed");
    return p;
}

static void*  g_stage[ST_COUNT];
static size_t g_stage_cap[ST_COUNT];

void* stage(int slot, size_t bytes) {
    if (bytes > g_stage_cap[slot]) {
        phip_free(g_stage[slot]);
        size_t cap = bytes + bytes / 4 + 256;
        g_stage[slot] = phip_malloc(cap);
        g_stage_cap[slot] = cap;
    }
    return g_stage[slot];
}

float* stage_up(int slot, const float* host, size_t count) {
    float* d = (float*)stage(slot, count * sizeof(float));
    if (host && count) phip_h2d(d, host, count * sizeof(float));
    return d;
}

int ppo_struct_sizes(long* out, int n) {
    const long s[7] = {(long)sizeof(Layer), (long)sizeof(NeuralNetwork), (long)sizeof(GaussianPolicy),
                       (long)sizeof(TrajectoryBuffer), (long)sizeof(Adam), (long)sizeof(PPO), (long)sizeof(Env)};
    for (int i = 0; i < n && i < 7; i++) out[i] = s[i];
    return 7;
}

/* main.c:18 calls openblas_set_num_threads(1) without declaring it; libppo has
 * no BLAS, so this only records the request. */
static int g_host_threads = 1;
void openblas_set_num_threads(int num_threads) { g_host_threads = num_threads > 0 ? num_threads : 1; }
