/*
 * trajectory_buffer.c — rollout storage with host and HBM mirrors.
 *
 * Reference: /root/reference/src/trajectory_buffer.cu.  The shuffles keep the
 * reference's libc rand() consumption (swap(i, rand() % N), D12) so seeded
 * runs reproduce its minibatch order; the gather is the coalesced
 * one-wave-per-row kernel of csrc/buffer.hip.
 */
#include "internal.h"

static float* get_action(TrajectoryBuffer* b, int i) { return b->action_p + (size_t)i * b->action_size; }
static float* get_state(TrajectoryBuffer* b, int i) { return b->state_p + (size_t)i * b->state_size; }
static float* get_next_state(TrajectoryBuffer* b, int i) { return b->next_state_p + (size_t)i * b->state_size; }
static float* get_reward(TrajectoryBuffer* b, int i) { return b->reward_p + i; }
static float* get_logprob(TrajectoryBuffer* b, int i) { return b->logprob_p + i; }
static float* get_advantage(TrajectoryBuffer* b, int i) { return b->advantage_p + i; }
static float* get_adv_target(TrajectoryBuffer* b, int i) { return b->adv_target_p + i; }
static bool* get_terminated(TrajectoryBuffer* b, int i) { return b->terminated_p + i; }
static bool* get_truncated(TrajectoryBuffer* b, int i) { return b->truncated_p + i; }

static void point_host(TrajectoryBuffer* b) {
    b->action_p = b->h_action_p;         b->state_p = b->h_state_p;
    b->next_state_p = b->h_next_state_p; b->reward_p = b->h_reward_p;
    b->logprob_p = b->h_logprob_p;       b->advantage_p = b->h_advantage_p;
    b->adv_target_p = b->h_adv_target_p; b->terminated_p = b->h_terminated_p;
    b->truncated_p = b->h_truncated_p;
    b->on_device = 0;
}

static void point_device(TrajectoryBuffer* b) {
    b->action_p = b->d_action_p;         b->state_p = b->d_state_p;
    b->next_state_p = b->d_next_state_p; b->reward_p = b->d_reward_p;
    b->logprob_p = b->d_logprob_p;       b->advantage_p = b->d_advantage_p;
    b->adv_target_p = b->d_adv_target_p; b->terminated_p = b->d_terminated_p;
    b->truncated_p = b->d_truncated_p;
    b->on_device = 1;
}

TrajectoryBuffer* create_trajectory_buffer(int capacity, int state_size, int action_size) {
    phip_init();
    TrajectoryBuffer* b = (TrajectoryBuffer*)xcalloc(1, sizeof(TrajectoryBuffer));
    b->capacity = capacity;
    b->idx = 0;
    b->full = false;
    b->state_size = state_size;
    b->action_size = action_size;
    const size_t N = (size_t)capacity, S = (size_t)state_size, A = (size_t)action_size;
    b->h_action_p = (float*)xcalloc(N * A, sizeof(float));
    b->h_state_p = (float*)xcalloc(N * S, sizeof(float));
    b->h_next_state_p = (float*)xcalloc(N * S, sizeof(float));
    b->h_reward_p = (float*)xcalloc(N, sizeof(float));
    b->h_logprob_p = (float*)xcalloc(N, sizeof(float));
    b->h_advantage_p = (float*)xcalloc(N, sizeof(float));
    b->h_adv_target_p = (float*)xcalloc(N, sizeof(float));
    b->h_terminated_p = (bool*)xcalloc(N, sizeof(bool));
    b->h_truncated_p = (bool*)xcalloc(N, sizeof(bool));
    b->d_action_p = (float*)phip_malloc(sizeof(float) * N * A);
    b->d_state_p = (float*)phip_malloc(sizeof(float) * N * S);
    b->d_next_state_p = (float*)phip_malloc(sizeof(float) * N * S);
    b->d_reward_p = (float*)phip_malloc(sizeof(float) * N);
    b->d_logprob_p = (float*)phip_malloc(sizeof(float) * N);
    b->d_advantage_p = (float*)phip_malloc(sizeof(float) * N);
    b->d_adv_target_p = (float*)phip_malloc(sizeof(float) * N);
    b->d_terminated_p = (bool*)phip_malloc(sizeof(bool) * N);
    b->d_truncated_p = (bool*)phip_malloc(sizeof(bool) * N);
    point_host(b);
    b->random_idx = NULL;
    b->h_random_idx = NULL;
    b->action = get_action;         b->state = get_state;
    b->next_state = get_next_state; b->reward = get_reward;
    b->logprob = get_logprob;       b->advantage = get_advantage;
    b->adv_target = get_adv_target; b->terminated = get_terminated;
    b->truncated = get_truncated;
    return b;
}

void free_trajectory_buffer(TrajectoryBuffer* b, bool use_cuda) {
    (void)use_cuda;
    if (!b) return;
    free(b->h_action_p); free(b->h_state_p); free(b->h_next_state_p); free(b->h_reward_p);
    free(b->h_logprob_p); free(b->h_advantage_p); free(b->h_adv_target_p);
    free(b->h_terminated_p); free(b->h_truncated_p);
    phip_free(b->d_action_p); phip_free(b->d_state_p); phip_free(b->d_next_state_p); phip_free(b->d_reward_p);
    phip_free(b->d_logprob_p); phip_free(b->d_advantage_p); phip_free(b->d_adv_target_p);
    phip_free(b->d_terminated_p); phip_free(b->d_truncated_p);
    if (b->random_idx_is_device) phip_free(b->random_idx);
    free(b->h_random_idx);
    free(b);
}

static int limit_of(const TrajectoryBuffer* b) { return b->full ? b->capacity : b->idx; }

/* trajectory_buffer.cu:126-146 */
static void rand_permutation(int* perm, int n) {
    for (int i = 0; i < n; i++) perm[i] = i;
    for (int i = 0; i < n; i++) {
        int j = rand() % n;
        int t = perm[i];
        perm[i] = perm[j];
        perm[j] = t;
    }
}

static int* ensure_host_perm(TrajectoryBuffer* b) {
    if (!b->h_random_idx) b->h_random_idx = (int*)xmalloc(sizeof(int) * (size_t)(b->capacity > 0 ? b->capacity : 1));
    return b->h_random_idx;
}

static int* ensure_dev_perm(TrajectoryBuffer* b) {
    if (!b->random_idx_is_device || !b->random_idx) {
        b->random_idx = (int*)phip_malloc(sizeof(int) * (size_t)(b->capacity > 0 ? b->capacity : 1));
        b->random_idx_is_device = 1;
    }
    return b->random_idx;
}

void shuffle_buffer(TrajectoryBuffer* b) {
    const int n = limit_of(b);
    int* h = ensure_host_perm(b);
    rand_permutation(h, n);
    if (!b->random_idx_is_device) b->random_idx = h;
}

void shuffle_buffer_cuda(TrajectoryBuffer* b) {
    const int n = limit_of(b);
    int* h = ensure_host_perm(b);
    rand_permutation(h, n);
    int* d = ensure_dev_perm(b);
    phip_h2d(d, h, sizeof(int) * (size_t)n);
}

/* trajectory_buffer.cu:188-200 — device pointers */
void get_batch_cuda(TrajectoryBuffer* b, int batch_idx, int batch_size, float* states, float* actions, float* logprobs,
                    float* advantages, float* adv_targets) {
    if (!b->random_idx_is_device) die("get_batch_cuda: call shuffle_buffer_cuda first");
    phip_gather(b->random_idx, 0, batch_idx * batch_size, limit_of(b), batch_size, b->state_size, b->action_size,
                b->state_p, b->action_p, b->logprob_p, b->advantage_p, b->adv_target_p, states, actions, logprobs,
                advantages, adv_targets);
}

/* trajectory_buffer.cu:202-220 — host pointers: the current (host) buffer and the host
 * permutation are staged into HBM, gathered on the GPU and copied back. */
void get_batch(TrajectoryBuffer* b, int batch_idx, int batch_size, float* states, float* actions, float* logprobs,
               float* advantages, float* adv_targets) {
    const int n = limit_of(b), S = b->state_size, A = b->action_size, B = batch_size;
    if (!b->h_random_idx) die("get_batch: call shuffle_buffer first");
    int* dperm = (int*)stage(ST_A, sizeof(int) * (size_t)n);
    phip_h2d(dperm, b->h_random_idx, sizeof(int) * (size_t)n);
    const float *ds, *da, *dl, *dv, *dt;
    if (b->on_device) {
        ds = b->state_p; da = b->action_p; dl = b->logprob_p; dv = b->advantage_p; dt = b->adv_target_p;
    } else {
        ds = stage_up(ST_B, b->state_p, (size_t)n * S);
        da = stage_up(ST_C, b->action_p, (size_t)n * A);
        dl = stage_up(ST_D, b->logprob_p, (size_t)n);
        dv = stage_up(ST_E, b->advantage_p, (size_t)n);
        dt = stage_up(ST_F, b->adv_target_p, (size_t)n);
    }
    float* out = (float*)stage(ST_G, sizeof(float) * (size_t)B * (S + A + 3));
    float *os = out, *oa = os + (size_t)B * S, *ol = oa + (size_t)B * A, *ov = ol + B, *ot = ov + B;
    phip_gather(dperm, 0, batch_idx * B, n, B, S, A, ds, da, dl, dv, dt, os, oa, ol, ov, ot);
    phip_d2h(states, os, sizeof(float) * (size_t)B * S);
    phip_d2h(actions, oa, sizeof(float) * (size_t)B * A);
    phip_d2h(logprobs, ol, sizeof(float) * (size_t)B);
    phip_d2h(advantages, ov, sizeof(float) * (size_t)B);
    phip_d2h(adv_targets, ot, sizeof(float) * (size_t)B);
}

void reset_buffer(TrajectoryBuffer* b) {
    b->idx = 0;
    b->full = false;
}

void buffer_to_device(TrajectoryBuffer* b) {
    const size_t N = (size_t)b->capacity, S = (size_t)b->state_size, A = (size_t)b->action_size;
    phip_h2d(b->d_action_p, b->h_action_p, sizeof(float) * N * A);
    phip_h2d(b->d_state_p, b->h_state_p, sizeof(float) * N * S);
    phip_h2d(b->d_next_state_p, b->h_next_state_p, sizeof(float) * N * S);
    phip_h2d(b->d_reward_p, b->h_reward_p, sizeof(float) * N);
    phip_h2d(b->d_logprob_p, b->h_logprob_p, sizeof(float) * N);
    phip_h2d(b->d_advantage_p, b->h_advantage_p, sizeof(float) * N);
    phip_h2d(b->d_adv_target_p, b->h_adv_target_p, sizeof(float) * N);
    phip_h2d(b->d_terminated_p, b->h_terminated_p, sizeof(bool) * N);
    phip_h2d(b->d_truncated_p, b->h_truncated_p, sizeof(bool) * N);
    point_device(b);
}

void buffer_to_host(TrajectoryBuffer* b) {
    const size_t N = (size_t)b->capacity, S = (size_t)b->state_size, A = (size_t)b->action_size;
    phip_d2h(b->h_action_p, b->d_action_p, sizeof(float) * N * A);
    phip_d2h(b->h_state_p, b->d_state_p, sizeof(float) * N * S);
    phip_d2h(b->h_next_state_p, b->d_next_state_p, sizeof(float) * N * S);
    phip_d2h(b->h_reward_p, b->d_reward_p, sizeof(float) * N);
    phip_d2h(b->h_logprob_p, b->d_logprob_p, sizeof(float) * N);
    phip_d2h(b->h_advantage_p, b->d_advantage_p, sizeof(float) * N);
    phip_d2h(b->h_adv_target_p, b->d_adv_target_p, sizeof(float) * N);
    phip_d2h(b->h_terminated_p, b->d_terminated_p, sizeof(bool) * N);
    phip_d2h(b->h_truncated_p, b->d_truncated_p, sizeof(bool) * N);
    point_host(b);
}

/* used by ppo_fill_synthetic: the device mirror was written directly */
void buffer_point_device(TrajectoryBuffer* b) { point_device(b); }
