/*
 * ppo.c — PPO orchestration (reference /root/reference/src/ppo.cu).
 *
 * The update (GAE → value epochs → policy epochs) is issued entirely on
 * libppo's HIP stream: no per-minibatch allocation, no device→host reads
 * (the reference blocks on 1–2 scalar copies per minibatch), the
 * losses accumulate on the device.  Per value minibatch:
 *     gather → L × fused linear(+bias+ReLU) → MSE+grad → L × bwd_W(+bias grad)
 *     → (L−1) × bwd_x(+ReLU′) → [RCCL all-reduce] → flat Adam
 * and per policy minibatch the same with the fused Gaussian/clipped-surrogate
 * head (csrc/kernels.hip) in place of the MSE.
 */
#include "internal.h"

#include <math.h>

void buffer_point_device(TrajectoryBuffer* b);

/* ------------------------------------------------------------------ */
/* device workspaces                                                   */
/* ------------------------------------------------------------------ */
typedef struct {
    int cap_B, S, A;
    float *states, *actions, *old_lp, *adv, *tgt, *gv, *gmu;
    int* rows;                    /* minibatch slot → buffer row (layer 0's fused gather) */
    int* rows_p;                  /* the policy loop's own rows / gathered states (it runs on the */
    float* states_p;              /* side stream beside the value loop) */
    int* perm[2];                 /* host rand() shuffle: every epoch's permutation (value, policy) */
    long perm_cap[2];
    int* ro_rows;                 /* rollout: rows[t·E + e] = e·T + t */
    float* tiny_steps[3];         /* small-network path: per-step Adam step sizes (value, entropy, policy) */
    int tiny_cap[3];
    float* env_state;             /* rollout: per-environment state */
    int ro_E, ro_T, ro_kind, ro_S;
    unsigned long long ro_step;   /* rollout step counter (Philox stream offset) */
    float* stats;                 /* [0] Σ value loss, [1] Σ policy loss */
    long n_v, n_p;
    long n_graph;                 /* minibatch steps replayed from captured graphs (PPO_GRAPH=1) */
    uint64_t key;                 /* device-shuffle epoch key */
    unsigned long long seed;
    int seeded;
    long max_v, max_p;            /* ppo_set_step_limit: cap on value / policy minibatch steps (−1: none) */
    /* launch-free minibatch steps (graph replay): per phase (0 value, 1 policy) a device step table,
     * its step counter and the Adam kernel's ticket */
    PhipStepArgs* tab[2];
    long tab_cap[2];
    int* ctr;                     /* [2] step counters, [2] tickets (as unsigned) */
    PhipStepArgs* h_tab;
    long h_tab_cap;
    /* phase gathers: every minibatch step's row indices and per-row inputs of a whole phase, gathered
     * by one launch per epoch before the loops (value: rows, targets; policy: rows, actions, old
     * log-probs, advantages) — step iv reads its B rows at iv·B */
    int* ph_rows[2];
    float *ph_tgt, *ph_act, *ph_olp, *ph_adv;
    long ph_cap[2];
} PPODev;

static float* g_v = NULL;         /* V(state), V(next_state) for compute_gae_cuda */
static float* g_vn = NULL;
static int* g_own = NULL;         /* transitions whose V(next_state) needs its own forward */
static long g_v_cap = 0;
static double* g_welford = NULL;  /* (n, mean, M2) */
static double* g_welford_all = NULL;
static int g_welford_world = 0;
static float* g_adv_stats = NULL; /* (mean, std) as used for normalisation */
static long g_gae_own_rows = 0;   /* rows of the last GAE's own V(next_state) forward */
static long g_gae_n = 0;          /* transitions of the last GAE */

static uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static void ensure_gae_ws(long n) {
    if (!g_welford) {
        g_welford = (double*)phip_malloc(4 * sizeof(double));
        g_adv_stats = (float*)phip_malloc(4 * sizeof(float));
    }
    const int world = phip_comm_world();
    if (world > g_welford_world) {
        phip_free(g_welford_all);
        g_welford_all = (double*)phip_malloc(sizeof(double) * 3 * (size_t)world);
        g_welford_world = world;
    }
    if (n > g_v_cap) {
        phip_free(g_v);
        phip_free(g_vn);
        phip_free(g_own);
        g_v = (float*)phip_malloc(sizeof(float) * (size_t)n);
        g_vn = (float*)phip_malloc(sizeof(float) * (size_t)n);
        g_own = (int*)phip_malloc(sizeof(int) * (size_t)n);
        g_v_cap = n;
    }
}

static PPODev* dev_ws(PPO* ppo, int B) {
    PPODev* d = (PPODev*)ppo->dev;
    const int S = ppo->buffer->state_size, A = ppo->buffer->action_size;
    if (!d) {
        d = (PPODev*)xcalloc(1, sizeof(PPODev));
        d->stats = (float*)phip_malloc(4 * sizeof(float));
        d->max_v = d->max_p = -1;
        ppo->dev = d;
    }
    if (B > d->cap_B) {
        phip_free(d->states); phip_free(d->actions); phip_free(d->old_lp); phip_free(d->adv);
        phip_free(d->tgt); phip_free(d->gv); phip_free(d->gmu); phip_free(d->rows);
        phip_free(d->rows_p); phip_free(d->states_p);
        d->rows = (int*)phip_malloc(sizeof(int) * (size_t)B);
        d->rows_p = (int*)phip_malloc(sizeof(int) * (size_t)B);
        d->states = (float*)phip_malloc(sizeof(float) * (size_t)B * S);
        d->states_p = (float*)phip_malloc(sizeof(float) * (size_t)B * S);
        d->actions = (float*)phip_malloc(sizeof(float) * (size_t)B * A);
        d->old_lp = (float*)phip_malloc(sizeof(float) * (size_t)B);
        d->adv = (float*)phip_malloc(sizeof(float) * (size_t)B);
        d->tgt = (float*)phip_malloc(sizeof(float) * (size_t)B);
        d->gv = (float*)phip_malloc(sizeof(float) * (size_t)B);
        d->gmu = (float*)phip_malloc(sizeof(float) * (size_t)B * A);
        d->cap_B = B;
    }
    d->S = S;
    d->A = A;
    return d;
}

static void free_dev_ws(PPO* ppo) {
    PPODev* d = (PPODev*)ppo->dev;
    if (!d) return;
    phip_free(d->states); phip_free(d->actions); phip_free(d->old_lp); phip_free(d->adv);
    phip_free(d->tgt); phip_free(d->gv); phip_free(d->gmu); phip_free(d->stats); phip_free(d->rows);
    phip_free(d->ro_rows); phip_free(d->env_state); phip_free(d->perm[0]); phip_free(d->perm[1]);
    phip_free(d->rows_p); phip_free(d->states_p);
    for (int i = 0; i < 3; i++) phip_free(d->tiny_steps[i]);
    phip_free(d->tab[0]); phip_free(d->tab[1]); phip_free(d->ctr);
    phip_free(d->ph_rows[0]); phip_free(d->ph_rows[1]); phip_free(d->ph_tgt); phip_free(d->ph_act);
    phip_free(d->ph_olp); phip_free(d->ph_adv);
    free(d->h_tab);
    free(d);
    ppo->dev = NULL;
}

/* ------------------------------------------------------------------ */
/* construction (ppo.cu:6-51)                                          */
/* ------------------------------------------------------------------ */
PPO* create_ppo(char** activation_functions, int* layer_sizes, int num_layers, int buffer_size, float lr_policy,
                float lr_v, float lambda, float epsilon, float ent_coeff, float init_std, bool use_cuda) {
    PPO* ppo = (PPO*)xcalloc(1, sizeof(PPO));
    ppo->buffer = create_trajectory_buffer(buffer_size, layer_sizes[0], layer_sizes[num_layers - 1]);
    ppo->policy = create_gaussian_policy(layer_sizes, activation_functions, num_layers, init_std);
    int* sizes_v = (int*)xmalloc(sizeof(int) * (size_t)num_layers);
    memcpy(sizes_v, layer_sizes, sizeof(int) * (size_t)(num_layers - 1));
    sizes_v[num_layers - 1] = 1;                                         /* ppo.cu:12-16 */
    ppo->V = create_neural_network(sizes_v, activation_functions, num_layers);
    free(sizes_v);
    ppo->adam_policy = create_adam_from_nn_cuda(ppo->policy->mu, 0.9f, 0.999f);
    ppo->adam_V = create_adam_from_nn_cuda(ppo->V, 0.9f, 0.999f);
    ppo->adam_entropy = create_adam_cuda(&ppo->policy->d_log_std, &ppo->policy->d_log_std_grad,
                                         &ppo->policy->action_size, 1, ppo->policy->action_size, 0.9f, 0.999f);
    ppo->lambda = lambda;
    ppo->epsilon = epsilon;
    ppo->ent_coeff = ent_coeff;
    ppo->lr_policy = lr_policy;
    ppo->lr_V = lr_v;
    ppo->use_cuda = use_cuda;
    ppo->dev = NULL;
    return ppo;
}

void free_ppo(PPO* ppo) {
    if (!ppo) return;
    free_adam_cuda(ppo->adam_policy);
    free_adam_cuda(ppo->adam_V);
    free_adam_cuda(ppo->adam_entropy);
    free_trajectory_buffer(ppo->buffer, ppo->use_cuda);
    free_gaussian_policy(ppo->policy);
    free_neural_network(ppo->V);
    free_dev_ws(ppo);
    free(ppo);
}

/* ------------------------------------------------------------------ */
/* rollout (ppo.cu:54-79) — host loop over the Env ABI, out of scope of the accelerated path */
/* ------------------------------------------------------------------ */
void collect_trajectories(TrajectoryBuffer* buffer, Env* env, GaussianPolicy* policy, int steps) {
    if (buffer->on_device) buffer_to_host(buffer);
    env->reset_env(buffer->state(buffer, buffer->idx));
    for (int i = 0; i < steps; i++) {
        sample_action(policy, buffer->state(buffer, buffer->idx), buffer->action(buffer, buffer->idx),
                      buffer->logprob(buffer, buffer->idx), 1);
        env->step_env(buffer->action(buffer, buffer->idx), buffer->next_state(buffer, buffer->idx),
                      buffer->reward(buffer, buffer->idx), buffer->terminated(buffer, buffer->idx),
                      buffer->truncated(buffer, buffer->idx), buffer->action_size);
        int new_idx = (buffer->idx + 1) % buffer->capacity;
        if (i < steps - 1) {
            if (*buffer->truncated(buffer, buffer->idx) || *buffer->terminated(buffer, buffer->idx))
                env->reset_env(buffer->state(buffer, new_idx));
            else
                memcpy(buffer->state(buffer, new_idx), buffer->next_state(buffer, buffer->idx),
                       sizeof(float) * (size_t)buffer->state_size);
        } else if (!*buffer->terminated(buffer, buffer->idx)) {
            *buffer->truncated(buffer, buffer->idx) = true;
        }
        buffer->idx = new_idx;
        buffer->full = buffer->full || buffer->idx == 0;
    }
}

/* ------------------------------------------------------------------ */
/* GAE (ppo.cu:261-369)                                                */
/* ------------------------------------------------------------------ */
/* PPO_GAE_FULL=1: evaluate V over every next_state row as the reference does (A/B checks) */
static int gae_full_forwards(void) {
    const char* e = getenv("PPO_GAE_FULL");
    return e && *e && *e != '0';
}

void ppo_gae_device(NeuralNetwork* V, TrajectoryBuffer* b, float gamma, float lambda) {
    const int n = b->full ? b->capacity : b->idx;
    g_gae_own_rows = 0;                     /* an empty buffer reports no own-row forward */
    g_gae_n = n;
    ensure_gae_ws(n);
    if (n > 0 && gae_full_forwards()) {     /* the reference's two full forwards (ppo.cu:333-336) */
        nn_forward_dev(V, b->next_state_p, n);
        phip_d2d(g_vn, V->d_output, sizeof(float) * (size_t)n);
        g_gae_own_rows = n;
        nn_forward_dev(V, b->state_p, n);
        phip_d2d(g_v, V->d_output, sizeof(float) * (size_t)n);
    } else if (n > 0) {
        /* V(state) once; V(next_state[t]) = V(state[t+1]) wherever the rows are bitwise equal
         * (every transition that did not end an episode); the rest get their own forward */
        nn_forward_dev(V, b->state_p, n);
        phip_d2d(g_v, V->d_output, sizeof(float) * (size_t)n);
        const int own = phip_next_value_map(b->next_state_p, b->state_p, g_v, g_vn, g_own, n, V->layers[0].input_size);
        g_gae_own_rows = own;
        if (own > 0) {
            nn_forward_dev_rows(V, b->next_state_p, g_own, NULL, own);
            phip_scatter_values(g_vn, g_own, V->d_output, own);
        }
    }
    phip_gae_scan(g_v, g_vn, b->reward_p, (const uint8_t*)b->terminated_p, (const uint8_t*)b->truncated_p, n, gamma,
                  lambda, b->advantage_p, b->adv_target_p, g_welford);
    const int world = phip_comm_world();
    if (world > 1) {       /* global advantage statistics across env shards */
        phip_allgather_f64(g_welford, g_welford_all, 3);
        phip_welford_combine(g_welford_all, world, g_welford);
    }
    phip_normalize(b->advantage_p, n, g_welford, g_adv_stats);
}

long ppo_gae_state(double* welford, float* v, float* v_next, long n) {
    phip_sync();
    if (n > g_gae_n) n = g_gae_n;
    if (welford) {
        double w[6] = {0, 0, 0, 0, 0, 0};
        if (g_welford) phip_d2h(w, g_welford, 3 * sizeof(double));
        if (phip_comm_world() > 1 && g_welford_all)
            phip_d2h(w + 3, g_welford_all + 3 * (size_t)phip_comm_rank(), 3 * sizeof(double));
        else
            memcpy(w + 3, w, 3 * sizeof(double));
        memcpy(welford, w, sizeof(w));
    }
    if (v && n > 0) phip_d2h(v, g_v, sizeof(float) * (size_t)n);
    if (v_next && n > 0) phip_d2h(v_next, g_vn, sizeof(float) * (size_t)n);
    return g_gae_n;
}

/* device buffer (after buffer_to_device); `horizon` is unused: the scan is exact (D7) */
void compute_gae_cuda(NeuralNetwork* V, TrajectoryBuffer* buffer, float gamma, float lambda, int horizon) {
    (void)horizon;
    ppo_gae_device(V, buffer, gamma, lambda);
}

/* host buffer: staged through the device mirror */
void compute_gae(NeuralNetwork* V, TrajectoryBuffer* buffer, float gamma, float lambda) {
    const int was_device = buffer->on_device;
    if (!was_device) buffer_to_device(buffer);
    ppo_gae_device(V, buffer, gamma, lambda);
    if (!was_device) buffer_to_host(buffer);
}

/* ------------------------------------------------------------------ */
/* clipped surrogate (ppo.cu:82-169)                                   */
/* ------------------------------------------------------------------ */
float policy_loss_and_grad_cuda(float* grad_logprob, float* grad_entropy, float* adv, float* logprobs,
                                float* old_logprobs, float entropy, float ent_coeff, float epsilon, int m) {
    float* d = (float*)stage(ST_H, 16);
    phip_h2d(d + 1, &entropy, sizeof(float));
    phip_policy_loss(adv, logprobs, old_logprobs, grad_logprob, m, epsilon, ent_coeff, d + 1, d, NULL);
    float loss = 0.f;
    phip_d2h(&loss, d, sizeof(float));
    *grad_entropy = -ent_coeff;
    return loss;
}

float policy_loss_and_grad(float* grad_logprob, float* grad_entropy, float* adv, float* logprobs,
                           float* old_logprobs, float entropy, float ent_coeff, float epsilon, int m) {
    float* da = stage_up(ST_A, adv, (size_t)m);
    float* dl = stage_up(ST_B, logprobs, (size_t)m);
    float* dol = stage_up(ST_C, old_logprobs, (size_t)m);
    float* dg = (float*)stage(ST_D, sizeof(float) * (size_t)(m > 0 ? m : 1));
    float loss = policy_loss_and_grad_cuda(dg, grad_entropy, da, dl, dol, entropy, ent_coeff, epsilon, m);
    phip_d2h(grad_logprob, dg, sizeof(float) * (size_t)m);
    return loss;
}

/* ------------------------------------------------------------------ */
/* the update                                                          */
/* ------------------------------------------------------------------ */
static const int* next_perm(PPO* ppo, PPODev* d, int shuffle_mode, uint64_t* key) {
    if (shuffle_mode == PPO_SHUFFLE_DEVICE) {
        *key = d->key++;
        return NULL;
    }
    shuffle_buffer_cuda(ppo->buffer);                   /* reference: host rand() swap shuffle */
    *key = 0;
    return ppo->buffer->random_idx;
}

/* ------------------------------------------------------------------ */
/* small networks: every minibatch step of a phase in one workgroup    */
/* (csrc/tiny.hip); same arithmetic, rand() order and Adam step counts  */
/* ------------------------------------------------------------------ */
/* max_w: widest layer the kernel takes (128 for the single-workgroup kernel; the multi-workgroup
 * cluster kernel checks its own shapes) */
static int tiny_net(NeuralNetwork* nn, Adam* adam, PhipTinyNet* t, int max_w) {
    const int L = nn->num_layers - 1;
    if (nn->dtype != 0 || L < 1 || L > 8 || !adam->flat || adam->weights[0] != nn->d_params ||
        adam->grad_weights[0] != nn->d_grads)
        return -1;
    for (int i = 0; i < L; i++)
        if (nn->layers[i].input_size > max_w || nn->layers[i].output_size > max_w) return -1;
    long nw = 0;
    for (int i = 0; i < L; i++) nw += (long)nn->layers[i].input_size * nn->layers[i].output_size;
    if (max_w <= 128 && nw > nn->tiny_wt_cap) {
        phip_free(nn->d_tiny_wt);
        nn->d_tiny_wt = (float*)phip_malloc(sizeof(float) * (size_t)nw);
        nn->tiny_wt_cap = nw;
    }
    memset(t, 0, sizeof(*t));
    t->L = L;
    for (int i = 0; i <= L; i++) t->sizes[i] = nn->layers[i].input_size;
    for (int i = 0; i < L; i++) {
        t->relu[i] = nn_is_relu(nn, i);
        t->woff[i] = nn->param_offset[i];
        t->boff[i] = nn->bias_offset[i];
    }
    if (t->sizes[L] > 32) return -1;
    t->params = nn->d_params;
    t->grads = nn->d_grads;
    t->wt = (float*)nn->d_tiny_wt;
    t->wt_cap = nn->tiny_wt_cap;
    t->m = adam->m;
    t->v = adam->v;
    t->span = adam->span;
    return 0;
}

/* Adam step of a network's flat span; in bf16 mode the same pass refreshes the bf16 parameter
 * shadow when the span starts at the network's parameters, else a separate conversion does.
 * zero_grads: the same pass clears the gradients it read (the next backward skips its memset) */
static int adam_update_net(Adam* adam, float lr, NeuralNetwork* nn, int zero_grads) {
    const int own = adam->flat && adam->weights[0] == nn->d_params && adam->grad_weights[0] == nn->d_grads;
    const int fused = nn->dtype == 1 && own;
    const int r = adam_update_cuda_w16(adam, lr, fused ? nn->d_w16 : NULL, nn->num_params, zero_grads && own);
    if (!(r & 1) && nn->dtype == 1) nn_sync_w16(nn);
    return (r & 2) != 0;                 /* the network's gradients are zero again */
}

/* the step-table form of adam_update_net / the entropy Adam (graph replay): flat span, gradients
 * cleared, step sizes from the table; which = 0 advances the step counter (the network's Adam,
 * the step's last kernel), 1 reads the entropy entry */
static void adam_net_tab(Adam* adam, NeuralNetwork* nn, PPODev* d, int ph, int which) {
    const int fused = nn && nn->dtype == 1;
    phip_adam_flat_tab(adam->weights[0], adam->grad_weights[0], adam->m, adam->v, adam->span, d->tab[ph], d->ctr + ph,
                       (unsigned*)(d->ctr + 2 + ph), which, adam->beta1, adam->beta2,
                       adam->grad_scale, fused ? nn->d_w16 : NULL, fused ? nn->num_params : 0, 1);
    nn_note_device_update(adam->weights[0]);
}

static float* tiny_steps(PPODev* d, int slot, Adam* adam, float lr, int n) {
    float* h = (float*)xmalloc(sizeof(float) * 2 * (size_t)n);
    for (int i = 0; i < n; i++) adam_next_step(adam, lr, &h[2 * i], &h[2 * i + 1]);
    if (n > d->tiny_cap[slot]) {
        phip_free(d->tiny_steps[slot]);
        d->tiny_steps[slot] = (float*)phip_malloc(sizeof(float) * 2 * (size_t)n);
        d->tiny_cap[slot] = n;
    }
    phip_h2d(d->tiny_steps[slot], h, sizeof(float) * 2 * (size_t)n);
    free(h);
    return d->tiny_steps[slot];
}

/* every epoch's minibatch order for one phase (slot 0 value, 1 policy), drawn in the reference's
 * order (one shuffle per epoch): device-shuffle keys into keys[], or host rand() permutations
 * copied into HBM, epoch e at the returned pointer + e·limit */
static const int* phase_perms(PPO* ppo, PPODev* d, int shuffle_mode, int n_epochs, int limit, int slot,
                              uint64_t* keys) {
    if (shuffle_mode == PPO_SHUFFLE_DEVICE) {
        for (int e = 0; e < n_epochs; e++) keys[e] = d->key++;
        return NULL;
    }
    const long need = (long)n_epochs * limit;
    if (need > d->perm_cap[slot]) {
        phip_free(d->perm[slot]);
        d->perm[slot] = (int*)phip_malloc(sizeof(int) * (size_t)need);
        d->perm_cap[slot] = need;
    }
    for (int e = 0; e < n_epochs; e++) {
        shuffle_buffer_cuda(ppo->buffer);
        phip_d2d(d->perm[slot] + (long)e * limit, ppo->buffer->random_idx, sizeof(int) * (size_t)limit);
        keys[e] = 0;
    }
    return d->perm[slot];
}

static const int* tiny_perms(PPO* ppo, PPODev* d, int shuffle_mode, int n_epochs, int limit, PhipTinyPhase* ph) {
    uint64_t keys[16];
    const int* perms = phase_perms(ppo, d, shuffle_mode, n_epochs, limit, ph->policy, keys);
    if (shuffle_mode == PPO_SHUFFLE_DEVICE)
        for (int e = 0; e < n_epochs; e++)
            for (int r = 0; r < 4; r++) ph->feistel_k[4 * e + r] = (uint32_t)splitmix64(keys[e] + (uint64_t)r);
    return perms;
}

static int ppo_update_tiny(PPO* ppo, PPODev* d, int B, int n_epochs_policy, int n_epochs_value, int shuffle_mode) {
    TrajectoryBuffer* buf = ppo->buffer;
    const int limit = buf->full ? buf->capacity : buf->idx;
    const int num_batches = buf->capacity / B;
    if (getenv("PPO_NO_TINY") || phip_comm_world() > 1 || n_epochs_value > 16 || n_epochs_policy > 16) return -1;
    PhipTinyNet nv, np;
    /* one workgroup per phase for networks ≤ 128 wide; otherwise the cluster kernel (S → 256 → 256 → O
     * at B = 64, cluster.hip) when it takes the shape */
    int cluster = 0;
    if (tiny_net(ppo->V, ppo->adam_V, &nv, 128) || tiny_net(ppo->policy->mu, ppo->adam_policy, &np, 128)) {
        if (tiny_net(ppo->V, ppo->adam_V, &nv, 1 << 20) || tiny_net(ppo->policy->mu, ppo->adam_policy, &np, 1 << 20))
            return -1;
        cluster = 1;
    }
    int (*phase_fn)(const PhipTinyNet*, const PhipTinyPhase*) = cluster ? phip_cluster_update : phip_tiny_update;
    if (!ppo->adam_entropy->flat || ppo->adam_entropy->grad_weights[0] != ppo->policy->d_log_std_grad) return -1;
    GaussianPolicy* pol = ppo->policy;
    np.log_std = pol->d_log_std;
    np.log_std_grad = pol->d_log_std_grad;
    np.m_ls = ppo->adam_entropy->m;
    np.v_ls = ppo->adam_entropy->v;
    PhipTinyPhase ph;
    memset(&ph, 0, sizeof(ph));
    ph.state = buf->state_p; ph.action = buf->action_p; ph.logprob = buf->logprob_p;
    ph.adv = buf->advantage_p; ph.adv_target = buf->adv_target_p;
    ph.limit = limit; ph.B = B; ph.num_batches = num_batches;
    ph.b1 = 0.9f; ph.b2 = 0.999f; ph.eps = ppo->epsilon; ph.ent_coeff = ppo->ent_coeff;
    ph.stats = d->stats;
    /* fit check before any state (rand() stream, Adam steps, keys) is consumed: a dry phase */
    {
        PhipTinyNet probe = nv;
        PhipTinyPhase pp = ph;
        pp.n_epochs = 0;
        if (phase_fn(&probe, &pp) != 0) return -1;
        probe = np;
        pp.policy = 1;
        if (phase_fn(&probe, &pp) != 0) return -1;
    }
    /* both phases' permutations and Adam step tables first, in the reference's order (value
     * epochs' shuffles, then the policy's); then the two single-workgroup phases run concurrently
     * (value on libppo's stream, policy on the side stream: they share only read-only buffer
     * arrays), each on its own CU.  PPO_SERIAL=1 runs them one after the other. */
    PhipTinyPhase pv = ph, pp = ph;
    /* step caps (ppo_set_step_limit): the first max steps of each phase, as in the multi-launch loop */
    long cap_v = (long)n_epochs_value * num_batches, cap_p = (long)n_epochs_policy * num_batches;
    if (d->max_v >= 0 && cap_v > d->max_v) cap_v = d->max_v;
    if (d->max_p >= 0 && cap_p > d->max_p) cap_p = d->max_p;
    const int run_v = cap_v > 0, run_p = cap_p > 0;
    if (run_v) {
        pv.policy = 0;
        pv.n_epochs = n_epochs_value;
        pv.max_steps = cap_v;
        pv.perms = tiny_perms(ppo, d, shuffle_mode, n_epochs_value, limit, &pv);
        pv.steps = tiny_steps(d, 0, ppo->adam_V, ppo->lr_V, (int)cap_v);
    } else if (n_epochs_value > 0) {
        for (int j = 0; j < n_epochs_value; j++) { uint64_t key; next_perm(ppo, d, shuffle_mode, &key); }
    }
    if (run_p) {
        pp.policy = 1;
        pp.n_epochs = n_epochs_policy;
        pp.max_steps = cap_p;
        pp.perms = tiny_perms(ppo, d, shuffle_mode, n_epochs_policy, limit, &pp);
        /* per step the entropy Adam steps before the policy Adam (ppo.cu:440-442); their step
         * counters are independent, so the two sequences can be generated one after the other */
        pp.steps_ls = tiny_steps(d, 1, ppo->adam_entropy, ppo->lr_policy, (int)cap_p);
        pp.steps = tiny_steps(d, 2, ppo->adam_policy, ppo->lr_policy, (int)cap_p);
    } else if (n_epochs_policy > 0) {
        for (int j = 0; j < n_epochs_policy; j++) { uint64_t key; next_perm(ppo, d, shuffle_mode, &key); }
    }
    const char* serial_env = getenv("PPO_SERIAL");
    const int concurrent = run_v && run_p && !(serial_env && *serial_env && *serial_env != '0');
    if (concurrent) phip_side_fork();
    if (run_v) {
        if (phase_fn(&nv, &pv) != 0) die("ppo_update: single-launch value phase failed to launch");
        d->n_v += cap_v;
    }
    if (run_p) {
        if (concurrent) phip_side_use(1);
        if (phase_fn(&np, &pp) != 0) die("ppo_update: single-launch policy phase failed to launch");
        if (concurrent) phip_side_use(0);
        d->n_p += cap_p;
    }
    if (concurrent) phip_side_join();
    if (cluster) {
        /* a barrier timeout leaves the phase's parameters and Adam state half-written (the workgroups
         * leave without their write-back): detect it before this update returns, so no caller reads,
         * checkpoints or continues from that state */
        phip_sync();
        if (phip_cluster_error())
            die("ppo_update: a multi-workgroup phase (cluster.hip) timed out at a grid barrier; "
                "the update's parameters and Adam state are incomplete");
        phip_cluster_report();
    }
    return 0;
}

/* ------------------------------------------------------------------ */
/* one value / policy minibatch step (ppo.cu:395-443 bodies)           */
/* ------------------------------------------------------------------ */
typedef struct {
    PPO* ppo;
    PPODev* d;
    int B, S, A, limit, num_batches, comm, fuse_v, fuse_p, wide_p, fold_v;
    const int *perms_v, *perms_p;
    const uint64_t *keys_v, *keys_p;
    long nv, np;
    void *gv, *gp;                /* captured graphs of K steps each (value, policy) */
    void *gv1, *gp1;              /* … and of one step (the remainder) */
    int K;                        /* requested steps per graph (PPO_GRAPH_STEPS, default 16) */
    long Kv, Kp;                  /* steps per graph as captured */
    int phg;                      /* the phases' inputs were gathered up front (PPODev ph_*) */
} StepCtx;

/* value step iv (tab: the step-table form captured into a graph: gather and Adam read their
 * per-step arguments from d->tab[0] at the device step counter); returns whether its Adam cleared
 * the gradients */
static int value_step(StepCtx* c, long iv, int v_zero, int tab) {
    PPO* ppo = c->ppo;
    PPODev* d = c->d;
    TrajectoryBuffer* buf = ppo->buffer;
    NeuralNetwork* V = ppo->V;
    const int B = c->B;
    const int* rows = d->rows;
    const float* tgt = d->tgt;
    if (tab) {
        phip_gather_rows_tab(d->tab[0], d->ctr + 0, c->perms_v, c->limit, B, c->A, buf->action_p, buf->logprob_p,
                             buf->advantage_p, buf->adv_target_p, NULL, NULL, NULL, d->tgt, d->rows);
    } else if (c->phg) {
        rows = d->ph_rows[0] + iv * B;
        tgt = d->ph_tgt + iv * B;
    } else {
        const int j = (int)(iv / c->num_batches), k = (int)(iv % c->num_batches);
        const int* perm = c->perms_v ? c->perms_v + (long)j * c->limit : NULL;
        /* gather fused into layer 0: the kernel emits row indices (+ targets); the layer-0 GEMM
         * reads the buffer rows through them and leaves the gathered copy for its grad_W */
        phip_gather_rows(perm, c->keys_v[j], k * B, c->limit, B, c->S, c->A, buf->state_p, buf->action_p,
                         buf->logprob_p, buf->advantage_p, buf->adv_target_p, NULL, NULL, NULL, NULL, d->tgt, d->rows);
    }
    /* with a communicator: the gradients all-reduced after the backward (comm.hip: one all-reduce in
     * this stream by default; PPO_COMM_ASYNC=1 per-layer buckets on the comm stream), joined before Adam */
    if (c->fold_v && !tab) {   /* output layer + MSE folded into the last hidden layer (nn_value_fold_step) */
        nn_value_fold_step(V, buf->state_p, rows, d->states, B, v_zero, c->comm ? 0 : -1, tgt, d->stats + 0);
    } else if (c->fuse_v) {    /* output layer + MSE + output-layer backward in one pass (out_head.hip) */
        nn_out_head_step(V, 0, buf->state_p, rows, d->states, B, v_zero, c->comm ? 0 : -1, tgt, NULL, NULL,
                         NULL, NULL, 0.f, 0.f, NULL, d->stats + 0);
    } else {
        nn_forward_dev_rows(V, buf->state_p, rows, d->states, B);
        phip_mse(V->d_output, tgt, B, d->gv, NULL, d->stats + 0);
        nn_backward_dev_z(V, d->gv, B, 0, v_zero, c->comm ? 0 : -1);
    }
    phip_allreduce_join();
    if (tab) {
        adam_net_tab(ppo->adam_V, V, d, 0, 0);
        return 1;
    }
    return adam_update_net(ppo->adam_V, ppo->lr_V, V, iv + 1 < c->nv);
}

static void policy_step(StepCtx* c, long ip, int* p_zero, int* ls_zero, int tab) {
    PPO* ppo = c->ppo;
    PPODev* d = c->d;
    TrajectoryBuffer* buf = ppo->buffer;
    GaussianPolicy* pol = ppo->policy;
    NeuralNetwork* mu = pol->mu;
    const int B = c->B, A = c->A;
    const int* rows = d->rows_p;
    const float *act = d->actions, *olp = d->old_lp, *adv = d->adv;
    if (tab) {
        phip_gather_rows_tab(d->tab[1], d->ctr + 1, c->perms_p, c->limit, B, A, buf->action_p, buf->logprob_p,
                             buf->advantage_p, buf->adv_target_p, d->actions, d->old_lp, d->adv, NULL, d->rows_p);
    } else if (c->phg) {
        rows = d->ph_rows[1] + ip * B;
        act = d->ph_act + ip * B * A;
        olp = d->ph_olp + ip * B;
        adv = d->ph_adv + ip * B;
    } else {
        const int j = (int)(ip / c->num_batches), k = (int)(ip % c->num_batches);
        const int* perm = c->perms_p ? c->perms_p + (long)j * c->limit : NULL;
        phip_gather_rows(perm, c->keys_p[j], k * B, c->limit, B, c->S, A, buf->state_p, buf->action_p,
                         buf->logprob_p, buf->advantage_p, buf->adv_target_p, NULL, d->actions, d->old_lp, d->adv,
                         NULL, d->rows_p);
    }
    /* μ grads + (top bucket) the log σ gradient behind them */
    if (c->fuse_p) {       /* output layer + clipped surrogate + output-layer backward (out_head.hip) */
        if (!*ls_zero) phip_memset(pol->d_log_std_grad, 0, sizeof(float) * (size_t)A);
        nn_out_head_step(mu, 1, buf->state_p, rows, d->states_p, B, *p_zero, c->comm ? align4(A) : -1, NULL,
                         pol->d_log_std, act, adv, olp, ppo->epsilon, ppo->ent_coeff,
                         pol->d_log_std_grad, d->stats + 1);
    } else if (c->wide_p) { /* A = 17: policy head + output-layer backward in one pass (out_head.hip) */
        if (!*ls_zero) phip_memset(pol->d_log_std_grad, 0, sizeof(float) * (size_t)A);
        nn_policy_wide_step(mu, buf->state_p, rows, d->states_p, B, *p_zero, c->comm ? align4(A) : -1,
                            pol->d_log_std, act, adv, olp, ppo->epsilon, ppo->ent_coeff,
                            pol->d_log_std_grad, d->stats + 1);
    } else {
        nn_forward_dev_rows(mu, buf->state_p, rows, d->states_p, B);
        phip_policy_head(mu->d_output, pol->d_log_std, act, adv, olp, B, A, ppo->epsilon,
                         ppo->ent_coeff, d->gmu, pol->d_log_std_grad, d->stats + 1, *ls_zero);
        nn_backward_dev_z(mu, d->gmu, B, 0, *p_zero, c->comm ? align4(A) : -1);
    }
    phip_allreduce_join();
    /* ppo.cu:440-442 order; the entropy Adam clears the log σ gradient it read (the next policy head
     * accumulates into zeros) */
    if (tab) {
        adam_net_tab(ppo->adam_entropy, NULL, d, 1, 1);
        adam_net_tab(ppo->adam_policy, mu, d, 1, 0);
        *ls_zero = *p_zero = 1;
        return;
    }
    /* both Adams in one launch where they qualify (flat spans, the network's 16-B aligned) */
    Adam* ap = ppo->adam_policy;
    const int own = ap->flat && ap->weights[0] == mu->d_params && ap->grad_weights[0] == mu->d_grads;
    const int fused = mu->dtype == 1 && own;
    const int ls_own = ppo->adam_entropy->flat && ppo->adam_entropy->grad_weights[0] == pol->d_log_std_grad;
    const int r = adam_update_pair_w16(ap, ppo->lr_policy, fused ? mu->d_w16 : NULL, mu->num_params,
                                         ip + 1 < c->np && own, ppo->adam_entropy, ppo->lr_policy,
                                         ip + 1 < c->np && ls_own);
    if (r >= 0) {
        if (!(r & 1) && mu->dtype == 1) nn_sync_w16(mu);
        *ls_zero = ls_own && (r & 4);
        *p_zero = (r & 2) != 0;
        return;
    }
    *ls_zero = ls_own && (adam_update_cuda_w16(ppo->adam_entropy, ppo->lr_policy, NULL, 0, ip + 1 < c->np) & 2);
    *p_zero = adam_update_net(ppo->adam_policy, ppo->lr_policy, mu, ip + 1 < c->np);
}

/* graph replay (opt-in, PPO_GRAPH=1; PPO_GRAPH_STEPS = steps per captured graph, default 16) for
 * small minibatches on one GPU when every Adam of the step is a flat, 16-B aligned span that owns its
 * network (the table kernels' form).  Measured at C3, B = 64 (profiles/r03_graph_replay.txt): eager
 * 2062 ms per update, graphs of 1 / 4 / 16 / 64 steps 2375 / 2156 / 2104 / 2091 ms — on this ROCm a
 * graph replays its kernel nodes at the eager launch cost, and the step is GPU-bound (≈ 36 µs for 8–9
 * dependent small kernels), so it stays off by default. */
static int step_graphs_ok(const StepCtx* c) {
    const char* e = getenv("PPO_GRAPH");
    if (!(e && *e && *e != '0') || c->comm || phip_comm_world() > 1 || c->B > 2048 || c->A > 32) return 0;
    PPO* ppo = c->ppo;
    Adam* ads[3] = {ppo->adam_V, ppo->adam_policy, ppo->adam_entropy};
    for (int i = 0; i < 3; i++) {
        Adam* a = ads[i];
        const uintptr_t al = (uintptr_t)a->weights[0] | (uintptr_t)a->grad_weights[0] | (uintptr_t)a->m |
                             (uintptr_t)a->v;
        if (!a->flat || (al & 15u)) return 0;
    }
    /* the table Adam always clears the gradient it read (the captured steps run their backward with
     * the gradients already zero), so every Adam must own its network's gradient span, as `own` in
     * adam_update_net requires on the eager path */
    if (ppo->adam_V->weights[0] != ppo->V->d_params || ppo->adam_V->grad_weights[0] != ppo->V->d_grads ||
        ppo->adam_policy->weights[0] != ppo->policy->mu->d_params ||
        ppo->adam_policy->grad_weights[0] != ppo->policy->mu->d_grads ||
        ppo->adam_entropy->grad_weights[0] != ppo->policy->d_log_std_grad)
        return 0;
    /* only the combination tests/test_gpu_update.py replays against eager launches: fp32 networks with
     * the fused output heads (value A = 1, policy A <= 6) */
    if (ppo->V->dtype != 0 || ppo->policy->mu->dtype != 0 || !c->fuse_v || !c->fuse_p || c->fold_v) return 0;
    return 1;
}

/* the step table of phase ph (0 value, 1 policy) for steps 1 … n−2 — epoch order, minibatch offset
 * and the Adam step sizes in the reference's step order (advancing the host Adam step counters as
 * the eager path does) — uploaded, the counter reset, and one step captured as a graph */
static void* capture_graph(StepCtx* c, int ph, int steps) {
    if (phip_graph_begin() != 0) return NULL;
    for (int s = 0; s < steps; s++) {
        if (ph) {
            int pz = 1, lz = 1;
            policy_step(c, 1, &pz, &lz, 1);
        } else {
            (void)value_step(c, 1, 1, 1);
        }
    }
    return phip_graph_end();
}

static void capture_steps(StepCtx* c, int ph) {
    PPO* ppo = c->ppo;
    PPODev* d = c->d;
    const long n = (ph ? c->np : c->nv) - 2;
    if (n <= 0) return;
    if (n > d->h_tab_cap) {
        free(d->h_tab);
        d->h_tab = (PhipStepArgs*)xmalloc(sizeof(PhipStepArgs) * (size_t)n);
        d->h_tab_cap = n;
    }
    if (n > d->tab_cap[ph]) {
        phip_free(d->tab[ph]);
        d->tab[ph] = (PhipStepArgs*)phip_malloc(sizeof(PhipStepArgs) * (size_t)n);
        d->tab_cap[ph] = n;
    }
    if (!d->ctr) d->ctr = (int*)phip_malloc(sizeof(int) * 4);
    const int* perms = ph ? c->perms_p : c->perms_v;
    const uint64_t* keys = ph ? c->keys_p : c->keys_v;
    /* the table advances the host Adam step counters as the eager steps would; kept to roll back if
     * the capture fails (the phase then runs every step eagerly) */
    const int t_v = ppo->adam_V->time_step, t_p = ppo->adam_policy->time_step, t_e = ppo->adam_entropy->time_step;
    for (long t = 0; t < n; t++) {
        const long i = t + 1;
        const int j = (int)(i / c->num_batches), k = (int)(i % c->num_batches);
        PhipStepArgs* e = &d->h_tab[t];
        memset(e, 0, sizeof(*e));
        e->perm_off = perms ? (long)j * c->limit : -1;
        if (!perms) phip_step_feistel(e, keys[j], c->limit);
        e->offset = k * c->B;
        if (ph) {
            adam_next_step(ppo->adam_entropy, ppo->lr_policy, &e->step_ls, &e->bc2_ls);   /* ppo.cu:440-442 */
            adam_next_step(ppo->adam_policy, ppo->lr_policy, &e->step, &e->bc2);
        } else {
            adam_next_step(ppo->adam_V, ppo->lr_V, &e->step, &e->bc2);
        }
    }
    phip_h2d(d->tab[ph], d->h_tab, sizeof(PhipStepArgs) * (size_t)n);
    phip_memset(d->ctr + ph, 0, sizeof(int));
    phip_memset(d->ctr + 2 + ph, 0, sizeof(int));
    const int K = (int)(n < c->K ? n : c->K);
    void* gk = capture_graph(c, ph, K);
    void* g1 = gk && K > 1 ? capture_graph(c, ph, 1) : NULL;
    if (!gk || (K > 1 && !g1)) {
        /* an opt-in speed feature must not end a training run: warn, drop the graphs, replay nothing */
        fprintf(stderr, "libppo: warning: graph capture of the %s steps failed (%s); running them eagerly\n",
                ph ? "policy" : "value", phip_graph_error());
        phip_graph_destroy(gk);
        phip_graph_destroy(g1);
        ppo->adam_V->time_step = t_v;
        ppo->adam_policy->time_step = t_p;
        ppo->adam_entropy->time_step = t_e;
        return;
    }
    if (ph) { c->gp = gk; c->gp1 = g1; c->Kp = K; } else { c->gv = gk; c->gv1 = g1; c->Kv = K; }
}

static void ppo_update_body(PPO* ppo, float gamma, int batch_size, int n_epochs_policy, int n_epochs_value,
                            int shuffle_mode, unsigned long long seed);

/* the phases' minibatch inputs, gathered before the loops: the rows of epoch j's steps are one gather
 * of num_batches·B consecutive list positions (step k's slot i is position k·B + i, modulo the buffer
 * length, as the per-step gather takes it — trajectory_buffer.cu get_batch), so ph_rows[p] + iv·B holds
 * exactly the rows step iv would have gathered */
static void phase_gather(StepCtx* c) {
    PPO* ppo = c->ppo;
    PPODev* d = c->d;
    TrajectoryBuffer* buf = ppo->buffer;
    const long B = c->B, A = c->A, per = (long)c->num_batches * B;
    for (int ph = 0; ph < 2; ph++) {
        const long n = ph ? c->np : c->nv;
        if (n <= 0) continue;
        if (n * B > d->ph_cap[ph]) {
            phip_free(d->ph_rows[ph]);
            d->ph_rows[ph] = (int*)phip_malloc(sizeof(int) * (size_t)(n * B));
            if (ph) {
                phip_free(d->ph_act); phip_free(d->ph_olp); phip_free(d->ph_adv);
                d->ph_act = (float*)phip_malloc(sizeof(float) * (size_t)(n * B * A));
                d->ph_olp = (float*)phip_malloc(sizeof(float) * (size_t)(n * B));
                d->ph_adv = (float*)phip_malloc(sizeof(float) * (size_t)(n * B));
            } else {
                phip_free(d->ph_tgt);
                d->ph_tgt = (float*)phip_malloc(sizeof(float) * (size_t)(n * B));
            }
            d->ph_cap[ph] = n * B;
        }
        const int* perms = ph ? c->perms_p : c->perms_v;
        const uint64_t* keys = ph ? c->keys_p : c->keys_v;
        for (long j = 0; j * c->num_batches < n; j++) {
            const long steps = n - j * c->num_batches < c->num_batches ? n - j * c->num_batches : c->num_batches;
            const long o = j * per;
            if (steps * B >= (1L << 31)) die("ppo_update: a phase epoch exceeds 2^31 rows");
            phip_gather_rows(perms ? perms + j * c->limit : NULL, keys[j], 0, c->limit, (int)(steps * B), c->S, c->A,
                             buf->state_p, buf->action_p, buf->logprob_p, buf->advantage_p, buf->adv_target_p, NULL,
                             ph ? d->ph_act + o * A : NULL, ph ? d->ph_olp + o : NULL, ph ? d->ph_adv + o : NULL,
                             ph ? NULL : d->ph_tgt + o, d->ph_rows[ph] + o);
        }
    }
    c->phg = 1;
}

/* the replica check's parameter spans in HBM: μ, log σ, V */
static void replica_hash(PPO* ppo) {
    GaussianPolicy* pol = ppo->policy;
    const float* spans[3] = {pol->mu->d_params, pol->d_log_std, ppo->V->d_params};
    const long lens[3] = {pol->mu->num_params, pol->action_size, ppo->V->num_params};
    phip_param_hash(spans, lens, 3);
}

unsigned long long ppo_param_hash(void* vppo) {
    unsigned long long h = 0;
    replica_hash((PPO*)vppo);
    char msg[8];
    (void)phip_comm_check_hash(0, &h, msg, 0);    /* this rank's hash only: no collective */
    return h;
}

int ppo_comm_check_replicas(void* vppo) {
    replica_hash((PPO*)vppo);
    char msg[400];
    if (phip_comm_check_hash(1, NULL, msg, (int)sizeof(msg)) == 0) return 0;
    char buf[480];
    snprintf(buf, sizeof(buf), "replica check: parameters differ across ranks: %s", msg);
    phip_record_error(buf);
    return -1;
}

/* PPO_REPLICA_CHECK=K: the replica check after every K-th update at world > 1 (default 1, 0 = off) */
static int replica_check_due(void) {
    static long n = 0;
    const char* e = getenv("PPO_REPLICA_CHECK");
    const long k = e && *e ? atol(e) : 1;
    if (k <= 0) return 0;
    return ++n % k == 0;
}

void ppo_update(void* vppo, float gamma, int batch_size, int n_epochs_policy, int n_epochs_value, int shuffle_mode,
                unsigned long long seed) {
    PPO* ppo = (PPO*)vppo;
    ppo_update_body(ppo, gamma, batch_size, n_epochs_policy, n_epochs_value, shuffle_mode, seed);
    ppo->V->dev_version++;               /* HBM parameters moved (also by the single-workgroup path) */
    ppo->policy->mu->dev_version++;
    /* replicated Adam must leave every rank with the same parameters; a rank that drifted
     * would otherwise train on its own weights silently */
    if (phip_comm_world() > 1 && replica_check_due() && ppo_comm_check_replicas(ppo) != 0)
        die(ppo_last_error());
}

static void ppo_update_body(PPO* ppo, float gamma, int batch_size, int n_epochs_policy, int n_epochs_value,
                            int shuffle_mode, unsigned long long seed) {
    TrajectoryBuffer* buf = ppo->buffer;
    if (phip_cluster_error()) die("ppo_update: a multi-workgroup phase (cluster.hip) timed out at a barrier");
    if (!buf->on_device) die("ppo_update: buffer must be device-resident (buffer_to_device / ppo_fill_synthetic)");
    if (batch_size <= 0) die("ppo_update: batch_size must be positive");
    PPODev* d = dev_ws(ppo, batch_size);
    if (shuffle_mode == PPO_SHUFFLE_DEVICE && (!d->seeded || d->seed != seed)) {
        d->seed = seed;
        d->key = splitmix64(seed);
        d->seeded = 1;
    }
    const int S = buf->state_size, A = buf->action_size, B = batch_size;
    const int limit = buf->full ? buf->capacity : buf->idx;
    const int num_batches = buf->capacity / B;                           /* D13 */
    const int world = phip_comm_world();
    const float gscale = 1.0f / (float)world;
    const int comm = phip_comm_active();
    ppo->adam_V->grad_scale = gscale;
    ppo->adam_policy->grad_scale = gscale;
    ppo->adam_entropy->grad_scale = gscale;
    NeuralNetwork* V = ppo->V;
    GaussianPolicy* pol = ppo->policy;
    NeuralNetwork* mu = pol->mu;

    ppo_gae_device(V, buf, gamma, ppo->lambda);
    /* D19: an empty buffer (idx = 0, not full) has nothing to train on; the reference would divide
     * by zero (rand() % 0 in shuffle_buffer, % limit in get_batch) — here the update ends after GAE.
     * At world > 1 the ranks agree first (min over ranks): one empty shard ends the update on every
     * rank, so no rank waits in a gradient all-reduce the others never issue. */
    if ((world > 1 ? phip_comm_min_i32(limit) : limit) <= 0) return;

    if (ppo_update_tiny(ppo, d, B, n_epochs_policy, n_epochs_value, shuffle_mode) == 0) return;

    /* The policy loop reads only the buffer and the advantages — nothing the value loop writes —
     * so on one GPU the two run concurrently: value steps on libppo's stream, policy steps on its
     * side stream (own workspaces), issued interleaved.  Every network sees exactly the reference's
     * sequence of minibatches and Adam steps; epochs' shuffles are drawn up front in the
     * reference's order (value epochs first).  PPO_SERIAL=1 runs them one after the other.  Under
     * data parallelism (world > 1) each loop issues one gradient all-reduce per step in its own
     * stream on its own communicator (comm.hip; PPO_COMM_ASYNC=1: per-layer buckets on one comm
     * stream).  The interleave below is a fixed function of (iv, ip, nv, np), never of timing, so
     * every rank issues the same total order of collectives — half of comm.hip's deadlock argument. */
    long nv = (long)n_epochs_value * num_batches, np = (long)n_epochs_policy * num_batches;
    if (d->max_v >= 0 && nv > d->max_v) nv = d->max_v;
    if (d->max_p >= 0 && np > d->max_p) np = d->max_p;
    uint64_t* keys = (uint64_t*)xmalloc(sizeof(uint64_t) * (size_t)(n_epochs_value + n_epochs_policy + 1));
    uint64_t* keys_v = keys;
    uint64_t* keys_p = keys + n_epochs_value;
    const int* perms_v = phase_perms(ppo, d, shuffle_mode, n_epochs_value, limit, 0, keys_v);
    const int* perms_p = phase_perms(ppo, d, shuffle_mode, n_epochs_policy, limit, 1, keys_p);
    const char* serial_env = getenv("PPO_SERIAL");
    const int concurrent = nv > 0 && np > 0 && !(serial_env && *serial_env && *serial_env != '0');
    const int fuse_p = nn_out_head_ok(mu, 1);
    StepCtx c = {ppo, d, B, S, A, limit, num_batches, comm, nn_out_head_ok(V, 0), fuse_p,
                 !fuse_p && nn_policy_wide_ok(mu, B), nn_value_fold_ok(V, B), perms_v, perms_p, keys_v, keys_p, nv, np,
                 NULL, NULL, NULL, NULL, 16, 1, 1, 0};
    {
        const char* ge = getenv("PPO_GRAPH_STEPS");
        if (ge && atoi(ge) > 0) c.K = atoi(ge);
    }
    /* graph replay (opt-in): steps 1 … n−2 of a phase replay captured graphs of K steps (the first
     * step runs eagerly — workspaces allocated, gradients cleared — and the last one too, so the
     * caller can read its gradients) */
    const int graphs = step_graphs_ok(&c);
    /* eager steps: every step's gathered inputs up front (one launch per epoch instead of one per
     * step; on libppo's stream before the fork, so both loops see them) */
    if (!graphs) phase_gather(&c);
    if (concurrent) phip_side_fork();
    long iv = 0, ip = 0;
    /* gradients cleared by the previous Adam step (not after a loop's last step: a caller may read
     * the last minibatch's gradients after the update) */
    int v_zero = 0, p_zero = 0, ls_zero = 0;
    while (iv < nv || ip < np) {
        /* serial: every value step first (the reference's order); concurrent: issue in proportion */
        const int take_v = iv < nv && (ip >= np || !concurrent || iv * np <= ip * nv);
        if (take_v) {
            long done = 1;
            if (c.gv && iv >= 1 && iv + 1 < nv) {
                if (nv - 1 - iv >= c.Kv) { phip_graph_launch(c.gv); done = c.Kv; }
                else phip_graph_launch(c.gv1 ? c.gv1 : c.gv);
                d->n_graph += done;
            } else {
                v_zero = value_step(&c, iv, v_zero, 0);
                if (iv == 0 && graphs && nv >= 3) capture_steps(&c, 0);
            }
            d->n_v += done;
            iv += done;
        } else {
            long done = 1;
            if (concurrent) phip_side_use(1);
            if (c.gp && ip >= 1 && ip + 1 < np) {
                if (np - 1 - ip >= c.Kp) { phip_graph_launch(c.gp); done = c.Kp; }
                else phip_graph_launch(c.gp1 ? c.gp1 : c.gp);
                d->n_graph += done;
            } else {
                policy_step(&c, ip, &p_zero, &ls_zero, 0);
                if (ip == 0 && graphs && np >= 3) capture_steps(&c, 1);
            }
            if (concurrent) phip_side_use(0);
            d->n_p += done;
            ip += done;
        }
    }
    phip_graph_destroy(c.gv);
    phip_graph_destroy(c.gp);
    phip_graph_destroy(c.gv1);
    phip_graph_destroy(c.gp1);
    if (concurrent) phip_side_join();
    free(keys);
}

void ppo_set_step_limit(void* vppo, long max_value_steps, long max_policy_steps) {
    PPODev* d = dev_ws((PPO*)vppo, 1);
    d->max_v = max_value_steps;
    d->max_p = max_policy_steps;
}

void ppo_reset_stats(void* vppo) {
    PPO* ppo = (PPO*)vppo;
    PPODev* d = dev_ws(ppo, 1);
    phip_memset(d->stats, 0, 4 * sizeof(float));
    d->n_v = d->n_p = d->n_graph = 0;
}

void ppo_read_stats(void* vppo, double* out, int n) {
    PPO* ppo = (PPO*)vppo;
    PPODev* d = dev_ws(ppo, 1);
    float s[4] = {0, 0, 0, 0}, a[2] = {0, 0};
    phip_d2h(s, d->stats, sizeof(s));
    if (g_adv_stats) phip_d2h(a, g_adv_stats, sizeof(a));
    double v[9] = {s[0], (double)d->n_v, s[1], (double)d->n_p, compute_entropy_cuda(ppo->policy), a[0], a[1],
                   (double)g_gae_own_rows, (double)d->n_graph};
    for (int i = 0; i < n && i < 9; i++) out[i] = v[i];
}

/* ppo.cu:451-558 */
void train_ppo_epoch(PPO* ppo, Env* env, int steps_per_epoch, int batch_size, int n_epochs_policy,
                     int n_epochs_value) {
    for (int i = 0; i < steps_per_epoch / ppo->buffer->capacity; i++) {
        collect_trajectories(ppo->buffer, env, ppo->policy, ppo->buffer->capacity);
        buffer_to_device(ppo->buffer);
        ppo_update(ppo, env->gamma, batch_size, n_epochs_policy, n_epochs_value, PPO_SHUFFLE_HOST_RAND, 0);
        buffer_to_host(ppo->buffer);
        policy_to_host(ppo->policy);
        nn_write_weights_to_host(ppo->V);
    }
}

/* ppo.cu:560-583: rollout `steps` and print the mean discounted return J and return R */
void eval_ppo(PPO* ppo, Env* env, int steps) {
    reset_buffer(ppo->buffer);
    collect_trajectories(ppo->buffer, env, ppo->policy, steps);
    TrajectoryBuffer* b = ppo->buffer;
    float rewards = *b->reward(b, steps - 1);
    float episode_J = *b->reward(b, steps - 1);
    int n_episodes = 1;
    float sum_J = 0;
    for (int i = steps - 2; i >= 0; i--) {
        rewards += *b->reward(b, i);
        episode_J = *b->reward(b, i) + env->gamma * episode_J;
        if (*b->terminated(b, i) || *b->truncated(b, i)) {
            n_episodes++;
            sum_J += episode_J;
            episode_J = 0;
        }
    }
    printf("J: %f R: %f Episodes: %d\n", sum_J / n_episodes, rewards / n_episodes, n_episodes);
    reset_buffer(ppo->buffer);
}

/* ------------------------------------------------------------------ */
/* batched sampling / synthetic rollouts (ppo_ext.h)                   */
/* ------------------------------------------------------------------ */
void ppo_sample_action_device(void* vpolicy, float* d_state, float* d_action, float* d_log_prob, int m,
                              unsigned long long seed, unsigned long long offset) {
    GaussianPolicy* p = (GaussianPolicy*)vpolicy;
    nn_forward_dev(p->mu, d_state, m);
    phip_sample(p->mu->d_output, p->d_log_std, d_action, d_log_prob, m, p->action_size, seed, offset);
}

void ppo_rollout_device(void* vppo, int n_envs, int horizon, int env_kind, unsigned long long seed) {
    PPO* ppo = (PPO*)vppo;
    TrajectoryBuffer* b = ppo->buffer;
    const int E = n_envs, T = horizon;
    const long N = (long)E * T;
    if (E <= 0 || T <= 0 || N > b->capacity) die("ppo_rollout_device: n_envs*horizon must be in [1, capacity]");
    if (env_kind != 0 && env_kind != 1) die("ppo_rollout_device: env_kind must be 0 (Pendulum-v1) or 1 (synthetic)");
    const int S = b->state_size, A = b->action_size;
    if (env_kind == 0 && (S != 3 || A != 1)) die("ppo_rollout_device: Pendulum-v1 needs state_size 3, action_size 1");
    PPODev* d = dev_ws(ppo, 1);
    if (d->ro_E != E || d->ro_T != T) {
        phip_free(d->ro_rows);
        d->ro_rows = (int*)phip_malloc(sizeof(int) * (size_t)N);
        phip_rollout_rows(d->ro_rows, E, T);
        d->ro_T = T;
    }
    if (d->ro_E != E || d->ro_kind != env_kind || d->ro_S != S || !d->env_state) {
        phip_free(d->env_state);
        d->env_state = (float*)phip_malloc(sizeof(float) * (size_t)E * (S > 3 ? S : 3));
        phip_env_reset(env_kind, d->env_state, b->d_state_p, E, T, S, splitmix64(seed));
        d->ro_E = E;
        d->ro_kind = env_kind;
        d->ro_S = S;
    }
    const uint64_t key = splitmix64(seed ^ 0x524F4C4CULL);
    GaussianPolicy* pol = ppo->policy;
    phip_env_first_obs(env_kind, d->env_state, b->d_state_p, E, T, S);
    for (int t = 0; t < T; t++) {
        const int* rows = d->ro_rows + (long)t * E;
        nn_forward_dev_rows(pol->mu, b->d_state_p, rows, NULL, E);
        phip_sample_rows(pol->mu->d_output, pol->d_log_std, rows, b->d_action_p, b->d_logprob_p, E, A, key,
                         d->ro_step++);
        phip_env_step(env_kind, d->env_state, b->d_state_p, b->d_action_p, b->d_next_state_p, b->d_reward_p,
                      (uint8_t*)b->d_terminated_p, (uint8_t*)b->d_truncated_p, E, T, t, S, A, key);
    }
    phip_memset(b->d_advantage_p, 0, sizeof(float) * (size_t)N);
    phip_memset(b->d_adv_target_p, 0, sizeof(float) * (size_t)N);
    b->idx = (int)(N % b->capacity);
    b->full = N == b->capacity;
    buffer_point_device(b);
}

void ppo_fill_synthetic(void* vppo, int n_envs, int horizon, unsigned long long seed, float p_terminate) {
    PPO* ppo = (PPO*)vppo;
    TrajectoryBuffer* b = ppo->buffer;
    const long N = (long)n_envs * horizon;
    if (N <= 0 || N > b->capacity) die("ppo_fill_synthetic: n_envs*horizon must be in [1, capacity]");
    const int S = b->state_size, A = b->action_size;
    const uint64_t s0 = splitmix64(seed);
    phip_fill_uniform(b->d_state_p, N * S, s0 ^ 0x1, -1.f, 1.f);
    phip_fill_rollout_flags((uint8_t*)b->d_terminated_p, (uint8_t*)b->d_truncated_p, n_envs, horizon, p_terminate,
                            s0 ^ 0x2);
    phip_link_next_state(b->d_next_state_p, b->d_state_p, (const uint8_t*)b->d_terminated_p, n_envs, horizon, S,
                         s0 ^ 0x3);
    phip_fill_normal(b->d_reward_p, N, s0 ^ 0x4, 0.1f);
    ppo_sample_action_device(ppo->policy, b->d_state_p, b->d_action_p, b->d_logprob_p, (int)N, s0 ^ 0x5, 0);
    phip_memset(b->d_advantage_p, 0, sizeof(float) * (size_t)N);
    phip_memset(b->d_adv_target_p, 0, sizeof(float) * (size_t)N);
    b->idx = (int)(N % b->capacity);
    b->full = N == b->capacity;
    buffer_point_device(b);
    (void)A;
}

/* ------------------------------------------------------------------ */
/* checkpoint (ppo.cu:585-648 byte layout)                             */
/* ------------------------------------------------------------------ */
void save_ppo(PPO* ppo, const char* filename) {
    FILE* f = fopen(filename, "wb");
    if (!f) die("save_ppo: cannot open file");
    policy_to_host(ppo->policy);
    nn_write_weights_to_host(ppo->V);
    fwrite(&ppo->lambda, sizeof(float), 1, f);
    fwrite(&ppo->epsilon, sizeof(float), 1, f);
    fwrite(&ppo->ent_coeff, sizeof(float), 1, f);
    fwrite(&ppo->lr_policy, sizeof(float), 1, f);
    fwrite(&ppo->lr_V, sizeof(float), 1, f);
    fwrite(&ppo->buffer->state_size, sizeof(int), 1, f);
    fwrite(&ppo->buffer->action_size, sizeof(int), 1, f);
    fwrite(&ppo->buffer->capacity, sizeof(int), 1, f);
    save_policy(ppo->policy, f);
    save_neural_network(ppo->V, f);
    save_adam(ppo->adam_policy, f, true);
    save_adam(ppo->adam_V, f, true);
    save_adam(ppo->adam_entropy, f, true);
    fclose(f);
}

PPO* load_ppo(const char* filename, bool use_cuda) {
    FILE* f = fopen(filename, "rb");
    if (!f) die("load_ppo: cannot open file");
    PPO* ppo = (PPO*)xcalloc(1, sizeof(PPO));
    ppo->use_cuda = use_cuda;
    int S, A, cap;
    if (fread(&ppo->lambda, sizeof(float), 1, f) != 1 || fread(&ppo->epsilon, sizeof(float), 1, f) != 1 ||
        fread(&ppo->ent_coeff, sizeof(float), 1, f) != 1 || fread(&ppo->lr_policy, sizeof(float), 1, f) != 1 ||
        fread(&ppo->lr_V, sizeof(float), 1, f) != 1 || fread(&S, sizeof(int), 1, f) != 1 ||
        fread(&A, sizeof(int), 1, f) != 1 || fread(&cap, sizeof(int), 1, f) != 1)
        die("load_ppo: unexpected end of file");
    if (S <= 0 || A <= 0 || cap < 0) die("load_ppo: bad header");
    ppo->buffer = create_trajectory_buffer(cap, S, A);
    ppo->policy = load_policy(f, S, A);
    ppo->V = load_neural_network(f);
    if (ppo->policy->mu->layers[0].input_size != S || ppo->policy->mu->output_size != A ||
        ppo->V->layers[0].input_size != S || ppo->V->output_size != 1)
        die("load_ppo: network shapes do not match the header");
    /* optimiser state always lives in HBM (use_cuda is kept for the ABI; both values run the HIP
     * path), so the moments are loaded as device Adams whatever use_cuda says */
    ppo->adam_policy = load_adam_from_nn(f, ppo->policy->mu, true);
    ppo->adam_V = load_adam_from_nn(f, ppo->V, true);
    ppo->adam_entropy = load_adam_ex(f, &ppo->policy->d_log_std, &ppo->policy->d_log_std_grad, &A, 1, true);
    fclose(f);
    return ppo;
}

/* ppo_ext.h: compute precision of both networks (bf16 MFMA for config C5) */
int ppo_set_compute_dtype(void* vppo, int dtype) {
    PPO* ppo = (PPO*)vppo;
    if (!ppo) return -1;
    if (nn_set_compute_dtype(ppo->V, dtype) != 0) return -1;
    return nn_set_compute_dtype(ppo->policy->mu, dtype);
}
