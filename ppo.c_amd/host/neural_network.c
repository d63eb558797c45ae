/*
 * neural_network.c — MLP objects over flat HBM parameter/gradient buffers.
 *
 * Reference: /root/reference/src/neural_network.cu.  Construction consumes
 * libc rand() in the reference's order and with its initialisers
 * (neural_network.cu:40-51) so seeded runs start from the same weights; the
 * forward/backward passes run the fused MFMA GEMMs of csrc/gemm.hip:
 *   forward  : y_{i+1} = act_i(y_i·W_iᵀ + b_i)                 (one kernel per layer)
 *   backward : gW_i, gb_i = g_{i+1}ᵀ·y_i, Σ g_{i+1}             (one kernel per layer)
 *              g_i = (g_{i+1}·W_i) ⊙ 1[y_i > 0]                (one kernel per layer, skipped
 *                                                               for layer 0 in the update)
 */
#include "internal.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

int nn_is_relu(const NeuralNetwork* nn, int layer) {
    const ActivationFunction* a = nn->layers[layer].d_activation_function;
    return a && a->activation != NULL;
}

/* ---- host mirror <-> HBM reconciliation ------------------------------------------------------
 * The reference's host-pointer functions compute from the host mirrors (Layer.weights, log_std);
 * libppo computes from HBM.  Every live network is registered so a device Adam step can mark the
 * network whose parameters it moved (dev_version); the host entry points then pull newer HBM
 * parameters into the mirrors, and push only mirror tensors the caller edited since the last sync
 * (compared with the h_sync snapshot) — HBM is never overwritten with stale host values. */
static NeuralNetwork** g_nets = NULL;
static int g_nets_n = 0, g_nets_cap = 0;

static void nn_registry_add(NeuralNetwork* nn) {
    if (g_nets_n == g_nets_cap) {
        g_nets_cap = g_nets_cap ? 2 * g_nets_cap : 16;
        NeuralNetwork** p = (NeuralNetwork**)realloc(g_nets, sizeof(NeuralNetwork*) * (size_t)g_nets_cap);
        if (!p) die("host allocation failed");
        g_nets = p;
    }
    g_nets[g_nets_n++] = nn;
}

static void nn_registry_remove(NeuralNetwork* nn) {
    for (int i = 0; i < g_nets_n; i++)
        if (g_nets[i] == nn) { g_nets[i] = g_nets[--g_nets_n]; return; }
}

void nn_note_device_update(const float* d_ptr) {
    for (int i = 0; i < g_nets_n; i++) {
        NeuralNetwork* nn = g_nets[i];
        if (d_ptr >= nn->d_params && d_ptr < nn->d_params + nn->num_params + nn->extra_floats) nn->dev_version++;
    }
}

/* h_sync offset of layer i's weights in the packed order */
static long packed_offset(const NeuralNetwork* nn, int layer) {
    long off = 0;
    for (int i = 0; i < layer; i++) off += (long)nn->layers[i].input_size * nn->layers[i].output_size + nn->layers[i].output_size;
    return off;
}

/* the caller edited a weight mirror since the last sync (it differs from the h_sync snapshot) */
static int nn_mirrors_edited(const NeuralNetwork* nn) {
    for (int i = 0; i < nn->num_layers - 1; i++) {
        const Layer* ly = &nn->layers[i];
        const size_t nw = (size_t)ly->input_size * ly->output_size, nb = (size_t)ly->output_size;
        const float* sw = nn->h_sync + packed_offset(nn, i);
        if (memcmp(sw, ly->weights, sizeof(float) * nw) || memcmp(sw + nw, ly->biases, sizeof(float) * nb)) return 1;
    }
    return 0;
}

/* Weights and the caller-owned extra floats (policy log σ behind μ) are reconciled separately:
 * host_version_w records the HBM version the weight mirrors were last pulled at, so a weights-only
 * sync (extra == NULL: forward_propagation / save_neural_network on μ itself) pulls once per HBM
 * update and afterwards pushes the caller's mirror edits, instead of pulling again on every call.
 * When HBM moved AND the caller edited a mirror since the last sync, HBM wins (it holds the
 * update's result) and the lost edit is reported on stderr. */
void nn_host_sync(NeuralNetwork* nn, float* extra) {
    const int L = nn->num_layers - 1;
    const long ne = extra ? nn->extra_floats : 0;
    int pushed = 0;
    if (nn->dev_version != nn->host_version_w) {          /* HBM weights are newer: pull */
        if (nn_mirrors_edited(nn))
            fprintf(stderr, "libppo: warning: host weight edits dropped: the device parameters were updated "
                            "since the last sync (ppo_update / Adam)\n");
        nn_write_weights_to_host(nn);
        nn->host_version_w = nn->dev_version;
    } else {                                              /* push the tensors the caller edited */
        for (int i = 0; i < L; i++) {
            Layer* ly = &nn->layers[i];
            const size_t nw = (size_t)ly->input_size * ly->output_size, nb = (size_t)ly->output_size;
            float* sw = nn->h_sync + packed_offset(nn, i);
            if (memcmp(sw, ly->weights, sizeof(float) * nw)) {
                phip_h2d(ly->d_weights, ly->weights, sizeof(float) * nw);
                memcpy(sw, ly->weights, sizeof(float) * nw);
                pushed = 1;
            }
            if (memcmp(sw + nw, ly->biases, sizeof(float) * nb)) {
                phip_h2d(ly->d_biases, ly->biases, sizeof(float) * nb);
                memcpy(sw + nw, ly->biases, sizeof(float) * nb);
                pushed = 1;
            }
        }
    }
    if (ne) {
        float* snap = nn->h_sync + nn->num_params_packed;
        if (nn->dev_version != nn->host_version) {        /* HBM extras newer: pull */
            phip_d2h(extra, nn->d_params + nn->num_params, sizeof(float) * (size_t)ne);
            memcpy(snap, extra, sizeof(float) * (size_t)ne);
        } else if (memcmp(snap, extra, sizeof(float) * (size_t)ne)) {
            phip_h2d(nn->d_params + nn->num_params, extra, sizeof(float) * (size_t)ne);
            memcpy(snap, extra, sizeof(float) * (size_t)ne);
        }
        nn->host_version = nn->dev_version;
    } else if (!nn->extra_floats) {
        nn->host_version = nn->dev_version;
    }
    if (pushed) nn_sync_w16(nn);
}

/* the caller's extra floats were written to HBM and the mirror (policy log_std at creation / load) */
void nn_sync_extra_snapshot(NeuralNetwork* nn, const float* extra) {
    if (nn->extra_floats) memcpy(nn->h_sync + nn->num_params_packed, extra, sizeof(float) * (size_t)nn->extra_floats);
}

/* neural_network.cu:40-51 restated: He-uniform hidden layers, Xavier-uniform output layer. */
static void init_layer_from_rand(Layer* ly, int is_last) {
    const int in = ly->input_size, out = ly->output_size;
    float gain = is_last ? 1 : sqrtf(2.0);
    float std = gain * sqrtf(2.0 / (in + out));
    for (long j = 0; j < (long)in * out; j++) ly->weights[j] = (2 * (float)rand() / RAND_MAX - 1) * sqrtf(3.0) * std;
    for (int j = 0; j < out; j++) ly->biases[j] = (2 * (float)rand() / RAND_MAX - 1) * (1. / sqrtf(in));
}

NeuralNetwork* nn_create_ex(int* layer_sizes, char** activation_functions, int num_layers, long extra_floats,
                            int init_from_rand) {
    if (num_layers < 2) die("create_neural_network: need at least 2 layer sizes");
    phip_init();
    const int L = num_layers - 1;
    NeuralNetwork* nn = (NeuralNetwork*)xcalloc(1, sizeof(NeuralNetwork));
    nn->num_layers = num_layers;
    nn->layers = (Layer*)xcalloc((size_t)num_layers, sizeof(Layer));
    nn->bits_m = -1;
    nn->activation_functions = (char**)xmalloc(sizeof(char*) * (size_t)L);
    nn->param_offset = (long*)xmalloc(sizeof(long) * (size_t)L);
    nn->bias_offset = (long*)xmalloc(sizeof(long) * (size_t)L);

    long off = 0, packed = 0;
    for (int i = 0; i < L; i++) {
        Layer* ly = &nn->layers[i];
        nn->activation_functions[i] = strdup(activation_functions[i]);
        ly->input_size = layer_sizes[i];
        ly->output_size = layer_sizes[i + 1];
        const long nw = (long)ly->input_size * ly->output_size;
        nn->param_offset[i] = off;
        off += align4(nw);
        nn->bias_offset[i] = off;
        off += align4(ly->output_size);
        packed += nw + ly->output_size;
        ly->weights = (float*)xmalloc(sizeof(float) * (size_t)nw);
        ly->biases = (float*)xmalloc(sizeof(float) * (size_t)ly->output_size);
        ly->grad_weights = (float*)xcalloc((size_t)nw, sizeof(float));
        ly->grad_biases = (float*)xcalloc((size_t)ly->output_size, sizeof(float));
        ly->activation_function = build_activation_function(activation_functions[i]);
        ly->d_activation_function = build_activation_function_cuda(activation_functions[i]);
        if (init_from_rand) init_layer_from_rand(ly, i == L - 1);
    }
    nn->layers[L].input_size = layer_sizes[L];
    nn->output_size = layer_sizes[L];
    nn->num_params = off;
    nn->num_params_packed = packed;
    nn->extra_floats = extra_floats;

    const size_t bytes = sizeof(float) * (size_t)(off + align4(extra_floats));
    nn->d_params = (float*)phip_malloc(bytes);
    nn->d_grads = (float*)phip_malloc(bytes);
    for (int i = 0; i < L; i++) {
        Layer* ly = &nn->layers[i];
        ly->d_weights = nn->d_params + nn->param_offset[i];
        ly->d_biases = nn->d_params + nn->bias_offset[i];
        ly->d_grad_weights = nn->d_grads + nn->param_offset[i];
        ly->d_grad_biases = nn->d_grads + nn->bias_offset[i];
    }
    nn->h_sync = (float*)xcalloc((size_t)(packed + extra_floats), sizeof(float));
    nn_registry_add(nn);
    if (init_from_rand) nn_write_weights_to_device(nn);
    nn->cublas_handle = NULL;
    return nn;
}

NeuralNetwork* create_neural_network(int* layer_sizes, char** activation_functions, int num_layers) {
    return nn_create_ex(layer_sizes, activation_functions, num_layers, 0, 1);
}

static long bits_words(const NeuralNetwork* nn, int upto, int m) {   /* words before layer `upto`'s block */
    long w = 0;
    for (int i = 0; i < upto; i++) w += (long)m * ((nn->layers[i].input_size + 31) / 32);
    return w;
}

/* ReLU′ bit mask of layers[i].d_input (written by the forward of layer i−1) */
static unsigned* act_bits(NeuralNetwork* nn, int i) { return nn->d_act_bits + bits_words(nn, i, nn->act_cap_m); }

void nn_ensure_act(NeuralNetwork* nn, int m) {
    if (m <= nn->act_cap_m) return;
    for (int i = 0; i < nn->num_layers; i++) {
        phip_free(nn->layers[i].d_input);
        nn->layers[i].d_input = (float*)phip_malloc(sizeof(float) * (size_t)m * nn->layers[i].input_size);
    }
    phip_free(nn->d_act_bits);
    nn->d_act_bits = (unsigned*)phip_malloc(sizeof(unsigned) * (size_t)bits_words(nn, nn->num_layers, m));
    nn->bits_m = -1;
    nn->act_cap_m = m;
}

void nn_ensure_grad(NeuralNetwork* nn, int m) {
    if (m <= nn->grad_cap_m) return;
    for (int i = 0; i < nn->num_layers; i++) {
        phip_free(nn->layers[i].d_grad_x);
        nn->layers[i].d_grad_x = (float*)phip_malloc(sizeof(float) * (size_t)m * nn->layers[i].input_size);
    }
    nn->grad_cap_m = m;
}

/* Forward over m rows.  With d_rows != NULL, input row r is d_x[d_rows[r]] (the minibatch gather
 * fused into layer 0), and the gathered rows are written to d_xcopy, which backward then uses as
 * layer 0's input. */
static void nn_forward_dev_bf16(NeuralNetwork* nn, const float* d_x, const int* d_rows, float* d_xcopy, int m,
                                int upto) {
    const int L = nn->num_layers - 1;
    nn->d_x0 = d_rows ? d_xcopy : d_x;
    nn->x0_dtype = d_rows ? 1 : 0;                 /* the gathered copy is written as bf16 */
    const void* in = d_x;
    int tin = 0;
    const int S = nn->layers[0].input_size;
    if (d_rows && d_xcopy && S % 4 == 0) {                    /* gather + round once, then a plain bf16 GEMM */
        phip_gather_rows_bf16((unsigned short*)d_xcopy, d_x, d_rows, m, S);
        in = d_xcopy;
        tin = 1;
        d_rows = NULL;
        d_xcopy = NULL;
    }
    for (int i = 0; i < upto; i++) {
        Layer* ly = &nn->layers[i];
        float* out = nn->layers[i + 1].d_input;    /* hidden: bf16 storage; network output: fp32 */
        const int tout = i == L - 1 ? 0 : 1;
        phip_linear16_fwd(out, tout, in, tin, i == 0 ? d_rows : NULL, i == 0 ? (void*)d_xcopy : NULL,
                          nn->d_w16 + nn->param_offset[i], ly->d_biases, m, ly->input_size, ly->output_size,
                          nn_is_relu(nn, i), act_bits(nn, i + 1));
        in = out;
        tin = tout;
    }
}

/* fp32 GEMM engine (ppo_ext.h ppo_gemm_f32_engine): -1 = not yet read from PPO_F32_GEMM */
static int g_f32_engine = -1;

int ppo_gemm_f32_engine(int engine) {
    if (g_f32_engine < 0) {
        const char* e = getenv("PPO_F32_GEMM");
        g_f32_engine = (e && strcmp(e, "exact") == 0) ? 0 : (e && strcmp(e, "x3") == 0) ? 1 : PPO_F32_ENGINE_DEFAULT;
    }
    const int old = g_f32_engine;
    if (engine == 0 || engine == 1) g_f32_engine = engine;
    return old;
}

/* the x3 engine serves the minibatch- and buffer-sized products; small-m forwards (rollout steps
 * over E environments) keep the exact kernel family's small-M path */
static int use_x3(int m) { return m > 1024 && ppo_gemm_f32_engine(-1) == 1; }
/* per layer: the 1- and A-wide output layers are latency-bound skinny products where the exact
 * kernels (and their paired backward launch) measure faster (profiles/r01_x3_sweep.txt) */
static int use_x3_layer(int m, int n, int l) { return use_x3(m) && n > 32 && l > 32; }
/* the reference-API products (mat_mul*_cuda, layers.c) through the same engine choice (fp32 storage).
 * Callers may pass any valid device pointer (a row or element offset into a buffer); the x3 kernels
 * need 16-B aligned operands, so an unaligned operand routes to the exact family, which has a scalar
 * path for it. */
static int al16(const void* p) { return ((uintptr_t)p & 15) == 0; }
void lin_fwd(float* y, const float* x, const float* W, const float* b, int m, int n, int l) {
    if (use_x3(m) && phip_x3_supported(0, m, n, l) && al16(y) && al16(x) && al16(W) && al16(b))
        phip_x3_fwd(y, x, NULL, NULL, W, b, m, n, l, 0, NULL);
    else phip_linear_fwd(y, x, W, b, m, n, l, 0);
}
void lin_bwd_x(float* gx, const float* g, const float* W, int m, int n, int l) {
    if (use_x3(m) && phip_x3_supported(1, m, n, l) && al16(gx) && al16(g) && al16(W))
        phip_x3_bwd_x(gx, g, W, NULL, m, n, l);
    else phip_linear_bwd_x(gx, g, W, NULL, m, n, l);
}
void lin_bwd_w(float* gW, const float* g, const float* x, int m, int n, int l) {
    if (use_x3(m) && phip_x3_supported(2, m, n, l) && al16(gW) && al16(g) && al16(x))
        phip_x3_bwd_w(gW, NULL, g, x, m, n, l, 0);
    else phip_linear_bwd_w(gW, NULL, g, x, m, n, l);
}

int ppo_nn_input_rows(void* vnn, float* out, int m) {
    NeuralNetwork* nn = (NeuralNetwork*)vnn;
    const int S = nn->layers[0].input_size;
    if (!nn->d_x0 || nn->x0_dtype != 0 || m <= 0 || m > nn->cache_m_forward) return -1;
    phip_d2h(out, nn->d_x0, sizeof(float) * (size_t)m * S);
    return 0;
}

/* value-head fold (nn_value_fold_step): the forward's last layer also forms the partial dots of the
 * 1-wide output layer (w) into ypart, and reports their slot count */
typedef struct { const float* w; float* ypart; int slots; } FoldFwd;

/* forward through the first `upto` linear layers (fp32 storage; upto = L: the whole network) */
static void nn_forward_dev_upto(NeuralNetwork* nn, const float* d_x, const int* d_rows, float* d_xcopy, int m,
                                int upto, FoldFwd* fold);

void nn_forward_dev_rows(NeuralNetwork* nn, const float* d_x, const int* d_rows, float* d_xcopy, int m) {
    nn_forward_dev_upto(nn, d_x, d_rows, d_xcopy, m, nn->num_layers - 1, NULL);
}

static void nn_forward_dev_upto(NeuralNetwork* nn, const float* d_x, const int* d_rows, float* d_xcopy, int m,
                                int upto, FoldFwd* fold) {
    nn_ensure_act(nn, m);
    const int L = nn->num_layers - 1;
    if (nn->dtype == 1) {
        nn_forward_dev_bf16(nn, d_x, d_rows, d_xcopy, m, upto);
        nn->bits_m = m;
        nn->cache_m_forward = m;
        nn->d_output = nn->layers[L].d_input;
        return;
    }
    /* (round 6: the gathered copy dropped, layer 0's grad_W reading the buffer rows through the indices —
     * the forward 6 µs faster, the grad_W 9 µs slower on random 1.5 KB rows: profiles/r06_x0_gather_rejected.txt) */
    nn->d_x0 = d_rows ? d_xcopy : d_x;
    nn->x0_dtype = 0;
    const float* in = d_x;
    for (int i = 0; i < upto; i++) {
        Layer* ly = &nn->layers[i];
        float* out = nn->layers[i + 1].d_input;
        const int n = ly->input_size, l = ly->output_size;
        if (fold && i == upto - 1) {            /* nn_value_fold_ok: the x3 engine takes this layer */
            fold->slots = phip_x3_fwd_vhead(out, in, i == 0 ? d_rows : NULL, i == 0 ? d_xcopy : NULL, ly->d_weights,
                                            ly->d_biases, m, n, l, nn_is_relu(nn, i), act_bits(nn, i + 1), fold->w,
                                            fold->ypart);
        } else if (use_x3_layer(m, n, l) && phip_x3_supported(0, m, n, l)) {
            phip_x3_fwd(out, in, i == 0 ? d_rows : NULL, i == 0 ? d_xcopy : NULL, ly->d_weights, ly->d_biases, m, n,
                        l, nn_is_relu(nn, i), act_bits(nn, i + 1));
        } else if (i == 0 && d_rows) {
            phip_linear_fwd_gather(out, in, d_rows, d_xcopy, ly->d_weights, ly->d_biases, m, n, l, nn_is_relu(nn, i),
                                   act_bits(nn, i + 1));
        } else {
            phip_linear_fwd_bits(out, in, ly->d_weights, ly->d_biases, m, n, l, nn_is_relu(nn, i), act_bits(nn, i + 1));
        }
        in = out;
    }
    nn->bits_m = m;
    nn->cache_m_forward = m;
    nn->d_output = nn->layers[L].d_input;
}

void nn_forward_dev(NeuralNetwork* nn, const float* d_x, int m) { nn_forward_dev_rows(nn, d_x, NULL, NULL, m); }

/* gradient buckets (nn_backward_dev_z): ≥ 1 MiB of consecutive layers per all-reduce */
#define GRAD_BUCKET_FLOATS (256L * 1024)

/* layer i's gradients are queued: all-reduce [param_offset[i], *hi) once it holds a bucket's worth,
 * or at the bottom layer (the flat layout [W0, b0, W1, b1, …] makes every bucket one span); with the
 * all-reduces in stream order (comm.hip, the default) only at the bottom: one collective per step */
static void bucket_flush(NeuralNetwork* nn, int i, long* hi) {
    const long lo = nn->param_offset[i];
    if (i > 0 && (*hi - lo < GRAD_BUCKET_FLOATS || phip_comm_inline())) return;
    phip_allreduce_sum_f32_async(nn->d_grads + lo, *hi - lo);
    *hi = lo;
}

void nn_backward_dev(NeuralNetwork* nn, const float* d_grad_out, int m, int want_grad_x0) {
    nn_backward_dev_z(nn, d_grad_out, m, want_grad_x0, 0, -1);
}

/* value-head fold: the backward's top layer (top - 1) takes its upper gradient g·w·1[h > 0] from g,
 * w and h's mask (nn_value_fold_step) */
typedef struct {
    float* g; const float* w; float* gw_out;
    /* the value head carried by the hidden layer's grad_W launch (phip_x3_bwd_w_vhead) */
    const float* ypart; int slots; const float* b; const float* tgt; float* y; float* gb; float* loss;
} FoldBwd;

static void nn_backward_dev_top(NeuralNetwork* nn, const float* d_grad_out, int m, int want_grad_x0,
                                int grads_zero, long reduce_extra, int top, const FoldBwd* fold);

void nn_backward_dev_z(NeuralNetwork* nn, const float* d_grad_out, int m, int want_grad_x0, int grads_zero,
                       long reduce_extra) {
    nn_backward_dev_top(nn, d_grad_out, m, want_grad_x0, grads_zero, reduce_extra, nn->num_layers - 1, NULL);
}

/* backward through layers top-1 … 0, starting from the gradient at layer top's input (top = L: the
 * whole network, from the output gradient; top = L-1: the output layer's backward already ran) */
static void nn_backward_dev_top(NeuralNetwork* nn, const float* d_grad_out, int m, int want_grad_x0,
                                int grads_zero, long reduce_extra, int top, const FoldBwd* fold) {
    nn_ensure_grad(nn, m);
    const int L = nn->num_layers - 1;
    const float* g = d_grad_out;
    if (top == L && nn_is_relu(nn, L - 1)) {      /* output activation: mask a copy (rare; the reference uses "none") */
        float* top = nn->layers[L].d_grad_x;
        if (top != d_grad_out) phip_d2d(top, d_grad_out, sizeof(float) * (size_t)m * nn->output_size);
        phip_relu_bwd(nn->layers[L].d_input, top, (long)m * nn->output_size);
        g = top;
    }
    /* one memset for every layer's gradient (split-K grad_W accumulates atomically);
     * the trailing extra_floats (policy log_std grad) are owned by the caller and left alone */
    if (!grads_zero) phip_memset(nn->d_grads, 0, sizeof(float) * (size_t)nn->num_params);
    if (nn->dtype == 1) {      /* bf16 mode: hidden gradients stored bf16, the top one (heads) fp32 */
        if (nn->bits_m != m) die("nn_backward_dev (bf16): backward must follow a forward over the same rows");
        int tg = top == L ? 0 : 1;             /* below a fused output layer: its bf16 grad_x */
        long hi = nn->num_params + (reduce_extra > 0 ? reduce_extra : 0);
        for (int i = top - 1; i >= 0; i--) {
            Layer* ly = &nn->layers[i];
            const void* x = i == 0 ? (const void*)nn->d_x0 : (const void*)ly->d_input;
            phip_linear16_bwd_w(ly->d_grad_weights, ly->d_grad_biases, g, tg, x, i == 0 ? nn->x0_dtype : 1, m,
                                ly->input_size, ly->output_size, 1);
            int tgx = tg;
            if (i > 0 || want_grad_x0) {
                const int relu_in = i > 0 && nn_is_relu(nn, i - 1);
                tgx = i > 0 ? 1 : 0;
                phip_linear16_bwd_x(ly->d_grad_x, tgx, g, tg, nn->d_w16 + nn->param_offset[i],
                                    relu_in ? act_bits(nn, i) : NULL, m, ly->input_size, ly->output_size);
            }
            g = ly->d_grad_x;
            tg = tgx;
            if (reduce_extra >= 0) bucket_flush(nn, i, &hi);
        }
        nn->cache_m_backward = m;
        return;
    }
    /* grad_W and grad_x of a layer are independent: with the ReLU′ bits of this forward they go
     * out as one launch (phip_linear_bwd_pair: grad_x tiles fill the CUs grad_W tiles leave).
     * (measured: grad_W on a second queue beside grad_x was slower than back to back) */
    long hi = nn->num_params + (reduce_extra > 0 ? reduce_extra : 0);
    for (int i = top - 1; i >= 0; i--) {
        Layer* ly = &nn->layers[i];
        const float* x = i == 0 ? nn->d_x0 : ly->d_input;
        const int n = ly->input_size, l = ly->output_size;
        const int want_gx = i > 0 || want_grad_x0;
        const int relu_in = i > 0 && nn_is_relu(nn, i - 1);
        const unsigned* bits = relu_in && nn->bits_m == m ? act_bits(nn, i) : NULL;   /* this forward's bits */
        if (fold && i == top - 1) {
            /* grad_W = diag(w)·(maskᵀ·diag(g)·x), grad_b = diag(w)·maskᵀ·g, the output layer's gW = Σ g·h;
             * grad_x = diag(g)·(mask·diag(w)·W) ⊙ the input mask (gemm_x3.hip) */
            const float* h = nn->layers[i + 1].d_input;
            phip_x3_defer_reduce(want_gx);                    /* its slab reduce rides on grad_x */
            phip_x3_bwd_w_vhead(ly->d_grad_weights, ly->d_grad_biases, h, fold->g, fold->w, fold->gw_out, x, m, n, l, 1,
                                fold->ypart, fold->slots, fold->b, fold->tgt, fold->y, fold->gb, fold->loss);
            if (want_gx) {
                if (relu_in && !bits) die("nn_value_fold_step: the forward's ReLU′ bits are missing");
                phip_x3_bwd_x_fold(ly->d_grad_x, NULL, act_bits(nn, i + 1), fold->g, fold->w, ly->d_weights, bits, m, n,
                                   l);
            }
        } else if (i == L - 1 && want_gx && (!relu_in || bits) &&
            phip_out_bwd_wide(ly->d_grad_weights, ly->d_grad_biases, ly->d_grad_x, g, x, ly->d_weights, relu_in, m, n,
                              l)) {
            /* wide output layer (A = 17): grad_x and grad_W in one pass over the rows (out_head.hip) */
        } else if (use_x3_layer(m, n, l) && phip_x3_supported(2, m, n, l)) {
            const int pair = want_gx && (!relu_in || bits);
            phip_x3_defer_reduce(pair);                       /* its slab reduce rides on grad_x */
            phip_x3_bwd_w(ly->d_grad_weights, ly->d_grad_biases, g, x, m, n, l, 1);
            if (pair) phip_x3_bwd_x(ly->d_grad_x, g, ly->d_weights, bits, m, n, l);
            else if (want_gx) phip_linear_bwd_x_bits(ly->d_grad_x, g, ly->d_weights, ly->d_input, NULL, m, n, l);
        } else if (want_gx && (!relu_in || bits)) {
            phip_linear_bwd_pair(ly->d_grad_weights, ly->d_grad_biases, ly->d_grad_x, g, x, ly->d_weights, bits, m, n,
                                 l, 1);
        } else {
            phip_linear_bwd_w_ex(ly->d_grad_weights, ly->d_grad_biases, g, x, m, n, l, 1);
            if (want_gx)
                phip_linear_bwd_x_bits(ly->d_grad_x, g, ly->d_weights, relu_in ? ly->d_input : NULL, NULL, m, n, l);
        }
        g = ly->d_grad_x;
        if (reduce_extra >= 0) bucket_flush(nn, i, &hi);
    }
    nn->cache_m_backward = m;
}

/* The output layer fused with the loss head (out_head.hip) for one minibatch step: at least one
 * hidden layer, identity output, a supported (width, A) — fp32 storage, or bf16 storage for the value
 * head — and no deterministic-GEMM request (ppo_gemm_tune(·, 1)); PPO_OUT_HEAD=0 disables it (read
 * per call). */
int nn_out_head_ok(const NeuralNetwork* nn, int head) {
    const char* e = getenv("PPO_OUT_HEAD");
    if ((e && e[0] == '0') || phip_gemm_deterministic()) return 0;     /* its gW sums use f32 atomics */
    const int L = nn->num_layers - 1;
    if (L < 2 || nn_is_relu(nn, L - 1)) return 0;
    if (nn->dtype == 1 && (head != 0 || nn->param_offset[L - 1] % 8 != 0)) return 0;   /* W shadow: 16-B rows */
    return phip_out_head_supported(head, nn->layers[L - 1].input_size, nn->layers[L - 1].output_size);
}

/* forward (all but the output layer), then the fused output layer + head + output-layer backward,
 * then the hidden layers' backward — the same results as nn_forward_dev_rows → head kernel →
 * nn_backward_dev_z up to fp32 re-association of the output layer's sums */
void nn_out_head_step(NeuralNetwork* nn, int head, const float* d_x, const int* d_rows, float* d_xcopy, int m,
                      int grads_zero, long reduce_extra, const float* tgt, const float* log_std, const float* action,
                      const float* adv, const float* old_lp, float eps, float ent_coeff, float* grad_log_std,
                      float* loss_accum) {
    const int L = nn->num_layers - 1;
    nn_forward_dev_upto(nn, d_x, d_rows, d_xcopy, m, L - 1, NULL);
    nn_ensure_grad(nn, m);
    if (!grads_zero) phip_memset(nn->d_grads, 0, sizeof(float) * (size_t)nn->num_params);
    Layer* ly = &nn->layers[L - 1];
    const int b16 = nn->dtype == 1;            /* bf16 mode: bf16 activation / gradient, the W shadow */

    phip_out_head(head, b16, ly->d_input, nn_is_relu(nn, L - 2), b16 ? (const void*)(nn->d_w16 + nn->param_offset[L - 1])
                                                                     : (const void*)ly->d_weights,
                  ly->d_biases, m, ly->input_size, ly->output_size, tgt, log_std, action, adv, old_lp, eps, ent_coeff,
                  nn->layers[L].d_input, ly->d_grad_x, ly->d_grad_weights, ly->d_grad_biases, grad_log_std,
                  loss_accum);
    nn->d_output = nn->layers[L].d_input;
    nn_backward_dev_top(nn, ly->d_grad_x, m, 0, 1, reduce_extra, L - 1, NULL);
}

/* The value network's 1-wide output layer and MSE head folded into its last hidden layer's x3
 * kernels (fp32, identity output after a ReLU hidden layer, the x3 engine at this m, no
 * deterministic-GEMM request; PPO_VALUE_FOLD=0 disables it, read per call).  With h = relu(z) the
 * last hidden activation, y = h·w + b and g = ∂L/∂y, the head's upper gradient is G = g·w·1[h > 0] —
 * rank one — so it is never formed: the forward's epilogue leaves partial dots of h·w, the hidden layer's
 * grad_W launch forms y, the loss, g and the output bias gradient from them before its mainloop (the head
 * carried: no launch of its own), and the hidden layer's backward GEMMs take the 0/1 mask of h as their
 * operand (one bf16 plane: three MFMA plane products instead of six) with g and w as row / column scales
 * (gemm_x3.hip FOLD; grad_x stages W scaled by w per k-row). */
int nn_value_fold_ok(const NeuralNetwork* nn, int m) {
    const char* e = getenv("PPO_VALUE_FOLD");
    if ((e && e[0] == '0') || phip_gemm_deterministic()) return 0;     /* atomics in the gradient sums */
    const int L = nn->num_layers - 1;
    if (nn->dtype != 0 || L < 2 || nn->output_size != 1 || nn_is_relu(nn, L - 1) || !nn_is_relu(nn, L - 2)) return 0;
    const Layer* hid = &nn->layers[L - 2];
    const int n = hid->input_size, l = hid->output_size;
    return use_x3_layer(m, n, l) && phip_x3_supported(0, m, n, l) && phip_x3_supported(1, m, n, l) &&
           phip_x3_supported(2, m, n, l);
}

void nn_value_fold_step(NeuralNetwork* nn, const float* d_x, const int* d_rows, float* d_xcopy, int m, int grads_zero,
                        long reduce_extra, const float* tgt, float* loss_accum) {
    const int L = nn->num_layers - 1;
    Layer* hid = &nn->layers[L - 2];
    Layer* out = &nn->layers[L - 1];
    const int l = hid->output_size;
    const size_t mp = ((size_t)m + 3) & ~(size_t)3;
    const size_t slots_max = 2 * (size_t)((l + 63) / 64);     /* column tiles (≥ 64 wide) × 2 waves along N */
    const size_t need = slots_max * mp + mp;
    if ((long)need > nn->fold_ws_cap) {        /* the network's own scratch, freed with it */
        phip_free(nn->d_fold_ws);
        nn->d_fold_ws = (float*)phip_malloc(sizeof(float) * need);
        nn->fold_ws_cap = (long)need;
    }
    float* ypart = nn->d_fold_ws;
    float* g = ypart + slots_max * mp;
    FoldFwd ff = {out->d_weights, ypart, 0};
    nn_forward_dev_upto(nn, d_x, d_rows, d_xcopy, m, L - 1, &ff);
    if (ff.slots <= 0 || (size_t)ff.slots > slots_max) die("nn_value_fold_step: unexpected partial-dot slots");
    nn_ensure_grad(nn, m);
    if (!grads_zero) phip_memset(nn->d_grads, 0, sizeof(float) * (size_t)nn->num_params);
    /* ypart rows are at stride m (phip_x3_fwd_vhead); the head itself runs inside the hidden layer's
     * grad_W launch (y, g, the output bias gradient, the loss) */
    nn->d_output = nn->layers[L].d_input;
    const FoldBwd fb = {g, out->d_weights, out->d_grad_weights, ypart, ff.slots, out->d_biases, tgt,
                        nn->layers[L].d_input, out->d_grad_biases, loss_accum};
    nn_backward_dev_top(nn, NULL, m, 0, 1, reduce_extra, L - 1, &fb);
}

/* The A = 17 policy network (C4): its output layer's backward fused with the policy head
 * (out_head.hip, phip_policy_head_bwd_wide) — fp32, identity output, at least one hidden layer, the
 * flat gradient layout (gb after gW), no deterministic-GEMM request (the head's f32 atomics) */
int nn_policy_wide_ok(const NeuralNetwork* nn, int m) {
    const int L = nn->num_layers - 1;
    if (nn->dtype != 0 || L < 2 || nn_is_relu(nn, L - 1) || phip_gemm_deterministic()) return 0;
    const Layer* ly = &nn->layers[L - 1];
    if (nn->param_offset[L - 1] % 4 != 0) return 0;                     /* 16-B aligned W / gW */
    return phip_out_bwd_wide_ok(m, ly->input_size, ly->output_size, 1);
}

/* forward through every layer, then the policy head + output-layer backward in one pass, then the
 * hidden layers' backward — the separate path's results (nn_forward_dev_rows → phip_policy_head →
 * nn_backward_dev_z) up to the order of the output layer's gradient sums */
void nn_policy_wide_step(NeuralNetwork* nn, const float* d_x, const int* d_rows, float* d_xcopy, int m,
                         int grads_zero, long reduce_extra, const float* log_std, const float* action,
                         const float* adv, const float* old_lp, float eps, float ent_coeff, float* grad_log_std,
                         float* loss_accum) {
    const int L = nn->num_layers - 1;
    Layer* ly = &nn->layers[L - 1];
    /* PPO_POLICY_FUSED (read per call): 1 the one-launch output layer, 0 the two launches, unset: one launch
     * up to 8192 rows (the G = 8 shard's policy step: 27.1 vs 19.4 + 17.2 µs) and two above (C4's 32768 rows:
     * 75 vs 42.6 + 19.1 µs — eight 16-row blocks per CU, each a chain of seven barrier-separated phases;
     * profiles/r06_policy_out_fused_ab.txt) */
    const char* pf = getenv("PPO_POLICY_FUSED");
    const int fused = pf && pf[0] ? pf[0] != '0' : m <= 8192;
    if (fused) {
        /* the output layer's forward, the head and its backward in one pass over h (out_head.hip
         * policy_out_fused_kernel): the hidden layers' forward only */
        nn_forward_dev_upto(nn, d_x, d_rows, d_xcopy, m, L - 1, NULL);
        nn_ensure_grad(nn, m);
        if (!grads_zero) phip_memset(nn->d_grads, 0, sizeof(float) * (size_t)nn->num_params);
        float* mu = nn->layers[L].d_input;
        if (!phip_policy_out_fused(ly->d_input, ly->d_weights, ly->d_biases, mu, log_std, action, adv, old_lp, eps,
                                   ent_coeff, grad_log_std, loss_accum, nn_is_relu(nn, L - 2), ly->d_grad_weights,
                                   ly->d_grad_biases, ly->d_grad_x, m, ly->input_size, ly->output_size))
            die("nn_policy_wide_step: the fused output layer declined a shape nn_policy_wide_ok accepted");
        nn->d_output = mu;
        nn_backward_dev_top(nn, ly->d_grad_x, m, 0, 1, reduce_extra, L - 1, NULL);
        return;
    }
    nn_forward_dev_rows(nn, d_x, d_rows, d_xcopy, m);
    nn_ensure_grad(nn, m);
    if (!grads_zero) phip_memset(nn->d_grads, 0, sizeof(float) * (size_t)nn->num_params);
    if (!phip_policy_head_bwd_wide(nn->d_output, log_std, action, adv, old_lp, eps, ent_coeff, grad_log_std,
                                   loss_accum, ly->d_input, ly->d_weights, nn_is_relu(nn, L - 2), ly->d_grad_weights,
                                   ly->d_grad_biases, ly->d_grad_x, m, ly->input_size, ly->output_size))
        die("nn_policy_wide_step: the wide head declined a shape nn_policy_wide_ok accepted");
    nn_backward_dev_top(nn, ly->d_grad_x, m, 0, 1, reduce_extra, L - 1, NULL);
}

/* neural_network.cu:74-105: copies the input into layers[0].d_input first. */
void forward_propagation_cuda(NeuralNetwork* nn, float* input, int m) {
    nn_ensure_act(nn, m);
    phip_d2d(nn->layers[0].d_input, input, sizeof(float) * (size_t)m * nn->layers[0].input_size);
    nn_forward_dev(nn, nn->layers[0].d_input, m);
}

/* neural_network.cu:121-161: grad_in is copied into the last layer's d_grad_x;
 * every layer's d_grad_x (including layer 0) is produced. */
void backward_propagation_cuda(NeuralNetwork* nn, float* grad_in, int m) {
    nn_ensure_grad(nn, m);
    const int L = nn->num_layers - 1;
    phip_d2d(nn->layers[L].d_grad_x, grad_in, sizeof(float) * (size_t)m * nn->output_size);
    nn_backward_dev(nn, nn->layers[L].d_grad_x, m, 1);
}

/* Host-pointer entry points (reference CPU path, neural_network.cu:163-231): host mirrors and HBM
 * are reconciled first (nn_host_sync: newer HBM parameters pulled, caller-edited mirror tensors
 * pushed); the output and gradients come back into the host mirrors. */
void forward_propagation(NeuralNetwork* nn, float* input, int m) {
    nn_host_sync(nn, NULL);
    nn_ensure_act(nn, m);
    phip_h2d(nn->layers[0].d_input, input, sizeof(float) * (size_t)m * nn->layers[0].input_size);
    nn_forward_dev(nn, nn->layers[0].d_input, m);
    free(nn->output);
    nn->output = (float*)xmalloc(sizeof(float) * (size_t)m * nn->output_size);
    phip_d2h(nn->output, nn->d_output, sizeof(float) * (size_t)m * nn->output_size);
}

void backward_propagation(NeuralNetwork* nn, float* grad_in, int m) {
    nn_host_sync(nn, NULL);
    nn_ensure_grad(nn, m);
    const int L = nn->num_layers - 1;
    phip_h2d(nn->layers[L].d_grad_x, grad_in, sizeof(float) * (size_t)m * nn->output_size);
    nn_backward_dev(nn, nn->layers[L].d_grad_x, m, 0);
    for (int i = 0; i < L; i++) {
        Layer* ly = &nn->layers[i];
        phip_d2h(ly->grad_weights, ly->d_grad_weights, sizeof(float) * (size_t)ly->input_size * ly->output_size);
        phip_d2h(ly->grad_biases, ly->d_grad_biases, sizeof(float) * (size_t)ly->output_size);
    }
}

void nn_sync_w16(NeuralNetwork* nn);

void nn_write_weights_to_device(NeuralNetwork* nn) {
    long off = 0;
    for (int i = 0; i < nn->num_layers - 1; i++) {
        Layer* ly = &nn->layers[i];
        const size_t nw = (size_t)ly->input_size * ly->output_size, nb = (size_t)ly->output_size;
        phip_h2d(ly->d_weights, ly->weights, sizeof(float) * nw);
        phip_h2d(ly->d_biases, ly->biases, sizeof(float) * nb);
        memcpy(nn->h_sync + off, ly->weights, sizeof(float) * nw);
        memcpy(nn->h_sync + off + nw, ly->biases, sizeof(float) * nb);
        off += (long)(nw + nb);
    }
    nn_sync_w16(nn);
}

/* bf16 mode: refresh the bf16 shadow of the parameters (after every parameter update) */
void nn_sync_w16(NeuralNetwork* nn) {
    if (nn && nn->dtype == 1) phip_f32_to_bf16(nn->d_w16, nn->d_params, nn->num_params);
}

int nn_set_compute_dtype(void* vnn, int dtype) {
    NeuralNetwork* nn = (NeuralNetwork*)vnn;
    if (!nn || (dtype != 0 && dtype != 1)) return -1;
    if (dtype == 1 && !nn->d_w16) nn->d_w16 = (unsigned short*)phip_malloc(sizeof(unsigned short) * (size_t)nn->num_params);
    nn->dtype = dtype;
    nn->bits_m = -1;
    nn_sync_w16(nn);
    return 0;
}

void nn_write_weights_to_host(NeuralNetwork* nn) {
    long off = 0;
    for (int i = 0; i < nn->num_layers - 1; i++) {
        Layer* ly = &nn->layers[i];
        const size_t nw = (size_t)ly->input_size * ly->output_size, nb = (size_t)ly->output_size;
        phip_d2h(ly->weights, ly->d_weights, sizeof(float) * nw);
        phip_d2h(ly->biases, ly->d_biases, sizeof(float) * nb);
        memcpy(nn->h_sync + off, ly->weights, sizeof(float) * nw);
        memcpy(nn->h_sync + off + nw, ly->biases, sizeof(float) * nb);
        off += (long)(nw + nb);
    }
    nn->host_version_w = nn->dev_version;
    if (!nn->extra_floats) nn->host_version = nn->dev_version;   /* with extras: the owner syncs them too */
}

void free_neural_network(NeuralNetwork* nn) {
    if (!nn) return;
    const int L = nn->num_layers - 1;
    for (int i = 0; i < L; i++) {
        Layer* ly = &nn->layers[i];
        free(ly->weights);
        free(ly->biases);
        free(ly->grad_weights);
        free(ly->grad_biases);
        free(ly->input);
        free(ly->activation_function);
        free(ly->d_activation_function);
        free(nn->activation_functions[i]);
    }
    for (int i = 0; i < nn->num_layers; i++) {
        phip_free(nn->layers[i].d_input);
        phip_free(nn->layers[i].d_grad_x);
    }
    phip_free(nn->d_act_bits);
    phip_free(nn->d_w16);
    phip_free(nn->d_tiny_wt);
    phip_free(nn->d_fold_ws);
    phip_free(nn->d_params);
    phip_free(nn->d_grads);
    nn_registry_remove(nn);
    free(nn->h_sync);
    free(nn->activation_functions);
    free(nn->param_offset);
    free(nn->bias_offset);
    free(nn->layers);
    free(nn->output);
    free(nn);
}

/* neural_network.cu:284-300 byte layout: num_layers, output_size, per activation
 * (len incl. NUL, chars), per layer (in, out, W[out·in], b[out]). */
void save_neural_network(NeuralNetwork* nn, FILE* file) {
    nn_host_sync(nn, NULL);
    fwrite(&nn->num_layers, sizeof(int), 1, file);
    fwrite(&nn->output_size, sizeof(int), 1, file);
    for (int i = 0; i < nn->num_layers - 1; i++) {
        int len = (int)strlen(nn->activation_functions[i]) + 1;
        fwrite(&len, sizeof(int), 1, file);
        fwrite(nn->activation_functions[i], 1, (size_t)len, file);
    }
    for (int i = 0; i < nn->num_layers - 1; i++) {
        Layer* ly = &nn->layers[i];
        fwrite(&ly->input_size, sizeof(int), 1, file);
        fwrite(&ly->output_size, sizeof(int), 1, file);
        fwrite(ly->weights, sizeof(float), (size_t)ly->input_size * ly->output_size, file);
        fwrite(ly->biases, sizeof(float), (size_t)ly->output_size, file);
    }
}

static void read_exact(void* dst, size_t sz, size_t n, FILE* f) {
    if (fread(dst, sz, n, f) != n) die("checkpoint: unexpected end of file");
}

/* neural_network.cu:303-358; extra_floats lets load_policy keep log_std beside μ's parameters */
NeuralNetwork* nn_load_ex(FILE* file, long extra_floats) {
    int num_layers, output_size;
    read_exact(&num_layers, sizeof(int), 1, file);
    read_exact(&output_size, sizeof(int), 1, file);
    if (num_layers < 2 || num_layers > 64) die("checkpoint: bad layer count");
    const int L = num_layers - 1;
    char** acts = (char**)xmalloc(sizeof(char*) * (size_t)L);
    for (int i = 0; i < L; i++) {
        int len;
        read_exact(&len, sizeof(int), 1, file);
        if (len <= 0 || len > 4096) die("checkpoint: bad activation name");
        acts[i] = (char*)xmalloc((size_t)len);
        read_exact(acts[i], 1, (size_t)len, file);
        acts[i][len - 1] = 0;
    }
    long pos = ftell(file);
    int* sizes = (int*)xmalloc(sizeof(int) * (size_t)num_layers);
    /* first pass: sizes */
    for (int i = 0; i < L; i++) {
        int in, out;
        read_exact(&in, sizeof(int), 1, file);
        read_exact(&out, sizeof(int), 1, file);
        sizes[i] = in;
        sizes[i + 1] = out;
        fseek(file, (long)sizeof(float) * ((long)in * out + out), SEEK_CUR);
    }
    fseek(file, pos, SEEK_SET);
    NeuralNetwork* nn = nn_create_ex(sizes, acts, num_layers, extra_floats, 0);
    for (int i = 0; i < L; i++) {
        Layer* ly = &nn->layers[i];
        int in, out;
        read_exact(&in, sizeof(int), 1, file);
        read_exact(&out, sizeof(int), 1, file);
        read_exact(ly->weights, sizeof(float), (size_t)in * out, file);
        read_exact(ly->biases, sizeof(float), (size_t)out, file);
    }
    nn_write_weights_to_device(nn);
    for (int i = 0; i < L; i++) free(acts[i]);
    free(acts);
    free(sizes);
    return nn;
}

NeuralNetwork* load_neural_network(FILE* file) { return nn_load_ex(file, 0); }
