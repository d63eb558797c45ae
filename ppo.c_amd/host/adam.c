/*
 * adam.c — Adam objects (reference /root/reference/src/adam.cu).
 *
 * Device Adams detect when their tensors form one contiguous span (the flat
 * per-network buffers, with ≤3 floats of zero-gradient alignment padding
 * between tensors) and then update the whole span with a single vectorised
 * kernel; m and v are flat HBM buffers covering that span.
 */
#include "internal.h"

#include <math.h>

static Adam* adam_alloc(float** weights, float** grads, int* length, int num_layers, int size, float beta1,
                        float beta2) {
    Adam* a = (Adam*)xcalloc(1, sizeof(Adam));
    a->weights = (float**)xmalloc(sizeof(float*) * (size_t)num_layers);
    a->grad_weights = (float**)xmalloc(sizeof(float*) * (size_t)num_layers);
    a->lengths = (int*)xmalloc(sizeof(int) * (size_t)num_layers);
    memcpy(a->weights, weights, sizeof(float*) * (size_t)num_layers);
    memcpy(a->grad_weights, grads, sizeof(float*) * (size_t)num_layers);
    memcpy(a->lengths, length, sizeof(int) * (size_t)num_layers);
    a->size = size;
    a->beta1 = beta1;
    a->beta2 = beta2;
    a->time_step = 0;
    a->num_layers = num_layers;
    a->grad_scale = 1.0f;
    return a;
}

/* contiguous with small (<4 float) padding gaps, identical param→grad offset for every tensor */
static long flat_span(float** w, float** g, const int* len, int n) {
    if (n <= 0) return -1;
    const ptrdiff_t dg = g[0] - w[0];
    for (int i = 0; i < n; i++) {
        if (g[i] - w[i] != dg) return -1;
        if (i + 1 < n) {
            const ptrdiff_t gap = w[i + 1] - (w[i] + len[i]);
            if (gap < 0 || gap > 3) return -1;
        }
    }
    return (long)((w[n - 1] + len[n - 1]) - w[0]);
}

/* ---------------- host-pointer Adam (adam.cu:6-74) ---------------- */
Adam* create_adam(float** weights, float** grad_weights, int* length, int num_layers, int size, float beta1,
                  float beta2) {
    Adam* a = adam_alloc(weights, grad_weights, length, num_layers, size, beta1, beta2);
    a->m = (float*)xcalloc((size_t)size, sizeof(float));
    a->v = (float*)xcalloc((size_t)size, sizeof(float));
    a->on_device = 0;
    a->span = size;
    return a;
}

Adam* create_adam_from_nn(NeuralNetwork* nn, float beta1, float beta2) {
    const int L = nn->num_layers - 1;
    float** w = (float**)xmalloc(sizeof(float*) * (size_t)(2 * L));
    float** g = (float**)xmalloc(sizeof(float*) * (size_t)(2 * L));
    int* len = (int*)xmalloc(sizeof(int) * (size_t)(2 * L));
    int size = 0;
    for (int i = 0; i < L; i++) {
        Layer* ly = &nn->layers[i];
        w[2 * i] = ly->weights;      g[2 * i] = ly->grad_weights;      len[2 * i] = ly->input_size * ly->output_size;
        w[2 * i + 1] = ly->biases;   g[2 * i + 1] = ly->grad_biases;   len[2 * i + 1] = ly->output_size;
        size += len[2 * i] + len[2 * i + 1];
    }
    Adam* a = create_adam(w, g, len, 2 * L, size, beta1, beta2);
    free(w); free(g); free(len);
    return a;
}

void free_adam(Adam* adam) {
    if (!adam) return;
    if (adam->on_device) { free_adam_cuda(adam); return; }
    free(adam->weights);
    free(adam->grad_weights);
    free(adam->lengths);
    free(adam->m);
    free(adam->v);
    free(adam);
}

static void bias_corrections(Adam* a, float* bc1, float* bc2) {
    a->time_step += 1;
    *bc1 = 1 - powf(a->beta1, a->time_step);     /* adam.cu:56-57 */
    *bc2 = 1 - powf(a->beta2, a->time_step);
}

/* the next step's bias-corrected step size and second-moment correction, as adam_update_cuda
 * computes them (advances time_step) — for kernels that run many Adam steps in one launch */
void adam_next_step(Adam* a, float lr, float* step, float* bc2) {
    float bc1;
    bias_corrections(a, &bc1, bc2);
    *step = lr / bc1;
}

/* host tensors: staged into HBM, updated by the multi-tensor kernel, copied back */
void adam_update(Adam* adam, float lr) {
    if (adam->on_device) { adam_update_cuda(adam, lr); return; }
    float bc1, bc2;
    bias_corrections(adam, &bc1, &bc2);
    const int n = adam->num_layers;
    long total = 0;
    for (int i = 0; i < n; i++) total += adam->lengths[i];
    float* dp = (float*)stage(ST_A, sizeof(float) * (size_t)total);
    float* dg = (float*)stage(ST_B, sizeof(float) * (size_t)total);
    float* dm = stage_up(ST_C, adam->m, (size_t)total);
    float* dv = stage_up(ST_D, adam->v, (size_t)total);
    long off = 0;
    for (int i = 0; i < n; i++) {
        phip_h2d(dp + off, adam->weights[i], sizeof(float) * (size_t)adam->lengths[i]);
        phip_h2d(dg + off, adam->grad_weights[i], sizeof(float) * (size_t)adam->lengths[i]);
        off += adam->lengths[i];
    }
    phip_adam_flat(dp, dg, dm, dv, total, lr, adam->beta1, adam->beta2, bc1, bc2, adam->grad_scale);
    off = 0;
    for (int i = 0; i < n; i++) {
        phip_d2h(adam->weights[i], dp + off, sizeof(float) * (size_t)adam->lengths[i]);
        off += adam->lengths[i];
    }
    phip_d2h(adam->m, dm, sizeof(float) * (size_t)total);
    phip_d2h(adam->v, dv, sizeof(float) * (size_t)total);
}

/* ---------------- device Adam (adam.cu:76-169) ---------------- */
Adam* create_adam_cuda(float** weights, float** grad_weights, int* length, int num_layers, int size, float beta1,
                       float beta2) {
    Adam* a = adam_alloc(weights, grad_weights, length, num_layers, size, beta1, beta2);
    a->on_device = 1;
    const long span = flat_span(weights, grad_weights, length, num_layers);
    a->flat = span >= 0;
    a->span = a->flat ? span : size;
    a->m = (float*)phip_malloc(sizeof(float) * (size_t)align4(a->span));
    a->v = (float*)phip_malloc(sizeof(float) * (size_t)align4(a->span));
    return a;
}

Adam* create_adam_from_nn_cuda(NeuralNetwork* nn, float beta1, float beta2) {
    const int L = nn->num_layers - 1;
    float** w = (float**)xmalloc(sizeof(float*) * (size_t)(2 * L));
    float** g = (float**)xmalloc(sizeof(float*) * (size_t)(2 * L));
    int* len = (int*)xmalloc(sizeof(int) * (size_t)(2 * L));
    int size = 0;
    for (int i = 0; i < L; i++) {
        Layer* ly = &nn->layers[i];
        w[2 * i] = ly->d_weights;    g[2 * i] = ly->d_grad_weights;    len[2 * i] = ly->input_size * ly->output_size;
        w[2 * i + 1] = ly->d_biases; g[2 * i + 1] = ly->d_grad_biases; len[2 * i + 1] = ly->output_size;
        size += len[2 * i] + len[2 * i + 1];
    }
    Adam* a = create_adam_cuda(w, g, len, 2 * L, size, beta1, beta2);
    free(w); free(g); free(len);
    return a;
}

void free_adam_cuda(Adam* adam) {
    if (!adam) return;
    phip_free(adam->m);
    phip_free(adam->v);
    free(adam->weights);
    free(adam->grad_weights);
    free(adam->lengths);
    free(adam);
}

void adam_update_cuda(Adam* adam, float lr) { adam_update_cuda_w16(adam, lr, NULL, 0, 0); }

/* w16 != NULL: also refresh the bf16 shadow of the first n16 parameters (flat spans only).
 * zero_g: clear the gradient span once read (flat spans only).  Returns bit 0: shadow refreshed,
 * bit 1: gradients cleared. */
int adam_update_cuda_w16(Adam* adam, float lr, unsigned short* w16, long n16, int zero_g) {
    float bc1, bc2;
    bias_corrections(adam, &bc1, &bc2);
    nn_note_device_update(adam->weights[0]);          /* the network's host mirrors are now stale */
    if (adam->flat) {
        /* the clearing pass is the vectorised kernel's: 16-B aligned spans only */
        const uintptr_t al = (uintptr_t)adam->weights[0] | (uintptr_t)adam->grad_weights[0] | (uintptr_t)adam->m |
                             (uintptr_t)adam->v;
        if (al & 15u) zero_g = 0;
        phip_adam_flat_w16(adam->weights[0], adam->grad_weights[0], adam->m, adam->v, adam->span, lr, adam->beta1,
                           adam->beta2, bc1, bc2, adam->grad_scale, w16, w16 ? n16 : 0, zero_g);
        return (w16 != NULL) | (zero_g ? 2 : 0);
    } else {
        phip_adam_multi(adam->weights, adam->grad_weights, adam->lengths, adam->num_layers, adam->m, adam->v, lr,
                        adam->beta1, adam->beta2, bc1, bc2, adam->grad_scale);
    }
    return 0;
}

/* a network's flat Adam (16-B aligned span) and a small flat side Adam (the entropy Adam's log σ) in
 * one launch; the side's step runs first in the step counters (ppo.cu:440-442 order; the spans are
 * independent).  Returns bit 0: shadow refreshed, bit 1: network gradients cleared, bit 2: side
 * gradients cleared; −1 (nothing done) when the pair does not qualify. */
int adam_update_pair_w16(Adam* adam, float lr, unsigned short* w16, long n16, int zero_g, Adam* side, float lr_side,
                         int zero_side) {
    const uintptr_t al = (uintptr_t)adam->weights[0] | (uintptr_t)adam->grad_weights[0] | (uintptr_t)adam->m |
                         (uintptr_t)adam->v;
    if (!adam->flat || !side->flat || (al & 15u) || side->span > 256 || side->span < 1 || adam->span < 1 ||
        adam->beta1 != side->beta1 || adam->beta2 != side->beta2 || ((uintptr_t)w16 & 7u))
        return -1;
    float bc1s, bc2s, bc1, bc2;
    bias_corrections(side, &bc1s, &bc2s);
    bias_corrections(adam, &bc1, &bc2);
    nn_note_device_update(adam->weights[0]);
    nn_note_device_update(side->weights[0]);
    phip_adam_flat_pair(adam->weights[0], adam->grad_weights[0], adam->m, adam->v, adam->span, lr, adam->beta1,
                        adam->beta2, bc1, bc2, adam->grad_scale, w16, w16 ? n16 : 0, zero_g, side->weights[0],
                        side->grad_weights[0], side->m, side->v, (int)side->span, lr_side, bc1s, bc2s,
                        side->grad_scale, zero_side);
    return (w16 != NULL) | (zero_g ? 2 : 0) | (zero_side ? 4 : 0);
}

/* ---------------- checkpoint (adam.cu:172-264 byte layout) ---------------- */
/* m / v are written packed by tensor (reference order), whatever the padding in HBM. */
static void moments_to_host(Adam* a, float* m, float* v) {
    if (!a->on_device) {
        memcpy(m, a->m, sizeof(float) * (size_t)a->size);
        memcpy(v, a->v, sizeof(float) * (size_t)a->size);
        return;
    }
    long src = 0, dst = 0;
    for (int i = 0; i < a->num_layers; i++) {
        if (a->flat) src = (long)(a->weights[i] - a->weights[0]);
        phip_d2h(m + dst, a->m + src, sizeof(float) * (size_t)a->lengths[i]);
        phip_d2h(v + dst, a->v + src, sizeof(float) * (size_t)a->lengths[i]);
        dst += a->lengths[i];
        if (!a->flat) src += a->lengths[i];
    }
}

void save_adam(Adam* adam, FILE* file, bool cuda) {
    (void)cuda;
    fwrite(&adam->size, sizeof(int), 1, file);
    fwrite(&adam->time_step, sizeof(int), 1, file);
    fwrite(&adam->beta1, sizeof(float), 1, file);
    fwrite(&adam->beta2, sizeof(float), 1, file);
    fwrite(&adam->num_layers, sizeof(int), 1, file);
    float* m = (float*)xmalloc(sizeof(float) * (size_t)adam->size);
    float* v = (float*)xmalloc(sizeof(float) * (size_t)adam->size);
    moments_to_host(adam, m, v);
    fwrite(m, sizeof(float), (size_t)adam->size, file);
    fwrite(v, sizeof(float), (size_t)adam->size, file);
    free(m);
    free(v);
}

/* n_expected: tensors the caller's arrays hold (−1: unknown, the reference signature) — a checkpoint
 * whose tensor count or size disagrees is rejected before anything is allocated or copied */
Adam* load_adam_ex(FILE* file, float** weights, float** grad_weights, int* length, int n_expected, bool cuda) {
    int size, t, n;
    float b1, b2;
    if (fread(&size, sizeof(int), 1, file) != 1 || fread(&t, sizeof(int), 1, file) != 1 ||
        fread(&b1, sizeof(float), 1, file) != 1 || fread(&b2, sizeof(float), 1, file) != 1 ||
        fread(&n, sizeof(int), 1, file) != 1)
        die("checkpoint: unexpected end of file");
    if (n <= 0 || (n_expected >= 0 && n != n_expected))
        die("checkpoint: Adam tensor count does not match the network");
    long total = 0;
    for (int i = 0; i < n; i++) {
        if (length[i] < 0) die("checkpoint: negative Adam tensor length");
        total += length[i];
    }
    if (size < 0 || (long)size != total) die("checkpoint: Adam size does not match the tensor lengths");
    float* m = (float*)xmalloc(sizeof(float) * (size_t)size);
    float* v = (float*)xmalloc(sizeof(float) * (size_t)size);
    if (fread(m, sizeof(float), (size_t)size, file) != (size_t)size ||
        fread(v, sizeof(float), (size_t)size, file) != (size_t)size)
        die("checkpoint: unexpected end of file");
    Adam* a;
    if (cuda) {
        a = create_adam_cuda(weights, grad_weights, length, n, size, b1, b2);
        long src = 0, dst = 0;
        for (int i = 0; i < n; i++) {
            if (a->flat) dst = (long)(a->weights[i] - a->weights[0]);
            phip_h2d(a->m + dst, m + src, sizeof(float) * (size_t)length[i]);
            phip_h2d(a->v + dst, v + src, sizeof(float) * (size_t)length[i]);
            src += length[i];
            if (!a->flat) dst += length[i];
        }
        free(m);
        free(v);
    } else {
        a = adam_alloc(weights, grad_weights, length, n, size, b1, b2);
        a->m = m;
        a->v = v;
        a->span = size;
    }
    a->time_step = t;
    return a;
}

Adam* load_adam(FILE* file, float** weights, float** grad_weights, int* length, bool cuda) {
    return load_adam_ex(file, weights, grad_weights, length, -1, cuda);
}

Adam* load_adam_from_nn(FILE* file, NeuralNetwork* nn, bool cuda) {
    const int L = nn->num_layers - 1;
    float** w = (float**)xmalloc(sizeof(float*) * (size_t)(2 * L));
    float** g = (float**)xmalloc(sizeof(float*) * (size_t)(2 * L));
    int* len = (int*)xmalloc(sizeof(int) * (size_t)(2 * L));
    for (int i = 0; i < L; i++) {
        Layer* ly = &nn->layers[i];
        w[2 * i] = cuda ? ly->d_weights : ly->weights;
        w[2 * i + 1] = cuda ? ly->d_biases : ly->biases;
        g[2 * i] = cuda ? ly->d_grad_weights : ly->grad_weights;
        g[2 * i + 1] = cuda ? ly->d_grad_biases : ly->grad_biases;
        len[2 * i] = ly->input_size * ly->output_size;
        len[2 * i + 1] = ly->output_size;
    }
    Adam* a = load_adam_ex(file, w, g, len, 2 * L, cuda);
    free(w); free(g); free(len);
    return a;
}
