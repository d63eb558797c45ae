/*
 * neural_network.h — MLP built from mat_mul layers.
 *
 * Drop-in for /root/reference/include/neural_network.h:18-72.  The struct
 * fields callers can touch keep their names and meaning; the CUDA/cuBLAS
 * includes are gone and `cublas_handle` is an opaque ppo_gpu_handle_t.
 *
 * MI355X layout (libppo): all weights and biases of one network live in ONE
 * flat, 16-byte aligned fp32 HBM buffer ([W0,b0,W1,b1,...], each tensor
 * padded to a multiple of 4 floats); Layer.d_weights / d_biases point into it.
 * Gradients use a second flat buffer with the same offsets.  This makes Adam
 * and the cross-GPU gradient all-reduce a single call per network.
 *
 * Semantics kept from the reference:
 *   - layers[i].input (host) / d_input (device) cache the POST-activation
 *     input of layer i; backward must follow a forward on the same network
 *     (neural_network.cu:74-105,163-189).
 *   - backward overwrites the gradients of every layer (not accumulated
 *     across calls) (neural_network.cu:121-161,192-231).
 */
#ifndef NEURAL_NETWORK_H
#define NEURAL_NETWORK_H

#include <stdlib.h>
#include <stdio.h>
#include <string.h>
#include <math.h>

#include "mat_mul.h"
#include "activation_function.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    float* weights;        /* host mirror [out*in]  */
    float* biases;         /* host mirror [out]     */
    float* grad_weights;
    float* grad_biases;
    float* input;          /* host cached post-activation input [m, input_size] */

    float* d_weights;      /* into NeuralNetwork.d_params  */
    float* d_biases;
    float* d_grad_weights; /* into NeuralNetwork.d_grads   */
    float* d_grad_biases;
    float* d_input;        /* device cached post-activation input [m, input_size] */

    float* d_grad_x;       /* device grad w.r.t. this layer's input [m, input_size] */

    ActivationFunction* activation_function;
    ActivationFunction* d_activation_function;
    int input_size;
    int output_size;
} Layer;

typedef struct {
    Layer* layers;          /* num_layers entries; the last one only carries the output */
    int num_layers;         /* number of layer SIZES (= linear layers + 1) */
    int output_size;

    int cache_m_forward;
    int cache_m_backward;

    float* output;          /* host [m, output_size] */
    float* d_output;        /* device [m, output_size] (aliases layers[num_layers-1].d_input) */
    char** activation_functions;

    ppo_gpu_handle_t cublas_handle;   /* name kept for source compatibility */

    /* ---- libppo extension (appended; not in the reference struct) ---- */
    float* d_params;        /* flat parameter buffer */
    float* d_grads;         /* flat gradient buffer (same offsets) */
    long   num_params;      /* floats in d_params including alignment padding */
    long   num_params_packed; /* Σ in·out + out (reference Adam size) */
    long*  param_offset;    /* per linear layer: offset of W in the flat buffer */
    long*  bias_offset;     /* per linear layer: offset of b */
    int    act_cap_m;       /* rows the device activation cache can hold */
    int    grad_cap_m;      /* rows the device grad cache can hold */
    int    host_cap_m;      /* rows the host staging arrays can hold */
    long   extra_floats;    /* trailing floats in d_params/d_grads owned by the caller (policy log_std) */
    const float* d_x0;      /* input of layer 0 used by the last device forward */
    unsigned* d_act_bits;   /* ReLU′ masks as bits, one [act_cap_m, ⌈size_i/32⌉] block per layer input */
    int    bits_m;          /* rows of the forward that wrote d_act_bits (−1: none valid) */
    int    dtype;           /* compute mode: 0 = fp32 (default), 1 = bf16 MFMA (C5) — see ppo_ext.h */
    int    x0_dtype;        /* storage of d_x0: 0 = fp32, 1 = bf16 (the gathered copy in bf16 mode) */
    unsigned short* d_w16;  /* bf16 mode: bf16 shadow of d_params (same offsets), refreshed after updates */
    float* d_tiny_wt;       /* small-network update path: transposed weights scratch */
    long   tiny_wt_cap;
    /* host mirror <-> HBM reconciliation for the host-pointer entry points (forward_propagation,
     * sample_action, ...): HBM parameters changed by Adam / ppo_update are pulled to the host
     * mirrors, host mirrors edited by the caller are pushed to HBM — never blindly overwritten */
    float* h_sync;          /* host-mirror snapshot at the last sync: packed [W0,b0,...] then extra_floats */
    long   dev_version;     /* bumped by every HBM parameter update */
    long   host_version;    /* dev_version the host mirrors (weights and extra floats) last matched */
    long   host_version_w;  /* dev_version the host weight mirrors last matched (a weights-only sync) */
    float* d_fold_ws;       /* value-head fold scratch (nn_value_fold_step): partial dots [slots][m] | g [m] */
    long   fold_ws_cap;     /* floats */
} NeuralNetwork;

typedef struct {
    float (*loss)(float* y, float* y_true, int m, int n);
    void (*loss_derivative)(float* grad, float* y, float* y_true, int m, int n);
} LossFunction;

NeuralNetwork* create_neural_network(int* layer_sizes, char** activation_functions, int num_layers);
void forward_propagation(NeuralNetwork* nn, float* input, int m);
void free_neural_network(NeuralNetwork* nn);
void backward_propagation(NeuralNetwork* nn, float* grad_in, int m);

void forward_propagation_cuda(NeuralNetwork* nn, float* input, int m);
void backward_propagation_cuda(NeuralNetwork* nn, float* grad_in, int m);

void nn_write_weights_to_device(NeuralNetwork* nn);
void nn_write_weights_to_host(NeuralNetwork* nn);

void save_neural_network(NeuralNetwork* nn, FILE* file);
NeuralNetwork* load_neural_network(FILE* file);

#ifdef __cplusplus
}
#endif
#endif /* NEURAL_NETWORK_H */
