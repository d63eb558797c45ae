/*
 * mat_mul.h — dense linear layer (y = x·Wᵀ + b) and its two backward products.
 *
 * Drop-in for the reference interface /root/reference/include/mat_mul.h:16-20.
 * Layouts are the reference's (row-major): x[m,n], W[l,n] (out×in, PyTorch
 * Linear convention), out[m,l].  The reference's `cublasHandle_t` parameter is
 * replaced by the opaque `ppo_gpu_handle_t` (a HIP stream context owned by
 * libppo); callers that pass `nn->cublas_handle` compile unchanged.
 *
 * In libppo every entry point executes on the MI355X:
 *   mat_mul_cuda / mat_mul_backwards_cuda   device pointers (reference mat_mul.cu:132-217)
 *   mat_mul / mat_mul_backwards             host pointers, staged through HBM
 *                                           (reference mat_mul.cu:39-80, CPU β=1 semantics)
 */
#ifndef MAT_MUL_H
#define MAT_MUL_H

#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Opaque GPU context (replaces cublasHandle_t, reference neural_network.h:52). */
typedef struct ppo_gpu_ctx* ppo_gpu_handle_t;

/* out[m,l] = x[m,n]·weight[l,n]ᵀ + bias[l]                        (mat_mul.cu:39-55) */
void mat_mul(float* out, float* x, float* weight, float* bias, int m, int n, int l);
/* grad_x[m,n] += grad_in[m,l]·weight[l,n];  grad_weight[l,n] += grad_inᵀ·x
 * (accumulating, like the reference's cblas β=1 calls, mat_mul.cu:57-80)   */
void mat_mul_backwards(float* grad_x, float* grad_weight, float* grad_in, float* x, float* weight, int m, int n, int l);

/* Device versions (mat_mul.cu:132-217): the backward OVERWRITES (β=0). */
void mat_mul_cuda(ppo_gpu_handle_t handle, float* out, float* x, float* weight, float* bias, int m, int n, int l);
void mat_mul_backwards_cuda(ppo_gpu_handle_t handle, float* grad_x, float* grad_weight, float* grad_in, float* x, float* weight, int m, int n, int l);

#ifdef __cplusplus
}
#endif
#endif /* MAT_MUL_H */
