/*
 * layers.c — mat_mul, activation and loss entry points of the reference API.
 *
 * References: /root/reference/src/mat_mul.cu:39-217, activation_function.cu:5-73,
 * loss.cu:5-83.  `_cuda` functions take device pointers; the plain names take
 * host pointers and are staged through HBM onto the same kernels.
 */
#include "internal.h"

/* ---------------- mat_mul.h ---------------- */
void mat_mul_cuda(ppo_gpu_handle_t handle, float* out, float* x, float* weight, float* bias, int m, int n, int l) {
    (void)handle;
    lin_fwd(out, x, weight, bias, m, n, l);
}

/* mat_mul.cu:165-217: both products overwrite (cuBLAS β = 0) */
void mat_mul_backwards_cuda(ppo_gpu_handle_t handle, float* grad_x, float* grad_weight, float* grad_in, float* x,
                            float* weight, int m, int n, int l) {
    (void)handle;
    if (grad_x) lin_bwd_x(grad_x, grad_in, weight, m, n, l);
    lin_bwd_w(grad_weight, grad_in, x, m, n, l);
}

void mat_mul(float* out, float* x, float* weight, float* bias, int m, int n, int l) {
    float* dx = stage_up(ST_A, x, (size_t)m * n);
    float* dw = stage_up(ST_B, weight, (size_t)l * n);
    float* db = stage_up(ST_C, bias, (size_t)l);
    float* dy = (float*)stage(ST_D, sizeof(float) * (size_t)m * l);
    lin_fwd(dy, dx, dw, db, m, n, l);
    phip_d2h(out, dy, sizeof(float) * (size_t)m * l);
}

/* mat_mul.cu:57-80: the CPU products ACCUMULATE into grad_x / grad_weight (β = 1) */
void mat_mul_backwards(float* grad_x, float* grad_weight, float* grad_in, float* x, float* weight, int m, int n,
                       int l) {
    float* dg = stage_up(ST_A, grad_in, (size_t)m * l);
    float* dx = stage_up(ST_B, x, (size_t)m * n);
    float* dw = stage_up(ST_C, weight, (size_t)l * n);
    float* tmp = (float*)stage(ST_D, sizeof(float) * ((size_t)m * n > (size_t)l * n ? (size_t)m * n : (size_t)l * n));
    if (grad_x) {
        float* acc = stage_up(ST_E, grad_x, (size_t)m * n);
        lin_bwd_x(tmp, dg, dw, m, n, l);
        phip_axpy(acc, tmp, (long)m * n);
        phip_d2h(grad_x, acc, sizeof(float) * (size_t)m * n);
    }
    float* accw = stage_up(ST_F, grad_weight, (size_t)l * n);
    lin_bwd_w(tmp, dg, dx, m, n, l);
    phip_axpy(accw, tmp, (long)l * n);
    phip_d2h(grad_weight, accw, sizeof(float) * (size_t)l * n);
}

/* ---------------- activation_function.h ---------------- */
void ReLU_cuda(float* x, int m, int n) { phip_relu(x, (long)m * n); }
void ReLU_derivative_cuda(float* x, float* grad, int m, int n) { phip_relu_bwd(x, grad, (long)m * n); }

void ReLU(float* x, int m, int n) {
    const size_t cnt = (size_t)m * n;
    float* d = stage_up(ST_A, x, cnt);
    phip_relu(d, (long)cnt);
    phip_d2h(x, d, sizeof(float) * cnt);
}

void ReLU_derivative(float* x, float* grad, int m, int n) {
    const size_t cnt = (size_t)m * n;
    float* dx = stage_up(ST_A, x, cnt);
    float* dg = stage_up(ST_B, grad, cnt);
    phip_relu_bwd(dx, dg, (long)cnt);
    phip_d2h(grad, dg, sizeof(float) * cnt);
}

static ActivationFunction* build(const char* name, int device) {
    ActivationFunction* a = (ActivationFunction*)xmalloc(sizeof(ActivationFunction));
    if (name && strcmp(name, "relu") == 0) {
        a->activation = device ? &ReLU_cuda : &ReLU;
        a->activation_derivative = device ? &ReLU_derivative_cuda : &ReLU_derivative;
    } else {                      /* any other name: identity (activation_function.cu:46-73) */
        a->activation = NULL;
        a->activation_derivative = NULL;
    }
    return a;
}
ActivationFunction* build_activation_function(char* name) { return build(name, 0); }
ActivationFunction* build_activation_function_cuda(char* name) { return build(name, 1); }

/* ---------------- loss.h ---------------- */
float mean_squared_error_cuda(float* y, float* y_true, int m, int n) {
    float* d_loss = (float*)stage(ST_H, 16);
    phip_mse(y, y_true, (long)m * n, NULL, d_loss, NULL);
    float loss = 0.f;
    phip_d2h(&loss, d_loss, sizeof(float));
    return loss;
}

void mean_squared_error_derivative_cuda(float* grad, float* y, float* y_true, int m, int n) {
    phip_mse(y, y_true, (long)m * n, grad, NULL, NULL);
}

float mean_squared_error(float* y, float* y_true, int m, int n) {
    const size_t cnt = (size_t)m * n;
    float* dy = stage_up(ST_A, y, cnt);
    float* dt = stage_up(ST_B, y_true, cnt);
    return mean_squared_error_cuda(dy, dt, m, n);
}

void mean_squared_error_derivative(float* grad, float* y, float* y_true, int m, int n) {
    const size_t cnt = (size_t)m * n;
    float* dy = stage_up(ST_A, y, cnt);
    float* dt = stage_up(ST_B, y_true, cnt);
    float* dg = (float*)stage(ST_C, sizeof(float) * cnt);
    phip_mse(dy, dt, (long)cnt, dg, NULL, NULL);
    phip_d2h(grad, dg, sizeof(float) * cnt);
}
