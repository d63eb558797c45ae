/*
 * loss.h — mean-squared-error value loss.
 *
 * Drop-in for /root/reference/include/loss.h:10-14 (loss.cu:5-83):
 *   L = Σ (y_true − y)² / (m·n);   grad = 2·(y − y_true)/(m·n)
 * The device version reduces on the GPU with no size limit (the reference's
 * 512-partial host array, loss.cu:56, is gone) and allocates nothing per call.
 */
#ifndef LOSS_H
#define LOSS_H

#include <math.h>

#ifdef __cplusplus
extern "C" {
#endif

float mean_squared_error(float* y, float* y_true, int m, int n);
void mean_squared_error_derivative(float* grad, float* y, float* y_true, int m, int n);

float mean_squared_error_cuda(float* y, float* y_true, int m, int n);
void mean_squared_error_derivative_cuda(float* grad, float* y, float* y_true, int m, int n);

#ifdef __cplusplus
}
#endif
#endif /* LOSS_H */
