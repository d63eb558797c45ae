/*
 * activation_function.h — ReLU and the name→function-pointer table.
 *
 * Drop-in for /root/reference/include/activation_function.h:10-22.
 * "relu" maps to ReLU/ReLU_derivative; any other name maps to NULL pointers,
 * meaning identity (reference activation_function.cu:46-73).
 * ReLU_derivative(x, grad) masks grad where the POST-activation x <= 0.
 */
#ifndef ACTIVATION_FUNCTION_H
#define ACTIVATION_FUNCTION_H

#include <string.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    void (*activation)(float* x, int m, int n);
    void (*activation_derivative)(float* x, float* grad, int m, int n);
} ActivationFunction;

/* host-pointer entry points (staged through HBM in libppo) */
void ReLU(float* x, int m, int n);
void ReLU_derivative(float* x, float* grad, int m, int n);

/* device-pointer entry points */
void ReLU_cuda(float* x, int m, int n);
void ReLU_derivative_cuda(float* x, float* grad, int m, int n);

ActivationFunction* build_activation_function(char* name);
ActivationFunction* build_activation_function_cuda(char* name);

#ifdef __cplusplus
}
#endif
#endif /* ACTIVATION_FUNCTION_H */
