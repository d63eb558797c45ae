/*
 * adam.h — Adam over a list of (pointer, length) tensors.
 *
 * Drop-in for /root/reference/include/adam.h:10-38.  Update rule (adam.cu:53-74):
 *   t += 1;  m = β1·m + (1−β1)·g;  v = β2·v + (1−β2)·g²
 *   θ −= (lr/(1−β1^t)) · m / (sqrt(v/(1−β2^t)) + 1e-8)
 *
 * libppo: when the tensors are contiguous in memory (the flat per-network
 * buffers of neural_network.h) the update is ONE vectorised streaming kernel
 * over the flat range; otherwise a multi-tensor kernel walks a small table.
 * m and v are always flat device buffers of `size` floats (`size` counts the
 * span including alignment padding for flat networks; padding gradients are 0).
 */
#ifndef ADAM_H
#define ADAM_H

#include <stdbool.h>
#include "neural_network.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    float** weights;        /* tensor base pointers (host array of pointers) */
    float** grad_weights;
    int* lengths;
    float* m;
    float* v;
    float beta1;
    float beta2;
    int time_step;
    int size;
    int num_layers;         /* number of tensors */

    /* ---- libppo extension ---- */
    int on_device;          /* 1: tensors/m/v are device pointers */
    int flat;               /* 1: tensors are one contiguous span starting at weights[0] */
    float grad_scale;       /* multiplies g before the update (1/world for data-parallel) */
    long span;              /* floats covered by the flat update (≥ size when tensors are padded) */
} Adam;

Adam* create_adam(float** weights, float** grad_weights, int* length, int num_layers, int size, float beta1, float beta2);
Adam* create_adam_from_nn(NeuralNetwork* nn, float beta1, float beta2);
void free_adam(Adam* adam);
void adam_update(Adam* adam, float lr);

Adam* create_adam_cuda(float** weights, float** grad_weights, int* length, int num_layers, int size, float beta1, float beta2);
Adam* create_adam_from_nn_cuda(NeuralNetwork* nn, float beta1, float beta2);
void free_adam_cuda(Adam* adam);
void adam_update_cuda(Adam* adam, float lr);

void save_adam(Adam* adam, FILE* file, bool cuda);
Adam* load_adam(FILE* file, float** weights, float** grad_weights, int* length, bool cuda);
Adam* load_adam_from_nn(FILE* file, NeuralNetwork* nn, bool cuda);

#ifdef __cplusplus
}
#endif
#endif /* ADAM_H */
