/*
 * internal.h — helpers shared by libppo's plain-C host code.
 *
 * The host side is orchestration only: object lifetime, the reference's
 * libc-rand() consumption order (weight init, shuffles, rollout noise) and
 * launch sequencing.  Every numeric operation of the PPO path runs in a HIP
 * kernel through ppo_hip.h; host-pointer entry points of the reference API
 * stage their operands through HBM (stage_*) and run the same kernels.
 */
#ifndef PPO_HOST_INTERNAL_H
#define PPO_HOST_INTERNAL_H

#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/ppo.h"
#include "../csrc/ppo_hip.h"

void* xmalloc(size_t n);
void* xcalloc(size_t n, size_t sz);
void  die(const char* msg);

/* grow-only device scratch slots for host-pointer (staged) entry points */
enum { ST_A = 0, ST_B, ST_C, ST_D, ST_E, ST_F, ST_G, ST_H, ST_COUNT };
void* stage(int slot, size_t bytes);
float* stage_up(int slot, const float* host, size_t count);   /* h2d into slot, returns device ptr */

static inline long align4(long n) { return (n + 3) & ~3L; }

/* fp32 GEMM engine used when PPO_F32_GEMM is unset (ppo_ext.h ppo_gemm_f32_engine): 1 = x3 */
#define PPO_F32_ENGINE_DEFAULT 1
int  ppo_gemm_f32_engine(int engine);
/* linear-layer products of the reference API through the engine choice (neural_network.c) */
void lin_fwd(float* y, const float* x, const float* W, const float* b, int m, int n, int l);
void lin_bwd_x(float* gx, const float* g, const float* W, int m, int n, int l);
void lin_bwd_w(float* gW, const float* g, const float* x, int m, int n, int l);

/* neural_network.c internals used by policy.c / ppo.c */
NeuralNetwork* nn_create_ex(int* layer_sizes, char** activation_functions, int num_layers, long extra_floats,
                            int init_from_rand);
int  nn_is_relu(const NeuralNetwork* nn, int layer);
void nn_ensure_act(NeuralNetwork* nn, int m);
void nn_ensure_grad(NeuralNetwork* nn, int m);
/* device forward using d_x as layer-0 input (no copy) */
void nn_forward_dev(NeuralNetwork* nn, const float* d_x, int m);
void nn_forward_dev_rows(NeuralNetwork* nn, const float* d_x, const int* d_rows, float* d_xcopy, int m);
/* device backward from d_grad_out (no copy unless the output activation needs masking) */
void nn_backward_dev(NeuralNetwork* nn, const float* d_grad_out, int m, int want_grad_x0);
/* the same; grads_zero: d_grads already hold zeros (cleared by the previous Adam step), no memset;
 * reduce_extra ≥ 0 (data parallelism): the gradients are all-reduced in buckets of consecutive
 * layers as the backward finishes them (top bucket: also the reduce_extra floats after the
 * network's parameters — the policy's log σ gradient); the caller joins before Adam */
void nn_backward_dev_z(NeuralNetwork* nn, const float* d_grad_out, int m, int want_grad_x0, int grads_zero,
                       long reduce_extra);
/* the output layer fused with the loss head (head 0 value / MSE, 1 policy), see neural_network.c */
int  nn_out_head_ok(const NeuralNetwork* nn, int head);
int  nn_value_fold_ok(const NeuralNetwork* nn, int m);
void nn_value_fold_step(NeuralNetwork* nn, const float* d_x, const int* d_rows, float* d_xcopy, int m, int grads_zero,
                        long reduce_extra, const float* tgt, float* loss_accum);
int  nn_policy_wide_ok(const NeuralNetwork* nn, int m);
void nn_policy_wide_step(NeuralNetwork* nn, const float* d_x, const int* d_rows, float* d_xcopy, int m,
                         int grads_zero, long reduce_extra, const float* log_std, const float* action,
                         const float* adv, const float* old_lp, float eps, float ent_coeff, float* grad_log_std,
                         float* loss_accum);
void nn_out_head_step(NeuralNetwork* nn, int head, const float* d_x, const int* d_rows, float* d_xcopy, int m,
                      int grads_zero, long reduce_extra, const float* tgt, const float* log_std, const float* action,
                      const float* adv, const float* old_lp, float eps, float ent_coeff, float* grad_log_std,
                      float* loss_accum);

NeuralNetwork* nn_load_ex(FILE* file, long extra_floats);
/* host mirror <-> HBM reconciliation (neural_network.c) */
void nn_note_device_update(const float* d_ptr);   /* an HBM parameter update touched d_ptr's network */
void nn_host_sync(NeuralNetwork* nn, float* extra); /* before a host-pointer entry point computes */
void nn_sync_extra_snapshot(NeuralNetwork* nn, const float* extra);
void policy_host_sync(GaussianPolicy* p);
void nn_sync_w16(NeuralNetwork* nn);       /* bf16 mode: refresh the bf16 weight shadow */

/* adam.c */
void adam_next_step(Adam* a, float lr, float* step, float* bc2);
/* device Adam that also writes the bf16 shadow w16[0, n16) in the same pass; returns 1 when it did */
int adam_update_cuda_w16(Adam* adam, float lr, unsigned short* w16, long n16, int zero_g);
int adam_update_pair_w16(Adam* adam, float lr, unsigned short* w16, long n16, int zero_g, Adam* side, float lr_side,
                         int zero_side);

/* checkpoint Adam with a known tensor count (n_expected < 0: unknown); rejects mismatches */
Adam* load_adam_ex(FILE* file, float** weights, float** grad_weights, int* length, int n_expected, bool cuda);

/* trajectory_buffer.c */
void buffer_point_device(TrajectoryBuffer* b);

/* policy.c */
GaussianPolicy* policy_create_ex(int* layer_sizes, char** activation_functions, int num_layers, float init_std,
                                 int init_from_rand);

/* ppo.c: GAE on the device buffer with explicit output of v / v_next scratch */
void ppo_gae_device(NeuralNetwork* V, TrajectoryBuffer* buffer, float gamma, float lambda);

#endif
