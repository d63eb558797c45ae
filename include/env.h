/*
 * env.h — environment ABI (function-pointer table).
 *
 * Drop-in for /root/reference/include/env.h:7-18.  Environments are outside
 * the accelerated path (OUT OF SCOPE); libppo ships the reference's
 * toy env (create_simple_env) and a native Pendulum-v1 behind create_gym_env
 * so the reference main.c links and runs.
 */
#ifndef ENV_H
#define ENV_H

#include <stdbool.h>
#include <stdlib.h>

typedef struct {
    void (*free_env)();
    void (*reset_env)(float* state);
    void (*step_env)(float* action, float* obs, float* reward, bool* terminated, bool* truncated, int action_size);
    int state_size;
    int action_size;
    int horizon;
    float gamma;
} Env;

#ifdef __cplusplus
extern "C" {
#endif

Env* create_simple_env(int id, int seed);

#ifdef __cplusplus
}
#endif

#endif /* ENV_H */
