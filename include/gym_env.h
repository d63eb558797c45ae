/*
 * gym_env.h — gymnasium-compatible environment constructor.
 *
 * Drop-in for /root/reference/include/gym_env.h:8.  The reference embeds
 * CPython and imports gymnasium (gym_env.c:5-35).  gymnasium is not available
 * on the build/GPU images, so libppo implements Pendulum-v1 (id 0) natively in
 * C with the gymnasium dynamics (max_episode_steps = 200, γ = 0.99).  This
 * header therefore does not pull in <Python.h>.
 */
#ifndef GYM_ENV_H
#define GYM_ENV_H

#include "env.h"
#include <stdbool.h>

#ifdef __cplusplus
extern "C" {
#endif

Env* create_gym_env(int id, int seed);

#ifdef __cplusplus
}
#endif

#endif /* GYM_ENV_H */
