/*
 * env.c — environments behind the reference's Env ABI (OUT OF SCOPE of the
 * accelerated path; present so the reference main.c links and runs).
 *
 *  create_simple_env : the reference's 1-D "reach 5" toy (src/env.c:6-51), restated.
 *  create_gym_env    : Pendulum-v1 (id 0) with gymnasium's dynamics, native C.  The reference
 *                      embeds CPython + gymnasium (src/gym_env.c, scripts/gym_env.py); gymnasium
 *                      is not installable here, so the dynamics are restated (classic_control
 *                      pendulum: g = 10, m = l = 1, dt = 0.05, max speed 8, max torque 2,
 *                      200-step time limit).  Its reset noise comes from a seeded xorshift, not
 *                      numpy's generator, so trajectories are not bit-identical to gymnasium.
 */
#include "internal.h"

#include <math.h>

/* ---------------- toy env (src/env.c) ---------------- */
static float g_simple_state = 0;
static int g_simple_step = 0;

static void reset_simple_env(float* obs) {
    g_simple_state = 0;
    g_simple_step = 0;
    obs[0] = 0;
}

static void step_simple_env(float* action, float* obs, float* reward, bool* terminated, bool* truncated,
                            int action_size) {
    (void)action_size;
    g_simple_state += fmaxf(fminf(action[0], 1), -1);
    obs[0] = g_simple_state;
    g_simple_step += 1;
    if (g_simple_state >= 5) {
        reward[0] = 1; terminated[0] = true; truncated[0] = false;
    } else if (g_simple_step >= 15) {
        reward[0] = 0; terminated[0] = false; truncated[0] = true;
    } else {
        reward[0] = 0; terminated[0] = false; truncated[0] = false;
    }
}

static void free_simple_env(void) {}

Env* create_simple_env(int id, int seed) {
    (void)id; (void)seed;
    Env* env = (Env*)xmalloc(sizeof(Env));
    env->state_size = 1;
    env->action_size = 1;
    env->reset_env = reset_simple_env;
    env->step_env = step_simple_env;
    env->free_env = free_simple_env;
    env->horizon = 15;
    env->gamma = 0.99f;
    return env;
}

/* ---------------- Pendulum-v1 ---------------- */
static double g_th = 0, g_thdot = 0;
static int g_pstep = 0;
static uint64_t g_rng = 0x9E3779B97F4A7C15ULL;

static double rng_uniform(double lo, double hi) {
    g_rng ^= g_rng << 13; g_rng ^= g_rng >> 7; g_rng ^= g_rng << 17;
    return lo + (hi - lo) * ((double)(g_rng >> 11) * (1.0 / 9007199254740992.0));
}

static void pendulum_obs(float* obs) {
    obs[0] = (float)cos(g_th);
    obs[1] = (float)sin(g_th);
    obs[2] = (float)g_thdot;
}

static void reset_pendulum(float* obs) {
    g_th = rng_uniform(-M_PI, M_PI);
    g_thdot = rng_uniform(-1.0, 1.0);
    g_pstep = 0;
    pendulum_obs(obs);
}

static void step_pendulum(float* action, float* obs, float* reward, bool* terminated, bool* truncated,
                          int action_size) {
    (void)action_size;
    const double g = 10.0, m = 1.0, l = 1.0, dt = 0.05, max_speed = 8.0, max_torque = 2.0;
    double u = action[0];
    if (u < -max_torque) u = -max_torque;
    if (u > max_torque) u = max_torque;
    double an = fmod(g_th + M_PI, 2 * M_PI);
    if (an < 0) an += 2 * M_PI;
    an -= M_PI;
    const double costs = an * an + 0.1 * g_thdot * g_thdot + 0.001 * u * u;
    double nthdot = g_thdot + (3 * g / (2 * l) * sin(g_th) + 3.0 / (m * l * l) * u) * dt;
    if (nthdot < -max_speed) nthdot = -max_speed;
    if (nthdot > max_speed) nthdot = max_speed;
    g_th = g_th + nthdot * dt;
    g_thdot = nthdot;
    g_pstep += 1;
    pendulum_obs(obs);
    *reward = (float)(-costs);
    *terminated = false;
    *truncated = g_pstep >= 200;
}

static void free_pendulum(void) {}

Env* create_gym_env(int id, int seed) {
    if (id != 0) die("create_gym_env: only Pendulum-v1 (id 0) is available natively");
    g_rng = 0x9E3779B97F4A7C15ULL ^ ((uint64_t)(uint32_t)seed * 0xBF58476D1CE4E5B9ULL);
    if (!g_rng) g_rng = 1;
    Env* env = (Env*)xmalloc(sizeof(Env));
    env->state_size = 3;
    env->action_size = 1;
    env->horizon = 200;
    env->reset_env = reset_pendulum;
    env->step_env = step_pendulum;
    env->free_env = free_pendulum;
    env->gamma = 0.99f;                                      /* gym_env.c:102 */
    return env;
}
