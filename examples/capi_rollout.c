/* capi_rollout.c — plain-C use of libmarlenv_hip.so (include/marlenv.h):
 * create a batch of intersection envs, roll them out with random actions on
 * host buffers, print per-step checksums.  No C++, no Python, no torch.
 *
 *   gcc -O2 -std=c11 -I include examples/capi_rollout.c \
 *       -L marl-traffic-intersection_amd -lmarlenv_hip \
 *       -Wl,-rpath,'$ORIGIN/../marl-traffic-intersection_amd' -o build/capi_rollout
 *   build/capi_rollout [envs] [agents] [rays] [steps]
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "marlenv.h"

#define CHECK(call)                                                                 \
    do {                                                                            \
        int rc_ = (call);                                                           \
        if (rc_ != MEV_OK) {                                                        \
            fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, mev_last_error());  \
            return 1;                                                               \
        }                                                                           \
    } while (0)

static uint32_t xs = 12345u;
static float urand(void) { /* xorshift32 in [-1, 1) */
    xs ^= xs << 13;
    xs ^= xs >> 17;
    xs ^= xs << 5;
    return (float)(xs >> 8) * (2.0f / 16777216.0f) - 1.0f;
}

int main(int argc, char** argv) {
    mev_config cfg;
    CHECK(mev_config_default(&cfg));
    cfg.num_envs = argc > 1 ? atoi(argv[1]) : 64;
    cfg.num_agents = argc > 2 ? atoi(argv[2]) : 8;
    cfg.lidar_rays = argc > 3 ? atoi(argv[3]) : 64;
    const int steps = argc > 4 ? atoi(argv[4]) : 20;
    cfg.use_team_reward = 1;
    mev_handle* h = NULL;
    CHECK(mev_create(&cfg, &h));
    int32_t D = 0;
    CHECK(mev_obs_dim(h, &D));
    const size_t E = (size_t)cfg.num_envs, EN = E * (size_t)cfg.num_agents;
    float* act = malloc(EN * 2 * sizeof(float));
    float* obs = malloc(EN * (size_t)D * sizeof(float));
    float* rew = malloc(EN * sizeof(float));
    uint8_t* status = malloc(EN);
    uint8_t* term = malloc(E);
    uint8_t* trunc = malloc(E);
    if (!act || !obs || !rew || !status || !term || !trunc) return 1;
    CHECK(mev_reset(h, NULL, obs, 0));
    for (int t = 0; t < steps; ++t) {
        for (size_t i = 0; i < EN * 2; ++i) act[i] = urand();
        mev_step_args a = {0};
        a.actions = act;
        a.dt = 1.0f / 60.0f;
        a.obs = obs;
        a.reward = rew;
        a.status = status;
        a.terminated = term;
        a.truncated = trunc;
        a.flags = MEV_AUTO_RESET;
        CHECK(mev_step(h, &a));
        double osum = 0.0, rsum = 0.0;
        int crashed = 0;
        for (size_t i = 0; i < EN * (size_t)D; ++i) osum += obs[i];
        for (size_t i = 0; i < EN; ++i) {
            rsum += rew[i];
            crashed += status[i] >= MEV_CRASH_WALL;
        }
        printf("step %3d obs_sum %.6f reward_sum %.6f crashes %d\n", t + 1, osum, rsum, crashed);
    }
    CHECK(mev_destroy(h));
    free(act); free(obs); free(rew); free(status); free(term); free(trunc);
    return 0;
}
