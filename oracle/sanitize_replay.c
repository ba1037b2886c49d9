/*
 * sanitize_replay.c — TEST INFRASTRUCTURE: the C restatement
 * (marl_oracle.c, included as one translation unit) built with
 * -fsanitize=address,undefined, replaying one scenario from a flat binary file
 * that tests/test_oracle_sanitized.py writes from a golden vector
 * (tests/golden/*.npz).  Writes every step's outputs to a second file the test
 * compares with the golden outputs bit for bit; any sanitizer report aborts
 * the process (the CPU restatement under ASan/UBSan).
 *
 * Input (little-endian): int32 hdr[13] = {lanes, n, rays, obs_dim, use_team,
 * respawn, max_steps, traffic, max_npcs, steps, n_traffic_routes, n_npcs, step_count};
 * float fhdr[10] = {density, dt, reward[8]}; int32 traffic_routes[n_tr];
 * orc_car egos[n]; orc_car npcs[n_npcs]; float actions[steps][n][2];
 * int32 spawned[steps].
 * Output: per step obs f32[n][D] | rew f32[n] | done u8[n] | status u8[n] | flags i32[4].
 * Usage: sanitize_replay IN OUT
 */
#include "marl_oracle.c"

#include <stdio.h>

static int rd(FILE* f, void* p, size_t n) { return fread(p, 1, n, f) == n ? 0 : -1; }

int main(int argc, char** argv) {
    if (argc != 3) return 2;
    FILE* in = fopen(argv[1], "rb");
    FILE* out = fopen(argv[2], "wb");
    if (!in || !out) return 2;
    int32_t h[13];
    float fh[10];
    if (rd(in, h, sizeof h) || rd(in, fh, sizeof fh)) return 3;
    const int lanes = h[0], n = h[1], rays = h[2], obs_dim = h[3], steps = h[9], ntr = h[10], nnpc = h[11];
    if (n < 1 || n > MAXCARS || nnpc < 0 || nnpc > MAXCARS || ntr < 0 || ntr > 4096 || steps < 0) return 3;
    orc_env* e = orc_create(lanes, n, rays, 360.0f, 250.0f, 4.0f, obs_dim, h[4], h[5], h[6], h[7], fh[0], fh + 2, h[8]);
    if (!e) return 4;
    int32_t* tr = (int32_t*)malloc(sizeof(int32_t) * (size_t)(ntr > 0 ? ntr : 1));
    orc_car* egos = (orc_car*)malloc(sizeof(orc_car) * (size_t)n);
    orc_car* npcs = (orc_car*)malloc(sizeof(orc_car) * (size_t)(nnpc > 0 ? nnpc : 1));
    float* act = (float*)malloc(sizeof(float) * 2 * (size_t)n * (size_t)(steps > 0 ? steps : 1));
    int32_t* sp = (int32_t*)malloc(sizeof(int32_t) * (size_t)(steps > 0 ? steps : 1));
    if (rd(in, tr, sizeof(int32_t) * (size_t)ntr) || rd(in, egos, sizeof(orc_car) * (size_t)n) ||
        rd(in, npcs, sizeof(orc_car) * (size_t)nnpc) || rd(in, act, sizeof(float) * 2 * (size_t)n * (size_t)steps) ||
        rd(in, sp, sizeof(int32_t) * (size_t)steps))
        return 3;
    orc_set_traffic_routes(e, tr, ntr);
    orc_set_state(e, egos, npcs, nnpc, h[12]);
    const int D = e->obs_dim;
    float* obs = (float*)malloc(sizeof(float) * (size_t)n * (size_t)D);
    float* rew = (float*)malloc(sizeof(float) * (size_t)n);
    uint8_t* done = (uint8_t*)malloc((size_t)n);
    uint8_t* st = (uint8_t*)malloc((size_t)n);
    int32_t fl[4];
    for (int t = 0; t < steps; ++t) {
        orc_step(e, act + (size_t)t * 2 * (size_t)n, fh[1], h[7] ? sp[t] : -1, obs, rew, done, st, fl);
        fwrite(obs, sizeof(float), (size_t)n * (size_t)D, out);
        fwrite(rew, sizeof(float), (size_t)n, out);
        fwrite(done, 1, (size_t)n, out);
        fwrite(st, 1, (size_t)n, out);
        fwrite(fl, sizeof(int32_t), 4, out);
    }
    fclose(out);
    fclose(in);
    free(obs); free(rew); free(done); free(st); free(tr); free(egos); free(npcs); free(act); free(sp);
    orc_destroy(e);
    return 0;
}
