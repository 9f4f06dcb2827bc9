/* oracle/san_driver.c — TEST INFRASTRUCTURE: drives the CPU restatement (cpu_ref.c) under
 * AddressSanitizer + UndefinedBehaviorSanitizer (the ASan/UBSan build of the oracle).
 *
 *   make -C oracle san        ->  oracle/build/san_driver (cpu_ref.c + this file, -fsanitize=address,undefined)
 *   oracle/build/san_driver <cn_config blob> <steps> <seed>
 *
 * The cn_config blob is the raw struct written by tests/test_oracle_sanitizers.py from make_cn_config (same
 * header, same layout). The driver resets every env, steps it with seeded actions (auto-resets, goal
 * changes, bounded rejection loops included), checks that every output is finite, and exits 0; any
 * sanitizer report aborts the process with a nonzero status. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../include/crowdnav.h"

typedef struct ref_engine ref_engine;
int cnref_create(const cn_config *cfg, ref_engine **out);
void cnref_destroy(ref_engine *g);
int cnref_reset(ref_engine *g, float *robot_node, float *temporal, float *spatial);
int cnref_step(ref_engine *g, const float *actions, float *robot_node, float *temporal, float *spatial,
               float *reward, uint8_t *done, int8_t *event, float *info, double *ep_return, int32_t *ep_len);
const char *cnref_last_error(void);
void cnref_set_threads(int n);

static uint64_t lcg = 88172645463325252ull;
static double urand(void)
{
    lcg ^= lcg << 13; lcg ^= lcg >> 7; lcg ^= lcg << 17;
    return (double)(lcg >> 11) * (1.0 / 9007199254740992.0);
}

int main(int argc, char **argv)
{
    if (argc < 4) { fprintf(stderr, "usage: san_driver <cfg blob> <steps> <seed>\n"); return 2; }
    cn_config c;
    FILE *f = fopen(argv[1], "rb");
    if (!f || fread(&c, sizeof c, 1, f) != 1) { fprintf(stderr, "cannot read %s\n", argv[1]); return 2; }
    fclose(f);
    const int steps = atoi(argv[2]);
    lcg += (uint64_t)atoll(argv[3]) * 0x9E3779B97F4A7C15ull;
    cnref_set_threads(1);
    ref_engine *g = NULL;
    if (cnref_create(&c, &g)) { fprintf(stderr, "create: %s\n", cnref_last_error()); return 3; }
    const int E = c.num_envs, N = c.human_num;
    float *rn = malloc(sizeof(float) * E * 7), *te = malloc(sizeof(float) * E * 2), *se = malloc(sizeof(float) * E * N * 2);
    float *act = malloc(sizeof(float) * E * 2), *rew = malloc(sizeof(float) * E), *info = malloc(sizeof(float) * E * CN_INFO_K);
    uint8_t *done = malloc(E);
    int8_t *ev = malloc(E);
    double *epr = malloc(sizeof(double) * E);
    int32_t *epl = malloc(sizeof(int32_t) * E);
    cnref_reset(g, rn, te, se);
    long episodes = 0;
    for (int t = 0; t < steps; ++t) {
        for (int k = 0; k < 2 * E; ++k)
            act[k] = (float)(c.kinematics == CN_UNICYCLE ? 0.3 * (urand() - 0.5) : 1.6 * (urand() - 0.5));
        cnref_step(g, act, rn, te, se, rew, done, ev, info, epr, epl);
        for (int e = 0; e < E; ++e) {
            if (!isfinite(rew[e])) { fprintf(stderr, "non-finite reward env %d step %d\n", e, t); return 4; }
            for (int k = 0; k < 7; ++k)
                if (!isfinite(rn[e * 7 + k])) { fprintf(stderr, "non-finite obs env %d step %d\n", e, t); return 4; }
            episodes += done[e];
        }
    }
    printf("ok: %d envs x %d steps, %ld episodes\n", E, steps, episodes);
    free(rn); free(te); free(se); free(act); free(rew); free(info); free(done); free(ev); free(epr); free(epl);
    cnref_destroy(g);
    return 0;
}
