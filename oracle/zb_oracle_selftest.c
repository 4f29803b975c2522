/*
 * zb_oracle_selftest.c — host-sanitizer driver of the CPU twin (TEST INFRASTRUCTURE ONLY; SURVEY.md
 * §5: the host twin under -fsanitize=address,undefined). Built by oracle/asan.mk together with
 * zb_oracle.c, run by tests/test_sanitizers.py.
 *
 *   zb_oracle_selftest <model.bin> <config.bin> <n_envs> <steps>
 *
 * Resets n_envs environments and steps them with the twin's synthetic actions (sigma 0.3, so
 * contacts, limits and automatic resets all occur), through every output (observations, reward
 * terms, statistics, solver iterations); then one debug forward and one constraint problem. Prints
 * a checksum line; any memory error or undefined behaviour aborts under the sanitizers.
 */
#include <stdio.h>
#include <stdlib.h>

#include "zbot_layout.h"
#include "zbot_model.h"

int zbo_reset(const ZbModel* m, const ZbEnvConfig* cfg, int n, int env_offset, uint64_t seed, float* state,
              float* rnd, const uint8_t* mask, float* obs_actor, float* obs_critic, float* obs_extra);
int zbo_step(const ZbModel* m, const ZbEnvConfig* cfg, int n, int env_offset, uint64_t seed, float* state,
             float* rnd, const float* action, float* obs_actor, float* obs_critic, float* obs_extra,
             float* reward_terms, float* reward, uint8_t* done, uint8_t* success, float curriculum, float* stats,
             int32_t* iters);
void zbo_synthetic_actions(const ZbModel* m, uint64_t seed, int n, int env_offset, uint32_t t, float std_,
                           float* out);

static int read_file(const char* path, void* dst, size_t bytes) {
  FILE* f = fopen(path, "rb");
  if (!f) return 0;
  size_t got = fread(dst, 1, bytes, f);
  int extra = fgetc(f);
  fclose(f);
  return got == bytes && extra == EOF;
}

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s model.bin config.bin n_envs steps\n", argv[0]);
    return 2;
  }
  ZbModel* m = (ZbModel*)malloc(sizeof(ZbModel));
  ZbEnvConfig cfg;
  if (!m || !read_file(argv[1], m, sizeof *m) || !read_file(argv[2], &cfg, sizeof cfg)) {
    fprintf(stderr, "cannot read the model / config blobs\n");
    return 2;
  }
  const int n = atoi(argv[3]), steps = atoi(argv[4]);
  float* state = (float*)calloc((size_t)n * ZB_STATE_STRIDE, sizeof(float));
  float* rnd = (float*)calloc((size_t)n * ZB_RAND_STRIDE, sizeof(float));
  float* act = (float*)malloc((size_t)n * ZB_NJ * sizeof(float));
  float* oa = (float*)malloc((size_t)n * ZB_OBS_ACTOR * sizeof(float));
  float* oc = (float*)malloc((size_t)n * ZB_OBS_CRITIC * sizeof(float));
  float* ox = (float*)malloc((size_t)n * ZB_OBS_EXTRA * sizeof(float));
  float* terms = (float*)malloc((size_t)n * ZB_NUM_TERMS * sizeof(float));
  float* rew = (float*)malloc((size_t)n * sizeof(float));
  float* stats = (float*)calloc((size_t)n * ZB_NUM_STATS, sizeof(float));
  uint8_t* done = (uint8_t*)malloc((size_t)n);
  uint8_t* succ = (uint8_t*)malloc((size_t)n);
  int32_t* iters = (int32_t*)malloc((size_t)n * sizeof(int32_t));
  uint8_t* mask = (uint8_t*)malloc((size_t)n);
  if (!state || !rnd || !act || !oa || !oc || !ox || !terms || !rew || !stats || !done || !succ || !iters || !mask)
    return 2;
  if (zbo_reset(m, &cfg, n, 0, 5, state, rnd, NULL, oa, oc, ox)) return 1;
  double sum = 0.0;
  long ends = 0;
  for (int t = 0; t < steps; t++) {
    zbo_synthetic_actions(m, 5, n, 0, (uint32_t)t, 0.3f, act);
    if (zbo_step(m, &cfg, n, 0, 5, state, rnd, act, oa, oc, ox, terms, rew, done, succ, 1.0f, stats, iters)) return 1;
    for (int e = 0; e < n; e++) {
      sum += rew[e];
      ends += done[e];
    }
    if (t == steps / 2) { /* a masked reset of every other env */
      for (int e = 0; e < n; e++) mask[e] = (uint8_t)(e & 1);
      if (zbo_reset(m, &cfg, n, 0, 5, state, rnd, mask, oa, oc, ox)) return 1;
    }
  }
  printf("zb_oracle_selftest ok: %d envs x %d steps, reward sum %.6f, episode ends %ld\n", n, steps, sum, ends);
  free(state); free(rnd); free(act); free(oa); free(oc); free(ox); free(terms); free(rew); free(stats);
  free(done); free(succ); free(iters); free(mask); free(m);
  return 0;
}
