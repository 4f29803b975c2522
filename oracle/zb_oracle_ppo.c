/*
 * zb_oracle_ppo.c — CPU restatement of the post-rollout PPO inputs
 * (TEST INFRASTRUCTURE: loaded by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg only; the product library never links it).
 *
 * Restates ksim 0.1.99 `compute_ppo_inputs` (un-vendored ksim/task/ppo.py
 * [U]) as called by PPOTask on the rollout's
 * rewards/dones and the critic values of get_ppo_variables
 * (train.py:1683-1729): a plain reverse scan per env, t = T-1 .. 0, in fp32
 * with no implicit contraction (-ffp-contract=off, oracle/Makefile) and one
 * explicit fmaf for the recurrence:
 *
 *   values_shifted[t] = values[t+1], last row: bootstrap (or values[T-1])
 *   mask[t]  = 1 - done[t]
 *   next[t]  = success[t] ? values[t] : values_shifted[t] * mask[t]
 *   delta[t] = (reward[t] + gamma * next[t]) - values[t]
 *   gae[t]   = fma((gamma * lam) * mask[t], gae[t+1], delta[t]),  gae[T] = 0
 *   target[t] = gae[t] + values[t]
 *
 * Batch moments (sum, sum of squares of gae, fp64): per env in the fixed
 * segment / row-group order of zbo_gae below, then a pairwise tree over envs
 * zero-padded to a power of two; the normalization (gae - mean) / (std + eps) uses the population std — both
 * as include/zbot_ppo.h specifies for the GPU path.
 *
 * Parity status vs the reference: UNPINNED (ksim is not importable here and
 * the reference holds no fixtures); pinned by hand-derived known answers in
 * tests/test_ppo.py.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* segment geometry of the moment order (zb_ppo.hip GSEG / GR / GJ) */
#define SEG 256
#define GR 64
#define GJ 4
#define NW 8 /* waves per workgroup: 8 row groups each */

static void tree_n(double* a, int m) { /* pairwise, m a power of two */
  for (int s = 1; s < m; s <<= 1)
    for (int i = 0; i + s < m; i += 2 * s) a[i] = a[i] + a[i + s];
}

void zbo_gae(const float* reward, const float* values, const uint8_t* done, const uint8_t* success,
             const float* bootstrap, int T, int n, float gamma, float lam, float* gae, float* vtarget,
             double* env_moments /* [n][2] or NULL */) {
  const float gl = gamma * lam;
  for (int e = 0; e < n; e++) {
    float g = 0.f;
    for (int t = T - 1; t >= 0; t--) {
      const size_t i = (size_t)t * n + e;
      const float v = values[i];
      const float vs = (t + 1 < T) ? values[i + n] : (bootstrap ? bootstrap[e] : v);
      const float mask = done[i] ? 0.f : 1.f;
      const float nxt = (success && success[i]) ? v : vs * mask;
      const float delta = (reward[i] + gamma * nxt) - v;
      const float c = gl * mask;
      g = fmaf(c, g, delta); /* one rounding, as the GPU's v_fma_f32 */
      gae[i] = g;
      if (vtarget) vtarget[i] = g + v;
    }
    if (!env_moments) continue;
    /* moments (zb_ppo.hip gae_kernel step 4/5): per 256-step segment, latest
       first, each row group r0 sums rows r0 + 64 j for j = 3..0; the 8 groups
       of wave w (r0 = 8w .. 8w+7) are combined by a pairwise tree and summed
       per wave over segments; the 8 wave sums by a pairwise tree at the end */
    double W1[NW], W2[NW];
    for (int w = 0; w < NW; w++) W1[w] = W2[w] = 0.0;
    const int nseg = (T + SEG - 1) / SEG;
    for (int sg = nseg - 1; sg >= 0; sg--) {
      const int tbase = sg * SEG;
      const int tl = T - tbase < SEG ? T - tbase : SEG;
      for (int w = 0; w < NW; w++) {
        double p1[8], p2[8];
        for (int i = 0; i < 8; i++) {
          const int r0 = 8 * w + i;
          p1[i] = 0.0;
          p2[i] = 0.0;
          for (int j = GJ - 1; j >= 0; j--) {
            const int row = r0 + GR * j;
            if (row >= tl) continue;
            const double gd = (double)gae[(size_t)(tbase + row) * n + e];
            p1[i] = p1[i] + gd;
            p2[i] = p2[i] + gd * gd;
          }
        }
        tree_n(p1, 8);
        tree_n(p2, 8);
        W1[w] = W1[w] + p1[0];
        W2[w] = W2[w] + p2[0];
      }
    }
    tree_n(W1, NW);
    tree_n(W2, NW);
    const double S1 = W1[0], S2 = W2[0];
    env_moments[2 * e] = S1;
    env_moments[2 * e + 1] = S2;
  }
}

/* pairwise tree over k (s1, s2) pairs, zero-padded to a power of two */
void zbo_moments_tree(const double* pairs, int k, double* out) {
  int p = 1;
  while (p < k) p <<= 1;
  double* a = (double*)calloc((size_t)2 * p, sizeof(double));
  if (k > 0) memcpy(a, pairs, (size_t)2 * k * sizeof(double));
  for (int s = 1; s < p; s <<= 1)
    for (int i = 0; i + s < p; i += 2 * s) {
      a[2 * i] = a[2 * i] + a[2 * (i + s)];
      a[2 * i + 1] = a[2 * i + 1] + a[2 * (i + s) + 1];
    }
  out[0] = a[0];
  out[1] = a[1];
  free(a);
}

void zbo_adv_normalize(const float* gae, float* adv, long long count, const double* mom, double total, float eps) {
  const double mean = mom[0] / total;
  double var = mom[1] / total - mean * mean;
  if (var < 0.0) var = 0.0;
  const float mean_f = (float)mean;
  const float denom = (float)sqrt(var) + eps;
  for (long long i = 0; i < count; i++) adv[i] = (gae[i] - mean_f) / denom;
}
