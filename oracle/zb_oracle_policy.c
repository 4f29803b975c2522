/*
 * zb_oracle_policy.c — CPU restatement of the GRU actor / critic and the
 * mixture-of-Gaussians action head (TEST INFRASTRUCTURE: loaded by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg only; the product
 * library never links it). SURVEY.md §8f row f1.
 *
 * Follows train.py:
 *   Actor.__init__/forward   train.py:885-967  (input_proj -> depth x GRUCell
 *                            -> output_proj; means + JOINT_BIASES, stds =
 *                            clip((softplus + min_std) * var_scale, max_std),
 *                            logits; slices of 100 reshaped [20][5])
 *   Critic.forward           train.py:970-1023 (same stack, one output)
 *   Model / get_model        train.py:1026-1057, 1604-1614 (min_std 0.01,
 *                            max_std 1.0, var_scale 1.0, hidden 128, depth 5,
 *                            5 mixtures)
 *   sample_action            train.py:1737-1763 (sample, or mode on argmax)
 *   get_ppo_variables        train.py:1683-1729 (log_prob of the taken
 *                            action; carry reset to zeros on done)
 * and, un-vendored [U]: equinox GRUCell / Linear (gate order r, z, n; bias on
 * the input gates, bias_n inside the reset product), ksim MixtureOfGaussians
 * (categorical over mixtures, then a Normal; mode = mean of the most likely
 * mixture).
 *
 * Arithmetic contract shared with csrc/zb_policy.hip (bit-identical):
 *   - every dot product is acc = 0; for k ascending: acc = fmaf(x_k, w_k, acc),
 *     then + bias (the matrix cores' k-ordered chain);
 *   - elementwise code is compiled without contraction (-ffp-contract=off);
 *   - exp/log/sigmoid/tanh/softplus/sincos, the RNG and the mixture head
 *     (zbf_mix_sample / zbf_mix_log_prob) come from include/zbot_fmath.h, so
 *     the head is shared code: tests/test_policy.py pins it against a float64
 *     numpy restatement and checks the sampler's distribution.
 *
 * Parity vs the reference: UNPINNED (jax/equinox/distrax/ksim are not
 * importable; no reference fixtures). Pinned by tests/test_policy.py
 * (hand-checked gates, a numpy float64 restatement, distribution moments).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "zbot_fmath.h"
#include "zbot_policy.h"

#define H ZB_POL_HIDDEN
#define D ZB_POL_DEPTH
#define NJ ZB_POL_JOINTS
#define NM ZB_POL_MIX

typedef struct {
  const float *win, *bin, *wih[D], *whh[D], *b[D], *bn[D], *wout, *bout, *mean_bias;
} Net;

static Net net_of(const float* P, int I, int O, int actor) {
  Net n;
  const float* p = P;
  n.win = p; p += (size_t)H * I;
  n.bin = p; p += H;
  for (int l = 0; l < D; l++) {
    n.wih[l] = p; p += (size_t)3 * H * H;
    n.whh[l] = p; p += (size_t)3 * H * H;
    n.b[l] = p; p += 3 * H;
    n.bn[l] = p; p += H;
  }
  n.wout = p; p += (size_t)O * H;
  n.bout = p; p += O;
  n.mean_bias = actor ? p : NULL;
  return n;
}

static float dotk(const float* x, const float* w, int K) {
  float acc = 0.0f;
  for (int k = 0; k < K; k++) acc = fmaf(x[k], w[k], acc);
  return acc;
}

/* one env, one step: carry [D][H] updated in place; out [O] */
static void gru_forward(const Net* nt, int I, int O, const float* obs, float* carry, float* out) {
  float x[H], xn[H];
  for (int u = 0; u < H; u++) x[u] = dotk(obs, nt->win + (size_t)u * I, I) + nt->bin[u];
  for (int l = 0; l < D; l++) {
    float* h = carry + l * H;
    for (int u = 0; u < H; u++) {
      float ig[3], hg[3];
      for (int g = 0; g < 3; g++) {
        ig[g] = dotk(x, nt->wih[l] + (size_t)(g * H + u) * H, H) + nt->b[l][g * H + u];
        hg[g] = dotk(h, nt->whh[l] + (size_t)(g * H + u) * H, H);
      }
      const float r = zbf_sigmoid(ig[0] + hg[0]);
      const float z = zbf_sigmoid(ig[1] + hg[1]);
      const float nn = zbf_tanh(ig[2] + r * (hg[2] + nt->bn[l][u]));
      xn[u] = nn + z * (h[u] - nn);
    }
    memcpy(h, xn, sizeof xn);
    memcpy(x, xn, sizeof xn);
  }
  for (int c = 0; c < O; c++) out[c] = dotk(x, nt->wout + (size_t)c * H, H) + nt->bout[c];
}

/* mixture head of one joint: mean/std/logit of its 5 components */
static void head(const Net* nt, const float* out, int j, float mu[NM], float sd[NM], float lg[NM]) {
  for (int m = 0; m < NM; m++) {
    mu[m] = out[j * NM + m] + nt->mean_bias[j];
    const float s = (zbf_softplus(out[NJ * NM + j * NM + m]) + 0.01f) * 1.0f;
    sd[m] = s < 1.0f ? s : 1.0f;
    lg[m] = out[2 * NJ * NM + j * NM + m];
  }
}

size_t zbo_policy_param_count(int kind) {
  const int I = kind == ZB_POL_ACTOR ? ZB_POL_ACTOR_IN : ZB_POL_CRITIC_IN;
  const int O = kind == ZB_POL_ACTOR ? ZB_POL_ACTOR_OUT : 1;
  return (size_t)H * I + H + (size_t)D * (6 * H * H + 4 * H) + (size_t)O * H + O + (kind == ZB_POL_ACTOR ? NJ : 0);
}

void zbo_policy_actor(const float* P, const float* obs, int T, int n, float* carry, const uint8_t* reset, int mode,
                      uint64_t seed, int env_offset, uint32_t step0, float* actions, float* log_prob) {
  const Net nt = net_of(P, ZB_POL_ACTOR_IN, ZB_POL_ACTOR_OUT, 1);
  float out[ZB_POL_ACTOR_OUT];
  for (int t = 0; t < T; t++)
    for (int e = 0; e < n; e++) {
      float* ce = carry + (size_t)e * D * H;
      if (reset && reset[(size_t)t * n + e]) memset(ce, 0, sizeof(float) * D * H);
      gru_forward(&nt, ZB_POL_ACTOR_IN, ZB_POL_ACTOR_OUT, obs + ((size_t)t * n + e) * ZB_POL_ACTOR_IN, ce, out);
      float* act = actions + ((size_t)t * n + e) * NJ;
      for (int j = 0; j < NJ; j++) {
        float mu[NM], sd[NM], lg[NM];
        head(&nt, out, j, mu, sd, lg);
        if (mode != ZB_POL_EVAL)
          act[j] = zbf_mix_sample(mu, sd, lg, mode == ZB_POL_MODE, seed, ZB_RNG_POLICY, (uint32_t)j,
                                  (uint32_t)(NJ + j), (uint32_t)(env_offset + e), step0 + (uint32_t)t);
        if (log_prob) log_prob[((size_t)t * n + e) * NJ + j] = zbf_mix_log_prob(mu, sd, lg, act[j]);
      }
    }
}

void zbo_policy_critic(const float* P, const float* obs, int T, int n, float* carry, const uint8_t* reset,
                       float* value) {
  const Net nt = net_of(P, ZB_POL_CRITIC_IN, 1, 0);
  for (int t = 0; t < T; t++)
    for (int e = 0; e < n; e++) {
      float* ce = carry + (size_t)e * D * H;
      if (reset && reset[(size_t)t * n + e]) memset(ce, 0, sizeof(float) * D * H);
      gru_forward(&nt, ZB_POL_CRITIC_IN, 1, obs + ((size_t)t * n + e) * ZB_POL_CRITIC_IN, ce,
                  value + (size_t)t * n + e);
    }
}

/* the shared math, exposed for known-answer tests */
float zbo_fm_exp(float x) { return zbf_exp(x); }
float zbo_fm_log(float x) { return zbf_log(x); }
float zbo_fm_tanh(float x) { return zbf_tanh(x); }
float zbo_fm_sigmoid(float x) { return zbf_sigmoid(x); }
float zbo_fm_softplus(float x) { return zbf_softplus(x); }
void zbo_fm_sincos_turns(float t, float* s, float* c) { zbf_sincos_turns(t, s, c); }
void zbo_fm_threefry(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1, uint32_t* o) {
  zbf_threefry2x32(k0, k1, c0, c1, &o[0], &o[1]);
}
float zbo_fm_normal(uint64_t seed, uint32_t purpose, uint32_t k, uint32_t env, uint32_t ctr) {
  return zbf_normal(seed, purpose, k, env, ctr);
}

float zbo_fm_mix_log_prob(const float* mu, const float* sd, const float* lg, float a) {
  return zbf_mix_log_prob(mu, sd, lg, a);
}
/* draws of joint j for global envs 0 .. n-1 at `step` */
void zbo_fm_mix_sample_batch(const float* mu, const float* sd, const float* lg, int argmax, uint64_t seed, int n,
                             uint32_t step, int j, float* out) {
  for (int e = 0; e < n; e++)
    out[e] = zbf_mix_sample(mu, sd, lg, argmax, seed, ZB_RNG_POLICY, (uint32_t)j, (uint32_t)(NJ + j), (uint32_t)e,
                            step);
}
void zbo_fm_normal_batch(uint64_t seed, uint32_t purpose, int n, float* out) {
  for (int e = 0; e < n; e++) out[e] = zbf_normal(seed, purpose, 0u, (uint32_t)e, 0u);
}
