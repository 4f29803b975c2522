/*
 * zbot_fmath.h — fp32 elementary functions and the counter-based RNG shared,
 * source-identical, by the HIP policy kernels (csrc/zb_policy.hip) and the
 * CPU oracle (oracle/zb_oracle_policy.c).
 *
 * Every function is a fixed sequence of IEEE-754 fp32 operations (+ - * /,
 * sqrtf, explicit fmaf, rintf, ldexpf, frexpf), all correctly rounded or exact
 * on both gfx950 (hipcc without fast-math flags) and the host (gcc with
 * -ffp-contract=off), so a result computed on the GPU is bit-identical to the
 * oracle's. Accuracy is a few ulp over the ranges the policy uses (sigmoid /
 * tanh / softplus gates, Box-Muller, log-probabilities); none of these are
 * claimed to equal jax's XLA implementations bit for bit — the reference
 * itself is not runnable here.
 */
#ifndef ZBOT_FMATH_H
#define ZBOT_FMATH_H

#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define ZBF_FN __host__ __device__ static inline
#else
#define ZBF_FN static inline
#endif

/* No implicit multiply-add contraction in anything below (the oracle is built
   with -ffp-contract=off; hipcc would otherwise fuse e.g. mu + sd * z). */
#if defined(__clang__)
#pragma clang fp contract(off)
#endif

#define ZBF_LN2_HI 0.693145751953125f   /* 0x3f317200: ln 2, 15 significant bits */
#define ZBF_LN2_LO 1.42860682e-06f      /* ln 2 - ZBF_LN2_HI */
#define ZBF_LOG2E 1.44269504088896341f
#define ZBF_TWO_PI 6.28318530717958648f
#define ZBF_HALF_LOG_2PI 0.918938533204672742f

/* e^x, x clamped to [-87, 88]: Cody-Waite reduction, degree-6 Horner polynomial */
ZBF_FN float zbf_exp(float x) {
  x = x < -87.0f ? -87.0f : (x > 88.0f ? 88.0f : x);
  const float n = rintf(x * ZBF_LOG2E);
  float r = fmaf(n, -ZBF_LN2_HI, x);
  r = fmaf(n, -ZBF_LN2_LO, r);
  float p = 1.3888949e-3f;
  p = fmaf(p, r, 8.3333715e-3f);
  p = fmaf(p, r, 4.1666664e-2f);
  p = fmaf(p, r, 1.6666667e-1f);
  p = fmaf(p, r, 0.5f);
  p = fmaf(p, r, 1.0f);
  p = fmaf(p, r, 1.0f);
  return ldexpf(p, (int)n);
}

/* natural log for x > 0 (x <= 0 returns -87.3, the log of the smallest value zbf_exp makes).
   Branch-free (selects), so a wavefront's lanes never diverge inside it. */
ZBF_FN float zbf_log(float x) {
  const int bad = !(x > 0.0f);
  int e;
  float m = frexpf(bad ? 1.0f : x, &e); /* x = m 2^e, m in [0.5, 1) */
  const int lo = m < 0.70710678f;
  m = lo ? m * 2.0f : m;
  e = lo ? e - 1 : e;
  /* log m = 2 atanh(s), s = (m - 1) / (m + 1), |s| < 0.1716 */
  const float s = (m - 1.0f) / (m + 1.0f);
  const float s2 = s * s;
  float p = 0.15148e0f;
  p = fmaf(p, s2, 0.18181258e0f);
  p = fmaf(p, s2, 0.22222393e0f);
  p = fmaf(p, s2, 0.28571427e0f);
  p = fmaf(p, s2, 0.40000000e0f);
  p = fmaf(p, s2, 0.66666669e0f);
  const float lm = fmaf(s * s2, p, 2.0f * s);
  const float fe = (float)e;
  const float r = fmaf(fe, ZBF_LN2_HI, fmaf(fe, ZBF_LN2_LO, lm));
  return bad ? -87.3365447f : r;
}

ZBF_FN float zbf_sigmoid(float x) { return 1.0f / (1.0f + zbf_exp(-x)); }

/* tanh(x) = sign(x) (1 - 2 / (e^{2|x|} + 1)); |x| < 2^-12 returns x */
ZBF_FN float zbf_tanh(float x) {
  const float ax = fabsf(x);
  const float t = 1.0f - 2.0f / (zbf_exp(2.0f * ax) + 1.0f);
  return ax < 2.44140625e-4f ? x : (x < 0.0f ? -t : t);
}

/* log(1 + y), y >= 0: log(u) * y / (u - 1) with u = 1 + y corrects the rounding of u */
ZBF_FN float zbf_log1p(float y) {
  const float u = 1.0f + y;
  const float d = u - 1.0f;
  const float r = zbf_log(u) * (y / (d == 0.0f ? 1.0f : d));
  return u == 1.0f ? y : r;
}

/* softplus(x) = max(x, 0) + log1p(e^{-|x|})  (jax.nn.softplus = logaddexp(x, 0)) */
ZBF_FN float zbf_softplus(float x) {
  const float mx = x > 0.0f ? x : 0.0f;
  return mx + zbf_log1p(zbf_exp(-fabsf(x)));
}

/* sin and cos of 2 pi t for t in [0, 1): octant reduction in turns, degree-7/8 polynomials */
ZBF_FN void zbf_sincos_turns(float t, float* s_out, float* c_out) {
  const float q = rintf(t * 4.0f); /* nearest quarter turn, 0..4 */
  const float f = fmaf(q, -0.25f, t); /* exact: |f| <= 1/8 */
  const float x = f * ZBF_TWO_PI;     /* |x| <= pi/4 */
  const float x2 = x * x;
  float sp = -1.9515296e-4f;
  sp = fmaf(sp, x2, 8.3321608e-3f);
  sp = fmaf(sp, x2, -1.6666654e-1f);
  const float sn = fmaf(x * x2, sp, x);
  float cp = 2.4433157e-5f;
  cp = fmaf(cp, x2, -1.3887316e-3f);
  cp = fmaf(cp, x2, 4.1666646e-2f);
  cp = fmaf(cp, x2, -0.5f);
  const float cs = fmaf(x2, cp, 1.0f);
  const int qi = ((int)q) & 3;
  float s, c;
  if (qi == 0) { s = sn; c = cs; }
  else if (qi == 1) { s = cs; c = -sn; }
  else if (qi == 2) { s = -sn; c = -cs; }
  else { s = -cs; c = sn; }
  *s_out = s;
  *c_out = c;
}

/* ---- threefry2x32-20 (Random123), the engine's counter-based RNG ---- */
ZBF_FN uint32_t zbf_rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

ZBF_FN void zbf_threefry2x32(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1, uint32_t* o0, uint32_t* o1) {
  const uint32_t ks2 = 0x1BD11BDAu ^ k0 ^ k1;
  uint32_t x0 = c0 + k0, x1 = c1 + k1;
  const int R[8] = {13, 15, 26, 6, 17, 29, 16, 24};
  const uint32_t ks[3] = {k0, k1, ks2};
  for (int blk = 0; blk < 5; blk++) {
    for (int i = 0; i < 4; i++) {
      x0 += x1;
      x1 = zbf_rotl32(x1, R[(blk & 1) * 4 + i]);
      x1 ^= x0;
    }
    x0 += ks[(blk + 1) % 3];
    x1 += ks[(blk + 2) % 3] + (uint32_t)(blk + 1);
  }
  *o0 = x0;
  *o1 = x1;
}

/* draw k of purpose `purpose` for global env `env` at counter `ctr` (engine convention) */
ZBF_FN void zbf_rng_bits(uint64_t seed, uint32_t purpose, uint32_t k, uint32_t env, uint32_t ctr, uint32_t* a,
                         uint32_t* b) {
  zbf_threefry2x32((uint32_t)seed ^ (purpose * 0x9E3779B9u), (uint32_t)(seed >> 32) ^ (k * 0x85EBCA6Bu), env, ctr,
                   a, b);
}

ZBF_FN float zbf_u01(uint32_t b) { return (float)(b >> 8) * (1.0f / 16777216.0f); }

/* one standard normal (Box-Muller, first output) from draw k */
ZBF_FN float zbf_normal(uint64_t seed, uint32_t purpose, uint32_t k, uint32_t env, uint32_t ctr) {
  uint32_t a, b;
  zbf_rng_bits(seed, purpose, k, env, ctr, &a, &b);
  const float u1 = 1.0f - zbf_u01(a); /* (0, 1] */
  const float u2 = zbf_u01(b);
  const float r = sqrtf(-2.0f * zbf_log(u1));
  float s, c;
  zbf_sincos_turns(u2, &s, &c);
  return r * c;
}

/* ---- mixture-of-Gaussians action head of one joint (ksim MixtureOfGaussians [U]) ---- */
#define ZBF_NMIX 5

/* log sum_m softmax(lg)_m N(a; mu_m, sd_m) */
ZBF_FN float zbf_mix_log_prob(const float* mu, const float* sd, const float* lg, float a) {
  float mx = lg[0];
  for (int m = 1; m < ZBF_NMIX; m++) mx = lg[m] > mx ? lg[m] : mx;
  float S = 0.0f;
  for (int m = 0; m < ZBF_NMIX; m++) S = S + zbf_exp(lg[m] - mx);
  const float logS = zbf_log(S);
  float v[ZBF_NMIX];
  float M = -3.0e38f;
  for (int m = 0; m < ZBF_NMIX; m++) {
    const float zm = (a - mu[m]) / sd[m];
    const float lnm = ((-0.5f * zm) * zm - zbf_log(sd[m])) - ZBF_HALF_LOG_2PI;
    v[m] = ((lg[m] - mx) - logS) + lnm;
    M = v[m] > M ? v[m] : M;
  }
  float acc = 0.0f;
  for (int m = 0; m < ZBF_NMIX; m++) acc = acc + zbf_exp(v[m] - M);
  return M + zbf_log(acc);
}

/* mode (argmax = 1): mean of the most likely mixture (first on ties).
   sample: mixture m by inverse CDF of softmax(lg) on the uniform of draw k_cat,
   then mu_m + sd_m * z with z the standard normal of draw k_normal. */
ZBF_FN float zbf_mix_sample(const float* mu, const float* sd, const float* lg, int argmax, uint64_t seed,
                            uint32_t purpose, uint32_t k_cat, uint32_t k_normal, uint32_t env, uint32_t step) {
  float mx = lg[0];
  int am = 0;
  for (int m = 1; m < ZBF_NMIX; m++)
    if (lg[m] > mx) {
      mx = lg[m];
      am = m;
    }
  if (argmax) return mu[am];
  float e[ZBF_NMIX];
  float S = 0.0f;
  for (int m = 0; m < ZBF_NMIX; m++) {
    e[m] = zbf_exp(lg[m] - mx);
    S = S + e[m];
  }
  uint32_t a, b;
  zbf_rng_bits(seed, purpose, k_cat, env, step, &a, &b);
  const float target = zbf_u01(a) * S;
  int pick = ZBF_NMIX - 1;
  int found = 0;
  float c = 0.0f;
  for (int m = 0; m < ZBF_NMIX; m++) { /* first m with target < c_m, as selects */
    c = c + e[m];
    const int hit = !found && target < c;
    pick = hit ? m : pick;
    found = found || hit;
  }
  const float z = zbf_normal(seed, purpose, k_normal, env, step);
  return mu[pick] + sd[pick] * z;
}

#endif /* ZBOT_FMATH_H */
