/*
 * zbot_ppo.h — C ABI of the post-rollout PPO inputs,
 * exported by libzbot_hip.so next to the engine (include/zbot.h).
 *
 * Replaces ksim 0.1.99's PPO input computation (un-vendored ksim/task/ppo.py
 * `compute_ppo_inputs` [U]; its caller is PPOTask after the rollout scan whose
 * per-step critic values come from get_ppo_variables, train.py:1683-1729):
 *
 *   values_shifted[t] = values[t+1]            (t < T-1)
 *                     = bootstrap[e] or values[T-1]   (t = T-1; ksim uses the
 *                                               last value as bootstrap [U])
 *   mask[t]  = 1 - done[t]
 *   next[t]  = success[t] ? values[t] : values_shifted[t] * mask[t]   [U]
 *   delta[t] = reward[t] + gamma * next[t] - values[t]
 *   gae[t]   = fma((gamma * lam) * mask[t], gae[t+1], delta[t])  (reverse
 *              scan, gae[T] = 0; one rounding per step)
 *   value_targets[t] = gae[t] + values[t]
 *   advantages = (gae - mean(gae)) / (std(gae) + eps)   (normalize_advantages,
 *                population std over the whole batch — every env, every step,
 *                every rank)
 *
 * Layout: every [T, n] array is time-major with the env axis contiguous, i.e.
 * exactly the buffers zb_step writes when the caller hands it row t of a
 * [T, n] reward / done rollout buffer. Values are the critic outputs for the
 * same rows. All pointers are device pointers; calls are asynchronous on
 * `stream` and allocate nothing (graph-capturable).
 *
 * Determinism: the batch moments are sums in fp64 over a fixed pairwise tree
 * whose leaves are envs (per-env time sums first, in an order fixed by T:
 * oracle/zb_oracle_ppo.c zbo_gae).
 * When every rank holds the same power-of-two number of envs (a multiple of
 * ZB_GAE_ENVS_PER_BLOCK), combining the per-rank moments with
 * zb_moments_combine in rank order reproduces the single-GPU tree bit for
 * bit, so normalized advantages do not depend on the world size.
 */
#ifndef ZBOT_PPO_H
#define ZBOT_PPO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZB_GAE_ENVS_PER_BLOCK 32  /* envs per workgroup of zb_gae (leaf group of the moment tree) */

/* Number of fp64 words of the `partials` scratch zb_gae needs for n envs. */
size_t zb_gae_partials_words(int n);

/*
 * GAE + value targets over a [T, n] rollout.
 *   reward, values  [T, n] fp32      done [T, n] uint8
 *   success         [T, n] uint8 (nullable: no successful terminations)
 *   bootstrap       [n] fp32 (nullable: values[T-1], ksim's convention [U])
 *   gae_out         [T, n] fp32  unnormalized GAE (may alias nothing else)
 *   value_targets   [T, n] fp32  (nullable)
 *   partials        [zb_gae_partials_words(n)] fp64 scratch (nullable: no
 *                   moments); filled with per-block (sum, sum of squares)
 *   moments_out     [2] fp64 (nullable): (sum, sum of squares) of gae over
 *                   this call's T*n elements, reduced over `partials` by the
 *                   fixed pairwise tree. Requires partials.
 */
int zb_gae(const float* reward, const float* values, const uint8_t* done, const uint8_t* success,
           const float* bootstrap, int T, int n, float gamma, float lam, float* gae_out,
           float* value_targets, double* partials, double* moments_out, void* stream);

/*
 * Pairwise-tree combine of `k` (sum, sum of squares) pairs stored as
 * moments[2*k] (device, fp64) into out[2] (device). Used for the per-rank
 * moments after an all-gather (rank order), so every rank normalizes with
 * the same bits.
 */
int zb_moments_combine(const double* moments, int k, double* out, void* stream);

/*
 * advantages[i] = (gae[i] - mean) / (std + eps) for i < count, where
 * mean = moments[0] / total, std = sqrt(max(moments[1] / total - mean^2, 0))
 * and `total` is the number of elements the moments cover (T * n_global).
 * In place when advantages == gae.
 */
int zb_adv_normalize(const float* gae, float* advantages, long long count, const double* moments,
                     double total, float eps, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ZBOT_PPO_H */
