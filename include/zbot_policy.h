/*
 * zbot_policy.h — C ABI of the GRU policy/value networks in the rollout loop
 * (SURVEY.md §8f row f1), exported by libzbot_hip.so next to the engine.
 *
 * Replaces, for N environments at once (train.py, ZbotWalkingTask):
 *   Actor.forward + MixtureOfGaussians sample / mode / log_prob
 *       train.py:885-967 (Actor), :1616-1643 (run_actor), :1737-1763
 *       (sample_action), :1683-1729 (get_ppo_variables' log_probs)
 *   Critic.forward   train.py:970-1023 (Critic), :1645-1681 (run_critic)
 * with hidden_size 128, depth 5, num_mixtures 5, min_std 0.01, max_std 1.0,
 * var_scale 1.0 (train.py:1068-1079, 1604-1614, 1040-1057).
 *
 * Per layer (equinox GRUCell, un-vendored equinox [U]):
 *   ig = W_ih x + b        hg = W_hh h
 *   r = sigmoid(ig_r + hg_r)   z = sigmoid(ig_z + hg_z)
 *   n = tanh(ig_n + r * (hg_n + b_n))      h' = n + z * (h - n)
 * Every matrix-vector product is the k-ordered fp32 fmaf chain the matrix
 * cores compute (v_mfma_f32_32x32x2_f32), so the GPU is bit-identical to the
 * CPU oracle (oracle/zb_oracle_policy.c), transcendental functions included
 * (include/zbot_fmath.h).
 *
 * Parameters are passed in equinox's natural layout, fp32, concatenated:
 *   input_proj.weight [H][I], input_proj.bias [H],
 *   per layer l < D: weight_ih [3H][H], weight_hh [3H][H], bias [3H], bias_n [H],
 *   output_proj.weight [O][H], output_proj.bias [O]
 * (zb_policy_param_count gives the total). Gate order r, z, n.
 *
 * Layouts (device, row-major): obs [T][n][I]; carry [n][D][H] (read and
 * written in place); reset [T][n] uint8 (nullable: carry zeroed before step
 * t for envs with reset[t][e] != 0 — pass the engine's done flags, which mark
 * envs whose observation is already the next episode's first);
 * actions [T][n][20]; log_prob [T][n][20] (per joint); value [T][n].
 */
#ifndef ZBOT_POLICY_H
#define ZBOT_POLICY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZB_POL_HIDDEN 128
#define ZB_POL_DEPTH 5
#define ZB_POL_MIX 5
#define ZB_POL_JOINTS 20
#define ZB_POL_ACTOR_IN 50     /* NUM_ACTOR_INPUTS train.py:51 */
#define ZB_POL_CRITIC_IN 484   /* NUM_CRITIC_INPUTS train.py:52 */
#define ZB_POL_ACTOR_OUT 300   /* NUM_JOINTS * 3 * num_mixtures train.py:934-938 */
#define ZB_POL_ENVS_PER_BLOCK 32   /* envs per workgroup (two 16-row matrix-core tiles) */

#define ZB_POL_ACTOR 0
#define ZB_POL_CRITIC 1

/* actor modes */
#define ZB_POL_SAMPLE 0        /* action_dist.sample(seed) -> actions (out) */
#define ZB_POL_MODE 1          /* action_dist.mode() (argmax=True) -> actions (out) */
#define ZB_POL_EVAL 2          /* log_prob of the given actions (in) */

#define ZB_RNG_POLICY 5u       /* RNG purpose of the action sample (engine uses 1-4) */

typedef struct ZbPolicy ZbPolicy;

/* Number of fp32 parameters of an actor (kind 0) or critic (kind 1). */
size_t zb_policy_param_count(int kind);

/* Upload `params` (host, natural layout above) to `device`, packed into
 * matrix-core fragment order. */
int zb_policy_create(int kind, const float* params, size_t n_params, int device, ZbPolicy** out);
int zb_policy_destroy(ZbPolicy* p);

/* Kernel layout of the handle's launches (bit-identical results either way):
 *   ZB_POL_LAYOUT_BLOCK  32 envs x 8 waves a workgroup, 89 KB (actor) / 116 KB (critic) of LDS:
 *                        the fastest alone on the GPU;
 *   ZB_POL_LAYOUT_WAVE   16 envs on one wave, <= 20 KB of LDS: a workgroup fits the slot of one
 *                        zb_step wave, so its launches fill the slots a concurrent step launch
 *                        frees (env groups on their own streams).
 * The default is ZB_POL_LAYOUT_BLOCK, or the environment's ZB_POLICY_LAYOUT=wave|block at
 * zb_policy_create. */
#define ZB_POL_LAYOUT_BLOCK 0
#define ZB_POL_LAYOUT_WAVE 1
#define ZB_POL_LAYOUT_WAVE2 2 /* the one-wave layout's unit tiles split over two waves (2 slots, 19 KB) */
#define ZB_POL_LAYOUT_WAVE4 3 /* ... over four waves (4 slots, 19 KB) */
int zb_policy_set_layout(ZbPolicy* p, int layout);

/* Persistent launches (round 5; default on): with the block layout a call over T steps is ONE launch
 * that runs the recurrence over the T steps with each layer's carry in registers (HBM sees the carry
 * once on entry and once after step T-1) instead of T launches. Bit-identical either way; 0 = one
 * launch per step. The slot-sized layouts always launch per step. No reference counterpart: ksim
 * scans the critic over the trajectory (get_ppo_variables, train.py:1683-1729). */
int zb_policy_set_persistent(ZbPolicy* p, int on);

/*
 * Actor over T consecutive steps of n envs (T = 1 in the rollout loop).
 *   mode ZB_POL_SAMPLE / ZB_POL_MODE: actions written; ZB_POL_EVAL: read.
 *   log_prob (nullable) receives log N-mixture(action) per joint.
 * Sampling draws are keyed by (seed, global env id = env_offset + e, step =
 * step0 + t): a pure function of its inputs, independent of n and sharding.
 */
int zb_policy_actor(ZbPolicy* p, const float* obs, int T, int n, float* carry, const uint8_t* reset, int mode,
                    uint64_t seed, int env_offset, uint32_t step0, float* actions, float* log_prob, void* stream);

/* Critic over T consecutive steps: value [T][n]. */
int zb_policy_critic(ZbPolicy* p, const float* obs, int T, int n, float* carry, const uint8_t* reset, float* value,
                     void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ZBOT_POLICY_H */
