/*
 * zbot.h — C ABI of libzbot_hip.so, the MI355X batched Z-Bot rollout engine.
 *
 * The engine replaces, for N environments at once, the ksim hot path that
 * train.py drives:
 *
 *   zb_step  <- ksim RLTask.step_engine (un-vendored ksim 0.1.99, task/rl.py)
 *               = for 20 substeps { FeetechActuators.get_stateful_ctrl
 *                 (train.py:1242-1280) -> mjx.step (MuJoCo-MJX 3.3.4) }
 *               -> terminations (train.py:1588-1593)
 *               -> observations (train.py:1478-1537, run_actor/run_critic
 *                  concatenations train.py:1624-1679)
 *               -> per-step reward terms (train.py:1546-1586)
 *               -> auto-reset of done envs (train.py:1471-1476)
 *   zb_reset <- ksim MjxEngine.reset + mjx.forward (train.py:1471-1476,
 *               FeetechActuators.get_initial_state train.py:1293-1298,
 *               ImuOrientationObservation.initial_carry train.py:843-845)
 *
 * Conventions
 *   - All device pointers are plain device addresses (e.g. torch
 *     tensor.data_ptr()), contiguous, env-major, on the handle's device.
 *   - `stream` is a hipStream_t passed as void* (0 = null stream). Every call
 *     is asynchronous on that stream; no allocation, copy or synchronisation
 *     happens inside zb_step / zb_reset (graph-capturable).
 *   - Return value: 0 on success, negative ZB_E* on failure; the message of
 *     the last failure on this thread is available from zb_last_error().
 *   - Handles are not thread-safe; distinct handles are independent.
 */
#ifndef ZBOT_H
#define ZBOT_H

#include <stddef.h>
#include <stdint.h>

#include "zbot_layout.h"
#include "zbot_model.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ZB_OK          0
#define ZB_EARG       -1   /* bad argument (null, size, layout mismatch) */
#define ZB_EDEVICE    -2   /* HIP runtime error (device, alloc, copy) */
#define ZB_ELAUNCH    -3   /* kernel launch failure */
#define ZB_EMODEL     -4   /* model outside the engine's limits */
#define ZB_ESTATE     -5   /* a launch flagged its results invalid (zb_check) */

typedef struct ZbHandle ZbHandle;

/* Library / layout introspection (host only, no GPU needed). */
int         zb_abi_version(void);
size_t      zb_model_struct_bytes(void);
size_t      zb_config_struct_bytes(void);
int         zb_state_stride(void);
int         zb_rand_stride(void);
const char* zb_last_error(void);

/* Fill `cfg` with the train.py defaults (train.py:1766-1788 + registered
 * components). Host only. */
void zb_default_config(ZbEnvConfig* cfg);

/*
 * The engine is compiled for the Z-Bot task topology and checks the model
 * against it (ZB_EMODEL otherwise): 26 bodies of which only the floating base
 * (body 1, free joint) branches; nu = 20 hinge actuators, nv = 26; the free
 * joint's 6 dofs form the root of the dof tree and every limb is an
 * unbranched chain of consecutive dofs of at most 6 (dof depth <= 12); body
 * depth <= 8; 1 to 16 floor colliders (ZB_MAX_GEOM, model version 9: boxes,
 * capsules, cylinders, spheres, ellipsoids, convex meshes = geom type 7 with
 * <= ZB_MAX_MESHV hull vertices; nskip_geom = 0), the touch sensors' geoms
 * (the soles) first. Exactly two box colliders (the soles) run the two-sole
 * kernels; any other collider set runs a general-collider instantiation with a
 * second bank of 32 contact-row lanes (Jacobian rows in per-env global scratch),
 * which holds, each substep, the first two of the other colliders within reach
 * of the floor. A model with more than two colliders beyond the soles (and no
 * self pair) adds a third bank of floor colliders: the first four within reach.
 * A substep with more within reach than the banks hold sets bit 1 of the state's
 * flag word (ZB_S_NAN; bit 0: non-finite; bit 2: the same, for the current
 * control step only). npair = 1 (the two box soles against each other,
 * geom-geom) holds the pair's contacts in that second bank when the soles are the
 * only colliders, and in a third bank beside the floor colliders' otherwise (the
 * floor colliders beyond the soles then keep the two of the second bank).
 *
 * Create a handle simulating `n_envs` environments whose global ids are
 * [env_offset, env_offset + n_envs) — RNG streams are keyed by global id, so
 * results for a given env do not depend on how envs are sharded over GPUs.
 * Copies the model to `device`, allocates persistent state, does NOT reset
 * (call zb_reset). Replaces ksim's mjx.put_model + engine construction.
 */
int zb_create(const ZbModel* model, const ZbEnvConfig* cfg, int n_envs,
              int env_offset, int device, uint64_t seed, ZbHandle** out);
int zb_destroy(ZbHandle* h);

/*
 * Reset environments (all when env_mask_dev is NULL, else those with
 * env_mask_dev[e] != 0) and write their observations. Output pointers may be
 * NULL to skip an output.
 *   obs_actor  [n_envs, 50]   obs_critic [n_envs, 484]   obs_extra [n_envs, 96]
 */
int zb_reset(ZbHandle* h, const uint8_t* env_mask_dev, float* obs_actor,
             float* obs_critic, float* obs_extra, void* stream);

/*
 * Advance every environment by one control step (n_substeps physics steps).
 *   action       [n_envs, 20]  joint position targets, ctrl order (in)
 *   obs_actor    [n_envs, 50]  observation of the next state (or of the reset
 *                              state for envs that terminated)
 *   obs_critic   [n_envs, 484]
 *   obs_extra    [n_envs, 96]  (nullable)
 *   reward_terms [n_envs, 12]  unscaled term values (nullable)
 *   reward       [n_envs]      sum_i scale_i * (curriculum if by_curr) * term_i
 *   done         [n_envs]      uint8 termination flag (failure or time limit)
 *   success      [n_envs]      uint8 (nullable): the episode ended by the
 *                              EpisodeLengthTermination time limit and not by a
 *                              failure (train.py:1588-1593, ksim's successful
 *                              termination [U]); ksim's compute_ppo_inputs
 *                              bootstraps these steps with V(s_t)
 *                              (include/zbot_ppo.h zb_gae `success`)
 *   curriculum_level           ksim curriculum scalar (one value for all envs)
 * ABI version 2 added `success` (version 1 had no such argument).
 */
int zb_step(ZbHandle* h, const float* action, float* obs_actor,
            float* obs_critic, float* obs_extra, float* reward_terms,
            float* reward, uint8_t* done, uint8_t* success,
            float curriculum_level, void* stream);

/* Run `n_steps` control steps back to back in ONE launch, with actions
 * action[t][n_envs][20]; outputs of the last step only (rollout benchmark /
 * fixed-policy rollouts). reward_sum [n_envs] (nullable) accumulates the
 * total reward of every step; done / success (nullable) are the last step's. */
int zb_rollout(ZbHandle* h, const float* actions, int n_steps,
               float* obs_actor, float* obs_critic, float* reward_sum,
               uint8_t* done, uint8_t* success, float curriculum_level,
               void* stream);

/*
 * ksim's FeetAirtimeReward, exactly, over a rollout of T steps
 * (FeetAirtimeReward.get_reward_stateful, train.py:515-546, evaluated by ksim
 * on the whole (T, ...) trajectory after the rollout).
 *
 * zb_step's FeetAirtime term is the causal per-step form
 * Σ_feet (air[t-1] − penalty)·[c_t ∧ ¬c_{t-1}]. That is ksim's term for every
 * t ≥ 1. At t = 0 ksim takes the previous contact as False
 * (`concatenate([False], c[:-1])`, train.py:527) and the airtime of
 * `roll(air, 1)` (train.py:533-534), i.e. air[T-1], known only after the last
 * step. To get ksim's rows:
 *   zb_mark_rollout_start(h);            before the rollout's first zb_step
 *                                        (or zb_rollout); host-side flag only
 *   ... T x zb_step ...
 *   zb_feet_airtime_exact(h, reward[0], reward_terms[0], level, stream);
 * which adds scale·(ksim term − causal term) to reward0[e] and writes ksim's
 * term into reward_terms0[e][ZB_T_FEET_AIRTIME] (either pointer nullable;
 * reward0 may be zb_rollout's reward_sum, the patch is additive). Rows t ≥ 1
 * are untouched. The handle's episode statistics get the same delta in their
 * reward sum (ZB_ST_REWARD, zb_get_stats); episode returns (ZB_ST_RETURN) keep
 * the causal row-0 term, as an episode can span the rollout boundary. curriculum_level is the level the first step ran at.
 * ZB_EARG if no marked step ran since the mark (or the rollout was already
 * patched). Added in ABI version 3.
 */
int zb_mark_rollout_start(ZbHandle* h);
int zb_feet_airtime_exact(ZbHandle* h, float* reward0, float* reward_terms0,
                          float curriculum_level, void* stream);

/* Persistent state access: [n_envs, ZB_STATE_STRIDE] fp32 words (device).
 * get copies out, set copies in (checkpoint / parity tests). */
int zb_get_state(ZbHandle* h, float* state_dev, void* stream);
int zb_set_state(ZbHandle* h, const float* state_dev, void* stream);
/* Randomized parameters [n_envs, ZB_RAND_STRIDE] (config 5). */
int zb_get_rand(ZbHandle* h, float* rand_dev, void* stream);
int zb_set_rand(ZbHandle* h, const float* rand_dev, void* stream);

/* Episode statistics [n_envs, ZB_NUM_STATS] accumulated by zb_step since the
 * last clear (deterministic per-env partials for the cross-GPU reduction). */
int zb_get_stats(ZbHandle* h, float* stats_dev, int clear, void* stream);

/* Synchronising health check: waits for the device, then reports ZB_ESTATE if a chunked
 * zb_step since the last check timed out waiting for a predecessor chunk (never
 * observed: the wait is bounded only as a guard). The unit that timed out stored no state, so the
 * envs' rows are stale and the launch's outputs invalid; the chunk counters are cleared for the
 * next launch. */
int zb_check(ZbHandle* h);

/* Solver diagnostics: total solver iterations of the last launch summed over
 * its substeps, per env ([n_envs] int32, device). */
int zb_get_solver_iters(ZbHandle* h, int32_t* iters_dev, void* stream);

/* Work units per pair of envs in the handle's zb_step launches: 0 restores the
 * automatic choice made at zb_create, 1 runs whole control steps, k > 1 splits every pair's
 * substeps into k chunks (clamped to the substep count). Results are the same bits for every k.
 * Env groups on their own streams fill the drain themselves and run unchunked. */
int zb_set_step_chunks(ZbHandle* h, int k);

/* Diagnostic: one forward pass (no integration) on the qpos/qvel stored in
 * state_dev [n_envs, ZB_STATE_STRIDE] with ctrl_dev [n_envs, 20] (nullable ->
 * zero ctrl); dumps M, bias, qacc_smooth, qacc, xpos, cinert, cvel and sensor
 * values into dbg_dev [n_envs, 1760] (layout: csrc/zb_internal.h ZB_DBG_*).
 * Used by the parity tests to localise differences to one pipeline stage. */
int zb_debug_forward(ZbHandle* h, float* state_dev, const float* ctrl_dev,
                     float* dbg_dev, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ZBOT_H */
