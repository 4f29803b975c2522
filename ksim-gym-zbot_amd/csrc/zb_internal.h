/*
 * zb_internal.h — declarations shared by the HIP engine (zb_engine.hip) and
 * the C-ABI host code (zb_capi.cpp). Not part of the public ABI.
 */
#ifndef ZB_INTERNAL_H
#define ZB_INTERNAL_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "zbot.h"
#include "zbot_policy.h"
#include "zbot_ppo.h"
#include "zb_host.h"

/* debug forward dump layout (zb_debug_forward), fp32 words per env */
#define ZB_DBG_QM      0     /* [nv*nv] dense symmetric mass matrix */
#define ZB_DBG_BIAS    1024  /* [nv] qfrc_bias */
#define ZB_DBG_QACCS   1056  /* [nv] qacc_smooth */
#define ZB_DBG_QACC    1088  /* [nv] constrained qacc */
#define ZB_DBG_XPOS    1120  /* [nbody*3] */
#define ZB_DBG_CINERT  1216  /* [nbody*10] */
#define ZB_DBG_CVEL    1536  /* [nbody*6] */
#define ZB_DBG_MISC    1728  /* nefc, ncon, touch_l, touch_r, imu quat(4), gyro(3), acc(3) */
#define ZB_DBG_STRIDE  1760
#define ZB_XJ_STRIDE   (32 * ZB_MAX_DEPTH) /* floats per env of StepArgs::xj */
#define ZB_NSTAMP      20    /* phase-stamp slots of the -DZB_STAMPS build (zb_engine.hip S_*) */

namespace zb {

struct StepArgs {
  const ZbModel* model;     /* device copy */
  const int32_t* topo;      /* [TP_NF][32] per-lane topology (device) */
  const ZbEnvConfig* cfg;   /* device copy */
  int n_envs;
  int env_offset;
  uint64_t seed;
  float* state;             /* [n, ZB_STATE_STRIDE] */
  float* rnd;               /* [n, ZB_RAND_STRIDE] */
  const float* action;      /* [nsteps, n, 20] */
  int nsteps;
  float* obs_actor;
  float* obs_critic;
  float* obs_extra;
  float* reward_terms;
  float* reward;            /* per step reward (nsteps==1) or reward sum (rollout) */
  uint8_t* done;
  uint8_t* success;         /* [n] or null: time-limit end without failure */
  float curriculum;
  float* stats;             /* [n, ZB_NUM_STATS] */
  int32_t* iters;           /* [n] */
  const uint8_t* reset_mask;
  float* dbg;               /* [n, ZB_DBG_STRIDE] */
  /* chunked step (nsteps == 1, step_kernel): the n_substeps of a control step split into
     nchunk work units per pair of envs, taken in chunk-major order from a counter */
  int nchunk;               /* 1: one workgroup per pair runs all substeps */
  uint32_t* sched;          /* [2 + npair]: units taken, pairs finished, per-pair chunks done */
  int32_t* itpart;          /* [n] Newton iterations of the chunks so far */
  int air_mark;             /* first step of a rollout: save its contacts + causal airtime term */
  int solver;               /* ZB_SOLVER_NEWTON / ZB_SOLVER_CG: which kernel instantiation runs */
  int xg;                   /* general colliders (zb_host.h needs_xg): 0 two-sole, 1 two banks, 2 two banks + cylinders / ellipsoids / meshes, 3 / 4 the sole pair, 5 three banks of floor colliders */
  float* xj;                /* xg: [n + 1, ZB_XJ_STRIDE] second-bank Jacobian rows (the last block: ghost teams) */
  int ed;                   /* ZB_F_EULERDAMP: the step kernel integrates the joint damping implicitly */
};

/* workgroups of step_kernel resident on the device at once (occupancy x CUs) */
int step_resident_blocks(int device, int xg, int solver, int ed);

hipError_t launch_step(const StepArgs& a, hipStream_t s);
hipError_t launch_reset(const StepArgs& a, hipStream_t s);
hipError_t launch_debug_forward(const StepArgs& a, hipStream_t s);
/* exact ksim FeetAirtime row 0 of a marked rollout (a.state, a.cfg, a.n_envs, a.curriculum,
   a.reward = reward row 0 or null, a.reward_terms = terms row 0 or null) */
hipError_t launch_airtime_exact(const StepArgs& a, hipStream_t s);

/* post-rollout PPO inputs (zb_ppo.hip, include/zbot_ppo.h) */
struct GaeArgs {
  const float* reward;      /* [T, n] */
  const float* values;      /* [T, n] */
  const uint8_t* done;      /* [T, n] */
  const uint8_t* success;   /* [T, n] or null */
  const float* bootstrap;   /* [n] or null */
  int T;
  int n;
  float gamma;
  float gl;                 /* gamma * lam, rounded once as the reference does */
  float* gae;               /* [T, n] */
  float* vtarget;           /* [T, n] or null */
  double* partials;         /* [ceil(n / ZB_GAE_ENVS_PER_BLOCK)][2] or null */
};

hipError_t launch_gae(const GaeArgs& a, double* moments_out, hipStream_t s);
hipError_t launch_moments(const double* in, int k, double* out, hipStream_t s);
/* GRU actor / critic, one step (zb_policy.hip, include/zbot_policy.h) */
struct PolicyArgs {
  const float* obs;       /* [n][I] of this step */
  float* carry;           /* [n][depth][hidden], read and written */
  const uint8_t* reset;   /* [n] or null: carry zeroed first */
  int n;
  int mode;               /* ZB_POL_SAMPLE / MODE / EVAL (actor) */
  uint64_t seed;
  int env_offset;
  uint32_t step;
  float* actions;         /* [n][20] (actor) */
  float* log_prob;        /* [n][20] or null (actor) */
  float* value;           /* [n] (critic) */
  const float* wpack;     /* fragment-packed weights */
  const float* bias;      /* biases and head constants */
  int layout;             /* ZB_POL_LAYOUT_BLOCK / ZB_POL_LAYOUT_WAVE */
  int T;                  /* block layout: steps run by one persistent launch (obs / reset / outputs
                             advance by one [n] step each; carry in registers between steps) */
};
hipError_t launch_policy(int kind, const PolicyArgs& a, hipStream_t s);

hipError_t launch_normalize(const float* gae, float* adv, long long count, const double* mom, double total,
                            float eps, hipStream_t s);

}  // namespace zb

#endif
