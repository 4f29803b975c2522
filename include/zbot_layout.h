/*
 * zbot_layout.h — environment configuration and the per-env memory layouts the
 * engine reads and writes in HBM (state, randomized parameters, outputs).
 *
 * Everything here is env-major: env e owns the contiguous row
 * [e * STRIDE, (e + 1) * STRIDE), so the team of lanes that simulates env e
 * loads/stores its row with consecutive addresses.
 *
 * Reference anchors:
 *   ZbEnvConfig fields      train.py:1766-1788 (dt, ctrl_dt, iterations, ls_iterations)
 *                           train.py:1439-1476 (randomizers, push event, resets)
 *                           train.py:1546-1593 (reward scales, terminations)
 *   state words             ksim PhysicsState (qpos/qvel/qacc_warmstart) +
 *                           PlannerState (train.py:1103-1108) + observation /
 *                           reward carries (train.py:843-845, 499-501)
 *   outputs                 ACTOR_DIM / CRITIC_DIM (train.py:30-54) and the
 *                           concatenations in run_actor/run_critic (train.py:1629-1679)
 */
#ifndef ZBOT_LAYOUT_H
#define ZBOT_LAYOUT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZB_NJ            20   /* NUM_JOINTS, train.py:27 */
#define ZB_NBODY_TASK    26   /* world + 25 observed bodies (CRITIC_DIM com_inertia=250) */
#define ZB_OBS_ACTOR     50   /* NUM_ACTOR_INPUTS, train.py:53 */
#define ZB_OBS_CRITIC    484  /* NUM_CRITIC_INPUTS, train.py:54 */
#define ZB_OBS_EXTRA     96   /* the remaining train.py:1478-1537 observations */
#define ZB_NUM_TERMS     12   /* reward terms registered in train.py:1546-1586 */
#define ZB_NUM_CMD       7    /* ConstantZeroCommand, train.py:423-427 */
#define ZB_NUM_STATS     4    /* per-env episode statistics (see ZB_ST_*) */

/* ---------------- per-env state, fp32 words (u32 slots bit-cast) ------------- */
#define ZB_STATE_STRIDE  192
#define ZB_S_QPOS        0    /* [nq]  (27) */
#define ZB_S_QVEL        32   /* [nv]  (26) */
#define ZB_S_QACCW       64   /* [nv]  qacc_warmstart */
#define ZB_S_PLAN_POS    96   /* [20]  PlannerState.position */
#define ZB_S_PLAN_VEL    116  /* [20]  PlannerState.velocity */
#define ZB_S_PLAN_TAU    136  /* [20]  PlannerState.last_computed_torque */
#define ZB_S_IMU_EMA     156  /* [4]   ImuOrientationObservation carry x */
#define ZB_S_IMU_LAG     160  /*       carry lag ~ U(lag_range) */
#define ZB_S_AIRTIME     161  /* [2]   FeetAirtimeReward carry (left, right) */
#define ZB_S_PUSH_TIMER  163  /*       seconds to the next push */
#define ZB_S_TOUCH       164  /* [2]   foot touch of the current observation */
#define ZB_S_FEET_DIST   166  /*       |feet_position_observation L-R| of current obs */
#define ZB_S_EP_RETURN   167  /*       running episode return */
#define ZB_S_EP_STEPS    168  /* u32   env-steps in the current episode */
#define ZB_S_RNG_STEP    169  /* u32   global per-env step counter (RNG counter) */
#define ZB_S_PREV_CONT   170  /* [2]   contact flags of the previous step (touchdown) */
#define ZB_S_EPISODE     172  /* u32   episode index of this env (RNG counter) */
#define ZB_S_NAN         173  /* u32   flags (diagnostic): bit 0 non-finite state (sticky); bit 1 more colliders beyond the soles within reach of the floor in a substep than its banks hold (four; two beside the sole pair), their contacts not simulated (zb_engine.hip select_bank2; sticky); bit 2 the same in the last control step (cleared at the start of each) */
#define ZB_S_AIR0_CONT   174  /* u32   first step of a marked rollout: contact bits (1 left, 2 right) */
#define ZB_S_AIR0_TERM   175  /*       ... and its causal FeetAirtime term (zb_feet_airtime_exact) */
#define ZB_S_END         176

/* -------------- per-env randomized model parameters (config 5) -------------- */
/* ksim randomizers named in train.py:1441-1454; sampled on every episode reset  */
#define ZB_RAND_STRIDE   160
#define ZB_R_MASS        0    /* [32] body mass scale   (AllBodiesMassMultiplication 0.95..1.15) */
#define ZB_R_ARMATURE    32   /* [32] dof armature scale (ArmatureRandomizer) */
#define ZB_R_DAMPING     64   /* [32] dof damping scale  (JointDampingRandomizer) */
#define ZB_R_FRICTION    96   /* [32] dof frictionloss scale (StaticFrictionRandomizer) */
#define ZB_R_QPOS0       128  /* [20] joint-zero offsets rad (JointZeroPositionRandomizer +-2 deg) */
#define ZB_R_FLOOR_MU    148  /*      floor friction scale (FloorFrictionRandomizer 0.3..1.5) */
#define ZB_R_IMU_QUAT    149  /* [4]  imu site rotation (IMUAlignmentRandomizer tilt/yaw) */
#define ZB_R_IMU_POS     153  /* [3]  imu site translation */
#define ZB_R_END         156

/* ---------------------------- observation extras ---------------------------- */
#define ZB_X_BASE_LINVEL   0   /* [3] BaseLinearVelocityObservation  */
#define ZB_X_BASE_ANGVEL   3   /* [3] BaseAngularVelocityObservation */
#define ZB_X_BASE_LINACC   6   /* [3] BaseLinearAccelerationObservation */
#define ZB_X_BASE_ANGACC   9   /* [3] BaseAngularAccelerationObservation */
#define ZB_X_BASE_HEIGHT   12  /* [1] BaseHeightObservation (train.py:876-882) */
#define ZB_X_TOUCH         13  /* [2] left/right_foot_touch */
#define ZB_X_FORCE         15  /* [6] left/right_foot_force */
#define ZB_X_FEET_POS      21  /* [6] FeetPositionObservation (train.py:430-465) */
#define ZB_X_FEETECH_TAU   27  /* [20] FeetechTorqueObservation (train.py:1301-1308) */
#define ZB_X_ACT_ACC       47  /* [20] ActuatorAccelerationObservation */
#define ZB_X_END           67

/* ------------------------------ reward terms -------------------------------- */
#define ZB_T_STAY_ALIVE      0
#define ZB_T_UPRIGHT         1
#define ZB_T_NAIVE_FORWARD   2
#define ZB_T_FWD_ORIENT      3
#define ZB_T_LINVEL_Y        4
#define ZB_T_SINGLE_FOOT     5
#define ZB_T_FEET_AIRTIME    6
#define ZB_T_FEET_ORIENT     7
#define ZB_T_FEET_TOO_CLOSE  8
#define ZB_T_STRAIGHT_LEG    9
#define ZB_T_ANKLE_KNEE      10
#define ZB_T_ARM_POSE        11

/* ----------------------------- episode statistics --------------------------- */
#define ZB_ST_RETURN   0   /* sum of returns of episodes finished since last clear */
#define ZB_ST_LENGTH   1   /* sum of their lengths (env-steps) */
#define ZB_ST_DONE     2   /* number of finished episodes */
#define ZB_ST_REWARD   3   /* sum of per-step total reward */

/* ZbEnvConfig.solver (mjtSolver order: mjSOL_CG = 1, mjSOL_NEWTON = 2). zb_default_config() sets
   ZB_SOLVER_CG (round 6: the solver ksim's MJX model uses); a zero-filled config is Newton */
#define ZB_SOLVER_NEWTON 0u  /* primal Newton, Hessian M + J'DJ (mj_solNewton) */
#define ZB_SOLVER_CG     1u  /* primal nonlinear CG, M^-1 preconditioned, Polak-Ribiere (mj_solCG) */

/* flag bits of ZbEnvConfig.flags */
#define ZB_F_OBS_NOISE   1u   /* ksim observation noise (train.py:1497,1503) */
#define ZB_F_PUSH        2u   /* PushEvent (train.py:1459-1468), config 3 */
#define ZB_F_RANDOMIZE   4u   /* physics randomizers (train.py:1441-1454), config 5 */
#define ZB_F_AUTORESET   8u   /* reset done envs inside zb_step (ksim auto-reset) */
#define ZB_F_EULERDAMP  16u   /* mj_Euler's implicit joint damping, qacc_e = (M + dt diag(damping))^-1 (qfrc_smooth +
                                 qfrc_constraint): MuJoCo's default (mjDSBL_EULERDAMP clear). Off here: ksim
                                 sets the disable bit on its MJX model [U]. train.py:1777-1781 */

typedef struct ZbEnvConfig {
  int32_t  struct_bytes;
  uint32_t flags;
  int32_t  n_substeps;        /* round(ctrl_dt / dt) = 20 */
  int32_t  iterations;        /* solver iterations, 8 */
  int32_t  ls_iterations;     /* line-search iterations, 8 */
  float    dt;                /* 0.001 */
  float    ctrl_dt;           /* 0.02 */
  float    tolerance;         /* MuJoCo opt.tolerance default 1e-8 */
  float    ls_tolerance;      /* MuJoCo opt.ls_tolerance default 0.01 */
  float    imu_noise_std;     /* radians(1)  train.py:1497 */
  float    acc_noise_std;     /* 0.5         train.py:1503 */
  float    reset_qvel_scale;  /* RandomJointVelocityReset scale [U] */
  float    max_episode_sec;   /* EpisodeLengthTermination 80 s, train.py:1592 */
  float    lag_range[2];      /* (0.0, 0.1) train.py:1496 */
  float    bad_z[2];          /* (0.05, 0.5) train.py:1590 */
  float    max_tilt_rad;      /* radians(60) train.py:1591 */
  float    push_linvel[4];    /* (0.1, 0.1, 0.05) train.py:1460-1462 */
  float    push_interval[2];  /* (2.0, 4.0) train.py:1467 */
  float    push_vel_range[2]; /* (0.05, 0.15) train.py:1466 */
  float    reward_scale[ZB_NUM_TERMS];
  int32_t  reward_by_curriculum[ZB_NUM_TERMS];
  float    feet_airtime_touchdown_penalty; /* 0.3 train.py:1562 */
  float    naive_forward_clip_max;         /* 0.2 train.py:1550 */
  float    feet_orient_error_scale;        /* 0.25 train.py:1568 */
  float    feet_too_close_threshold;       /* 0.12 train.py:1573 */
  float    touch_threshold;                /* 0.1 train.py:516,702 */
  float    stay_alive_balance;             /* ksim StayAliveReward balance [U] */
  /* randomizer ranges (config 5) [U: ksim 0.1.99 defaults] */
  float    rand_mass[2];        /* (0.95, 1.15) train.py:1443 */
  float    rand_armature[2];
  float    rand_damping[2];
  float    rand_friction[2];
  float    rand_qpos0[2];       /* (-2, +2) deg train.py:1445 */
  float    rand_floor_mu[2];    /* (0.3, 1.5) train.py:1447 */
  float    rand_imu_tilt_std;   /* radians(5)  train.py:1453 */
  float    rand_imu_yaw_std;    /* radians(1)  */
  float    rand_imu_pos_std;    /* 0.005 m     */
  int32_t  solver;             /* ZB_SOLVER_CG (zb_default_config) or ZB_SOLVER_NEWTON: the [U] solver
                                  type ksim sets on the MJX model */
  float    pad[2];
} ZbEnvConfig;

#ifdef __cplusplus
}
#endif
#endif /* ZBOT_LAYOUT_H */
