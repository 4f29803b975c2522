/*
 * zb_oracle.c — CPU restatement of the reference hot path (TEST INFRASTRUCTURE).
 *
 * ORACLE ONLY: this file is the parity checker and the CPU baseline. It is
 * loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * and by nothing else; the product path (libzbot_hip.so) never links it.
 *
 * What it restates (reference = ksim-gym-zbot train.py driving ksim 0.1.99 +
 * MuJoCo-MJX 3.3.4, both un-vendored — see SURVEY.md §8c):
 *   - train.py pure functions, from the reference text:
 *       trapezoidal_step            train.py:1137-1196   -> zbo_trapezoidal_step
 *       get_servo_deadband          train.py:1111-1118   -> ZB_DEADBAND
 *       Feetech duty -> torque      train.py:1260-1269   -> feetech_ctrl
 *       rotate_quat_by_quat         train.py:751-787     -> rotate_quat_by_quat
 *       ImuOrientationObservation   train.py:847-873     -> observe()
 *       custom rewards              train.py:485-748     -> rewards()
 *   - MuJoCo's published computation pipeline for mj_step (Euler), function
 *     by function (names follow MuJoCo's engine_*.c):
 *       mj_kinematics, mj_comPos, mj_crb, mj_factorM (sparse L'DL),
 *       mj_solveM, mj_comVel, mj_passive, mj_rne, actuation,
 *       plane-box collision, mj_makeConstraint (frictionloss, limits,
 *       pyramidal contacts), mj_makeImpedance/diagApprox (invweight0),
 *       mj_solNewton (primal Newton, dense Cholesky of the Hessian, exact
 *       line search on the piecewise-quadratic cost), mj_rnePostConstraint,
 *       sensors (framequat, gyro, accelerometer, touch, force), mj_Euler.
 *   - ksim semantics [U] for the engine loop / terminations / resets / noise.
 *
 * Parity status: UNPINNED against the reference (no jax/mujoco/ksim in the
 * container and the reference has no tests or golden vectors, SURVEY.md §4,
 * §8c). Pinned pieces: threefry2x32-20 known-answer vectors (Random123), the
 * train.py pure functions (hand-derived KATs in tests/test_oracle_kat.py) and
 * physics invariants (free fall, M SPD vs kinetic energy, static stand).
 *
 * Build: oracle/Makefile (float: liboracle_zbot.so, double: liboracle_zbot_f64.so).
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "zbot_layout.h"
#include "zbot_model.h"

#if defined(ZBO_COUNT)
/* oracle/zb_flops.cpp: `real` is a float that counts its arithmetic, and the math macros
   (SQRT ... ASIN) are its counting overloads; defined by the including file */
#elif defined(ZBO_DOUBLE)
typedef double real;
#define RS(x) x
#define SQRT sqrt
#define SIN sin
#define COS cos
#define EXP exp
#define LOG log
#define POW pow
#define FABS fabs
#define ATAN2 atan2
#define ASIN asin
#else
typedef float real;
#define SQRT sqrtf
#define SIN sinf
#define COS cosf
#define EXP expf
#define LOG logf
#define POW powf
#define FABS fabsf
#define ATAN2 atan2f
#define ASIN asinf
#endif

#define NB ZB_MAX_BODY
#define NDOF ZB_MAX_DOF
#define NCON (ZB_MAX_CON + ZB_CON_PER_PAIR) /* floor contacts + the sole pair's */
#define MAXEFC (2 * ZB_MAX_DOF + 4 * NCON)
#define MINVAL ((real)1e-15)
#define MINIMP ((real)0.0001)
#define MAXIMP ((real)0.9999)
#define ZB_DEADBAND ((real)(2.0 * 0.087 * 3.14159265358979323846 / 180.0)) /* train.py:1113-1116 */

enum { EFC_FRICTION = 0, EFC_LIMIT = 1, EFC_CONTACT = 2 };

/* --------------------------------------------------------------------------
 * threefry2x32-20 (Random123; JAX's PRNG primitive). Keys/counters are the
 * build's own stream layout (SURVEY.md §7 "RNG seed parity"): key =
 * (seed_lo ^ purpose*0x9E3779B9, seed_hi ^ k*0x85EBCA6B), ctr = (env, counter).
 * -------------------------------------------------------------------------- */
static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

void zbo_threefry2x32(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1, uint32_t out[2]) {
  static const int R[8] = {13, 15, 26, 6, 17, 29, 16, 24};
  uint32_t ks[3] = {k0, k1, 0x1BD11BDAu ^ k0 ^ k1};
  uint32_t x0 = c0 + ks[0], x1 = c1 + ks[1];
  for (int blk = 0; blk < 5; blk++) {
    for (int r = 0; r < 4; r++) {
      x0 += x1;
      x1 = rotl32(x1, R[(blk & 1) * 4 + r]);
      x1 ^= x0;
    }
    x0 += ks[(blk + 1) % 3];
    x1 += ks[(blk + 2) % 3] + (uint32_t)(blk + 1);
  }
  out[0] = x0;
  out[1] = x1;
}

#define P_OBS 1u
#define P_PUSH 2u
#define P_RESET 3u
#define P_RAND 4u
#define P_ACTION 5u

static void rng_bits(uint64_t seed, uint32_t purpose, uint32_t k, uint32_t env, uint32_t ctr, uint32_t out[2]) {
  zbo_threefry2x32((uint32_t)seed ^ (purpose * 0x9E3779B9u), (uint32_t)(seed >> 32) ^ (k * 0x85EBCA6Bu), env, ctr,
                   out);
}
static inline float u01(uint32_t b) { return (float)(b >> 8) * (1.0f / 16777216.0f); }
/* Box-Muller pair from one threefry call */
static void normal2(uint64_t seed, uint32_t purpose, uint32_t k, uint32_t env, uint32_t ctr, float out[2]) {
  uint32_t b[2];
  rng_bits(seed, purpose, k, env, ctr, b);
  float u1 = 1.0f - u01(b[0]); /* (0,1] */
  float u2 = u01(b[1]);
  float r = sqrtf(-2.0f * logf(u1));
  float th = 6.283185307179586f * u2;
  out[0] = r * cosf(th);
  out[1] = r * sinf(th);
}
static void uniform2(uint64_t seed, uint32_t purpose, uint32_t k, uint32_t env, uint32_t ctr, float out[2]) {
  uint32_t b[2];
  rng_bits(seed, purpose, k, env, ctr, b);
  out[0] = u01(b[0]);
  out[1] = u01(b[1]);
}

/* synthetic policy used by bench/tests: a = JOINT_BIASES + std * N(0,1), clipped to range */
void zbo_synthetic_actions(const ZbModel* m, uint64_t seed, int n, int env_offset, uint32_t t, float std_,
                           float* action) {
  for (int e = 0; e < n; e++) {
    for (int k = 0; k < ZB_NJ / 2; k++) {
      float z[2];
      normal2(seed, P_ACTION, (uint32_t)k, (uint32_t)(env_offset + e), t, z);
      for (int h = 0; h < 2; h++) {
        int j = 2 * k + h;
        int d = m->act_dof[j];
        float a = m->joint_bias[j] + std_ * z[h];
        if (m->dof_limited[d]) {
          if (a < m->dof_range[d][0]) a = m->dof_range[d][0];
          if (a > m->dof_range[d][1]) a = m->dof_range[d][1];
        }
        action[(size_t)e * ZB_NJ + j] = a;
      }
    }
  }
}

/* -------------------------------------------------------------------------- */
/* small vector / quaternion helpers (MuJoCo mju_* restatements)              */
/* -------------------------------------------------------------------------- */
static inline void cross3(real r[3], const real a[3], const real b[3]) {
  real t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
static inline real dot3(const real a[3], const real b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static inline void quat_mul(real r[4], const real a[4], const real b[4]) {
  real w = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  real x = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  real y = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  real z = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  r[0] = w; r[1] = x; r[2] = y; r[3] = z;
}
static inline void quat_normalize(real q[4]) {
  real n = SQRT(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < MINVAL) { q[0] = 1; q[1] = q[2] = q[3] = 0; return; }
  real s = (real)1 / n;
  q[0] *= s; q[1] *= s; q[2] *= s; q[3] *= s;
}
/* mju_quat2Mat: row-major */
static inline void quat2mat(real m[9], const real q[4]) {
  real w = q[0], x = q[1], y = q[2], z = q[3];
  m[0] = 1 - 2 * (y * y + z * z); m[1] = 2 * (x * y - w * z); m[2] = 2 * (x * z + w * y);
  m[3] = 2 * (x * y + w * z); m[4] = 1 - 2 * (x * x + z * z); m[5] = 2 * (y * z - w * x);
  m[6] = 2 * (x * z - w * y); m[7] = 2 * (y * z + w * x); m[8] = 1 - 2 * (x * x + y * y);
}
static inline void mulmv3(real r[3], const real m[9], const real v[3]) {
  real t0 = m[0] * v[0] + m[1] * v[1] + m[2] * v[2];
  real t1 = m[3] * v[0] + m[4] * v[1] + m[5] * v[2];
  real t2 = m[6] * v[0] + m[7] * v[1] + m[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
static inline void mulmtv3(real r[3], const real m[9], const real v[3]) { /* m^T v */
  real t0 = m[0] * v[0] + m[3] * v[1] + m[6] * v[2];
  real t1 = m[1] * v[0] + m[4] * v[1] + m[7] * v[2];
  real t2 = m[2] * v[0] + m[5] * v[1] + m[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
static inline void rotvec_quat(real r[3], const real q[4], const real v[3]) {
  real m[9];
  quat2mat(m, q);
  mulmv3(r, m, v);
}
/* mju_axisAngle2Quat */
static inline void axis_angle_quat(real q[4], const real axis[3], real angle) {
  real s = SIN(angle * (real)0.5);
  q[0] = COS(angle * (real)0.5); q[1] = axis[0] * s; q[2] = axis[1] * s; q[3] = axis[2] * s;
}
/* spatial algebra, 6-vectors [ang(3), lin(3)] (MuJoCo conventions) */
static inline void cross_motion(real r[6], const real v[6], const real u[6]) {
  real a[3], b[3], c[3];
  cross3(a, v, u);
  cross3(b, v, u + 3);
  cross3(c, v + 3, u);
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2];
  r[3] = b[0] + c[0]; r[4] = b[1] + c[1]; r[5] = b[2] + c[2];
}
static inline void cross_force(real r[6], const real v[6], const real f[6]) {
  real a[3], b[3], c[3];
  cross3(a, v, f);
  cross3(b, v + 3, f + 3);
  cross3(c, v, f + 3);
  r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2];
  r[3] = c[0]; r[4] = c[1]; r[5] = c[2];
}
/* mju_mulInertVec: cinert = [Ixx Iyy Izz Ixy Ixz Iyz, m*dx m*dy m*dz, m] */
static inline void mul_inert_vec(real r[6], const real i[10], const real v[6]) {
  r[0] = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  r[1] = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  r[2] = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  r[3] = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  r[4] = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  r[5] = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
}
static inline real dot6(const real a[6], const real b[6]) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}

/* -------------------------------------------------------------------------- */
/* per-env working data (mjData subset)                                        */
/* -------------------------------------------------------------------------- */
typedef struct {
  /* effective (possibly randomized) model parameters */
  real body_mass[NB], body_inertia[NB][3];
  real dof_armature[NDOF], dof_damping[NDOF], dof_frictionloss[NDOF];
  real qpos0[ZB_MAX_QPOS];
  real floor_mu;
  real imu_quat[4], imu_pos[3];

  real qpos[ZB_MAX_QPOS], qvel[NDOF], qacc[NDOF], qacc_smooth[NDOF], qacc_warm[NDOF];
  real ctrl[ZB_MAX_ACT], act_force[ZB_MAX_ACT];
  real xpos[NB][3], xquat[NB][4], xmat[NB][9], xipos[NB][3], ximat[NB][9];
  real xanchor[NB][3], xaxis[NB][3];
  real subtree_com[NB][3];
  real cinert[NB][10], crb[NB][10], cdof[NDOF][6], cdof_dot[NDOF][6];
  real cvel[NB][6], cacc[NB][6], cfrc[NB][6], cfrc_ext[NB][6];
  real qM[NDOF][NDOF], qLD[NDOF][NDOF], qLDinv[NDOF];
  real qfrc_bias[NDOF], qfrc_passive[NDOF], qfrc_actuator[NDOF], qfrc_smooth[NDOF], qfrc_constraint[NDOF];
  real geom_xpos[ZB_MAX_GEOM][3], geom_xmat[ZB_MAX_GEOM][9];
  real site_xpos[ZB_MAX_SITE][3], site_xmat[ZB_MAX_SITE][9], site_xquat[ZB_MAX_SITE][4];
  /* contacts */
  int ncon;
  real con_pos[NCON][3], con_dist[NCON], con_mu[NCON], con_n[NCON][3], con_t1[NCON][3], con_t2[NCON][3];
  int con_geom[NCON], con_geom1[NCON], con_efc[NCON]; /* geom1 -1: the floor (world) */
  /* constraints */
  int nefc;
  int efc_type[MAXEFC], efc_id[MAXEFC];
  real efc_J[MAXEFC][NDOF], efc_pos[MAXEFC], efc_D[MAXEFC], efc_R[MAXEFC], efc_aref[MAXEFC];
  real efc_floss[MAXEFC], efc_force[MAXEFC], efc_jar[MAXEFC];
  int efc_active[MAXEFC];
  /* sensors */
  real imu_framequat[4], imu_gyro[3], imu_acc[3], touch[2], force[2][3];
  int solver_iters;
  /* test infrastructure (zbo_set_clearance_out): the smallest |distance - margin| of a floor contact
     candidate over a control step's substeps: a contact that close to its activation boundary starts
     or not by rounding */
  real clearance;
} ZbData;

static float* g_clearance_out = NULL; /* zbo_set_clearance_out; NULL: not recorded */
static inline void track_clearance(ZbData* d, real dist, real margin) {
  const real c = dist > margin ? dist - margin : margin - dist;
  if (c < d->clearance) d->clearance = c;
}

/* ----------------------------- mj_kinematics ------------------------------ */
static void kinematics(const ZbModel* m, ZbData* d) {
  d->xpos[0][0] = d->xpos[0][1] = d->xpos[0][2] = 0;
  d->xquat[0][0] = 1; d->xquat[0][1] = d->xquat[0][2] = d->xquat[0][3] = 0;
  quat2mat(d->xmat[0], d->xquat[0]);
  for (int i = 1; i < m->nbody; i++) {
    int p = m->body_parent[i];
    real pos[3], quat[4];
    if (m->body_jnttype[i] == ZB_JNT_FREE) {
      int a = m->body_qposadr[i];
      pos[0] = d->qpos[a]; pos[1] = d->qpos[a + 1]; pos[2] = d->qpos[a + 2];
      quat[0] = d->qpos[a + 3]; quat[1] = d->qpos[a + 4]; quat[2] = d->qpos[a + 5]; quat[3] = d->qpos[a + 6];
      quat_normalize(quat);
      d->xanchor[i][0] = pos[0]; d->xanchor[i][1] = pos[1]; d->xanchor[i][2] = pos[2];
    } else {
      real bp[3] = {m->body_pos[i][0], m->body_pos[i][1], m->body_pos[i][2]};
      real bq[4] = {m->body_quat[i][0], m->body_quat[i][1], m->body_quat[i][2], m->body_quat[i][3]};
      real t[3];
      mulmv3(t, d->xmat[p], bp);
      pos[0] = d->xpos[p][0] + t[0]; pos[1] = d->xpos[p][1] + t[1]; pos[2] = d->xpos[p][2] + t[2];
      quat_mul(quat, d->xquat[p], bq);
      if (m->body_jnttype[i] == ZB_JNT_HINGE) {
        real mat[9], ax[3] = {m->jnt_axis[i][0], m->jnt_axis[i][1], m->jnt_axis[i][2]};
        real jp[3] = {m->jnt_pos[i][0], m->jnt_pos[i][1], m->jnt_pos[i][2]};
        quat2mat(mat, quat);
        /* anchor and axis in world, before applying the joint rotation */
        mulmv3(t, mat, jp);
        d->xanchor[i][0] = pos[0] + t[0]; d->xanchor[i][1] = pos[1] + t[1]; d->xanchor[i][2] = pos[2] + t[2];
        mulmv3(d->xaxis[i], mat, ax);
        int qa = m->body_qposadr[i];
        real qloc[4], qn[4];
        axis_angle_quat(qloc, ax, d->qpos[qa] - d->qpos0[qa]);
        quat_mul(qn, quat, qloc);
        quat[0] = qn[0]; quat[1] = qn[1]; quat[2] = qn[2]; quat[3] = qn[3];
        quat_normalize(quat);
        quat2mat(mat, quat);
        mulmv3(t, mat, jp);
        pos[0] = d->xanchor[i][0] - t[0]; pos[1] = d->xanchor[i][1] - t[1]; pos[2] = d->xanchor[i][2] - t[2];
      }
    }
    for (int k = 0; k < 3; k++) d->xpos[i][k] = pos[k];
    for (int k = 0; k < 4; k++) d->xquat[i][k] = quat[k];
    quat2mat(d->xmat[i], quat);
    /* inertial frame (body_iquat identity in compiled models) */
    real ip[3] = {m->body_ipos[i][0], m->body_ipos[i][1], m->body_ipos[i][2]}, t2[3];
    mulmv3(t2, d->xmat[i], ip);
    for (int k = 0; k < 3; k++) d->xipos[i][k] = pos[k] + t2[k];
    real iq[4] = {m->body_iquat[i][0], m->body_iquat[i][1], m->body_iquat[i][2], m->body_iquat[i][3]}, qi[4];
    quat_mul(qi, quat, iq);
    quat2mat(d->ximat[i], qi);
  }
  /* geoms */
  for (int g = 0; g < m->ngeom; g++) {
    int b = m->geom_body[g];
    real gp[3] = {m->geom_pos[g][0], m->geom_pos[g][1], m->geom_pos[g][2]}, t[3];
    real gq[4] = {m->geom_quat[g][0], m->geom_quat[g][1], m->geom_quat[g][2], m->geom_quat[g][3]}, q[4];
    mulmv3(t, d->xmat[b], gp);
    for (int k = 0; k < 3; k++) d->geom_xpos[g][k] = d->xpos[b][k] + t[k];
    quat_mul(q, d->xquat[b], gq);
    quat2mat(d->geom_xmat[g], q);
  }
  /* sites (imu site pose may be randomized) */
  for (int s = 0; s < m->nsite; s++) {
    int b = m->site_body[s];
    real sp[3] = {m->site_pos[s][0], m->site_pos[s][1], m->site_pos[s][2]};
    real sq[4] = {m->site_quat[s][0], m->site_quat[s][1], m->site_quat[s][2], m->site_quat[s][3]}, t[3], q[4];
    if (s == m->site_imu) {
      for (int k = 0; k < 3; k++) sp[k] = d->imu_pos[k];
      for (int k = 0; k < 4; k++) sq[k] = d->imu_quat[k];
    }
    mulmv3(t, d->xmat[b], sp);
    for (int k = 0; k < 3; k++) d->site_xpos[s][k] = d->xpos[b][k] + t[k];
    quat_mul(q, d->xquat[b], sq);
    for (int k = 0; k < 4; k++) d->site_xquat[s][k] = q[k];
    quat2mat(d->site_xmat[s], q);
  }
}

/* ------------------------------- mj_comPos -------------------------------- */
static void com_pos(const ZbModel* m, ZbData* d) {
  real msum[NB];
  for (int i = 0; i < m->nbody; i++) {
    msum[i] = d->body_mass[i];
    for (int k = 0; k < 3; k++) d->subtree_com[i][k] = d->body_mass[i] * d->xipos[i][k];
  }
  for (int i = m->nbody - 1; i > 0; i--) {
    int p = m->body_parent[i];
    msum[p] += msum[i];
    for (int k = 0; k < 3; k++) d->subtree_com[p][k] += d->subtree_com[i][k];
  }
  for (int i = 0; i < m->nbody; i++) {
    if (msum[i] < MINVAL) {
      for (int k = 0; k < 3; k++) d->subtree_com[i][k] = d->xipos[i][k];
    } else {
      for (int k = 0; k < 3; k++) d->subtree_com[i][k] /= msum[i];
    }
  }
  /* cinert: inertia about the root subtree com, world orientation (mju_inertCom) */
  const real* c = d->subtree_com[1]; /* every robot body has rootid 1 */
  for (int k = 0; k < 10; k++) d->cinert[0][k] = 0;
  for (int i = 1; i < m->nbody; i++) {
    const real* R = d->ximat[i];
    real mass = d->body_mass[i];
    const real* in = d->body_inertia[i];
    real dif[3] = {d->xipos[i][0] - c[0], d->xipos[i][1] - c[1], d->xipos[i][2] - c[2]};
    /* I = R diag(in) R^T + mass (|dif|^2 E - dif dif^T) */
    real I[9];
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) I[3 * a + b] = R[3 * a] * in[0] * R[3 * b] + R[3 * a + 1] * in[1] * R[3 * b + 1] +
                                                  R[3 * a + 2] * in[2] * R[3 * b + 2];
    real dd = dot3(dif, dif);
    real* ci = d->cinert[i];
    ci[0] = I[0] + mass * (dd - dif[0] * dif[0]);
    ci[1] = I[4] + mass * (dd - dif[1] * dif[1]);
    ci[2] = I[8] + mass * (dd - dif[2] * dif[2]);
    ci[3] = I[1] - mass * dif[0] * dif[1];
    ci[4] = I[2] - mass * dif[0] * dif[2];
    ci[5] = I[5] - mass * dif[1] * dif[2];
    ci[6] = mass * dif[0]; ci[7] = mass * dif[1]; ci[8] = mass * dif[2];
    ci[9] = mass;
  }
  /* cdof (mju_dofCom) */
  for (int i = 1; i < m->nbody; i++) {
    int j0 = m->body_dofadr[i];
    if (j0 < 0) continue;
    if (m->body_jnttype[i] == ZB_JNT_FREE) {
      real off[3] = {c[0] - d->xpos[i][0], c[1] - d->xpos[i][1], c[2] - d->xpos[i][2]};
      for (int k = 0; k < 3; k++) {
        real* cd = d->cdof[j0 + k];
        cd[0] = cd[1] = cd[2] = 0; cd[3] = cd[4] = cd[5] = 0;
        cd[3 + k] = 1;
      }
      for (int k = 0; k < 3; k++) {
        real* cd = d->cdof[j0 + 3 + k];
        real ax[3] = {d->xmat[i][k], d->xmat[i][3 + k], d->xmat[i][6 + k]};
        cd[0] = ax[0]; cd[1] = ax[1]; cd[2] = ax[2];
        cross3(cd + 3, ax, off);
      }
    } else {
      real off[3] = {c[0] - d->xanchor[i][0], c[1] - d->xanchor[i][1], c[2] - d->xanchor[i][2]};
      real* cd = d->cdof[j0];
      cd[0] = d->xaxis[i][0]; cd[1] = d->xaxis[i][1]; cd[2] = d->xaxis[i][2];
      cross3(cd + 3, d->xaxis[i], off);
    }
  }
}

/* ------------------------------- mj_crb ----------------------------------- */
static void crb(const ZbModel* m, ZbData* d) {
  int nv = m->nv;
  memcpy(d->crb, d->cinert, sizeof(d->crb));
  for (int i = m->nbody - 1; i > 0; i--) {
    int p = m->body_parent[i];
    if (p > 0)
      for (int k = 0; k < 10; k++) d->crb[p][k] += d->crb[i][k];
  }
  memset(d->qM, 0, sizeof(d->qM));
  for (int i = 0; i < nv; i++) {
    real buf[6];
    mul_inert_vec(buf, d->crb[m->dof_body[i]], d->cdof[i]);
    for (int j = i; j >= 0; j = m->dof_parent[j]) {
      d->qM[i][j] = dot6(d->cdof[j], buf);
    }
    d->qM[i][i] += d->dof_armature[i];
  }
}

/* mj_factorM: in-place L'DL over the dof tree (qM lower, j ancestor of i) */
static void factor_m(const ZbModel* m, real LD[NDOF][NDOF], real* LDinv) {
  for (int k = m->nv - 1; k >= 0; k--) {
    real Dk = LD[k][k];
    for (int i = m->dof_parent[k]; i >= 0; i = m->dof_parent[i]) {
      real tmp = LD[k][i] / Dk;
      for (int j = i; j >= 0; j = m->dof_parent[j]) LD[i][j] -= tmp * LD[k][j];
      LD[k][i] = tmp;
    }
  }
  for (int k = 0; k < m->nv; k++) LDinv[k] = (real)1 / LD[k][k];
}
/* mj_solveM: x = M^-1 b using the L'DL factor */
static void solve_m(const ZbModel* m, const real LD[NDOF][NDOF], const real* LDinv, real* x) {
  for (int k = m->nv - 1; k >= 0; k--)
    for (int i = m->dof_parent[k]; i >= 0; i = m->dof_parent[i]) x[i] -= LD[k][i] * x[k];
  for (int k = 0; k < m->nv; k++) x[k] *= LDinv[k];
  for (int k = 0; k < m->nv; k++)
    for (int i = m->dof_parent[k]; i >= 0; i = m->dof_parent[i]) x[k] -= LD[k][i] * x[i];
}
/* y = M x using the lower-triangular tree storage of qM */
static void mul_m(const ZbModel* m, const real M[NDOF][NDOF], const real* x, real* y) {
  for (int i = 0; i < m->nv; i++) y[i] = M[i][i] * x[i];
  for (int i = 0; i < m->nv; i++)
    for (int j = m->dof_parent[i]; j >= 0; j = m->dof_parent[j]) {
      y[i] += M[i][j] * x[j];
      y[j] += M[i][j] * x[i];
    }
}

/* ------------------------------- mj_comVel -------------------------------- */
static void com_vel(const ZbModel* m, ZbData* d) {
  for (int k = 0; k < 6; k++) d->cvel[0][k] = 0;
  for (int i = 1; i < m->nbody; i++) {
    int p = m->body_parent[i];
    real cv[6];
    for (int k = 0; k < 6; k++) cv[k] = d->cvel[p][k];
    int j0 = m->body_dofadr[i];
    if (j0 >= 0) {
      if (m->body_jnttype[i] == ZB_JNT_FREE) {
        for (int j = j0; j < j0 + 3; j++) {
          for (int k = 0; k < 6; k++) d->cdof_dot[j][k] = 0;
          for (int k = 0; k < 6; k++) cv[k] += d->cdof[j][k] * d->qvel[j];
        }
        for (int j = j0 + 3; j < j0 + 6; j++) cross_motion(d->cdof_dot[j], cv, d->cdof[j]);
        for (int j = j0 + 3; j < j0 + 6; j++)
          for (int k = 0; k < 6; k++) cv[k] += d->cdof[j][k] * d->qvel[j];
      } else {
        cross_motion(d->cdof_dot[j0], cv, d->cdof[j0]);
        for (int k = 0; k < 6; k++) cv[k] += d->cdof[j0][k] * d->qvel[j0];
      }
    }
    for (int k = 0; k < 6; k++) d->cvel[i][k] = cv[k];
  }
}

/* --------------------------------- mj_rne --------------------------------- */
static void rne(const ZbModel* m, ZbData* d, int with_acc, real cacc_out[NB][6], real cfrc_out[NB][6]) {
  cacc_out[0][0] = cacc_out[0][1] = cacc_out[0][2] = 0;
  cacc_out[0][3] = -m->gravity[0]; cacc_out[0][4] = -m->gravity[1]; cacc_out[0][5] = -m->gravity[2];
  for (int i = 1; i < m->nbody; i++) {
    int p = m->body_parent[i];
    real a[6];
    for (int k = 0; k < 6; k++) a[k] = cacc_out[p][k];
    int j0 = m->body_dofadr[i];
    for (int j = j0; j >= 0 && j < j0 + m->body_dofnum[i]; j++) {
      for (int k = 0; k < 6; k++) a[k] += d->cdof_dot[j][k] * d->qvel[j];
      if (with_acc)
        for (int k = 0; k < 6; k++) a[k] += d->cdof[j][k] * d->qacc[j];
    }
    for (int k = 0; k < 6; k++) cacc_out[i][k] = a[k];
    real f1[6], f2[6], tmp[6];
    mul_inert_vec(f1, d->cinert[i], a);
    mul_inert_vec(tmp, d->cinert[i], d->cvel[i]);
    cross_force(f2, d->cvel[i], tmp);
    for (int k = 0; k < 6; k++) cfrc_out[i][k] = f1[k] + f2[k];
  }
  for (int k = 0; k < 6; k++) cfrc_out[0][k] = 0;
  if (with_acc)
    for (int i = 1; i < m->nbody; i++)
      for (int k = 0; k < 6; k++) cfrc_out[i][k] -= d->cfrc_ext[i][k];
  for (int i = m->nbody - 1; i > 0; i--) {
    int p = m->body_parent[i];
    if (p > 0)
      for (int k = 0; k < 6; k++) cfrc_out[p][k] += cfrc_out[i][k];
  }
}

/* ------------------ actuation + passive + smooth acceleration -------------- */
static void smooth_forces(const ZbModel* m, ZbData* d) {
  int nv = m->nv;
  for (int j = 0; j < nv; j++) {
    d->qfrc_passive[j] = -d->dof_damping[j] * d->qvel[j];
    d->qfrc_actuator[j] = 0;
  }
  for (int a = 0; a < m->nu; a++) {
    real c = d->ctrl[a];
    if (c < m->act_ctrlrange[a][0]) c = m->act_ctrlrange[a][0];
    if (c > m->act_ctrlrange[a][1]) c = m->act_ctrlrange[a][1];
    d->act_force[a] = m->act_gear[a] * c;
    d->qfrc_actuator[m->act_dof[a]] += m->act_gear[a] * d->act_force[a];
  }
  rne(m, d, 0, d->cacc, d->cfrc);
  for (int j = 0; j < nv; j++) d->qfrc_bias[j] = dot6(d->cdof[j], d->cfrc[m->dof_body[j]]);
  for (int j = 0; j < nv; j++) {
    d->qfrc_smooth[j] = d->qfrc_passive[j] - d->qfrc_bias[j] + d->qfrc_actuator[j];
    d->qacc_smooth[j] = d->qfrc_smooth[j];
  }
  solve_m(m, d->qLD, d->qLDinv, d->qacc_smooth);
}

/* ------------------------------- collision -------------------------------- */
/* The floor plane (z = 0, normal +z, train.py:1326-1331 floor with geom_priority 2) against each
 * collider, as MuJoCo's primitive colliders (engine_collision_primitive.c, MuJoCo 3.3):
 *   box (mjc_PlaneBox): the 8 corners in index order (bit 0: +x, bit 1: +y, bit 2: +z half
 *     size), a corner kept when its offset from the centre along the normal is <= 0 and its
 *     distance is within the margin, at most 4;
 *   capsule (mjc_PlaneCapsule): the end spheres, the +half-length end first; tangent frame along
 *     the capsule axis projected on the plane (mjx plane_capsule: +y when that projection is
 *     shorter than 0.5, i.e. the axis is within 30 degrees of the normal);
 *   sphere (mjc_PlaneSphere): one contact;
 *   cylinder (mjc_PlaneCylinder): the axis a turned toward the plane, v the radius vector in the
 *     disk planes toward it (a prj(a) - n normalised to the radius; the geom's x axis times the
 *     radius when the disks are parallel to the plane), then up to 4 points, each kept within the
 *     margin, none when the first is not: the near disk's deepest point c + v + a, the far disk's
 *     c + v - a, and the two points of the near disk 120 degrees away from the first,
 *     c + a - v / 2 +- v1 (v1 = (v x a) normalised to sqrt(3)/2 of the radius);
 *   ellipsoid (mjc_PlaneEllipsoid): one contact at the support point along -n, in the geom frame
 *     -s .* sn / |sn| with sn = s .* (R' n) (s the three semi-axes).
 * Contact point: the deepest point moved back along the normal by half the distance. Frames other
 * than the capsule's are mju_makeFrame(+z): t1 = +y, t2 = n x t1 = -x. */
static void add_contact(const ZbModel* m, ZbData* d, int g, const real p[3], real dist, const real t1[3]) {
  if (d->ncon >= ZB_MAX_CON) return;
  int n = d->ncon++;
  d->con_pos[n][0] = p[0];
  d->con_pos[n][1] = p[1];
  d->con_pos[n][2] = p[2] - (real)0.5 * dist;
  d->con_dist[n] = dist;
  d->con_geom[n] = g;
  d->con_geom1[n] = -1;
  d->con_mu[n] = m->floor_friction[0] * d->floor_mu;
  /* frame (n, t1, t2 = n x t1) with n = +z */
  d->con_n[n][0] = 0; d->con_n[n][1] = 0; d->con_n[n][2] = 1;
  for (int k = 0; k < 3; k++) d->con_t1[n][k] = t1[k];
  d->con_t2[n][0] = -t1[1]; d->con_t2[n][1] = t1[0]; d->con_t2[n][2] = 0;
}

/* ------------------------- box-box (the sole pair) --------------------------
 * [U: MuJoCo's mjc_BoxBox and MJX's box_box are not on disk; this restates the published
 * separating-axis + face-clipping method they build on (Gottschalk's OBB test, ODE's dBoxBox), with
 * MJX's four-point manifold selection. The HIP engine (zb_engine.hip pair_contacts) computes the same
 * candidates in the same order.]
 *  1. Separating axes: box 1's three face normals, box 2's, then the nine edge cross products
 *     A_i x B_j (skipped when |A_i x B_j| < 1e-6, parallel edges), normalised.
 *     sep(L) = |d.L| - (sum_k a_k |A_k.L| + sum_k b_k |B_k.L|), d = c2 - c1. Any sep > margin: no
 *     contact. The largest sep (least penetration) wins, faces in order first; an edge axis replaces
 *     the best only if sep > best + 0.05 |best| (ODE's preference for face contacts, 1.05 sep > best
 *     for a penetration, kept for a gap inside the margin). The normal n = +-L
 *     points from box 1 to box 2 (n.d >= 0).
 *  2. Face axis k of the reference box R (I: the incident box): nr points from R toward I (n for
 *     box 1, -n for box 2); the reference face centre o = cR + r_k nr, its axes u, v (R's axes k+1,
 *     k+2, half sizes hu, hv). The incident face: I's axis j with the largest |I_j.nr|, on the side
 *     facing R; its vertices in cyclic order (+,+) (-,+) (-,-) (+,-) along I's axes j+1, j+2. In
 *     the frame (u, v, nr) at o, the candidates in this order:
 *       (a) the incident vertices with |x| <= hu and |y| <= hv;
 *       (b) for each incident edge k -> k+1, its crossings of the sides x = -hu, x = +hu, y = -hv,
 *           y = +hv (strictly between the edge's ends) within the other coordinate's extent;
 *       (c) the rectangle corners (-,-) (+,-) (+,+) (-,+) inside the incident quadrilateral, lifted
 *           onto its plane.
 *     A candidate at height z is a contact when z <= margin: dist = z, position o + x u + y v +
 *     (z / 2) nr (halfway between the faces). A candidate within 1e-6 in x and y of an earlier one
 *     within the margin is dropped. Of more than 4, MJX's manifold points: a the deepest (smallest z, first on ties), b the
 *     farthest from a, c the farthest from the line ab, d the farthest from the line bc or, failing
 *     that, ac (the first maximum of |cross(b - c, b - p)| over p followed by |cross(a - c, a - p)|),
 *     keeping distinct points in the order a, b, c, d.
 *  3. Edge axis A_i x B_j: one contact at the midpoint of the closest points of box 1's edge along
 *     A_i that is most extreme toward box 2 and box 2's edge along B_j most extreme toward box 1 (the
 *     line parameters clamped to the half lengths), dist = sep.
 * Returns the contact count (<= 4): positions, distances, the common normal. */
#define BB_MAXC 24
static int box_box(const real c1[3], const real R1[9], const float* s1, const real c2[3], const real R2[9],
                   const float* s2, real margin, real pos[4][3], real dist[4], real nrm[3]) {
  real A[3][3], B[3][3], a[3] = {s1[0], s1[1], s1[2]}, b[3] = {s2[0], s2[1], s2[2]};
  for (int k = 0; k < 3; k++)
    for (int r = 0; r < 3; r++) {
      A[k][r] = R1[3 * r + k]; /* column k of the rotation: the box's axis k in the world */
      B[k][r] = R2[3 * r + k];
    }
  const real dv[3] = {c2[0] - c1[0], c2[1] - c1[1], c2[2] - c1[2]};
  real best = -1e30, L[3] = {0, 0, 0};
  int code = -1; /* 0-2: face of box 1, 3-5: face of box 2, 6 + 3 i + j: edge A_i x B_j */
  for (int ax = 0; ax < 15; ax++) {
    real l[3];
    if (ax < 3) {
      for (int r = 0; r < 3; r++) l[r] = A[ax][r];
    } else if (ax < 6) {
      for (int r = 0; r < 3; r++) l[r] = B[ax - 3][r];
    } else {
      const int i = (ax - 6) / 3, j = (ax - 6) % 3;
      cross3(l, A[i], B[j]);
      const real ln = SQRT(dot3(l, l));
      if (ln < (real)1e-6) continue;
      for (int r = 0; r < 3; r++) l[r] /= ln;
    }
    real ra = 0, rb = 0;
    for (int k = 0; k < 3; k++) {
      ra += a[k] * FABS(dot3(A[k], l));
      rb += b[k] * FABS(dot3(B[k], l));
    }
    const real dl = dot3(dv, l);
    const real sep = FABS(dl) - (ra + rb);
    if (sep > margin) return 0;
    const int better = ax < 6 ? sep > best : sep > best + (real)0.05 * FABS(best);
    if (better) {
      best = sep;
      code = ax;
      const real sg = dl < 0 ? (real)-1 : (real)1;
      for (int r = 0; r < 3; r++) L[r] = sg * l[r];
    }
  }
  for (int r = 0; r < 3; r++) nrm[r] = L[r];
  if (code >= 6) {
    const int i = (code - 6) / 3, j = (code - 6) % 3;
    real p1[3] = {c1[0], c1[1], c1[2]}, p2[3] = {c2[0], c2[1], c2[2]};
    for (int k = 0; k < 3; k++) {
      if (k != i) {
        const real sg = dot3(A[k], L) > 0 ? (real)1 : (real)-1;
        for (int r = 0; r < 3; r++) p1[r] += sg * a[k] * A[k][r];
      }
      if (k != j) {
        const real sg = dot3(B[k], L) > 0 ? (real)-1 : (real)1;
        for (int r = 0; r < 3; r++) p2[r] += sg * b[k] * B[k][r];
      }
    }
    const real w[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]};
    const real ab = dot3(A[i], B[j]), d1 = dot3(A[i], w), d2 = dot3(B[j], w);
    const real den = 1 - ab * ab;
    real t = den > (real)1e-12 ? (real)((ab * d2 - d1) / den) : (real)0;
    if (t < -a[i]) t = -a[i];
    if (t > a[i]) t = a[i];
    real u = d2 + t * ab;
    if (u < -b[j]) u = -b[j];
    if (u > b[j]) u = b[j];
    for (int r = 0; r < 3; r++) pos[0][r] = (real)0.5 * (p1[r] + t * A[i][r] + p2[r] + u * B[j][r]);
    dist[0] = best;
    return 1;
  }
  /* face contact */
  const int ref2 = code >= 3, k = ref2 ? code - 3 : code;
  const real(*Rx)[3] = ref2 ? B : A;
  const real(*Ix)[3] = ref2 ? A : B;
  const real* rs = ref2 ? b : a;
  const real* is = ref2 ? a : b;
  const real* cR = ref2 ? c2 : c1;
  const real* cI = ref2 ? c1 : c2;
  real nr[3];
  for (int r = 0; r < 3; r++) nr[r] = ref2 ? -L[r] : L[r];
  const int ku = (k + 1) % 3, kv = (k + 2) % 3;
  real o[3];
  for (int r = 0; r < 3; r++) o[r] = cR[r] + rs[k] * nr[r];
  const real hu = rs[ku], hv = rs[kv];
  int jj = 0;
  real bestd = -1;
  for (int q = 0; q < 3; q++) {
    const real v = FABS(dot3(Ix[q], nr));
    if (v > bestd) { bestd = v; jj = q; }
  }
  const real sgi = dot3(Ix[jj], nr) > 0 ? (real)-1 : (real)1; /* the face of I facing R */
  const int ja = (jj + 1) % 3, jb = (jj + 2) % 3;
  static const real va[4] = {1, -1, -1, 1}, vb[4] = {1, 1, -1, -1};
  real px[4], py[4], pz[4];
  for (int q = 0; q < 4; q++) {
    real V[3];
    for (int r = 0; r < 3; r++)
      V[r] = cI[r] + sgi * is[jj] * Ix[jj][r] + va[q] * is[ja] * Ix[ja][r] + vb[q] * is[jb] * Ix[jb][r] - o[r];
    px[q] = dot3(V, Rx[ku]);
    py[q] = dot3(V, Rx[kv]);
    pz[q] = dot3(V, nr);
  }
  real cx[BB_MAXC], cy[BB_MAXC], cz[BB_MAXC];
  int nc = 0;
  /* (a) incident vertices inside the rectangle */
  for (int q = 0; q < 4; q++)
    if (FABS(px[q]) <= hu && FABS(py[q]) <= hv) { cx[nc] = px[q]; cy[nc] = py[q]; cz[nc] = pz[q]; nc++; }
  /* (b) incident edges crossing the rectangle's sides */
  for (int q = 0; q < 4; q++) {
    const int q1 = (q + 1) & 3;
    for (int sd = 0; sd < 4; sd++) {
      const int isx = sd < 2;
      const real X = (sd & 1) ? (isx ? hu : hv) : (isx ? -hu : -hv);
      const real e0 = isx ? px[q] : py[q], e1 = isx ? px[q1] : py[q1];
      if (!((e0 - X) * (e1 - X) < 0)) continue;
      const real t = (X - e0) / (e1 - e0);
      const real oth = isx ? py[q] + t * (py[q1] - py[q]) : px[q] + t * (px[q1] - px[q]);
      if (FABS(oth) > (isx ? hv : hu)) continue;
      cx[nc] = isx ? X : oth;
      cy[nc] = isx ? oth : X;
      cz[nc] = pz[q] + t * (pz[q1] - pz[q]);
      nc++;
    }
  }
  /* (c) rectangle corners inside the incident quadrilateral, on its plane */
  {
    real ni[3];
    for (int r = 0; r < 3; r++) ni[r] = sgi * Ix[jj][r];
    const real nx = dot3(ni, Rx[ku]), ny = dot3(ni, Rx[kv]), nz = dot3(ni, nr);
    static const real ca[4] = {-1, 1, 1, -1}, cb[4] = {-1, -1, 1, 1};
    for (int q = 0; q < 4; q++) {
      const real X = ca[q] * hu, Y = cb[q] * hv;
      int pos_ = 0, neg_ = 0;
      for (int e = 0; e < 4; e++) {
        const int e1 = (e + 1) & 3;
        const real cr = (px[e1] - px[e]) * (Y - py[e]) - (py[e1] - py[e]) * (X - px[e]);
        pos_ += cr >= 0;
        neg_ += cr <= 0;
      }
      if (pos_ < 4 && neg_ < 4) continue;
      cx[nc] = X;
      cy[nc] = Y;
      cz[nc] = pz[0] - (nx * (X - px[0]) + ny * (Y - py[0])) / nz;
      nc++;
    }
  }
  /* contacts within the margin; a candidate within 1e-6 (x and y) of an earlier one within the margin
     is a duplicate and dropped */
  int keep[BB_MAXC], nk = 0;
  for (int q = 0; q < nc; q++) {
    if (!(cz[q] <= margin)) continue;
    int dup = 0;
    for (int e = 0; e < q; e++)
      if (cz[e] <= margin && FABS(cx[q] - cx[e]) <= (real)1e-6 && FABS(cy[q] - cy[e]) <= (real)1e-6) dup = 1;
    if (!dup) keep[nk++] = q;
  }
  int sel[4], ns = 0;
  if (nk <= 4) {
    for (int q = 0; q < nk; q++) sel[ns++] = keep[q];
  } else {
    int ia = keep[0];
    for (int q = 1; q < nk; q++)
      if (cz[keep[q]] < cz[ia]) ia = keep[q];
    int ib = ia;
    real bm = -1;
    for (int q = 0; q < nk; q++) {
      const int p = keep[q];
      const real dd = (cx[p] - cx[ia]) * (cx[p] - cx[ia]) + (cy[p] - cy[ia]) * (cy[p] - cy[ia]);
      if (dd > bm) { bm = dd; ib = p; }
    }
    int ic = ia;
    bm = -1;
    for (int q = 0; q < nk; q++) {
      const int p = keep[q];
      const real dd = FABS((cx[ib] - cx[ia]) * (cy[p] - cy[ia]) - (cy[ib] - cy[ia]) * (cx[p] - cx[ia]));
      if (dd > bm) { bm = dd; ic = p; }
    }
    int id = ia;
    bm = -1;
    for (int pass = 0; pass < 2; pass++) {
      const int s0 = pass == 0 ? ib : ia;
      for (int q = 0; q < nk; q++) {
        const int p = keep[q];
        const real dd = FABS((cx[s0] - cx[ic]) * (cy[s0] - cy[p]) - (cy[s0] - cy[ic]) * (cx[s0] - cx[p]));
        if (dd > bm) { bm = dd; id = p; }
      }
    }
    const int cand[4] = {ia, ib, ic, id};
    for (int q = 0; q < 4; q++) {
      int dup = 0;
      for (int e = 0; e < ns; e++) dup |= sel[e] == cand[q];
      if (!dup) sel[ns++] = cand[q];
    }
  }
  for (int q = 0; q < ns; q++) {
    const int p = sel[q];
    for (int r = 0; r < 3; r++)
      pos[q][r] = o[r] + cx[p] * Rx[ku][r] + cy[p] * Rx[kv][r] + (real)0.5 * cz[p] * nr[r];
    dist[q] = cz[p];
  }
  return ns;
}

/* mju_makeFrame for a contact normal: t1 = (0,1,0) (or (0,0,1) when |n_y| >= 0.5) made orthogonal to
   n and normalised, t2 = n x t1 */
static void make_frame(const real n[3], real t1[3], real t2[3]) {
  real y[3] = {0, 1, 0};
  if (!(FABS(n[1]) < (real)0.5)) { y[1] = 0; y[2] = 1; }
  const real d = dot3(n, y);
  for (int k = 0; k < 3; k++) t1[k] = y[k] - d * n[k];
  const real ln = SQRT(dot3(t1, t1));
  for (int k = 0; k < 3; k++) t1[k] /= ln;
  cross3(t2, n, t1);
}

/* the sole pair's contacts (ZbModel.npair): box-box of geoms pair_geom[0] (geom1) and [1] (geom2) */
static void pair_collision(const ZbModel* m, ZbData* d) {
  if (m->npair < 1) return;
  const int g1 = m->pair_geom[0], g2 = m->pair_geom[1];
  real pos[4][3], dist[4], n[3];
  const int nc = box_box(d->geom_xpos[g1], d->geom_xmat[g1], m->geom_size[g1], d->geom_xpos[g2], d->geom_xmat[g2],
                         m->geom_size[g2], m->pair_margin, pos, dist, n);
  real t1[3], t2[3];
  if (nc > 0) make_frame(n, t1, t2);
  for (int q = 0; q < nc && d->ncon < NCON; q++) {
    const int c = d->ncon++;
    for (int k = 0; k < 3; k++) {
      d->con_pos[c][k] = pos[q][k];
      d->con_n[c][k] = n[k];
      d->con_t1[c][k] = t1[k];
      d->con_t2[c][k] = t2[k];
    }
    d->con_dist[c] = dist[q];
    d->con_geom[c] = g2;
    d->con_geom1[c] = g1;
    d->con_mu[c] = m->pair_friction[0];
  }
}

/* box_box for the known-answer tests (tests/test_colliders.py); frames as 3x3 row-major rotations */
int zbo_box_box(const float* c1, const float* R1, const float* s1, const float* c2, const float* R2, const float* s2,
                float margin, float* pos, float* dist, float* nrm) {
  real a[3], b[3], Ra[9], Rb[9], p[4][3], dd[4], n[3];
  for (int k = 0; k < 3; k++) { a[k] = c1[k]; b[k] = c2[k]; }
  for (int k = 0; k < 9; k++) { Ra[k] = R1[k]; Rb[k] = R2[k]; }
  const int nc = box_box(a, Ra, s1, b, Rb, s2, margin, p, dd, n);
  for (int q = 0; q < nc; q++) {
    for (int k = 0; k < 3; k++) pos[3 * q + k] = (float)p[q][k];
    dist[q] = (float)dd[q];
  }
  for (int k = 0; k < 3; k++) nrm[k] = (float)n[k];
  return nc;
}

/* ------------------------- plane - convex mesh -------------------------------
 * MJX's plane_convex with its _manifold_points (mjx/_src/collision_convex.py) [U: mujoco-mjx 3.3.4
 * is not on disk; restated from its published method]. In the geom frame (R, c the geom's world
 * rotation and centre; v_i its hull vertices, i < nv, in the model's order):
 *   n = R' e_z, the plane normal; p = R' (0 - c), the plane's origin;
 *   support_i = (p - v_i) . n, the depth of vertex i below the plane;
 *   mask_i = support_i > max(0, max_j support_j - 1e-3): penetrating, within a 1 mm skin of the deepest;
 *   every argmax below is over w_i = value_i + (mask_i ? 0 : -1e6), the first index on ties:
 *   a = argmax w (the first masked vertex); b = argmax |a - v_i|^2 (the farthest from a);
 *   c = argmax |(a - v_i) . (n x (a - b))| (the farthest from the line ab);
 *   d = the first maximum of |(b - v_i) . (n x (b - c))| over i, then of |(a - v_i) . (n x (a - c))|.
 * Contacts q = a, b, c, d (in this order): dist = -support (1 for a repeat of an earlier index),
 * position the vertex in the world moved by -dist/2 along the plane normal, frame mju_makeFrame(+z).
 * As for the other colliders, a contact exists where dist <= the margin. Writes the four candidates'
 * vertex indices, distances and world positions (before the half-distance shift); returns how many
 * pass the margin. */
static int plane_mesh(const float (*vert)[4], int nv, const real R[9], const real c[3], real margin, int idx[4],
                      real dist[4], real pos[4][3]) {
  const real n[3] = {R[6], R[7], R[8]};
  const real mc[3] = {-c[0], -c[1], -c[2]};
  real p[3];
  mulmtv3(p, R, mc);
  real sup[ZB_MAX_MESHV], smax = (real)-1e30;
  for (int i = 0; i < nv; i++) {
    const real dv[3] = {p[0] - vert[i][0], p[1] - vert[i][1], p[2] - vert[i][2]};
    sup[i] = dot3(dv, n);
    if (sup[i] > smax) smax = sup[i];
  }
  const real thr = smax - (real)1e-3 > 0 ? smax - (real)1e-3 : (real)0;
  real dm[ZB_MAX_MESHV];
  for (int i = 0; i < nv; i++) dm[i] = sup[i] > thr ? (real)0 : (real)-1e6;
  int ia = 0;
  for (int i = 1; i < nv; i++)
    if (dm[i] > dm[ia]) ia = i;
  const real A[3] = {vert[ia][0], vert[ia][1], vert[ia][2]};
  int ib = 0;
  real best = 0;
  for (int i = 0; i < nv; i++) {
    const real e0 = A[0] - vert[i][0], e1 = A[1] - vert[i][1], e2 = A[2] - vert[i][2];
    const real w = (e0 * e0 + e1 * e1 + e2 * e2) + dm[i];
    if (i == 0 || w > best) { best = w; ib = i; }
  }
  const real B[3] = {vert[ib][0], vert[ib][1], vert[ib][2]};
  real ab[3];
  {
    const real amb[3] = {A[0] - B[0], A[1] - B[1], A[2] - B[2]};
    cross3(ab, n, amb);
  }
  int ic = 0;
  for (int i = 0; i < nv; i++) {
    const real ap[3] = {A[0] - vert[i][0], A[1] - vert[i][1], A[2] - vert[i][2]};
    const real w = FABS(dot3(ap, ab)) + dm[i];
    if (i == 0 || w > best) { best = w; ic = i; }
  }
  const real C[3] = {vert[ic][0], vert[ic][1], vert[ic][2]};
  real ac[3], bc[3];
  {
    const real amc[3] = {A[0] - C[0], A[1] - C[1], A[2] - C[2]};
    const real bmc[3] = {B[0] - C[0], B[1] - C[1], B[2] - C[2]};
    cross3(ac, n, amc);
    cross3(bc, n, bmc);
  }
  int id = 0;
  for (int j = 0; j < 2 * nv; j++) {
    const int i = j < nv ? j : j - nv;
    const real* o = j < nv ? B : A;
    const real* ax = j < nv ? bc : ac;
    const real op[3] = {o[0] - vert[i][0], o[1] - vert[i][1], o[2] - vert[i][2]};
    const real w = FABS(dot3(op, ax)) + dm[i];
    if (j == 0 || w > best) { best = w; id = i; }
  }
  idx[0] = ia; idx[1] = ib; idx[2] = ic; idx[3] = id;
  int cnt = 0;
  for (int q = 0; q < 4; q++) {
    int uniq = 1;
    for (int r = 0; r < q; r++)
      if (idx[r] == idx[q]) uniq = 0;
    dist[q] = uniq ? -sup[idx[q]] : (real)1;
    const real v[3] = {vert[idx[q]][0], vert[idx[q]][1], vert[idx[q]][2]};
    real w[3];
    mulmv3(w, R, v);
    for (int k = 0; k < 3; k++) pos[q][k] = c[k] + w[k];
    if (dist[q] <= margin) cnt++;
  }
  return cnt;
}

/* plane_mesh for the known-answer tests (tests/test_colliders.py): R row-major, verts [nv][4] */
int zbo_plane_mesh(const float* verts, int nv, const float* R, const float* c, float margin, int* idx, float* dist,
                   float* pos) {
  real Rr[9], cr[3], dd[4], pp[4][3];
  for (int k = 0; k < 9; k++) Rr[k] = R[k];
  for (int k = 0; k < 3; k++) cr[k] = c[k];
  if (nv < 1 || nv > ZB_MAX_MESHV) return -1;
  const int cnt = plane_mesh((const float(*)[4])verts, nv, Rr, cr, margin, idx, dd, pp);
  for (int q = 0; q < 4; q++) {
    dist[q] = (float)dd[q];
    for (int k = 0; k < 3; k++) pos[3 * q + k] = (float)pp[q][k];
  }
  return cnt;
}

static void collision(const ZbModel* m, ZbData* d) {
  static const real ty[3] = {0, 1, 0};
  d->ncon = 0;
  const real margin = m->floor_margin;
  for (int g = 0; g < m->ngeom; g++) {
    const real* R = d->geom_xmat[g];
    const real* c = d->geom_xpos[g];
    const float* sz = m->geom_size[g];
    if (m->geom_type[g] == ZB_GEOM_BOX) {
      int cnt = 0;
      for (int i = 0; i < 8 && cnt < 4; i++) {
        real loc[3] = {(i & 1) ? sz[0] : -sz[0], (i & 2) ? sz[1] : -sz[1], (i & 4) ? sz[2] : -sz[2]}, w[3];
        mulmv3(w, R, loc);
        const real dist = c[2] + w[2];
        if (w[2] <= 0) track_clearance(d, dist, margin);
        if (dist > margin || w[2] > 0) continue;
        real p[3] = {c[0] + w[0], c[1] + w[1], c[2] + w[2]};
        add_contact(m, d, g, p, dist, ty);
        cnt++;
      }
    } else if (m->geom_type[g] == ZB_GEOM_CAPSULE) {
      /* axis = local z in the world; b = its projection on the plane, normalised */
      real ax[3] = {R[2], R[5], R[8]};
      real b[3] = {ax[0], ax[1], 0};
      real bn = SQRT(b[0] * b[0] + b[1] * b[1]);
      real t1[3];
      if (bn < (real)0.5) {
        t1[0] = 0; t1[1] = 1; t1[2] = 0;
      } else {
        t1[0] = b[0] / bn; t1[1] = b[1] / bn; t1[2] = 0;
      }
      for (int e = 0; e < 2; e++) {
        const real sg = e == 0 ? 1 : -1;
        real p[3] = {c[0] + sg * sz[1] * ax[0], c[1] + sg * sz[1] * ax[1], c[2] + sg * sz[1] * ax[2] - sz[0]};
        const real dist = p[2];
        track_clearance(d, dist, margin);
        if (dist > margin) continue;
        add_contact(m, d, g, p, dist, t1);
      }
    } else if (m->geom_type[g] == ZB_GEOM_SPHERE) {
      real p[3] = {c[0], c[1], c[2] - sz[0]};
      const real dist = p[2];
      track_clearance(d, dist, margin);
      if (dist <= margin) add_contact(m, d, g, p, dist, ty);
    } else if (m->geom_type[g] == ZB_GEOM_ELLIPSOID) {
      /* R' n with n = +z: the z components of the geom's axes, row 2 of R */
      real sn[3], loc[3], w[3];
      for (int k = 0; k < 3; k++) sn[k] = sz[k] * R[6 + k];
      const real nrm = SQRT(sn[0] * sn[0] + sn[1] * sn[1] + sn[2] * sn[2]);
      for (int k = 0; k < 3; k++) loc[k] = -sz[k] * sn[k] / nrm;
      mulmv3(w, R, loc);
      real p[3] = {c[0] + w[0], c[1] + w[1], c[2] + w[2]};
      const real dist = p[2];
      track_clearance(d, dist, margin);
      if (dist <= margin) add_contact(m, d, g, p, dist, ty);
    } else if (m->geom_type[g] == ZB_GEOM_CYLINDER) {
      /* the plane: normal n = +z through the origin, so dot(x, n) = x[2] */
      real a[3] = {R[2], R[5], R[8]};
      real prja = a[2];
      if (prja > 0) {
        for (int k = 0; k < 3; k++) a[k] = -a[k];
        prja = -prja;
      }
      const real dist0 = c[2];
      real v[3] = {a[0] * prja, a[1] * prja, a[2] * prja - 1};
      const real len = SQRT(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
      if (len >= MINVAL) {
        for (int k = 0; k < 3; k++) v[k] *= sz[0] / len;
      } else {
        v[0] = R[0] * sz[0];
        v[1] = R[3] * sz[0];
        v[2] = R[6] * sz[0];
      }
      const real prjv = v[2];
      for (int k = 0; k < 3; k++) a[k] *= sz[1];
      prja *= sz[1];
      const real d1 = dist0 + prja + prjv;
      track_clearance(d, d1, margin);
      if (d1 <= margin) {
        real p[3] = {c[0] + v[0] + a[0], c[1] + v[1] + a[1], c[2] + v[2] + a[2]};
        add_contact(m, d, g, p, d1, ty);
        const real d2 = dist0 - prja + prjv;
        if (d2 <= margin) {
          real q[3] = {c[0] + v[0] - a[0], c[1] + v[1] - a[1], c[2] + v[2] - a[2]};
          add_contact(m, d, g, q, d2, ty);
        }
        const real d3 = dist0 + prja - (real)0.5 * prjv;
        if (d3 <= margin) {
          real v1[3] = {v[1] * a[2] - v[2] * a[1], v[2] * a[0] - v[0] * a[2], v[0] * a[1] - v[1] * a[0]};
          const real n1 = SQRT(v1[0] * v1[0] + v1[1] * v1[1] + v1[2] * v1[2]);
          const real s1 = n1 > 0 ? sz[0] * SQRT((real)3) * (real)0.5 / n1 : (real)0;
          for (int k = 0; k < 3; k++) v1[k] *= s1;
          for (int e = 0; e < 2; e++) {
            const real sg = e == 0 ? (real)1 : (real)-1;
            real q[3] = {c[0] + a[0] - (real)0.5 * v[0] + sg * v1[0], c[1] + a[1] - (real)0.5 * v[1] + sg * v1[1],
                         c[2] + a[2] - (real)0.5 * v[2] + sg * v1[2]};
            add_contact(m, d, g, q, d3, ty);
          }
        }
      }
    } else if (m->geom_type[g] == ZB_GEOM_MESH) {
      int idx[4];
      real dist[4], pos[4][3];
      plane_mesh((const float(*)[4])m->mesh_vert[m->geom_vertadr[g]], m->geom_vertnum[g], R, c, margin, idx, dist, pos);
      for (int q = 0; q < 4; q++) {
        if (dist[q] < (real)1e29) track_clearance(d, dist[q], margin);
        if (dist[q] <= margin) add_contact(m, d, g, pos[q], dist[q], ty);
      }
    }
  }
  pair_collision(m, d);
}

/* ----------------------- constraint construction -------------------------- */
static real impedance(const float* solimp, real x_abs) {
  real dmin = solimp[0], dmax = solimp[1], width = solimp[2], mid = solimp[3], power = solimp[4];
  real imp;
  if (width <= MINVAL || x_abs >= width) {
    imp = dmax;
  } else {
    real x = x_abs / width, y;
    if (power == 1) {
      y = x;
    } else if (x <= mid) {
      y = POW(x, power) / POW(mid, power - 1);
    } else {
      y = 1 - POW(1 - x, power) / POW(1 - mid, power - 1);
    }
    imp = dmin + y * (dmax - dmin);
  }
  if (imp < MINIMP) imp = MINIMP;
  if (imp > MAXIMP) imp = MAXIMP;
  return imp;
}

static void add_row_params(ZbData* d, int r, const float* solref, const float* solimp, real dA, real dt) {
  real timeconst = solref[0], dampratio = solref[1], dmax = solimp[1];
  if (timeconst < 2 * dt) timeconst = 2 * dt; /* refsafe */
  real b = 2 / (dmax * timeconst);
  real k = 1 / (dmax * dmax * timeconst * timeconst * dampratio * dampratio);
  real imp = impedance(solimp, FABS(d->efc_pos[r]));
  real R = (1 - imp) / imp * dA;
  if (R < MINVAL) R = MINVAL;
  d->efc_R[r] = R;
  d->efc_D[r] = 1 / R;
  real vel = 0;
  for (int j = 0; j < NDOF; j++) vel += d->efc_J[r][j] * d->qvel[j];
  d->efc_aref[r] = -b * vel - k * imp * d->efc_pos[r];
}

static void point_jac_row(const ZbModel* m, const ZbData* d, int body, const real pt[3], const real dir[3],
                          real* row) {
  const real* c = d->subtree_com[1];
  real off[3] = {pt[0] - c[0], pt[1] - c[1], pt[2] - c[2]};
  for (int j = 0; j < NDOF; j++) row[j] = 0;
  for (int j = m->body_lastdof[body]; j >= 0; j = m->dof_parent[j]) {
    real t[3];
    cross3(t, d->cdof[j], off);
    real jp[3] = {d->cdof[j][3] + t[0], d->cdof[j][4] + t[1], d->cdof[j][5] + t[2]};
    row[j] = dot3(jp, dir);
  }
}

static void make_constraint(const ZbModel* m, ZbData* d, real dt) {
  int nv = m->nv, r = 0;
  /* frictionloss rows (dofs) */
  for (int j = 0; j < nv; j++) {
    if (d->dof_frictionloss[j] > 0) {
      memset(d->efc_J[r], 0, sizeof(d->efc_J[r]));
      d->efc_J[r][j] = 1;
      d->efc_type[r] = EFC_FRICTION;
      d->efc_id[r] = j;
      d->efc_pos[r] = 0;
      d->efc_floss[r] = d->dof_frictionloss[j];
      add_row_params(d, r, m->dof_solref, m->dof_solimp, m->dof_invweight0[j], dt);
      r++;
    }
  }
  /* joint limits (hinges): active when violated (margin 0) */
  for (int j = 0; j < nv; j++) {
    if (!m->dof_limited[j]) continue;
    real q = d->qpos[m->dof_qposadr[j]];
    for (int side = 0; side < 2; side++) {
      real dist = side == 0 ? q - m->dof_range[j][0] : m->dof_range[j][1] - q;
      if (dist < 0) {
        memset(d->efc_J[r], 0, sizeof(d->efc_J[r]));
        d->efc_J[r][j] = side == 0 ? 1 : -1;
        d->efc_type[r] = EFC_LIMIT;
        d->efc_id[r] = j;
        d->efc_pos[r] = dist;
        d->efc_floss[r] = 0;
        add_row_params(d, r, m->dof_solref, m->dof_solimp, m->dof_invweight0[j], dt);
        r++;
      }
    }
  }
  /* contacts: pyramidal cone, condim 3 -> 4 rows (+t1, -t1, +t2, -t2). A contact between two robot
     geoms (the sole pair) has J = J(body2) - J(body1) at the contact point (mj_jacDifPair; the root
     dofs' columns cancel exactly) and diagApprox from both bodies' translational invweight0 */
  for (int c = 0; c < d->ncon; c++) {
    int body = m->geom_body[d->con_geom[c]];
    const int b1 = d->con_geom1[c] >= 0 ? m->geom_body[d->con_geom1[c]] : -1;
    /* frame (n, t1, t2 = n x t1), collision() */
    const real* n = d->con_n[c];
    const real* t1 = d->con_t1[c];
    const real* t2 = d->con_t2[c];
    real Jn[NDOF], Jt1[NDOF], Jt2[NDOF];
    point_jac_row(m, d, body, d->con_pos[c], n, Jn);
    point_jac_row(m, d, body, d->con_pos[c], t1, Jt1);
    point_jac_row(m, d, body, d->con_pos[c], t2, Jt2);
    if (b1 >= 0) {
      real K[NDOF];
      point_jac_row(m, d, b1, d->con_pos[c], n, K);
      for (int j = 0; j < NDOF; j++) Jn[j] -= K[j];
      point_jac_row(m, d, b1, d->con_pos[c], t1, K);
      for (int j = 0; j < NDOF; j++) Jt1[j] -= K[j];
      point_jac_row(m, d, b1, d->con_pos[c], t2, K);
      for (int j = 0; j < NDOF; j++) Jt2[j] -= K[j];
    }
    real mu = d->con_mu[c];
    real tran = m->body_invweight0[body][0] + (b1 >= 0 ? m->body_invweight0[b1][0] : 0);
    real dA = tran * (1 + mu * mu);
    d->con_efc[c] = r;
    for (int e = 0; e < 4; e++) {
      const real* Jt = e < 2 ? Jt1 : Jt2;
      real s = (e & 1) ? -mu : mu;
      for (int j = 0; j < NDOF; j++) d->efc_J[r][j] = Jn[j] + s * Jt[j];
      d->efc_type[r] = EFC_CONTACT;
      d->efc_id[r] = c;
      d->efc_pos[r] = d->con_dist[c];
      d->efc_floss[r] = 0;
      if (b1 >= 0) add_row_params(d, r, m->pair_solref, m->pair_solimp, dA, dt);
      else add_row_params(d, r, m->floor_solref, m->floor_solimp, dA, dt);
      r++;
    }
  }
  d->nefc = r;
}

/* ------------------------------ Newton solver ------------------------------ */
/* constraint state at jar: force, cost, hessian activity */
static real efc_eval(const ZbData* d, int r, real jar, real* force, int* active) {
  real D = d->efc_D[r];
  if (d->efc_type[r] == EFC_FRICTION) {
    real f = d->efc_floss[r], Rf = d->efc_R[r] * f;
    if (jar <= -Rf) { *force = f; *active = 0; return -f * ((real)0.5 * Rf + jar); }
    if (jar >= Rf) { *force = -f; *active = 0; return f * (jar - (real)0.5 * Rf); }
    *force = -D * jar; *active = 1; return (real)0.5 * D * jar * jar;
  }
  if (jar < 0) { *force = -D * jar; *active = 1; return (real)0.5 * D * jar * jar; }
  *force = 0; *active = 0; return 0;
}

typedef struct {
  real Ma[NDOF], grad[NDOF], Mgrad[NDOF], search[NDOF], Mv[NDOF], Jv[MAXEFC];
  real H[NDOF][NDOF];
  real cost;
} Solver;

static real update_constraint(const ZbModel* m, ZbData* d, Solver* s) {
  int nv = m->nv;
  real cost = 0;
  for (int i = 0; i < nv; i++) cost += (real)0.5 * (s->Ma[i] - d->qfrc_smooth[i]) * (d->qacc[i] - d->qacc_smooth[i]);
  for (int r = 0; r < d->nefc; r++) cost += efc_eval(d, r, d->efc_jar[r], &d->efc_force[r], &d->efc_active[r]);
  for (int i = 0; i < nv; i++) {
    real q = 0;
    for (int r = 0; r < d->nefc; r++) q += d->efc_J[r][i] * d->efc_force[r];
    d->qfrc_constraint[i] = q;
    s->grad[i] = s->Ma[i] - d->qfrc_smooth[i] - q;
  }
  return cost;
}

/* dense Cholesky of H = M + J' D_active J (mju_cholFactor) and solve */
static void hessian_solve(const ZbModel* m, ZbData* d, Solver* s) {
  int nv = m->nv;
  for (int i = 0; i < nv; i++)
    for (int j = 0; j <= i; j++) {
      real v = d->qM[i][j]; /* zero unless j is i or an ancestor of i */
      for (int r = 0; r < d->nefc; r++)
        if (d->efc_active[r]) v += d->efc_J[r][i] * d->efc_D[r] * d->efc_J[r][j];
      s->H[i][j] = v;
    }
  for (int j = 0; j < nv; j++) {
    real v = s->H[j][j];
    for (int k = 0; k < j; k++) v -= s->H[j][k] * s->H[j][k];
    if (v < MINVAL) v = MINVAL;
    real L = SQRT(v);
    s->H[j][j] = L;
    for (int i = j + 1; i < nv; i++) {
      real w = s->H[i][j];
      for (int k = 0; k < j; k++) w -= s->H[i][k] * s->H[j][k];
      s->H[i][j] = w / L;
    }
  }
  real y[NDOF];
  for (int i = 0; i < nv; i++) {
    real v = s->grad[i];
    for (int k = 0; k < i; k++) v -= s->H[i][k] * y[k];
    y[i] = v / s->H[i][i];
  }
  for (int i = nv - 1; i >= 0; i--) {
    real v = y[i];
    for (int k = i + 1; k < nv; k++) v -= s->H[k][i] * s->Mgrad[k];
    s->Mgrad[i] = v / s->H[i][i];
  }
}

/* derivative and curvature of the line-search cost at alpha */
static void ls_eval(const ZbModel* m, const ZbData* d, const Solver* s, real c1, real c2, real alpha, real* d1,
                    real* d2) {
  (void)m;
  real g1 = c1 + alpha * c2, g2 = c2;
  for (int r = 0; r < d->nefc; r++) {
    real jv = s->Jv[r];
    if (jv == 0) continue;
    real x = d->efc_jar[r] + alpha * jv, D = d->efc_D[r];
    if (d->efc_type[r] == EFC_FRICTION) {
      real Rf = d->efc_R[r] * d->efc_floss[r];
      if (x <= -Rf) g1 -= d->efc_floss[r] * jv;
      else if (x >= Rf) g1 += d->efc_floss[r] * jv;
      else { g1 += D * x * jv; g2 += D * jv * jv; }
    } else if (x < 0) {
      g1 += D * x * jv;
      g2 += D * jv * jv;
    }
  }
  *d1 = g1;
  *d2 = g2;
}

static real line_search(const ZbModel* m, const ZbData* d, Solver* s, const ZbEnvConfig* cfg) {
  int nv = m->nv;
  mul_m(m, d->qM, s->search, s->Mv);
  for (int r = 0; r < d->nefc; r++) {
    real v = 0;
    for (int j = 0; j < nv; j++) v += d->efc_J[r][j] * s->search[j];
    s->Jv[r] = v;
  }
  real c1 = 0, c2 = 0;
  for (int i = 0; i < nv; i++) {
    c1 += s->search[i] * (s->Ma[i] - d->qfrc_smooth[i]);
    c2 += s->search[i] * s->Mv[i];
  }
  real d1, d2;
  ls_eval(m, d, s, c1, c2, 0, &d1, &d2);
  if (!(d1 < 0) || !(d2 > 0)) return 0;
  real gtol = (real)cfg->ls_tolerance * (-d1);
  real lo = 0, hi = -1; /* hi < 0: unbounded */
  real alpha = -d1 / d2;
  for (int it = 0; it < cfg->ls_iterations; it++) {
    ls_eval(m, d, s, c1, c2, alpha, &d1, &d2);
    if (FABS(d1) <= gtol) break;
    if (d1 < 0) lo = alpha; else hi = alpha;
    real an = alpha - d1 / d2;
    if (!(an > lo) || (hi >= 0 && !(an < hi))) an = (real)0.5 * (lo + (hi >= 0 ? hi : 2 * alpha));
    alpha = an;
  }
  return alpha;
}

/* warmstart: qacc_warmstart vs qacc_smooth, keep the cheaper (mj_fwdConstraint); sets qacc,
   s->Ma and efc_jar */
static void warmstart(const ZbModel* m, ZbData* d, Solver* sp) {
  int nv = m->nv;
  Solver* s = sp;
  {
    real jar_w[MAXEFC], cost_w = 0, cost_s = 0, f;
    int act;
    for (int i = 0; i < nv; i++) d->qacc[i] = d->qacc_warm[i];
    mul_m(m, d->qM, d->qacc, s->Ma);
    for (int i = 0; i < nv; i++) cost_w += (real)0.5 * (s->Ma[i] - d->qfrc_smooth[i]) * (d->qacc[i] - d->qacc_smooth[i]);
    for (int r = 0; r < d->nefc; r++) {
      real v = 0, v2 = 0;
      for (int j = 0; j < nv; j++) {
        v += d->efc_J[r][j] * d->qacc[j];
        v2 += d->efc_J[r][j] * d->qacc_smooth[j];
      }
      jar_w[r] = v - d->efc_aref[r];
      cost_w += efc_eval(d, r, jar_w[r], &f, &act);
      cost_s += efc_eval(d, r, v2 - d->efc_aref[r], &f, &act);
    }
    if (cost_w > cost_s) {
      for (int i = 0; i < nv; i++) d->qacc[i] = d->qacc_smooth[i];
      mul_m(m, d->qM, d->qacc, s->Ma);
      for (int r = 0; r < d->nefc; r++) {
        real v = 0;
        for (int j = 0; j < nv; j++) v += d->efc_J[r][j] * d->qacc[j];
        d->efc_jar[r] = v - d->efc_aref[r];
      }
    } else {
      for (int r = 0; r < d->nefc; r++) d->efc_jar[r] = jar_w[r];
    }
  }
}

static void solve_newton(const ZbModel* m, ZbData* d, const ZbEnvConfig* cfg) {
  int nv = m->nv;
  Solver s;
  warmstart(m, d, &s);
  real scale = (real)1 / (m->meaninertia * (nv > 1 ? nv : 1));
  s.cost = update_constraint(m, d, &s);
  hessian_solve(m, d, &s);
  for (int i = 0; i < nv; i++) s.search[i] = -s.Mgrad[i];
  int iter = 0;
  while (iter < cfg->iterations) {
    real alpha = line_search(m, d, &s, cfg);
    if (alpha == 0) break;
    for (int i = 0; i < nv; i++) {
      d->qacc[i] += alpha * s.search[i];
      s.Ma[i] += alpha * s.Mv[i];
    }
    for (int r = 0; r < d->nefc; r++) d->efc_jar[r] += alpha * s.Jv[r];
    real oldcost = s.cost;
    s.cost = update_constraint(m, d, &s);
    hessian_solve(m, d, &s);
    iter++;
    real improvement = scale * (oldcost - s.cost);
    real gn = 0;
    for (int i = 0; i < nv; i++) gn += s.grad[i] * s.grad[i];
    real gradient = scale * SQRT(gn);
    if (improvement < cfg->tolerance || gradient < cfg->tolerance) break;
    for (int i = 0; i < nv; i++) s.search[i] = -s.Mgrad[i];
  }
  d->solver_iters += iter;
}

/* Primal nonlinear conjugate gradient (mj_solCG; MJX solver.py with SolverType.CG): the same
   warmstart, cost, exact line search and termination test as Newton; the direction is the
   M^-1-preconditioned gradient (mj_solveM with the smooth factor qLD) with Polak-Ribiere
   beta = max(0, grad . (Mgrad - Mgrad_prev) / max(MINVAL, grad_prev . Mgrad_prev)), and no
   Hessian. As in solve_newton, an iteration that terminates skips the direction update, which
   only feeds the next iteration. */
static void solve_cg(const ZbModel* m, ZbData* d, const ZbEnvConfig* cfg) {
  int nv = m->nv;
  Solver s;
  warmstart(m, d, &s);
  real scale = (real)1 / (m->meaninertia * (nv > 1 ? nv : 1));
  s.cost = update_constraint(m, d, &s);
  for (int i = 0; i < nv; i++) s.Mgrad[i] = s.grad[i];
  solve_m(m, d->qLD, d->qLDinv, s.Mgrad);
  for (int i = 0; i < nv; i++) s.search[i] = -s.Mgrad[i];
  int iter = 0;
  while (iter < cfg->iterations) {
    real alpha = line_search(m, d, &s, cfg);
    if (alpha == 0) break;
    for (int i = 0; i < nv; i++) {
      d->qacc[i] += alpha * s.search[i];
      s.Ma[i] += alpha * s.Mv[i];
    }
    for (int r = 0; r < d->nefc; r++) d->efc_jar[r] += alpha * s.Jv[r];
    real oldcost = s.cost, gold[NDOF], mgold[NDOF];
    for (int i = 0; i < nv; i++) {
      gold[i] = s.grad[i];
      mgold[i] = s.Mgrad[i];
    }
    s.cost = update_constraint(m, d, &s);
    iter++;
    real improvement = scale * (oldcost - s.cost);
    real gn = 0;
    for (int i = 0; i < nv; i++) gn += s.grad[i] * s.grad[i];
    real gradient = scale * SQRT(gn);
    if (improvement < cfg->tolerance || gradient < cfg->tolerance) break;
    for (int i = 0; i < nv; i++) s.Mgrad[i] = s.grad[i];
    solve_m(m, d->qLD, d->qLDinv, s.Mgrad);
    real num = 0, den = 0;
    for (int i = 0; i < nv; i++) {
      num += s.grad[i] * (s.Mgrad[i] - mgold[i]);
      den += gold[i] * mgold[i];
    }
    real beta = num / (den > MINVAL ? den : MINVAL);
    if (!(beta > 0)) beta = 0;
    for (int i = 0; i < nv; i++) s.search[i] = -s.Mgrad[i] + beta * s.search[i];
  }
  d->solver_iters += iter;
}

/* --------------------------- full forward pass ----------------------------- */
static void forward(const ZbModel* m, ZbData* d, real dt, const ZbEnvConfig* cfg) {
  kinematics(m, d);
  com_pos(m, d);
  crb(m, d);
  memcpy(d->qLD, d->qM, sizeof(d->qM));
  factor_m(m, d->qLD, d->qLDinv);
  collision(m, d);
  com_vel(m, d);
  make_constraint(m, d, dt);
  smooth_forces(m, d);
  if (d->nefc == 0) {
    for (int i = 0; i < m->nv; i++) {
      d->qacc[i] = d->qacc_smooth[i];
      d->qfrc_constraint[i] = 0;
    }
  } else if (cfg->solver == ZB_SOLVER_CG) {
    solve_cg(m, d, cfg);
  } else {
    solve_newton(m, d, cfg);
  }
}

/* --------------------- sensors (after the constraint solve) ----------------- */
static void sensors(const ZbModel* m, ZbData* d) {
  /* contact forces on bodies (cfrc_ext) and touch */
  memset(d->cfrc_ext, 0, sizeof(d->cfrc_ext));
  d->touch[0] = d->touch[1] = 0;
  const real* c = d->subtree_com[1];
  for (int k = 0; k < d->ncon; k++) {
    int r = d->con_efc[k];
    real f0 = d->efc_force[r], f1 = d->efc_force[r + 1], f2 = d->efc_force[r + 2], f3 = d->efc_force[r + 3];
    real fn = f0 + f1 + f2 + f3, mu = d->con_mu[k];
    real ft1 = mu * (f0 - f1), ft2 = mu * (f2 - f3);
    /* world force on geom2's body = fn*n + ft1*t1 + ft2*t2 (geom1's body, when it is not the
       floor, takes the opposite: mj_rnePostConstraint) */
    const real *nn = d->con_n[k], *t1 = d->con_t1[k], *t2 = d->con_t2[k];
    real F[3];
    for (int a = 0; a < 3; a++) F[a] = fn * nn[a] + ft1 * t1[a] + ft2 * t2[a];
    int g = d->con_geom[k], g1 = d->con_geom1[k];
    int body = m->geom_body[g];
    real off[3] = {d->con_pos[k][0] - c[0], d->con_pos[k][1] - c[1], d->con_pos[k][2] - c[2]}, tq[3];
    cross3(tq, off, F);
    for (int a = 0; a < 3; a++) {
      d->cfrc_ext[body][a] += tq[a];
      d->cfrc_ext[body][3 + a] += F[a];
    }
    if (g1 >= 0) {
      const int b1 = m->geom_body[g1];
      for (int a = 0; a < 3; a++) {
        d->cfrc_ext[b1][a] -= tq[a];
        d->cfrc_ext[b1][3 + a] -= F[a];
      }
    }
    /* touch: the normal force of the contacts of the sensor's geom (either side of the pair) */
    if (g == m->geom_left_foot || g1 == m->geom_left_foot) d->touch[0] += fn;
    if (g == m->geom_right_foot || g1 == m->geom_right_foot) d->touch[1] += fn;
  }
  /* mj_rnePostConstraint: cacc with qacc, cfrc_int */
  real cacc[NB][6], cfrc[NB][6];
  rne(m, d, 1, cacc, cfrc);
  /* imu: framequat, gyro, accelerometer */
  int s = m->site_imu, b = m->site_body[s];
  for (int k = 0; k < 4; k++) d->imu_framequat[k] = d->site_xquat[s][k];
  const real* R = d->site_xmat[s];
  real dif[3] = {d->site_xpos[s][0] - c[0], d->site_xpos[s][1] - c[1], d->site_xpos[s][2] - c[2]};
  real w[3] = {d->cvel[b][0], d->cvel[b][1], d->cvel[b][2]}, t[3];
  mulmtv3(d->imu_gyro, R, w);
  /* linear velocity and acceleration at the site (mju_transformSpatial) */
  real v[3], a[3];
  cross3(t, w, dif);
  for (int k = 0; k < 3; k++) v[k] = d->cvel[b][3 + k] + t[k];
  real aw[3] = {cacc[b][0], cacc[b][1], cacc[b][2]};
  cross3(t, aw, dif);
  for (int k = 0; k < 3; k++) a[k] = cacc[b][3 + k] + t[k];
  cross3(t, w, v);
  for (int k = 0; k < 3; k++) a[k] += t[k];
  mulmtv3(d->imu_acc, R, a);
  /* force sensors at the foot sites: interaction force of the foot body, site frame */
  int fs[2] = {m->site_left_foot, m->site_right_foot};
  for (int side = 0; side < 2; side++) {
    int ss = fs[side], fb = m->site_body[ss];
    real F[3] = {cfrc[fb][3], cfrc[fb][4], cfrc[fb][5]};
    mulmtv3(d->force[side], d->site_xmat[ss], F);
  }
}

/* -------------------------------- mj_Euler ---------------------------------- */
/* eulerdamp (ZB_F_EULERDAMP, MuJoCo's default when mjDSBL_EULERDAMP is clear; engine_forward.c
   mj_Euler, MJX forward.py euler): the joint damping is integrated implicitly,
   qacc_e = (M + dt diag(dof_damping))^-1 (qfrc_smooth + qfrc_constraint), by the same tree L'DL as
   mj_factorM / mj_solveM, and qvel advances with qacc_e. d->qacc (sensors, the warmstart saved by
   mj_advance) stays the solver's. Without it qvel advances with qacc (explicit damping, inside
   qfrc_smooth's passive force). */
static void integrate(const ZbModel* m, ZbData* d, real dt, int eulerdamp) {
  int nv = m->nv;
  real qacc_e[NDOF];
  if (eulerdamp) {
    real H[NDOF][NDOF], Hinv[NDOF];
    memcpy(H, d->qM, sizeof(H));
    for (int j = 0; j < nv; j++) {
      H[j][j] += dt * d->dof_damping[j];
      qacc_e[j] = d->qfrc_smooth[j] + d->qfrc_constraint[j];
    }
    factor_m(m, H, Hinv);
    solve_m(m, H, Hinv, qacc_e);
  } else {
    for (int j = 0; j < nv; j++) qacc_e[j] = d->qacc[j];
  }
  for (int j = 0; j < nv; j++) d->qvel[j] += dt * qacc_e[j];
  for (int i = 1; i < m->nbody; i++) {
    int qa = m->body_qposadr[i], da = m->body_dofadr[i];
    if (m->body_jnttype[i] == ZB_JNT_FREE) {
      for (int k = 0; k < 3; k++) d->qpos[qa + k] += dt * d->qvel[da + k];
      /* mju_quatIntegrate: q <- q * exp(0.5 * w * dt), body-frame w */
      real w[3] = {d->qvel[da + 3], d->qvel[da + 4], d->qvel[da + 5]};
      real nw = SQRT(dot3(w, w));
      real* q = &d->qpos[qa + 3];
      if (nw > MINVAL) {
        real ax[3] = {w[0] / nw, w[1] / nw, w[2] / nw}, qr[4], qn[4];
        axis_angle_quat(qr, ax, nw * dt);
        real qq[4] = {q[0], q[1], q[2], q[3]};
        quat_mul(qn, qq, qr);
        q[0] = qn[0]; q[1] = qn[1]; q[2] = qn[2]; q[3] = qn[3];
      }
      quat_normalize(q);
    } else if (m->body_jnttype[i] == ZB_JNT_HINGE) {
      d->qpos[qa] += dt * d->qvel[da];
    }
  }
}

/* ---------------------- Feetech actuator (train.py) -------------------------- */
/* trapezoidal_step, train.py:1137-1196 (elementwise) */
void zbo_trapezoidal_step(const float* pos, const float* vel, const float* target, float dt, const float* vmax,
                          const float* amax, int n, float* new_pos, float* new_vel) {
  for (int j = 0; j < n; j++) {
    real err = (real)target[j] - pos[j];
    real thr = err >= 0 ? ZB_DEADBAND : ZB_DEADBAND; /* positive / negative deadband */
    int in_db = FABS(err) <= thr;
    real db_vel = (real)vel[j] * (real)0.8;
    real db_pos = pos[j] + db_vel * dt;
    real tdir = (real)((err > 0) - (err < 0));
    real stop = FABS((real)vel[j] * vel[j]) / (2 * (real)amax[j]);
    real vdir = (real)((vel[j] > 0) - (vel[j] < 0));
    int towards = vdir * tdir >= 0;
    int accel = towards && FABS(err) > stop;
    real acc = accel ? tdir * amax[j] : -vdir * amax[j];
    if (FABS((real)vel[j]) < (real)1e-6) acc = tdir * amax[j];
    real pv = vel[j] + acc * dt;
    if (pv < -vmax[j]) pv = -vmax[j];
    if (pv > vmax[j]) pv = vmax[j];
    real pp = pos[j] + pv * dt;
    new_vel[j] = (float)(in_db ? db_vel : pv);
    new_pos[j] = (float)(in_db ? db_pos : pp);
  }
}

/* FeetechActuators.get_stateful_ctrl, train.py:1242-1280 */
static void feetech_ctrl(const ZbModel* m, ZbData* d, float* plan_pos, float* plan_vel, float* plan_tau,
                         const float* action, real dt) {
  float np[ZB_MAX_ACT], nvv[ZB_MAX_ACT];
  zbo_trapezoidal_step(plan_pos, plan_vel, action, (float)dt, m->fe_vmax, m->fe_amax, m->nu, np, nvv);
  for (int a = 0; a < m->nu; a++) {
    int d0 = m->act_dof[a];
    real q = d->qpos[m->dof_qposadr[d0]], qd = d->qvel[d0];
    real perr = (real)np[a] - q, verr = (real)nvv[a] - qd;
    real duty = (real)m->fe_kp[a] * m->fe_error_gain[a] * perr + (real)m->fe_kd[a] * verr;
    if (duty < -m->fe_max_pwm[a]) duty = -m->fe_max_pwm[a];
    if (duty > m->fe_max_pwm[a]) duty = m->fe_max_pwm[a];
    real tau = duty * m->fe_vin[a] * m->fe_kt[a] / m->fe_R[a];
    plan_pos[a] = np[a];
    plan_vel[a] = nvv[a];
    plan_tau[a] = (float)tau;
    d->ctrl[a] = tau; /* noise type "none" (train.py:1433-1436) */
  }
}

/* FeetechActuators.get_stateful_ctrl on raw arrays (KAT entry point) */
void zbo_feetech(const ZbModel* m, float dt, const float* plan_pos, const float* plan_vel, const float* action,
                 const float* q, const float* qd, float* npos, float* nvel, float* tau) {
  zbo_trapezoidal_step(plan_pos, plan_vel, action, dt, m->fe_vmax, m->fe_amax, m->nu, npos, nvel);
  for (int a = 0; a < m->nu; a++) {
    real duty = (real)m->fe_kp[a] * m->fe_error_gain[a] * ((real)npos[a] - q[a]) + (real)m->fe_kd[a] * ((real)nvel[a] - qd[a]);
    if (duty < -m->fe_max_pwm[a]) duty = -m->fe_max_pwm[a];
    if (duty > m->fe_max_pwm[a]) duty = m->fe_max_pwm[a];
    tau[a] = (float)(duty * m->fe_vin[a] * m->fe_kt[a] / m->fe_R[a]);
  }
}

/* ------------------------------- quaternions (train.py) ---------------------- */
/* rotate_quat_by_quat, train.py:751-787 */
static void rotate_quat_by_quat(const real qr_[4], const real rq_[4], int inverse, real out[4]) {
  const real eps = (real)1e-6;
  real n1 = SQRT(qr_[0] * qr_[0] + qr_[1] * qr_[1] + qr_[2] * qr_[2] + qr_[3] * qr_[3]) + eps;
  real n2 = SQRT(rq_[0] * rq_[0] + rq_[1] * rq_[1] + rq_[2] * rq_[2] + rq_[3] * rq_[3]) + eps;
  real a[4] = {rq_[0] / n2, rq_[1] / n2, rq_[2] / n2, rq_[3] / n2};
  real b[4] = {qr_[0] / n1, qr_[1] / n1, qr_[2] / n1, qr_[3] / n1};
  if (inverse) { a[1] = -a[1]; a[2] = -a[2]; a[3] = -a[3]; }
  real r[4];
  quat_mul(r, a, b);
  real n = SQRT(r[0] * r[0] + r[1] * r[1] + r[2] * r[2] + r[3] * r[3]) + eps;
  for (int k = 0; k < 4; k++) out[k] = r[k] / n;
}
void zbo_rotate_quat_by_quat(const float* q, const float* r, int inverse, float* out) {
  real a[4] = {q[0], q[1], q[2], q[3]}, b[4] = {r[0], r[1], r[2], r[3]}, o[4];
  rotate_quat_by_quat(a, b, inverse, o);
  for (int k = 0; k < 4; k++) out[k] = (float)o[k];
}

/* xax.quat_to_euler (roll, pitch) [U: xax 0.3.4] */
static void quat_roll_pitch(const real q_[4], real* roll, real* pitch) {
  real q[4] = {q_[0], q_[1], q_[2], q_[3]};
  quat_normalize(q);
  real w = q[0], x = q[1], y = q[2], z = q[3];
  *roll = ATAN2(2 * (w * x + y * z), 1 - 2 * (x * x + y * y));
  real sp = 2 * (w * y - z * x);
  if (sp > 1) sp = 1;
  if (sp < -1) sp = -1;
  *pitch = ASIN(sp);
}

/* -------------------------------------------------------------------------- */
/* env-level logic (ksim step_engine semantics [U])                            */
/* -------------------------------------------------------------------------- */
typedef struct {
  const ZbModel* m;
  const ZbEnvConfig* cfg;
  uint64_t seed;
  uint32_t env;
} EnvCtx;

static inline uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float bitsf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

static void load_params(const EnvCtx* c, ZbData* d, const float* rnd) {
  const ZbModel* m = c->m;
  int randomize = (c->cfg->flags & ZB_F_RANDOMIZE) && rnd;
  for (int i = 0; i < m->nbody; i++) {
    real s = randomize ? rnd[ZB_R_MASS + i] : 1;
    d->body_mass[i] = m->body_mass[i][0] * s;
    for (int k = 0; k < 3; k++) d->body_inertia[i][k] = m->body_inertia[i][k] * s;
  }
  for (int j = 0; j < m->nv; j++) {
    d->dof_armature[j] = m->dof_armature[j] * (randomize ? rnd[ZB_R_ARMATURE + j] : 1);
    d->dof_damping[j] = m->dof_damping[j] * (randomize ? rnd[ZB_R_DAMPING + j] : 1);
    d->dof_frictionloss[j] = m->dof_frictionloss[j] * (randomize ? rnd[ZB_R_FRICTION + j] : 1);
  }
  for (int q = 0; q < m->nq; q++) d->qpos0[q] = m->qpos0[q];
  if (randomize)
    for (int a = 0; a < m->nu; a++) d->qpos0[m->dof_qposadr[m->act_dof[a]]] += rnd[ZB_R_QPOS0 + a];
  d->floor_mu = randomize ? rnd[ZB_R_FLOOR_MU] : 1;
  int s = m->site_imu;
  for (int k = 0; k < 3; k++) d->imu_pos[k] = m->site_pos[s][k] + (randomize ? rnd[ZB_R_IMU_POS + k] : 0);
  real sq[4] = {m->site_quat[s][0], m->site_quat[s][1], m->site_quat[s][2], m->site_quat[s][3]};
  if (randomize) {
    real rq[4] = {rnd[ZB_R_IMU_QUAT], rnd[ZB_R_IMU_QUAT + 1], rnd[ZB_R_IMU_QUAT + 2], rnd[ZB_R_IMU_QUAT + 3]};
    real o[4];
    quat_mul(o, sq, rq);
    for (int k = 0; k < 4; k++) sq[k] = o[k];
  }
  for (int k = 0; k < 4; k++) d->imu_quat[k] = sq[k];
}

/* randomizer sampling (train.py:1441-1454; exact ksim laws [U]) */
static void sample_rand(const EnvCtx* c, uint32_t episode, float* rnd) {
  const ZbEnvConfig* cfg = c->cfg;
  float u[2];
  for (int i = 0; i < ZB_RAND_STRIDE; i++) rnd[i] = 0;
  for (int i = 0; i < ZB_MAX_BODY; i += 2) {
    uniform2(c->seed, P_RAND, (uint32_t)(i / 2), c->env, episode, u);
    for (int h = 0; h < 2; h++) rnd[ZB_R_MASS + i + h] = cfg->rand_mass[0] + (cfg->rand_mass[1] - cfg->rand_mass[0]) * u[h];
  }
  for (int j = 0; j < ZB_MAX_DOF; j += 2) {
    uniform2(c->seed, P_RAND, (uint32_t)(16 + j / 2), c->env, episode, u);
    for (int h = 0; h < 2; h++)
      rnd[ZB_R_ARMATURE + j + h] = cfg->rand_armature[0] + (cfg->rand_armature[1] - cfg->rand_armature[0]) * u[h];
    uniform2(c->seed, P_RAND, (uint32_t)(32 + j / 2), c->env, episode, u);
    for (int h = 0; h < 2; h++)
      rnd[ZB_R_DAMPING + j + h] = cfg->rand_damping[0] + (cfg->rand_damping[1] - cfg->rand_damping[0]) * u[h];
    uniform2(c->seed, P_RAND, (uint32_t)(48 + j / 2), c->env, episode, u);
    for (int h = 0; h < 2; h++)
      rnd[ZB_R_FRICTION + j + h] = cfg->rand_friction[0] + (cfg->rand_friction[1] - cfg->rand_friction[0]) * u[h];
  }
  for (int a = 0; a < ZB_NJ; a += 2) {
    uniform2(c->seed, P_RAND, (uint32_t)(64 + a / 2), c->env, episode, u);
    for (int h = 0; h < 2; h++) rnd[ZB_R_QPOS0 + a + h] = cfg->rand_qpos0[0] + (cfg->rand_qpos0[1] - cfg->rand_qpos0[0]) * u[h];
  }
  uniform2(c->seed, P_RAND, 74u, c->env, episode, u);
  rnd[ZB_R_FLOOR_MU] = cfg->rand_floor_mu[0] + (cfg->rand_floor_mu[1] - cfg->rand_floor_mu[0]) * u[0];
  /* imu alignment: small rotation from (tilt x, tilt y, yaw z) normals, translation normals */
  float z0[2], z1[2], z2[2];
  normal2(c->seed, P_RAND, 75u, c->env, episode, z0);
  normal2(c->seed, P_RAND, 76u, c->env, episode, z1);
  normal2(c->seed, P_RAND, 77u, c->env, episode, z2);
  real rv[3] = {cfg->rand_imu_tilt_std * z0[0], cfg->rand_imu_tilt_std * z0[1], cfg->rand_imu_yaw_std * z1[0]};
  real ang = SQRT(dot3(rv, rv)), q[4] = {1, 0, 0, 0};
  if (ang > MINVAL) {
    real ax[3] = {rv[0] / ang, rv[1] / ang, rv[2] / ang};
    axis_angle_quat(q, ax, ang);
  }
  for (int k = 0; k < 4; k++) rnd[ZB_R_IMU_QUAT + k] = (float)q[k];
  rnd[ZB_R_IMU_POS + 0] = cfg->rand_imu_pos_std * z1[1];
  rnd[ZB_R_IMU_POS + 1] = cfg->rand_imu_pos_std * z2[0];
  rnd[ZB_R_IMU_POS + 2] = cfg->rand_imu_pos_std * z2[1];
}

/* observation assembly (train.py:1478-1537, 1624-1679) */
static void observe(const EnvCtx* c, ZbData* d, float* st, float* oa, float* oc, float* ox) {
  const ZbModel* m = c->m;
  const ZbEnvConfig* cfg = c->cfg;
  uint32_t ctr = fbits(st[ZB_S_RNG_STEP]);
  /* ImuOrientationObservation.observe_stateful, train.py:853-873 (heading cmd = 0) */
  real hq[4] = {1, 0, 0, 0}, bq[4];
  rotate_quat_by_quat(d->imu_framequat, hq, 1, bq);
  if (bq[0] < 0) for (int k = 0; k < 4; k++) bq[k] = -bq[k];
  real lag = st[ZB_S_IMU_LAG];
  float imu[4];
  for (int k = 0; k < 4; k++) {
    real x = (real)st[ZB_S_IMU_EMA + k] * lag + bq[k] * (1 - lag);
    st[ZB_S_IMU_EMA + k] = (float)x;
    imu[k] = (float)x;
  }
  float acc[3] = {(float)d->imu_acc[0], (float)d->imu_acc[1], (float)d->imu_acc[2]};
  if (cfg->flags & ZB_F_OBS_NOISE) {
    float z[2];
    normal2(c->seed, P_OBS, 0, c->env, ctr, z);
    imu[0] += cfg->imu_noise_std * z[0]; imu[1] += cfg->imu_noise_std * z[1];
    normal2(c->seed, P_OBS, 1, c->env, ctr, z);
    imu[2] += cfg->imu_noise_std * z[0]; imu[3] += cfg->imu_noise_std * z[1];
    normal2(c->seed, P_OBS, 2, c->env, ctr, z);
    acc[0] += cfg->acc_noise_std * z[0]; acc[1] += cfg->acc_noise_std * z[1];
    normal2(c->seed, P_OBS, 3, c->env, ctr, z);
    acc[2] += cfg->acc_noise_std * z[0];
  }
  /* feet position in the robot frame (train.py:451-465) and touch */
  real bquat[4] = {d->qpos[3], d->qpos[4], d->qpos[5], d->qpos[6]}, bm[9];
  quat_normalize(bquat);
  quat2mat(bm, bquat);
  real fl[3], fr[3];
  mulmtv3(fl, bm, d->site_xpos[m->site_left_foot]);
  mulmtv3(fr, bm, d->site_xpos[m->site_right_foot]);
  real dfx = fl[0] - fr[0], dfy = fl[1] - fr[1], dfz = fl[2] - fr[2];
  st[ZB_S_FEET_DIST] = (float)SQRT(dfx * dfx + dfy * dfy + dfz * dfz);
  st[ZB_S_TOUCH] = (float)d->touch[0];
  st[ZB_S_TOUCH + 1] = (float)d->touch[1];

  if (oa) {
    for (int j = 0; j < ZB_NJ; j++) {
      oa[j] = (float)d->qpos[7 + j];
      oa[ZB_NJ + j] = (float)d->qvel[6 + j];
    }
    for (int k = 0; k < 4; k++) oa[40 + k] = imu[k];
    for (int k = 44; k < 50; k++) oa[k] = 0; /* zero command (train.py:1634-1636) */
  }
  if (oc) {
    int o = 0;
    for (int j = 0; j < ZB_NJ; j++) oc[o++] = (float)d->qpos[7 + j];
    for (int j = 0; j < ZB_NJ; j++) oc[o++] = (float)(d->qvel[6 + j] / 10);
    for (int i = 1; i < m->nbody; i++)
      for (int k = 0; k < 10; k++) oc[o++] = (float)d->cinert[i][k];
    for (int i = 1; i < m->nbody; i++)
      for (int k = 0; k < 6; k++) oc[o++] = (float)d->cvel[i][k];
    for (int k = 0; k < 3; k++) oc[o++] = acc[k];
    for (int k = 0; k < 3; k++) oc[o++] = (float)d->imu_gyro[k];
    for (int k = 0; k < 4; k++) oc[o++] = imu[k];
    for (int k = 0; k < ZB_NUM_CMD; k++) oc[o++] = 0;
    for (int a = 0; a < ZB_NJ; a++) oc[o++] = (float)(d->act_force[a] / 100);
    for (int k = 0; k < 3; k++) oc[o++] = (float)d->qpos[k];
    for (int k = 0; k < 4; k++) oc[o++] = (float)d->qpos[3 + k];
  }
  if (ox) {
    for (int k = 0; k < ZB_OBS_EXTRA; k++) ox[k] = 0;
    for (int k = 0; k < 3; k++) {
      ox[ZB_X_BASE_LINVEL + k] = (float)d->qvel[k];
      ox[ZB_X_BASE_ANGVEL + k] = (float)d->qvel[3 + k];
      ox[ZB_X_BASE_LINACC + k] = (float)d->qacc[k];
      ox[ZB_X_BASE_ANGACC + k] = (float)d->qacc[3 + k];
      ox[ZB_X_FORCE + k] = (float)d->force[0][k];
      ox[ZB_X_FORCE + 3 + k] = (float)d->force[1][k];
      ox[ZB_X_FEET_POS + k] = (float)fl[k];
      ox[ZB_X_FEET_POS + 3 + k] = (float)fr[k];
    }
    ox[ZB_X_BASE_HEIGHT] = (float)d->xpos[1][2];
    ox[ZB_X_TOUCH] = (float)d->touch[0];
    ox[ZB_X_TOUCH + 1] = (float)d->touch[1];
    for (int a = 0; a < ZB_NJ; a++) {
      ox[ZB_X_FEETECH_TAU + a] = st[ZB_S_PLAN_TAU + a];
      ox[ZB_X_ACT_ACC + a] = (float)d->qacc[6 + a];
    }
  }
}

static void state_to_data(const ZbModel* m, const float* st, ZbData* d) {
  for (int q = 0; q < m->nq; q++) d->qpos[q] = st[ZB_S_QPOS + q];
  for (int j = 0; j < m->nv; j++) {
    d->qvel[j] = st[ZB_S_QVEL + j];
    d->qacc_warm[j] = st[ZB_S_QACCW + j];
  }
}
static void data_to_state(const ZbModel* m, const ZbData* d, float* st) {
  for (int q = 0; q < m->nq; q++) st[ZB_S_QPOS + q] = (float)d->qpos[q];
  for (int j = 0; j < m->nv; j++) {
    st[ZB_S_QVEL + j] = (float)d->qvel[j];
    st[ZB_S_QACCW + j] = (float)d->qacc_warm[j];
  }
}

/* one physics step: ctrl given in d->ctrl; sensors when requested */
static void physics_substep(const ZbModel* m, ZbData* d, const ZbEnvConfig* cfg, int with_sensors, int do_integrate) {
  real dt = cfg->dt;
  forward(m, d, dt, cfg);
  if (with_sensors) sensors(m, d);
  if (do_integrate) { /* mj_advance saves qacc for warmstart, then integrates */
    for (int j = 0; j < m->nv; j++) d->qacc_warm[j] = d->qacc[j];
    integrate(m, d, dt, (cfg->flags & ZB_F_EULERDAMP) != 0);
  }
}

/* ksim reset (train.py:1471-1476) + forward; writes state, keeps RNG counters */
static void env_reset(const EnvCtx* c, ZbData* d, float* st, float* rnd) {
  const ZbModel* m = c->m;
  const ZbEnvConfig* cfg = c->cfg;
  uint32_t episode = fbits(st[ZB_S_EPISODE]);
  if ((cfg->flags & ZB_F_RANDOMIZE) && rnd) sample_rand(c, episode, rnd);
  load_params(c, d, rnd);
  /* qpos: base at qpos0, joints at JOINT_BIASES (+ randomized joint zero: qpos0 shift) */
  for (int q = 0; q < m->nq; q++) d->qpos[q] = m->qpos0[q];
  for (int a = 0; a < m->nu; a++) {
    int qa = m->dof_qposadr[m->act_dof[a]];
    d->qpos[qa] = m->joint_bias[a] + (d->qpos0[qa] - m->qpos0[qa]);
  }
  for (int j = 0; j < m->nv; j++) { d->qvel[j] = 0; d->qacc_warm[j] = 0; }
  float u[2];
  for (int a = 0; a < m->nu; a += 2) {
    uniform2(c->seed, P_RESET, (uint32_t)(a / 2), c->env, episode, u);
    for (int h = 0; h < 2 && a + h < m->nu; h++)
      d->qvel[m->act_dof[a + h]] = cfg->reset_qvel_scale * (2 * u[h] - 1);
  }
  uniform2(c->seed, P_RESET, 15u, c->env, episode, u);
  st[ZB_S_IMU_LAG] = cfg->lag_range[0] + (cfg->lag_range[1] - cfg->lag_range[0]) * u[0];
  st[ZB_S_PUSH_TIMER] = cfg->push_interval[0] + (cfg->push_interval[1] - cfg->push_interval[0]) * u[1];
  for (int k = 0; k < 4; k++) st[ZB_S_IMU_EMA + k] = 0;
  for (int a = 0; a < m->nu; a++) {
    st[ZB_S_PLAN_POS + a] = (float)d->qpos[m->dof_qposadr[m->act_dof[a]]];
    st[ZB_S_PLAN_VEL + a] = (float)d->qvel[m->act_dof[a]];
    st[ZB_S_PLAN_TAU + a] = 0;
  }
  st[ZB_S_EP_RETURN] = 0;
  st[ZB_S_EP_STEPS] = bitsf(0);
  st[ZB_S_EPISODE] = bitsf(episode + 1);
  for (int a = 0; a < m->nu; a++) d->ctrl[a] = 0;
  physics_substep(m, d, cfg, 1, 0); /* mjx.forward at the reset state */
  data_to_state(m, d, st);
}

static void rewards_and_done(const EnvCtx* c, ZbData* d, float* st, float cur, float* terms, float* rew_out,
                             uint8_t* done_out, int* done_flag, int* success_flag) {
  const ZbModel* m = c->m;
  const ZbEnvConfig* cfg = c->cfg;
  /* terminations on the next state (train.py:1588-1593) */
  real z = d->qpos[2];
  real bq[4] = {d->qpos[3], d->qpos[4], d->qpos[5], d->qpos[6]};
  quat_normalize(bq);
  real upz = 1 - 2 * (bq[1] * bq[1] + bq[2] * bq[2]);
  uint32_t steps = fbits(st[ZB_S_EP_STEPS]) + 1;
  int fail = (z < cfg->bad_z[0]) || (z > cfg->bad_z[1]) || (upz < COS((real)cfg->max_tilt_rad));
  int trunc = (real)steps * cfg->ctrl_dt >= cfg->max_episode_sec;
  if (!(z == z)) fail = 1; /* NaN state terminates */
  int done = fail || trunc;
  *done_flag = done;
  *success_flag = !fail && trunc;

  real t[ZB_NUM_TERMS];
  /* 0 StayAliveReward [U] */
  t[ZB_T_STAY_ALIVE] = fail ? (real)-1 : (real)1 / cfg->stay_alive_balance;
  /* 1 UprightReward [U]: world-z component of the base z axis (xquat[1]) */
  real xq[4] = {d->xquat[1][0], d->xquat[1][1], d->xquat[1][2], d->xquat[1][3]};
  t[ZB_T_UPRIGHT] = 1 - 2 * (xq[1] * xq[1] + xq[2] * xq[2]);
  /* 2 NaiveForwardReward clip_max 0.2 [U] */
  real vx = d->qvel[0];
  t[ZB_T_NAIVE_FORWARD] = vx > cfg->naive_forward_clip_max ? (real)cfg->naive_forward_clip_max : vx;
  /* 3 NaiveForwardOrientationReward [U]: world-x component of the base x axis */
  t[ZB_T_FWD_ORIENT] = 1 - 2 * (xq[2] * xq[2] + xq[3] * xq[3]);
  /* 4 LinearVelocityPenalty(y, robot frame, l1) [U] */
  real bm[9], vb[3], vw[3] = {d->qvel[0], d->qvel[1], d->qvel[2]};
  quat2mat(bm, bq);
  mulmtv3(vb, bm, vw);
  t[ZB_T_LINVEL_Y] = FABS(vb[1]);
  /* 5 SimpleSingleFootContactReward, train.py:698-712 (obs of the current state) */
  int lc = st[ZB_S_TOUCH] > cfg->touch_threshold, rc = st[ZB_S_TOUCH + 1] > cfg->touch_threshold;
  t[ZB_T_SINGLE_FOOT] = (real)(lc != rc);
  /* 6 FeetAirtimeReward, train.py:503-546 (causal per-step form) */
  {
    int cont[2] = {lc, rc};
    real r = 0;
    for (int s = 0; s < 2; s++) {
      real air_prev = st[ZB_S_AIRTIME + s];
      int prev = st[ZB_S_PREV_CONT + s] > (float)0.5;
      int td = cont[s] && !prev;
      r += (air_prev - cfg->feet_airtime_touchdown_penalty) * (real)td;
      real air = (cont[s] || done) ? (real)0 : air_prev + cfg->ctrl_dt;
      st[ZB_S_AIRTIME + s] = (float)air;
      st[ZB_S_PREV_CONT + s] = (float)cont[s];
    }
    t[ZB_T_FEET_AIRTIME] = r;
  }
  /* 7 FeetOrientationReward, train.py:679-688 */
  {
    real rl, pl, rr, pr;
    quat_roll_pitch(d->xquat[m->body_left_foot], &rl, &pl);
    quat_roll_pitch(d->xquat[m->body_right_foot], &rr, &pr);
    real err = FABS(rl) + FABS(pl) + FABS(rr) + FABS(pr);
    t[ZB_T_FEET_ORIENT] = EXP(-err / cfg->feet_orient_error_scale);
  }
  /* 8 FeetTooClosePenalty, train.py:740-748 */
  t[ZB_T_FEET_TOO_CLOSE] = st[ZB_S_FEET_DIST] < cfg->feet_too_close_threshold ? 1 : 0;
  /* 9-11 JointDeviationPenalty groups (sum w*(q - bias)^2) [U norm] */
  {
    static const int straight[4] = {7, 6, 1, 0};
    static const int ankle[6] = {9, 10, 11, 3, 4, 5};
    static const int arm[8] = {12, 13, 14, 15, 16, 17, 18, 19};
    real s1 = 0, s2 = 0, s3 = 0;
    for (int i = 0; i < 4; i++) { int j = straight[i]; real e = d->qpos[7 + j] - m->joint_bias[j]; s1 += m->joint_weight[j] * e * e; }
    for (int i = 0; i < 6; i++) { int j = ankle[i]; real e = d->qpos[7 + j] - m->joint_bias[j]; s2 += m->joint_weight[j] * e * e; }
    for (int i = 0; i < 8; i++) { int j = arm[i]; real e = d->qpos[7 + j] - m->joint_bias[j]; s3 += m->joint_weight[j] * e * e; }
    t[ZB_T_STRAIGHT_LEG] = s1;
    t[ZB_T_ANKLE_KNEE] = s2;
    t[ZB_T_ARM_POSE] = s3;
  }
  real total = 0;
  for (int i = 0; i < ZB_NUM_TERMS; i++) {
    real sc = cfg->reward_scale[i] * (cfg->reward_by_curriculum[i] ? (real)cur : (real)1);
    total += sc * t[i];
    if (terms) terms[i] = (float)t[i];
  }
  *rew_out = (float)total;
  *done_out = (uint8_t)done;
  st[ZB_S_EP_STEPS] = bitsf(steps);
  st[ZB_S_EP_RETURN] += (float)total;
}

/* push event (train.py:1459-1468; exact ksim law [U]) */
static void push_event(const EnvCtx* c, ZbData* d, float* st, float cur) {
  const ZbEnvConfig* cfg = c->cfg;
  uint32_t ctr = fbits(st[ZB_S_RNG_STEP]);
  float timer = st[ZB_S_PUSH_TIMER] - cfg->ctrl_dt;
  if (timer <= 0) {
    float u[2], v[2];
    uniform2(c->seed, P_PUSH, 0, c->env, ctr, u);
    uniform2(c->seed, P_PUSH, 1, c->env, ctr, v);
    real mag = (cfg->push_vel_range[0] + (cfg->push_vel_range[1] - cfg->push_vel_range[0]) * v[1]) /
               cfg->push_vel_range[1];
    d->qvel[0] += (real)cur * mag * cfg->push_linvel[0] * (2 * u[0] - 1);
    d->qvel[1] += (real)cur * mag * cfg->push_linvel[1] * (2 * u[1] - 1);
    d->qvel[2] += (real)cur * mag * cfg->push_linvel[2] * (2 * v[0] - 1);
    timer = cfg->push_interval[0] + (cfg->push_interval[1] - cfg->push_interval[0]) * v[1];
  }
  st[ZB_S_PUSH_TIMER] = timer;
}

static int nonfinite(const ZbModel* m, const ZbData* d) {
  for (int q = 0; q < m->nq; q++) if (!isfinite((double)d->qpos[q])) return 1;
  for (int j = 0; j < m->nv; j++) if (!isfinite((double)d->qvel[j])) return 1;
  return 0;
}

/* -------------------------------------------------------------------------- */
/* public oracle API                                                           */
/* -------------------------------------------------------------------------- */
int zbo_real_bytes(void) { return (int)sizeof(real); }

int zbo_reset(const ZbModel* m, const ZbEnvConfig* cfg, int n, int env_offset, uint64_t seed, float* state,
              float* rnd, const uint8_t* mask, float* obs_actor, float* obs_critic, float* obs_extra) {
  if (!m || !cfg || !state || n < 0) return -1;
#pragma omp parallel for schedule(dynamic, 4)
  for (int e = 0; e < n; e++) {
    if (mask && !mask[e]) continue;
    ZbData* d = (ZbData*)calloc(1, sizeof(ZbData));
    EnvCtx c = {m, cfg, seed, (uint32_t)(env_offset + e)};
    float* st = state + (size_t)e * ZB_STATE_STRIDE;
    float* rr = rnd ? rnd + (size_t)e * ZB_RAND_STRIDE : NULL;
    env_reset(&c, d, st, rr);
    observe(&c, d, st, obs_actor ? obs_actor + (size_t)e * ZB_OBS_ACTOR : NULL,
            obs_critic ? obs_critic + (size_t)e * ZB_OBS_CRITIC : NULL,
            obs_extra ? obs_extra + (size_t)e * ZB_OBS_EXTRA : NULL);
    free(d);
  }
  return 0;
}

/* test infrastructure: record each env's smallest floor-contact clearance over the next zbo_step calls'
   substeps into out[e] (NULL: stop) */
void zbo_set_clearance_out(float* out) { g_clearance_out = out; }

int zbo_step(const ZbModel* m, const ZbEnvConfig* cfg, int n, int env_offset, uint64_t seed, float* state,
             float* rnd, const float* action, float* obs_actor, float* obs_critic, float* obs_extra,
             float* reward_terms, float* reward, uint8_t* done, uint8_t* success, float curriculum, float* stats,
             int32_t* iters) {
  if (!m || !cfg || !state || !action || n < 0) return -1;
#pragma omp parallel for schedule(dynamic, 4)
  for (int e = 0; e < n; e++) {
    ZbData* d = (ZbData*)calloc(1, sizeof(ZbData));
    EnvCtx c = {m, cfg, seed, (uint32_t)(env_offset + e)};
    float* st = state + (size_t)e * ZB_STATE_STRIDE;
    float* rr = rnd ? rnd + (size_t)e * ZB_RAND_STRIDE : NULL;
    load_params(&c, d, rr);
    state_to_data(m, st, d);
    if (cfg->flags & ZB_F_PUSH) push_event(&c, d, st, curriculum);
    const float* act = action + (size_t)e * ZB_NJ;
    d->clearance = (real)1e30;
    for (int s = 0; s < cfg->n_substeps; s++) {
      feetech_ctrl(m, d, st + ZB_S_PLAN_POS, st + ZB_S_PLAN_VEL, st + ZB_S_PLAN_TAU, act, cfg->dt);
      physics_substep(m, d, cfg, s == cfg->n_substeps - 1, 1);
    }
    if (g_clearance_out) g_clearance_out[e] = (float)d->clearance;
    if (nonfinite(m, d)) st[ZB_S_NAN] = bitsf(1);
    data_to_state(m, d, st);
    float rew;
    uint8_t dn;
    int dflag, sflag;
    rewards_and_done(&c, d, st, curriculum, reward_terms ? reward_terms + (size_t)e * ZB_NUM_TERMS : NULL, &rew, &dn,
                     &dflag, &sflag);
    if (reward) reward[e] = rew;
    if (done) done[e] = dn;
    if (success) success[e] = (uint8_t)sflag;
    if (stats) {
      float* sp = stats + (size_t)e * ZB_NUM_STATS;
      sp[ZB_ST_REWARD] += rew;
      if (dflag) {
        sp[ZB_ST_RETURN] += st[ZB_S_EP_RETURN];
        sp[ZB_ST_LENGTH] += (float)fbits(st[ZB_S_EP_STEPS]);
        sp[ZB_ST_DONE] += 1;
      }
    }
    if (iters) iters[e] = d->solver_iters;
    if (dflag && (cfg->flags & ZB_F_AUTORESET)) env_reset(&c, d, st, rr);
    observe(&c, d, st, obs_actor ? obs_actor + (size_t)e * ZB_OBS_ACTOR : NULL,
            obs_critic ? obs_critic + (size_t)e * ZB_OBS_CRITIC : NULL,
            obs_extra ? obs_extra + (size_t)e * ZB_OBS_EXTRA : NULL);
    st[ZB_S_RNG_STEP] = bitsf(fbits(st[ZB_S_RNG_STEP]) + 1);
    free(d);
  }
  return 0;
}

/* ---------------------- debug / invariant-test entry points ----------------- */
/*
 * Run one forward pass on (qpos, qvel, ctrl) with the unrandomized model and
 * return internals: qM dense symmetric [nv*nv], qfrc_bias [nv], qacc_smooth [nv],
 * qacc [nv], xpos [nbody*3], cinert [nbody*10], cvel [nbody*6], nefc, ncon,
 * contact normal force per foot (touch[2]).
 */
int zbo_forward_debug(const ZbModel* m, const ZbEnvConfig* cfg, const float* qpos, const float* qvel,
                      const float* ctrl, float* qM, float* qfrc_bias, float* qacc_smooth, float* qacc, float* xpos,
                      float* cinert, float* cvel, int* nefc_ncon, float* touch) {
  ZbData* d = (ZbData*)calloc(1, sizeof(ZbData));
  EnvCtx c = {m, cfg, 0, 0};
  load_params(&c, d, NULL);
  for (int q = 0; q < m->nq; q++) d->qpos[q] = qpos[q];
  for (int j = 0; j < m->nv; j++) d->qvel[j] = qvel[j];
  for (int a = 0; a < m->nu; a++) d->ctrl[a] = ctrl ? ctrl[a] : 0;
  forward(m, d, cfg->dt, cfg);
  sensors(m, d);
  int nv = m->nv;
  if (qM)
    for (int i = 0; i < nv; i++)
      for (int j = 0; j < nv; j++) qM[i * nv + j] = 0;
  for (int i = 0; i < nv; i++) {
    if (qM) {
      qM[i * nv + i] = (float)d->qM[i][i];
      for (int j = m->dof_parent[i]; j >= 0; j = m->dof_parent[j]) {
        qM[i * nv + j] = (float)d->qM[i][j];
        qM[j * nv + i] = (float)d->qM[i][j];
      }
    }
    if (qfrc_bias) qfrc_bias[i] = (float)d->qfrc_bias[i];
    if (qacc_smooth) qacc_smooth[i] = (float)d->qacc_smooth[i];
    if (qacc) qacc[i] = (float)d->qacc[i];
  }
  for (int b = 0; b < m->nbody; b++) {
    if (xpos) for (int k = 0; k < 3; k++) xpos[b * 3 + k] = (float)d->xpos[b][k];
    if (cinert) for (int k = 0; k < 10; k++) cinert[b * 10 + k] = (float)d->cinert[b][k];
    if (cvel) for (int k = 0; k < 6; k++) cvel[b * 6 + k] = (float)d->cvel[b][k];
  }
  if (nefc_ncon) { nefc_ncon[0] = d->nefc; nefc_ncon[1] = d->ncon; }
  if (touch) { touch[0] = (float)d->touch[0]; touch[1] = (float)d->touch[1]; }
  free(d);
  return 0;
}

/*
 * Contacts of the collision stage alone at qpos, with the env's randomization row (rnd may be NULL):
 * kinematics, com_pos, collision; returns ncon. The GPU parity tests count them at the root lowered
 * and raised by a few fp32 ulps to find envs whose step starts with a contact at its activation
 * boundary (tests/test_gpu_parity.py boundary_envs).
 */
int zbo_contact_count(const ZbModel* m, const ZbEnvConfig* cfg, const float* qpos, const float* rnd) {
  ZbData* d = (ZbData*)calloc(1, sizeof(ZbData));
  EnvCtx c = {m, cfg, 0, 0};
  load_params(&c, d, rnd);
  for (int q = 0; q < m->nq; q++) d->qpos[q] = qpos[q];
  kinematics(m, d);
  com_pos(m, d);
  collision(m, d);
  const int n = d->ncon;
  free(d);
  return n;
}

/*
 * The constrained-acceleration problem of one forward pass, for the solver
 * optimality tests (tests/test_solver_optimality.py): qacc_smooth, the dense
 * mass matrix and the constraint rows (J [nefc][nv], D, R, aref, frictionloss,
 * type: 0 frictionloss, 1 limit, 2 contact edge), plus the Newton solution
 * qacc. Returns nefc.
 */
int zbo_constraint_debug(const ZbModel* m, const ZbEnvConfig* cfg, const float* qpos, const float* qvel,
                         const float* ctrl, const float* qacc_warm, float* qM, float* qacc_smooth, float* qacc,
                         float* J, float* D, float* R, float* aref, float* floss, int* type) {
  ZbData* d = (ZbData*)calloc(1, sizeof(ZbData));
  EnvCtx c = {m, cfg, 0, 0};
  load_params(&c, d, NULL);
  for (int q = 0; q < m->nq; q++) d->qpos[q] = qpos[q];
  for (int j = 0; j < m->nv; j++) {
    d->qvel[j] = qvel[j];
    d->qacc_warm[j] = qacc_warm ? qacc_warm[j] : 0;
  }
  for (int a = 0; a < m->nu; a++) d->ctrl[a] = ctrl ? ctrl[a] : 0;
  forward(m, d, cfg->dt, cfg);
  const int nv = m->nv, ne = d->nefc;
  for (int i = 0; i < nv; i++) {
    qacc_smooth[i] = (float)d->qacc_smooth[i];
    qacc[i] = (float)d->qacc[i];
    for (int j = 0; j < nv; j++) qM[i * nv + j] = 0;
  }
  for (int i = 0; i < nv; i++) {
    qM[i * nv + i] = (float)d->qM[i][i];
    for (int j = m->dof_parent[i]; j >= 0; j = m->dof_parent[j]) {
      qM[i * nv + j] = (float)d->qM[i][j];
      qM[j * nv + i] = (float)d->qM[i][j];
    }
  }
  for (int r = 0; r < ne; r++) {
    for (int j = 0; j < nv; j++) J[r * nv + j] = (float)d->efc_J[r][j];
    D[r] = (float)d->efc_D[r];
    R[r] = (float)d->efc_R[r];
    aref[r] = (float)d->efc_aref[r];
    floss[r] = (float)d->efc_floss[r];
    type[r] = d->efc_type[r];
  }
  free(d);
  return ne;
}

/* advance (qpos, qvel, qacc_warmstart) by n physics steps at fixed ctrl */
int zbo_simulate(const ZbModel* m, const ZbEnvConfig* cfg, float* qpos, float* qvel, float* qaccw, const float* ctrl,
                 int nsteps) {
  ZbData* d = (ZbData*)calloc(1, sizeof(ZbData));
  EnvCtx c = {m, cfg, 0, 0};
  load_params(&c, d, NULL);
  for (int q = 0; q < m->nq; q++) d->qpos[q] = qpos[q];
  for (int j = 0; j < m->nv; j++) { d->qvel[j] = qvel[j]; d->qacc_warm[j] = qaccw ? qaccw[j] : 0; }
  for (int s = 0; s < nsteps; s++) {
    for (int a = 0; a < m->nu; a++) d->ctrl[a] = ctrl ? ctrl[a] : 0;
    physics_substep(m, d, cfg, 0, 1);
  }
  for (int q = 0; q < m->nq; q++) qpos[q] = (float)d->qpos[q];
  for (int j = 0; j < m->nv; j++) { qvel[j] = (float)d->qvel[j]; if (qaccw) qaccw[j] = (float)d->qacc_warm[j]; }
  free(d);
  return 0;
}

/* ABI check helpers: the compiled layout of ZbModel / ZbEnvConfig */
#define OFF(T, f) {#f, offsetof(T, f)}
typedef struct { const char* name; size_t off; } FieldOff;
static const FieldOff model_fields[] = {
    OFF(ZbModel, magic), OFF(ZbModel, version), OFF(ZbModel, struct_bytes), OFF(ZbModel, nbody), OFF(ZbModel, nq),
    OFF(ZbModel, nv), OFF(ZbModel, nu), OFF(ZbModel, ngeom), OFF(ZbModel, nsite), OFF(ZbModel, max_depth),
    OFF(ZbModel, gravity), OFF(ZbModel, timestep), OFF(ZbModel, meaninertia), OFF(ZbModel, pad_opt),
    OFF(ZbModel, body_parent), OFF(ZbModel, body_depth), OFF(ZbModel, body_jnttype), OFF(ZbModel, body_dofadr),
    OFF(ZbModel, body_dofnum), OFF(ZbModel, body_qposadr), OFF(ZbModel, body_lastdof), OFF(ZbModel, body_pos),
    OFF(ZbModel, body_quat), OFF(ZbModel, body_ipos), OFF(ZbModel, body_iquat), OFF(ZbModel, body_mass),
    OFF(ZbModel, body_inertia), OFF(ZbModel, body_invweight0), OFF(ZbModel, jnt_axis), OFF(ZbModel, jnt_pos),
    OFF(ZbModel, dof_body), OFF(ZbModel, dof_parent), OFF(ZbModel, dof_depth), OFF(ZbModel, dof_anc),
    OFF(ZbModel, dof_limited), OFF(ZbModel, dof_qposadr), OFF(ZbModel, dof_armature), OFF(ZbModel, dof_damping),
    OFF(ZbModel, dof_frictionloss), OFF(ZbModel, dof_invweight0), OFF(ZbModel, dof_range), OFF(ZbModel, dof_solref),
    OFF(ZbModel, dof_solimp), OFF(ZbModel, qpos0), OFF(ZbModel, pad_q), OFF(ZbModel, act_dof), OFF(ZbModel, act_gear),
    OFF(ZbModel, act_ctrlrange), OFF(ZbModel, fe_kp), OFF(ZbModel, fe_kd), OFF(ZbModel, fe_error_gain),
    OFF(ZbModel, fe_max_pwm), OFF(ZbModel, fe_vin), OFF(ZbModel, fe_kt), OFF(ZbModel, fe_R), OFF(ZbModel, fe_vmax),
    OFF(ZbModel, fe_amax), OFF(ZbModel, fe_max_torque), OFF(ZbModel, fe_max_velocity), OFF(ZbModel, geom_body),
    OFF(ZbModel, geom_type), OFF(ZbModel, geom_pos), OFF(ZbModel, geom_quat), OFF(ZbModel, geom_size), OFF(ZbModel, floor_friction),
    OFF(ZbModel, floor_solref), OFF(ZbModel, floor_solimp), OFF(ZbModel, floor_margin), OFF(ZbModel, pad_floor),
    OFF(ZbModel, npair), OFF(ZbModel, pair_geom), OFF(ZbModel, pair_margin), OFF(ZbModel, pair_friction),
    OFF(ZbModel, pair_solref), OFF(ZbModel, pair_solimp),
    OFF(ZbModel, site_body), OFF(ZbModel, site_pos), OFF(ZbModel, site_quat), OFF(ZbModel, site_imu),
    OFF(ZbModel, site_left_foot), OFF(ZbModel, site_right_foot), OFF(ZbModel, body_base), OFF(ZbModel, body_left_foot),
    OFF(ZbModel, body_right_foot), OFF(ZbModel, geom_left_foot), OFF(ZbModel, geom_right_foot),
    OFF(ZbModel, max_body_depth), OFF(ZbModel, mrow_size), OFF(ZbModel, nskip_geom), OFF(ZbModel, nskip_pair), OFF(ZbModel, body_nchild),
    OFF(ZbModel, body_child), OFF(ZbModel, depth_maxchild), OFF(ZbModel, dof_desc), OFF(ZbModel, dof_ancpk),
    OFF(ZbModel, dof_rowmask), OFF(ZbModel, dof_act), OFF(ZbModel, dof_rowoff), OFF(ZbModel, geom_lastdof),
    OFF(ZbModel, nlevel), OFF(ZbModel, pad_lvl), OFF(ZbModel, level_nmem), OFF(ZbModel, level_mem),
    OFF(ZbModel, joint_bias), OFF(ZbModel, joint_weight), OFF(ZbModel, geom_vertadr), OFF(ZbModel, geom_vertnum),
    OFF(ZbModel, mesh_vert), OFF(ZbModel, pad_end),
};
static const FieldOff config_fields[] = {
    OFF(ZbEnvConfig, struct_bytes), OFF(ZbEnvConfig, flags), OFF(ZbEnvConfig, n_substeps),
    OFF(ZbEnvConfig, iterations), OFF(ZbEnvConfig, ls_iterations), OFF(ZbEnvConfig, dt), OFF(ZbEnvConfig, ctrl_dt),
    OFF(ZbEnvConfig, tolerance), OFF(ZbEnvConfig, ls_tolerance), OFF(ZbEnvConfig, imu_noise_std),
    OFF(ZbEnvConfig, acc_noise_std), OFF(ZbEnvConfig, reset_qvel_scale), OFF(ZbEnvConfig, max_episode_sec),
    OFF(ZbEnvConfig, lag_range), OFF(ZbEnvConfig, bad_z), OFF(ZbEnvConfig, max_tilt_rad), OFF(ZbEnvConfig, push_linvel),
    OFF(ZbEnvConfig, push_interval), OFF(ZbEnvConfig, push_vel_range), OFF(ZbEnvConfig, reward_scale),
    OFF(ZbEnvConfig, reward_by_curriculum), OFF(ZbEnvConfig, feet_airtime_touchdown_penalty),
    OFF(ZbEnvConfig, naive_forward_clip_max), OFF(ZbEnvConfig, feet_orient_error_scale),
    OFF(ZbEnvConfig, feet_too_close_threshold), OFF(ZbEnvConfig, touch_threshold),
    OFF(ZbEnvConfig, stay_alive_balance), OFF(ZbEnvConfig, rand_mass), OFF(ZbEnvConfig, rand_armature),
    OFF(ZbEnvConfig, rand_damping), OFF(ZbEnvConfig, rand_friction), OFF(ZbEnvConfig, rand_qpos0),
    OFF(ZbEnvConfig, rand_floor_mu), OFF(ZbEnvConfig, rand_imu_tilt_std), OFF(ZbEnvConfig, rand_imu_yaw_std),
    OFF(ZbEnvConfig, rand_imu_pos_std), OFF(ZbEnvConfig, solver), OFF(ZbEnvConfig, pad),
};
long zbo_field_offset(int which, const char* name) {
  const FieldOff* f = which == 0 ? model_fields : config_fields;
  size_t n = which == 0 ? sizeof(model_fields) / sizeof(FieldOff) : sizeof(config_fields) / sizeof(FieldOff);
  for (size_t i = 0; i < n; i++)
    if (strcmp(f[i].name, name) == 0) return (long)f[i].off;
  return -1;
}
size_t zbo_struct_bytes(int which) { return which == 0 ? sizeof(ZbModel) : sizeof(ZbEnvConfig); }
