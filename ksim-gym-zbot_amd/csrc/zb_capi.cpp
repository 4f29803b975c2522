/*
 * zb_capi.cpp — C ABI of libzbot_hip.so (declared in include/zbot.h).
 *
 * Host-side handle management: validates the compiled model against the
 * engine's limits, owns the persistent per-env device buffers, and launches
 * the kernels of zb_engine.hip asynchronously on the caller's stream. Nothing
 * here allocates, copies or synchronises inside zb_step / zb_reset.
 */
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "zb_internal.h"

#define ZB_ABI_VERSION 2

struct ZbHandle {
  int device;
  int n;
  int env_offset;
  uint64_t seed;
  ZbModel hmodel;
  ZbEnvConfig cfg;
  ZbModel* dmodel;
  ZbEnvConfig* dcfg;
  int32_t* dtopo; /* [TP_NF][32] per-lane topology */
  float* state;
  float* rnd;
  float* stats;
  int32_t* iters;
  float* stamps; /* ZB_STAMPS diagnostic build only */
  uint32_t* sched; /* chunked step: [2 + npair] counters and per-pair progress (zb_internal.h) */
  int32_t* itpart; /* chunked step: [n] Newton iterations so far */
  int nchunk;      /* work units per pair of envs in zb_step (1: unchunked) */
};

/* Chunks per control step for zb_step. The launch runs its pairs of envs in
   rounds of `resident` workgroups. When the last round is partial, its pairs run their whole
   control step while most of the chip idles; splitting every pair's substeps into chunks, taken
   in chunk-major order, spreads that last round over the chip at the price of one state hand-off
   per extra chunk (≈1.6 % of a pair's step each, measured). Measured on MI355X (2048 resident):
   1.25 rounds +24 % (4 chunks), 1.5 +15 % (2), 1.75 +6 % (4), 2.5 +5 % (2), 3.5 +2 % (2); whole
   rounds lose 1-3 %, so they stay unchunked. ZB_STEP_CHUNKS overrides (1 = unchunked); the count
   is clamped to [1, n_substeps]. */
static int choose_chunks(int n_envs, int n_substeps, int resident) {
  int k = 1;
  const char* ov = getenv("ZB_STEP_CHUNKS");
  if (ov && *ov) {
    k = atoi(ov);
  } else if (resident > 0) {
    const long npair = (n_envs + 1) / 2;
    const double rounds = (double)npair / resident;
    const double f = rounds - (long)rounds; /* filled fraction of the last round */
    if (rounds > 1.0 && rounds < 4.0 && f > 0.0 && f < 0.9) k = (f <= 0.3 || f >= 0.7) ? 4 : 2;
  }
  if (k > n_substeps) k = n_substeps;
  return k < 1 ? 1 : k;
}

static thread_local std::string g_err;

static int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
static int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}
#define HIPCHK(expr)                                                                       \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess) return fail(ZB_EDEVICE, "%s: %s", #expr, hipGetErrorString(_e)); \
  } while (0)

static int use_device(const ZbHandle* h) {
  int cur = -1;
  HIPCHK(hipGetDevice(&cur));
  if (cur != h->device) HIPCHK(hipSetDevice(h->device));
  return ZB_OK;
}

extern "C" {

int zb_abi_version(void) { return ZB_ABI_VERSION; }
size_t zb_model_struct_bytes(void) { return sizeof(ZbModel); }
size_t zb_config_struct_bytes(void) { return sizeof(ZbEnvConfig); }
int zb_state_stride(void) { return ZB_STATE_STRIDE; }
int zb_rand_stride(void) { return ZB_RAND_STRIDE; }
const char* zb_last_error(void) { return g_err.c_str(); }

void zb_default_config(ZbEnvConfig* c) {
  if (!c) return;
  memset(c, 0, sizeof *c);
  const double PI = 3.14159265358979323846;
  c->struct_bytes = (int32_t)sizeof(ZbEnvConfig);
  c->flags = ZB_F_OBS_NOISE | ZB_F_AUTORESET;
  c->n_substeps = 20;
  c->iterations = 8;
  c->ls_iterations = 8;
  c->dt = 0.001f;
  c->ctrl_dt = 0.02f;
  c->tolerance = 1e-8f;
  c->ls_tolerance = 0.01f;
  c->imu_noise_std = (float)(PI / 180.0);
  c->acc_noise_std = 0.5f;
  c->reset_qvel_scale = 0.01f;
  c->max_episode_sec = 80.f;
  c->lag_range[0] = 0.f; c->lag_range[1] = 0.1f;
  c->bad_z[0] = 0.05f; c->bad_z[1] = 0.5f;
  c->max_tilt_rad = (float)(60.0 * PI / 180.0);
  c->push_linvel[0] = 0.1f; c->push_linvel[1] = 0.1f; c->push_linvel[2] = 0.05f;
  c->push_interval[0] = 2.f; c->push_interval[1] = 4.f;
  c->push_vel_range[0] = 0.05f; c->push_vel_range[1] = 0.15f;
  const float scales[ZB_NUM_TERMS] = {1.0f, 1.0f, 5.0f, 0.3f, -2.0f, 0.3f, 2.5f, 0.3f, -0.5f, -0.5f, -0.05f, -2.0f};
  const int by_cur[ZB_NUM_TERMS] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1};
  for (int i = 0; i < ZB_NUM_TERMS; i++) {
    c->reward_scale[i] = scales[i];
    c->reward_by_curriculum[i] = by_cur[i];
  }
  c->feet_airtime_touchdown_penalty = 0.3f;
  c->naive_forward_clip_max = 0.2f;
  c->feet_orient_error_scale = 0.25f;
  c->feet_too_close_threshold = 0.12f;
  c->touch_threshold = 0.1f;
  c->stay_alive_balance = 10.f;
  c->rand_mass[0] = 0.95f; c->rand_mass[1] = 1.15f;
  c->rand_armature[0] = 1.0f; c->rand_armature[1] = 1.05f;
  c->rand_damping[0] = 0.95f; c->rand_damping[1] = 1.05f;
  c->rand_friction[0] = 0.5f; c->rand_friction[1] = 1.5f;
  c->rand_qpos0[0] = (float)(-2.0 * PI / 180.0); c->rand_qpos0[1] = (float)(2.0 * PI / 180.0);
  c->rand_floor_mu[0] = 0.3f; c->rand_floor_mu[1] = 1.5f;
  c->rand_imu_tilt_std = (float)(5.0 * PI / 180.0);
  c->rand_imu_yaw_std = (float)(1.0 * PI / 180.0);
  c->rand_imu_pos_std = 0.005f;
}

static int check_model(const ZbModel* m) {
  if (m->magic != ZB_MODEL_MAGIC) return fail(ZB_EARG, "model magic mismatch");
  if (m->version != ZB_MODEL_VERSION) return fail(ZB_EARG, "model version %d != %d", m->version, ZB_MODEL_VERSION);
  if (m->struct_bytes != (int32_t)sizeof(ZbModel))
    return fail(ZB_EARG, "model struct_bytes %d != %zu (layout mismatch)", m->struct_bytes, sizeof(ZbModel));
  if (m->nbody > 32 || m->nv > 32 || m->nq > ZB_MAX_QPOS)
    return fail(ZB_EMODEL, "model too large for a 32-lane team (nbody=%d nv=%d nq=%d)", m->nbody, m->nv, m->nq);
  if (m->ngeom * ZB_CON_PER_GEOM * 4 > 32)
    return fail(ZB_EMODEL, "ngeom=%d: contact rows exceed the 32-lane team", m->ngeom);
  if (m->max_depth > ZB_MAX_DEPTH) return fail(ZB_EMODEL, "dof depth %d > %d", m->max_depth, ZB_MAX_DEPTH);
  if (m->nu != ZB_NJ || m->nbody != ZB_NBODY_TASK)
    return fail(ZB_EMODEL, "task layout needs nu=%d nbody=%d (got %d, %d)", ZB_NJ, ZB_NBODY_TASK, m->nu, m->nbody);
  if (m->body_jnttype[1] != ZB_JNT_FREE) return fail(ZB_EMODEL, "body 1 must carry the free joint");
  int maxbd = 0;
  for (int b = 0; b < m->nbody; b++) {
    if (m->body_depth[b] > maxbd) maxbd = m->body_depth[b];
    int nch = 0;
    for (int c = 1; c < m->nbody; c++)
      if (m->body_parent[c] == b) nch++;
    if (nch > 8) return fail(ZB_EMODEL, "body %d has %d children (max 8)", b, nch);
    /* subtree sums are chain suffix sums below the base (zb_engine.hip subtree_sum) */
    if (b != 1 && nch > 1) return fail(ZB_EMODEL, "body %d branches (%d children): only the base may", b, nch);
  }
  if (maxbd > 15) return fail(ZB_EMODEL, "body depth %d > 15", maxbd);
  /* dof tree shape the factorization relies on (zb_engine.hip factor_ldl):
     a root chain 0..R-1 (R <= 6, one dof per top elimination level) and
     unbranched limb chains of consecutive dofs hanging off dof R-1 */
  int nroot = 0;
  for (int k = 0; k < 6 && k < m->nlevel; k++) {
    const int lv = m->nlevel - 1 - k;
    if (m->level_nmem[lv] == 1 && m->level_mem[lv][0] == k && m->dof_depth[k] == k) nroot++;
    else break;
  }
  if (nroot != 6) return fail(ZB_EMODEL, "dof tree: the free joint's 6 dofs must form the root chain (got %d)", nroot);
  if (m->nv != 6 + ZB_NJ) return fail(ZB_EMODEL, "task layout needs nv=%d (got %d)", 6 + ZB_NJ, m->nv);
  /* depths / counts the engine is compiled for (zb_engine.hip NGEOM, MAXBD, MAXDD, NLIMBLV) */
  if (m->ngeom != 2 || maxbd != 8 || m->max_depth != 12 || m->nlevel != 12)
    return fail(ZB_EMODEL, "engine compiled for ngeom 2, body depth 8, dof depth 12, 12 levels (got %d, %d, %d, %d)",
                m->ngeom, maxbd, m->max_depth, m->nlevel);
  for (int k = nroot; k < m->nv; k++) {
    const int p = m->dof_parent[k];
    int nchild_prev = 0;
    for (int j = nroot; j < m->nv; j++) nchild_prev += (m->dof_parent[j] == k - 1);
    const bool head = p == nroot - 1;
    const bool cont = p == k - 1 && k - 1 >= nroot && nchild_prev == 1;
    if (!head && !cont)
      return fail(ZB_EMODEL, "dof %d: limbs must be unbranched chains of consecutive dofs off dof %d", k, nroot - 1);
  }
  return ZB_OK;
}

static int check_cfg(const ZbEnvConfig* c) {
  if (c->struct_bytes != (int32_t)sizeof(ZbEnvConfig))
    return fail(ZB_EARG, "config struct_bytes %d != %zu", c->struct_bytes, sizeof(ZbEnvConfig));
  if (c->n_substeps < 1 || c->iterations < 0 || c->ls_iterations < 0 || !(c->dt > 0.f))
    return fail(ZB_EARG, "invalid solver/timestep configuration");
  return ZB_OK;
}

/* The per-lane roles of a 32-lane team (body lane, dof lane, limb-chain position, contact
   rows holding the dof, actuator), computed once here instead of by every wave at the top
   of every launch. Field-major [TP_NF][32]; the checks of check_model hold. */
static void build_topology(const ZbModel* m, int32_t t[zb::TP_NF][zb::TOPO_LANES]) {
  using namespace zb;
  const int NB = ZB_NBODY_TASK, NV = 6 + ZB_NJ;
  memset(t, 0, sizeof(int32_t) * TP_NF * TOPO_LANES);
  int nch_of[TOPO_LANES], bdep_of[TOPO_LANES];
  for (int l = 0; l < TOPO_LANES; l++) {
    const bool isb = l < NB;
    t[TP_BPAR][l] = isb ? m->body_parent[l] : 0;
    t[TP_BDEP][l] = bdep_of[l] = isb ? m->body_depth[l] : 1000;
    t[TP_BJT][l] = isb ? m->body_jnttype[l] : ZB_JNT_NONE;
    t[TP_BDOFADR][l] = isb ? m->body_dofadr[l] : -1;
    t[TP_BLAST][l] = isb ? m->body_lastdof[l] : -1;
    int nch = 0;
    uint32_t ch0 = 0, ch1 = 0;
    for (int b = 1; b < NB; b++)
      if (isb && m->body_parent[b] == l && nch < 8) {
        if (nch < 4) ch0 |= (uint32_t)b << (8 * nch);
        else ch1 |= (uint32_t)b << (8 * (nch - 4));
        nch++;
      }
    t[TP_NCH][l] = nch_of[l] = nch;
    t[TP_CH0][l] = (int32_t)ch0;
    t[TP_CH1][l] = (int32_t)ch1;
  }
  /* per body depth: the largest child count among the bodies at that depth (4 bits each) */
  uint64_t lv = 0;
  for (int d = 0; d <= TOPO_MAXBD && d < 16; d++) {
    int mx = 0;
    for (int l = 0; l < TOPO_LANES; l++)
      if (bdep_of[l] == d && nch_of[l] > mx) mx = nch_of[l];
    lv |= (uint64_t)(mx & 0xf) << (4 * d);
  }
  for (int l = 0; l < TOPO_LANES; l++) {
    t[TP_LVL_LO][l] = (int32_t)(uint32_t)lv;
    t[TP_LVL_HI][l] = (int32_t)(uint32_t)(lv >> 32);
    const bool isd = l < NV;
    const int ddep = isd ? m->dof_depth[l] : 0;
    const int dbody = isd ? m->dof_body[l] : 0;
    t[TP_DDEP][l] = ddep;
    t[TP_DBODY][l] = dbody;
    t[TP_QADR][l] = isd ? m->dof_qposadr[l] : -1;
    int act = -1;
    for (int a = 0; a < m->nu; a++)
      if (isd && m->act_dof[a] == l) act = a;
    t[TP_ACT][l] = act;
    uint32_t desc = 0;
    for (int k = 0; k < NV; k++)
      if (isd && k != l && m->dof_depth[k] > ddep && m->dof_anc[k][ddep] == l) desc |= 1u << k;
    uint32_t rm = 0;
    for (int g = 0; g < TOPO_NGEOM; g++) {
      const int kd = m->body_lastdof[m->geom_body[g]];
      if (isd && kd >= 0 && (kd == l || ((desc >> kd) & 1u))) rm |= 0xFFFFu << (16 * g);
    }
    t[TP_ROWMASK][l] = (int32_t)rm;
    t[TP_DK0][l] = isd ? l - m->body_dofadr[dbody] : 0;
    t[TP_DFREE][l] = (isd && m->body_jnttype[dbody] == ZB_JNT_FREE) ? 1 : 0;
    int hd = -1, ln = 0;
    if (isd && l >= TOPO_NROOT) {
      hd = l;
      while (m->dof_parent[hd] >= TOPO_NROOT) hd = m->dof_parent[hd];
      int k = hd;
      while (k + 1 < NV && m->dof_parent[k + 1] == k) k++;
      ln = k - hd + 1;
    }
    t[TP_CHD][l] = hd;
    t[TP_CPS][l] = hd >= 0 ? l - hd : 0;
    t[TP_CLN][l] = ln;
  }
}

int zb_create(const ZbModel* model, const ZbEnvConfig* cfg, int n_envs, int env_offset, int device, uint64_t seed,
              ZbHandle** out) {
  if (!model || !cfg || !out || n_envs < 0 || env_offset < 0) return fail(ZB_EARG, "zb_create: bad argument");
  *out = nullptr;
  int rc = check_model(model);
  if (rc) return rc;
  rc = check_cfg(cfg);
  if (rc) return rc;
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(ZB_EDEVICE, "device %d not available (%d devices)", device, ndev);
  HIPCHK(hipSetDevice(device));
  ZbHandle* h = new ZbHandle();
  h->device = device;
  h->n = n_envs;
  h->env_offset = env_offset;
  h->seed = seed;
  h->hmodel = *model;
  h->cfg = *cfg;
  size_t n = (size_t)(n_envs > 0 ? n_envs : 1);
  hipError_t e = hipMalloc(&h->dmodel, sizeof(ZbModel));
  if (e == hipSuccess) e = hipMalloc(&h->dcfg, sizeof(ZbEnvConfig));
  if (e == hipSuccess) e = hipMemcpy(h->dcfg, cfg, sizeof(ZbEnvConfig), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMalloc(&h->state, n * ZB_STATE_STRIDE * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&h->rnd, n * ZB_RAND_STRIDE * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&h->stats, n * ZB_NUM_STATS * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&h->iters, n * sizeof(int32_t));
  if (e == hipSuccess) e = hipMemcpy(h->dmodel, model, sizeof(ZbModel), hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    int32_t topo[zb::TP_NF][zb::TOPO_LANES];
    build_topology(model, topo);
    e = hipMalloc(&h->dtopo, sizeof topo);
    if (e == hipSuccess) e = hipMemcpy(h->dtopo, topo, sizeof topo, hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) e = hipMemset(h->state, 0, n * ZB_STATE_STRIDE * sizeof(float));
  if (e == hipSuccess) e = hipMemset(h->rnd, 0, n * ZB_RAND_STRIDE * sizeof(float));
  if (e == hipSuccess) e = hipMemset(h->stats, 0, n * ZB_NUM_STATS * sizeof(float));
  if (e == hipSuccess) e = hipMemset(h->iters, 0, n * sizeof(int32_t));
  if (e == hipSuccess) e = hipMalloc(&h->sched, (2 + (n + 1) / 2) * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemset(h->sched, 0, (2 + (n + 1) / 2) * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMalloc(&h->itpart, n * sizeof(int32_t));
  if (e == hipSuccess) e = hipMemset(h->itpart, 0, n * sizeof(int32_t));
  h->nchunk = choose_chunks(n_envs, cfg->n_substeps, zb::step_resident_blocks(device));
#if defined(ZB_STAMPS) || defined(ZB_WAVETIME)
  if (e == hipSuccess) e = hipMalloc(&h->stamps, n * ZB_NSTAMP * sizeof(unsigned long long));
#endif
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    zb_destroy(h);
    return fail(ZB_EDEVICE, "zb_create: %s", hipGetErrorString(e));
  }
  *out = h;
  return ZB_OK;
}

int zb_destroy(ZbHandle* h) {
  if (!h) return ZB_OK;
  (void)hipSetDevice(h->device);
  if (h->dmodel) (void)hipFree(h->dmodel);
  if (h->dcfg) (void)hipFree(h->dcfg);
  if (h->dtopo) (void)hipFree(h->dtopo);
  if (h->state) (void)hipFree(h->state);
  if (h->rnd) (void)hipFree(h->rnd);
  if (h->stats) (void)hipFree(h->stats);
  if (h->iters) (void)hipFree(h->iters);
  if (h->stamps) (void)hipFree(h->stamps);
  if (h->sched) (void)hipFree(h->sched);
  if (h->itpart) (void)hipFree(h->itpart);
  delete h;
  return ZB_OK;
}

static zb::StepArgs base_args(ZbHandle* h) {
  zb::StepArgs a;
  memset(&a, 0, sizeof a);
  a.model = h->dmodel;
  a.topo = h->dtopo;
  a.cfg = h->dcfg;
  a.n_envs = h->n;
  a.env_offset = h->env_offset;
  a.seed = h->seed;
  a.state = h->state;
  a.rnd = h->rnd;
  a.stats = h->stats;
  a.iters = h->iters;
  a.dbg = h->stamps;
  a.nsteps = 1;
  a.curriculum = 1.f;
  a.nchunk = 1;
  a.sched = h->sched;
  a.itpart = h->itpart;
  return a;
}

int zb_reset(ZbHandle* h, const uint8_t* env_mask_dev, float* obs_actor, float* obs_critic, float* obs_extra,
             void* stream) {
  if (!h) return fail(ZB_EARG, "zb_reset: null handle");
  int rc = use_device(h);
  if (rc) return rc;
  zb::StepArgs a = base_args(h);
  a.reset_mask = env_mask_dev;
  a.obs_actor = obs_actor;
  a.obs_critic = obs_critic;
  a.obs_extra = obs_extra;
  hipError_t e = zb::launch_reset(a, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ZB_ELAUNCH, "zb_reset launch: %s", hipGetErrorString(e));
  return ZB_OK;
}

int zb_step(ZbHandle* h, const float* action, float* obs_actor, float* obs_critic, float* obs_extra,
            float* reward_terms, float* reward, uint8_t* done, uint8_t* success, float curriculum_level,
            void* stream) {
  if (!h || !action) return fail(ZB_EARG, "zb_step: null handle or action");
  if (!(curriculum_level == curriculum_level)) return fail(ZB_EARG, "zb_step: curriculum is NaN");
  int rc = use_device(h);
  if (rc) return rc;
  zb::StepArgs a = base_args(h);
  a.action = action;
  a.obs_actor = obs_actor;
  a.obs_critic = obs_critic;
  a.obs_extra = obs_extra;
  a.reward_terms = reward_terms;
  a.reward = reward;
  a.done = done;
  a.success = success;
  a.curriculum = curriculum_level;
  a.nchunk = h->nchunk;
  hipError_t e = zb::launch_step(a, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ZB_ELAUNCH, "zb_step launch: %s", hipGetErrorString(e));
  return ZB_OK;
}

int zb_rollout(ZbHandle* h, const float* actions, int n_steps, float* obs_actor, float* obs_critic, float* reward_sum,
               uint8_t* done, uint8_t* success, float curriculum_level, void* stream) {
  if (!h || !actions || n_steps < 1) return fail(ZB_EARG, "zb_rollout: bad argument");
  int rc = use_device(h);
  if (rc) return rc;
  zb::StepArgs a = base_args(h);
  a.action = actions;
  a.nsteps = n_steps;
  a.obs_actor = obs_actor;
  a.obs_critic = obs_critic;
  a.reward = reward_sum;
  a.done = done;
  a.success = success;
  a.curriculum = curriculum_level;
  hipError_t e = zb::launch_step(a, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ZB_ELAUNCH, "zb_rollout launch: %s", hipGetErrorString(e));
  return ZB_OK;
}

static int copy_rows(ZbHandle* h, void* dst, const void* src, size_t bytes, void* stream) {
  if (!h || !dst || !src) return fail(ZB_EARG, "null pointer");
  int rc = use_device(h);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return ZB_OK;
}

int zb_get_state(ZbHandle* h, float* state_dev, void* stream) {
  if (!h) return fail(ZB_EARG, "null handle");
  return copy_rows(h, state_dev, h->state, (size_t)h->n * ZB_STATE_STRIDE * sizeof(float), stream);
}
int zb_set_state(ZbHandle* h, const float* state_dev, void* stream) {
  if (!h) return fail(ZB_EARG, "null handle");
  return copy_rows(h, h->state, state_dev, (size_t)h->n * ZB_STATE_STRIDE * sizeof(float), stream);
}
int zb_get_rand(ZbHandle* h, float* rand_dev, void* stream) {
  if (!h) return fail(ZB_EARG, "null handle");
  return copy_rows(h, rand_dev, h->rnd, (size_t)h->n * ZB_RAND_STRIDE * sizeof(float), stream);
}
int zb_set_rand(ZbHandle* h, const float* rand_dev, void* stream) {
  if (!h) return fail(ZB_EARG, "null handle");
  return copy_rows(h, h->rnd, rand_dev, (size_t)h->n * ZB_RAND_STRIDE * sizeof(float), stream);
}
int zb_get_stats(ZbHandle* h, float* stats_dev, int clear, void* stream) {
  if (!h) return fail(ZB_EARG, "null handle");
  int rc = copy_rows(h, stats_dev, h->stats, (size_t)h->n * ZB_NUM_STATS * sizeof(float), stream);
  if (rc) return rc;
  if (clear) HIPCHK(hipMemsetAsync(h->stats, 0, (size_t)h->n * ZB_NUM_STATS * sizeof(float), (hipStream_t)stream));
  return ZB_OK;
}
int zb_set_step_chunks(ZbHandle* h, int k) {
  if (!h) return fail(ZB_EARG, "null handle");
  if (k < 0) return fail(ZB_EARG, "zb_set_step_chunks: k = %d < 0", k);
  if (k == 0) {
    int rc = use_device(h);
    if (rc) return rc;
    h->nchunk = choose_chunks(h->n, h->cfg.n_substeps, zb::step_resident_blocks(h->device));
  } else {
    h->nchunk = k > h->cfg.n_substeps ? h->cfg.n_substeps : k;
  }
  return ZB_OK;
}

int zb_get_solver_iters(ZbHandle* h, int32_t* iters_dev, void* stream) {
  if (!h) return fail(ZB_EARG, "null handle");
  return copy_rows(h, iters_dev, h->iters, (size_t)h->n * sizeof(int32_t), stream);
}

int zb_debug_forward(ZbHandle* h, float* state_dev, const float* ctrl_dev, float* dbg_dev, void* stream) {
  if (!h || !state_dev || !dbg_dev) return fail(ZB_EARG, "zb_debug_forward: null pointer");
  int rc = use_device(h);
  if (rc) return rc;
  zb::StepArgs a = base_args(h);
  a.state = state_dev;
  a.action = ctrl_dev;
  a.dbg = dbg_dev;
  hipError_t e = zb::launch_debug_forward(a, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ZB_ELAUNCH, "zb_debug_forward launch: %s", hipGetErrorString(e));
  return ZB_OK;
}

/* ---- post-rollout PPO inputs (include/zbot_ppo.h) ---- */

size_t zb_gae_partials_words(int n) {
  return n > 0 ? 2 * (size_t)((n + ZB_GAE_ENVS_PER_BLOCK - 1) / ZB_GAE_ENVS_PER_BLOCK) : 0;
}

int zb_gae(const float* reward, const float* values, const uint8_t* done, const uint8_t* success,
           const float* bootstrap, int T, int n, float gamma, float lam, float* gae_out, float* value_targets,
           double* partials, double* moments_out, void* stream) {
  if (T < 0 || n < 0) return fail(ZB_EARG, "zb_gae: negative size (T=%d n=%d)", T, n);
  if (moments_out && !partials) return fail(ZB_EARG, "zb_gae: moments_out needs the partials scratch");
  if ((size_t)zb_gae_partials_words(n) / 2 > (size_t)1024 * 1024)
    return fail(ZB_EARG, "zb_gae: n=%d exceeds the moment tree (%d envs)", n, 1024 * 1024 * ZB_GAE_ENVS_PER_BLOCK);
  if (T == 0 || n == 0) {
    if (moments_out) HIPCHK(hipMemsetAsync(moments_out, 0, 2 * sizeof(double), (hipStream_t)stream));
    return ZB_OK;
  }
  if (!reward || !values || !done || !gae_out) return fail(ZB_EARG, "zb_gae: null input/output pointer");
  zb::GaeArgs a;
  a.reward = reward;
  a.values = values;
  a.done = done;
  a.success = success;
  a.bootstrap = bootstrap;
  a.T = T;
  a.n = n;
  a.gamma = gamma;
  a.gl = gamma * lam;
  a.gae = gae_out;
  a.vtarget = value_targets;
  a.partials = partials;
  hipError_t e = zb::launch_gae(a, moments_out, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ZB_ELAUNCH, "zb_gae launch: %s", hipGetErrorString(e));
  return ZB_OK;
}

int zb_moments_combine(const double* moments, int k, double* out, void* stream) {
  if (!out || k < 0 || (k > 0 && !moments)) return fail(ZB_EARG, "zb_moments_combine: bad argument");
  if (k > 1024 * 1024) return fail(ZB_EARG, "zb_moments_combine: k=%d > %d", k, 1024 * 1024);
  if (k == 0) {
    HIPCHK(hipMemsetAsync(out, 0, 2 * sizeof(double), (hipStream_t)stream));
    return ZB_OK;
  }
  hipError_t e = zb::launch_moments(moments, k, out, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ZB_ELAUNCH, "zb_moments_combine launch: %s", hipGetErrorString(e));
  return ZB_OK;
}

int zb_adv_normalize(const float* gae, float* advantages, long long count, const double* moments, double total,
                     float eps, void* stream) {
  if (count < 0) return fail(ZB_EARG, "zb_adv_normalize: negative count");
  if (count == 0) return ZB_OK;
  if (!gae || !advantages || !moments) return fail(ZB_EARG, "zb_adv_normalize: null pointer");
  if (!(total > 0.0)) return fail(ZB_EARG, "zb_adv_normalize: total must be > 0");
  hipError_t e = zb::launch_normalize(gae, advantages, count, moments, total, eps, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ZB_ELAUNCH, "zb_adv_normalize launch: %s", hipGetErrorString(e));
  return ZB_OK;
}

/* ---- GRU policy / value networks (include/zbot_policy.h) ---- */

struct ZbPolicy {
  int kind;
  int device;
  float* wpack;
  float* bias;
  int layout; /* ZB_POL_LAYOUT_* */
};

static int pol_in(int kind) { return kind == ZB_POL_ACTOR ? ZB_POL_ACTOR_IN : ZB_POL_CRITIC_IN; }
static int pol_out(int kind) { return kind == ZB_POL_ACTOR ? ZB_POL_ACTOR_OUT : 1; }

size_t zb_policy_param_count(int kind) {
  if (kind != ZB_POL_ACTOR && kind != ZB_POL_CRITIC) return 0;
  const size_t H = ZB_POL_HIDDEN, D = ZB_POL_DEPTH, I = (size_t)pol_in(kind), O = (size_t)pol_out(kind);
  return H * I + H + D * (6 * H * H + 4 * H) + O * H + O + (kind == ZB_POL_ACTOR ? ZB_POL_JOINTS : 0);
}

/* W [N][K] (natural layout) -> B fragments of v_mfma_f32_16x16x4_f32 [ceil(N/16)][ceil(K/16)][64][4]:
   element u of lane l in k-group g of tile t is W[16t + (l & 15)][16g + 4u + (l >> 4)]
   (zero outside W), so a lane reads 4 consecutive MFMA k-steps with one 16-B load */
static void pack_b(const float* W, int N, int K, std::vector<float>& out) {
  const int NT = (N + 15) / 16, G = (K + 15) / 16;
  for (int t = 0; t < NT; t++)
    for (int g = 0; g < G; g++)
      for (int l = 0; l < 64; l++)
        for (int u = 0; u < 4; u++) {
          const int row = 16 * t + (l & 15), k = 16 * g + 4 * u + (l >> 4);
          out.push_back(row < N && k < K ? W[(size_t)row * K + k] : 0.f);
        }
}

int zb_policy_create(int kind, const float* params, size_t n_params, int device, ZbPolicy** out) {
  if (!out || !params) return fail(ZB_EARG, "zb_policy_create: null argument");
  *out = nullptr;
  if (kind != ZB_POL_ACTOR && kind != ZB_POL_CRITIC) return fail(ZB_EARG, "zb_policy_create: unknown kind %d", kind);
  const size_t need = zb_policy_param_count(kind);
  if (n_params != need) return fail(ZB_EARG, "zb_policy_create: %zu parameters, expected %zu", n_params, need);
  const int H = ZB_POL_HIDDEN, D = ZB_POL_DEPTH, I = pol_in(kind), O = pol_out(kind);
  std::vector<float> wp, bias;
  const float* p = params;
  pack_b(p, H, I, wp); /* input_proj.weight */
  p += (size_t)H * I;
  bias.insert(bias.end(), p, p + H); /* input_proj.bias */
  p += H;
  for (int l = 0; l < D; l++) {
    pack_b(p, 3 * H, H, wp); /* weight_ih */
    p += (size_t)3 * H * H;
    pack_b(p, 3 * H, H, wp); /* weight_hh */
    p += (size_t)3 * H * H;
    bias.insert(bias.end(), p, p + 4 * H); /* bias [3H], bias_n [H] */
    p += 4 * H;
  }
  const float* wout = p;
  p += (size_t)O * H;
  bias.insert(bias.end(), p, p + O); /* output_proj.bias */
  p += O;
  if (kind == ZB_POL_ACTOR) {
    pack_b(wout, O, H, wp);
    bias.insert(bias.end(), p, p + ZB_POL_JOINTS); /* mean offsets (JOINT_BIASES) */
  } else {
    bias.insert(bias.end(), wout, wout + H); /* value head, natural layout */
  }
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(ZB_EDEVICE, "device %d not available (%d devices)", device, ndev);
  HIPCHK(hipSetDevice(device));
  ZbPolicy* h = new ZbPolicy();
  h->kind = kind;
  {
    const char* lay = getenv("ZB_POLICY_LAYOUT");
    h->layout = (lay && lay[0] == 'w') ? ZB_POL_LAYOUT_WAVE : ZB_POL_LAYOUT_BLOCK;
  }
  h->device = device;
  h->wpack = nullptr;
  h->bias = nullptr;
  hipError_t e = hipMalloc(&h->wpack, wp.size() * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&h->bias, bias.size() * sizeof(float));
  if (e == hipSuccess) e = hipMemcpy(h->wpack, wp.data(), wp.size() * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(h->bias, bias.data(), bias.size() * sizeof(float), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    zb_policy_destroy(h);
    return fail(ZB_EDEVICE, "zb_policy_create: %s", hipGetErrorString(e));
  }
  *out = h;
  return ZB_OK;
}

int zb_policy_destroy(ZbPolicy* h) {
  if (!h) return ZB_OK;
  (void)hipSetDevice(h->device);
  if (h->wpack) (void)hipFree(h->wpack);
  if (h->bias) (void)hipFree(h->bias);
  delete h;
  return ZB_OK;
}

static int policy_run(ZbPolicy* h, int kind, const float* obs, int T, int n, float* carry, const uint8_t* reset,
                      int mode, uint64_t seed, int env_offset, uint32_t step0, float* actions, float* log_prob,
                      float* value, void* stream) {
  if (!h) return fail(ZB_EARG, "null policy handle");
  if (h->kind != kind) return fail(ZB_EARG, "policy handle is a%s", h->kind == ZB_POL_ACTOR ? "n actor" : " critic");
  if (T < 0 || n < 0 || env_offset < 0) return fail(ZB_EARG, "bad size (T=%d n=%d offset=%d)", T, n, env_offset);
  if (T == 0 || n == 0) return ZB_OK;
  if (!obs || !carry) return fail(ZB_EARG, "null obs or carry");
  if (kind == ZB_POL_ACTOR) {
    if (!actions) return fail(ZB_EARG, "actor: null actions");
    if (mode != ZB_POL_SAMPLE && mode != ZB_POL_MODE && mode != ZB_POL_EVAL)
      return fail(ZB_EARG, "actor: unknown mode %d", mode);
  } else if (!value) {
    return fail(ZB_EARG, "critic: null value");
  }
  if ((uintptr_t)carry % 16) return fail(ZB_EARG, "carry must be 16-byte aligned");
  int cur = -1;
  HIPCHK(hipGetDevice(&cur));
  if (cur != h->device) HIPCHK(hipSetDevice(h->device));
  const size_t I = (size_t)pol_in(kind);
  for (int t = 0; t < T; t++) {
    zb::PolicyArgs a;
    memset(&a, 0, sizeof a);
    a.obs = obs + (size_t)t * n * I;
    a.carry = carry;
    a.reset = reset ? reset + (size_t)t * n : nullptr;
    a.n = n;
    a.mode = mode;
    a.seed = seed;
    a.env_offset = env_offset;
    a.step = step0 + (uint32_t)t;
    a.actions = actions ? actions + (size_t)t * n * ZB_POL_JOINTS : nullptr;
    a.log_prob = log_prob ? log_prob + (size_t)t * n * ZB_POL_JOINTS : nullptr;
    a.value = value ? value + (size_t)t * n : nullptr;
    a.wpack = h->wpack;
    a.bias = h->bias;
    a.layout = h->layout;
    hipError_t e = zb::launch_policy(kind, a, (hipStream_t)stream);
    if (e != hipSuccess) return fail(ZB_ELAUNCH, "policy launch: %s", hipGetErrorString(e));
  }
  return ZB_OK;
}

int zb_policy_set_layout(ZbPolicy* p, int layout) {
  if (!p) return fail(ZB_EARG, "null policy handle");
  if (layout != ZB_POL_LAYOUT_BLOCK && layout != ZB_POL_LAYOUT_WAVE && layout != ZB_POL_LAYOUT_WAVE2 &&
      layout != ZB_POL_LAYOUT_WAVE4)
    return fail(ZB_EARG, "unknown layout %d", layout);
  p->layout = layout;
  return ZB_OK;
}

int zb_policy_actor(ZbPolicy* p, const float* obs, int T, int n, float* carry, const uint8_t* reset, int mode,
                    uint64_t seed, int env_offset, uint32_t step0, float* actions, float* log_prob, void* stream) {
  return policy_run(p, ZB_POL_ACTOR, obs, T, n, carry, reset, mode, seed, env_offset, step0, actions, log_prob,
                    nullptr, stream);
}

int zb_policy_critic(ZbPolicy* p, const float* obs, int T, int n, float* carry, const uint8_t* reset, float* value,
                     void* stream) {
  return policy_run(p, ZB_POL_CRITIC, obs, T, n, carry, reset, ZB_POL_SAMPLE, 0, 0, 0, nullptr, nullptr, value,
                    stream);
}

#if defined(ZB_STAMPS) || defined(ZB_WAVETIME)
int zb_get_stamps(ZbHandle* h, void* out_dev, void* stream) {
  if (!h || !h->stamps) return fail(ZB_EARG, "no stamps");
  return copy_rows(h, out_dev, h->stamps, (size_t)h->n * ZB_NSTAMP * sizeof(unsigned long long), stream);
}
#endif

}  // extern "C"
