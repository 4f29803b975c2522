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

using zb::build_topology;
using zb::check_cfg;
using zb::check_model;
using zb::fail;

#define ZB_ABI_VERSION 3

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
  float* xj;       /* general colliders: [n + 1, ZB_XJ_STRIDE] second-bank Jacobian rows (zb_internal.h) */
  int xg;          /* needs_xg(model), decided once in zb_create: every launch uses the instantiation that
                      xj was (or was not) allocated for, whatever ZB_FORCE_XG says later */
  int nchunk;      /* work units per pair of envs in zb_step (1: unchunked) */
  int air_mark;    /* zb_mark_rollout_start: the next zb_step / zb_rollout is a rollout's step 0 */
  int air_marked;  /* a marked step has been launched since the last zb_feet_airtime_exact */
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
  /* [0] units taken, [1] pairs finished, [2 + pair] per-pair progress, [2 + npair] sticky error */
  if (e == hipSuccess) e = hipMalloc(&h->sched, (3 + (n + 1) / 2) * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemset(h->sched, 0, (3 + (n + 1) / 2) * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMalloc(&h->itpart, n * sizeof(int32_t));
  if (e == hipSuccess) e = hipMemset(h->itpart, 0, n * sizeof(int32_t));
  h->xg = zb::needs_xg(model);
  /* XG 4: two banks in global scratch per env (the floor selection, the sole pair) */
  if (e == hipSuccess && h->xg) e = hipMalloc(&h->xj, (n + 1) * ZB_XJ_STRIDE * (h->xg == 4 || h->xg == 5 ? 2 : 1) * sizeof(float));
  h->nchunk = choose_chunks(n_envs, cfg->n_substeps, zb::step_resident_blocks(device, h->xg, cfg->solver, (cfg->flags & ZB_F_EULERDAMP) ? 1 : 0));
#if defined(ZB_STAMPS) || defined(ZB_WAVETIME)
  {
    /* phase stamps: ZB_NSTAMP per env; wave times: 4 words per (chunk, pair), up to one chunk per
       substep (zb_set_step_chunks clamps to n_substeps) */
    size_t words = n * ZB_NSTAMP, wt = 4 * (size_t)cfg->n_substeps * ((n + 1) / 2);
    if (e == hipSuccess) e = hipMalloc(&h->stamps, (words > wt ? words : wt) * sizeof(unsigned long long));
  }
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
  if (h->xj) (void)hipFree(h->xj);
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
  a.solver = h->cfg.solver;
  a.xg = h->xg;
  a.ed = (h->cfg.flags & ZB_F_EULERDAMP) ? 1 : 0;
  a.xj = h->xj;
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
  if (!h || (!action && h->n > 0)) return fail(ZB_EARG, "zb_step: null handle or action");
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
  a.air_mark = h->air_mark;
  hipError_t e = zb::launch_step(a, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ZB_ELAUNCH, "zb_step launch: %s", hipGetErrorString(e));
  if (h->air_mark) h->air_marked = 1;
  h->air_mark = 0;
  return ZB_OK;
}

int zb_rollout(ZbHandle* h, const float* actions, int n_steps, float* obs_actor, float* obs_critic, float* reward_sum,
               uint8_t* done, uint8_t* success, float curriculum_level, void* stream) {
  if (!h || (!actions && h->n > 0) || n_steps < 1) return fail(ZB_EARG, "zb_rollout: bad argument");
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
  a.air_mark = h->air_mark;
  hipError_t e = zb::launch_step(a, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ZB_ELAUNCH, "zb_rollout launch: %s", hipGetErrorString(e));
  if (h->air_mark) h->air_marked = 1;
  h->air_mark = 0;
  return ZB_OK;
}

int zb_mark_rollout_start(ZbHandle* h) {
  if (!h) return fail(ZB_EARG, "zb_mark_rollout_start: null handle");
  h->air_mark = 1;
  h->air_marked = 0;
  return ZB_OK;
}

int zb_feet_airtime_exact(ZbHandle* h, float* reward0, float* reward_terms0, float curriculum_level, void* stream) {
  if (!h) return fail(ZB_EARG, "zb_feet_airtime_exact: null handle");
  if (!h->air_marked)
    return fail(ZB_EARG, "zb_feet_airtime_exact: no step of a marked rollout since zb_mark_rollout_start "
                         "(or already patched)");
  if (!(curriculum_level == curriculum_level)) return fail(ZB_EARG, "zb_feet_airtime_exact: curriculum is NaN");
  int rc = use_device(h);
  if (rc) return rc;
  zb::StepArgs a = base_args(h);
  a.reward = reward0;
  a.reward_terms = reward_terms0;
  a.curriculum = curriculum_level;
  hipError_t e = zb::launch_airtime_exact(a, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ZB_ELAUNCH, "zb_feet_airtime_exact launch: %s", hipGetErrorString(e));
  h->air_marked = 0;
  return ZB_OK;
}

static int copy_rows(ZbHandle* h, void* dst, const void* src, size_t bytes, void* stream) {
  if (h && bytes == 0) return ZB_OK; /* a handle over zero envs (an empty shard) */
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
    h->nchunk = choose_chunks(h->n, h->cfg.n_substeps, zb::step_resident_blocks(h->device, h->xg, h->cfg.solver, (h->cfg.flags & ZB_F_EULERDAMP) ? 1 : 0));
  } else {
    h->nchunk = k > h->cfg.n_substeps ? h->cfg.n_substeps : k;
  }
  return ZB_OK;
}

int zb_check(ZbHandle* h) {
  if (!h) return fail(ZB_EARG, "zb_check: null handle");
  int rc = use_device(h);
  if (rc) return rc;
  const size_t npair = ((size_t)(h->n > 0 ? h->n : 1) + 1) / 2;
  uint32_t err = 0;
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(&err, h->sched + 2 + npair, sizeof err, hipMemcpyDeviceToHost));
  if (err) {
    /* the chunk counters may be left mid-protocol: clear them so the next launch starts clean */
    HIPCHK(hipMemset(h->sched, 0, (3 + npair) * sizeof(uint32_t)));
    return fail(ZB_ESTATE, "a chunked zb_step timed out waiting for a predecessor chunk: the state of the "
                           "launches since the last zb_check is invalid (zb_set_state / zb_reset to recover)");
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
  int persistent; /* block layout: one launch per call over all T steps */
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
  h->persistent = 1;
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
  /* the 8-wave block layout runs all T steps in one persistent launch (carry kept in registers,
     zb_policy.hip); the slot-sized layouts launch once per step */
  const int per_launch = (h->layout == ZB_POL_LAYOUT_BLOCK && h->persistent) ? T : 1;
  for (int t = 0; t < T; t += per_launch) {
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
    a.T = per_launch;
    hipError_t e = zb::launch_policy(kind, a, (hipStream_t)stream);
    if (e != hipSuccess) return fail(ZB_ELAUNCH, "policy launch: %s", hipGetErrorString(e));
  }
  return ZB_OK;
}

int zb_policy_set_persistent(ZbPolicy* p, int on) {
  if (!p) return fail(ZB_EARG, "null policy handle");
  p->persistent = on ? 1 : 0;
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
