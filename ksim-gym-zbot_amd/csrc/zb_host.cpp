/*
 * zb_host.cpp — the host-only half of the C ABI (include/zbot.h): the error string, the
 * train.py default configuration, model / config validation and the per-lane team topology.
 * Plain C++ (no HIP): the product library links it, and csrc/sanitize.mk builds it with the host
 * sanitizers for tests/test_sanitizers.py.
 */
#include <cmath>
#include <cstdlib>
#include "zb_host.h"

#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <string>

namespace zb {

static thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

static bool in(int v, int lo, int hi) { return v >= lo && v < hi; } /* lo <= v < hi */

/* Every integer the kernels use as an index lies inside the array it indexes, so that no field of
   a model handed to zb_create can send a kernel outside its model copy, LDS rows or team lanes
   (an out-of-bounds access in a kernel faults the GPU). Counts first, then each table over the
   entries the engine reads. Found necessary by the mutation driver zb_host_selftest.cpp. */
static int check_indices(const ZbModel* m) {
  if (!in(m->nbody, 2, ZB_MAX_BODY + 1) || !in(m->nv, 1, ZB_MAX_DOF + 1) || !in(m->nq, 1, ZB_MAX_QPOS + 1) ||
      !in(m->nu, 0, ZB_MAX_ACT + 1) || !in(m->ngeom, 0, ZB_MAX_GEOM + 1) || !in(m->nsite, 0, ZB_MAX_SITE + 1) ||
      !in(m->max_depth, 1, ZB_MAX_DEPTH + 1) || !in(m->nlevel, 0, ZB_MAX_DEPTH + 1))
    return fail(ZB_EMODEL, "model counts out of range (nbody=%d nv=%d nq=%d nu=%d ngeom=%d nsite=%d depth=%d nlevel=%d)",
                m->nbody, m->nv, m->nq, m->nu, m->ngeom, m->nsite, m->max_depth, m->nlevel);
  const int NB = m->nbody, NV = m->nv, NQ = m->nq;
  if (m->body_parent[0] != -1) return fail(ZB_EMODEL, "body 0 (world) must have parent -1");
  for (int b = 0; b < NB; b++) {
    if (b > 0 && !in(m->body_parent[b], 0, b)) return fail(ZB_EMODEL, "body %d: parent %d not an earlier body", b, m->body_parent[b]);
    const int jt = m->body_jnttype[b];
    if (jt != ZB_JNT_NONE && jt != ZB_JNT_FREE && jt != ZB_JNT_HINGE) return fail(ZB_EMODEL, "body %d: joint type %d", b, jt);
    if (!in(m->body_depth[b], 0, 16) || !in(m->body_dofadr[b], -1, NV) || !in(m->body_dofnum[b], 0, 7) ||
        !in(m->body_qposadr[b], -1, NQ) || !in(m->body_lastdof[b], -1, NV) || !in(m->body_nchild[b], 0, 9))
      return fail(ZB_EMODEL, "body %d: a depth / dof / qpos index out of range", b);
    if (m->body_dofadr[b] >= 0 && m->body_dofadr[b] + m->body_dofnum[b] > NV)
      return fail(ZB_EMODEL, "body %d: dofs [%d, %d) past nv", b, m->body_dofadr[b], m->body_dofadr[b] + m->body_dofnum[b]);
    for (int c = 0; c < 8; c++)
      if (!in(m->body_child[b][c], -1, NB)) return fail(ZB_EMODEL, "body %d: child %d out of range", b, c);
  }
  for (int k = 0; k < NV; k++) {
    if (!in(m->dof_body[k], 1, NB) || !in(m->dof_parent[k], -1, k) || !in(m->dof_depth[k], 0, m->max_depth) ||
        !in(m->dof_qposadr[k], -1, NQ) || !in(m->dof_act[k], -1, m->nu) || !in(m->dof_rowoff[k], 0, 248 - 8) ||
        (m->dof_limited[k] != 0 && m->dof_limited[k] != 1))
      return fail(ZB_EMODEL, "dof %d: a body / parent / depth / qpos / actuator / row index out of range", k);
    for (int d = 0; d < ZB_MAX_DEPTH; d++)
      if (!in(m->dof_anc[k][d], -1, NV)) return fail(ZB_EMODEL, "dof %d: ancestor at depth %d out of range", k, d);
    if (m->dof_anc[k][m->dof_depth[k]] != k) return fail(ZB_EMODEL, "dof %d: not its own ancestor at its depth", k);
  }
  for (int a = 0; a < m->nu; a++)
    if (!in(m->act_dof[a], 0, NV)) return fail(ZB_EMODEL, "actuator %d: dof %d out of range", a, m->act_dof[a]);
  for (int g = 0; g < m->ngeom; g++)
    if (!in(m->geom_body[g], 1, NB) || !in(m->geom_lastdof[g], -1, NV) ||
        m->geom_lastdof[g] != m->body_lastdof[m->geom_body[g]])
      return fail(ZB_EMODEL, "geom %d: body / dof out of range", g);
  for (int s = 0; s < m->nsite; s++)
    if (!in(m->site_body[s], 0, NB)) return fail(ZB_EMODEL, "site %d: body %d out of range", s, m->site_body[s]);
  if (!in(m->site_imu, 0, m->nsite) || !in(m->site_left_foot, 0, m->nsite) || !in(m->site_right_foot, 0, m->nsite) ||
      !in(m->body_base, 1, NB) || !in(m->body_left_foot, 1, NB) || !in(m->body_right_foot, 1, NB) ||
      !in(m->geom_left_foot, 0, m->ngeom) || !in(m->geom_right_foot, 0, m->ngeom))
    return fail(ZB_EMODEL, "a named site / body / geom index is out of range");
  if (!in(m->max_body_depth, 0, 16) || !in(m->mrow_size, 0, 248 - 8 + 1))
    return fail(ZB_EMODEL, "max_body_depth %d / mrow_size %d out of range", m->max_body_depth, m->mrow_size);
  for (int d = 0; d < 16; d++)
    if (!in(m->depth_maxchild[d], 0, 9)) return fail(ZB_EMODEL, "depth_maxchild[%d] out of range", d);
  for (int l = 0; l < m->nlevel; l++) {
    if (!in(m->level_nmem[l], 0, 9)) return fail(ZB_EMODEL, "level %d: %d members", l, m->level_nmem[l]);
    for (int i = 0; i < m->level_nmem[l]; i++)
      if (!in(m->level_mem[l][i], 0, NV)) return fail(ZB_EMODEL, "level %d member %d out of range", l, i);
  }
  return ZB_OK;
}

int check_model(const ZbModel* m) {
  if (m->magic != ZB_MODEL_MAGIC) return fail(ZB_EARG, "model magic mismatch");
  if (m->version != ZB_MODEL_VERSION) return fail(ZB_EARG, "model version %d != %d", m->version, ZB_MODEL_VERSION);
  if (m->struct_bytes != (int32_t)sizeof(ZbModel))
    return fail(ZB_EARG, "model struct_bytes %d != %zu (layout mismatch)", m->struct_bytes, sizeof(ZbModel));
  if (int rc = check_indices(m)) return rc;
  if (m->nskip_geom != 0)
    return fail(ZB_EMODEL, "the source model has %d colliding geoms the engine does not collide with the floor (it "
                           "collides the 2 box soles): compile_model(..., drop_colliders=True) to simulate without "
                           "them knowingly", m->nskip_geom);
  if (m->nskip_pair != 0)
    return fail(ZB_EMODEL, "the source model collides %d pairs of its own geoms with each other; the engine "
                           "collides the robot with itself only as the two box soles against each other: "
                           "compile_model(..., drop_self_contacts=True) to simulate without them knowingly",
                m->nskip_pair);
  if (m->nbody > 32 || m->nv > 32 || m->nq > ZB_MAX_QPOS)
    return fail(ZB_EMODEL, "model too large for a 32-lane team (nbody=%d nv=%d nq=%d)", m->nbody, m->nv, m->nq);
  /* colliders: two banks of 32 contact-row lanes, 16 rows (4 contacts x 4 pyramid edges) per geom; the
     first bank holds geoms 0-1 (the soles), the second the first two others within reach of the floor
     each substep (zb_engine.hip select_bank2) */
  if (m->ngeom < 1 || m->ngeom > ZB_MAX_GEOM)
    return fail(ZB_EMODEL, "ngeom=%d: 1 to %d floor colliders", m->ngeom, ZB_MAX_GEOM);
  for (int g = 0; g < m->ngeom; g++) {
    const int ty = m->geom_type[g];
    const int nsz = (ty == ZB_GEOM_BOX || ty == ZB_GEOM_ELLIPSOID) ? 3
                    : (ty == ZB_GEOM_CAPSULE || ty == ZB_GEOM_CYLINDER) ? 2
                    : (ty == ZB_GEOM_SPHERE || ty == ZB_GEOM_MESH) ? 1 : 0;
    if (nsz == 0)
      return fail(ZB_EMODEL, "geom %d: type %d (mesh 7, box 6, cylinder 5, ellipsoid 4, capsule 3, sphere 2)", g, ty);
    for (int k = 0; k < nsz; k++)
      if (!(m->geom_size[g][k] > 0.f)) return fail(ZB_EMODEL, "geom %d: size[%d] must be positive", g, k);
    if (ty == ZB_GEOM_MESH) {
      /* the hull's vertices: a range of the pool, within the kernel's per-mesh limit */
      const int adr = m->geom_vertadr[g], num = m->geom_vertnum[g];
      if (num < 1 || num > ZB_MAX_MESHV || adr < 0 || adr + num > ZB_MAX_MESHVERT)
        return fail(ZB_EMODEL, "geom %d: mesh vertices [%d, %d + %d) (1 to %d hull vertices in a pool of %d)", g, adr,
                    adr, num, ZB_MAX_MESHV, ZB_MAX_MESHVERT);
      for (int i = adr; i < adr + num; i++)
        for (int k = 0; k < 3; k++)
          if (!std::isfinite(m->mesh_vert[i][k])) return fail(ZB_EMODEL, "geom %d: mesh vertex %d not finite", g, i - adr);
    }
  }
  if (m->max_depth > ZB_MAX_DEPTH) return fail(ZB_EMODEL, "dof depth %d > %d", m->max_depth, ZB_MAX_DEPTH);
  if (m->npair < 0 || m->npair > 1) return fail(ZB_EMODEL, "npair=%d: the sole pair at most", m->npair);
  if (m->npair == 1) {
    /* the sole pair (zb_engine.hip pair_rows): the two box soles (geoms 0 and 1, the touch sensors'),
       on two different limbs (its contact rows are one half-row per limb chain); with other floor
       colliders beside them its rows take a bank of their own (XG 4) */
    const int g1 = m->pair_geom[0], g2 = m->pair_geom[1];
    if (m->ngeom < 2 || !((g1 == 0 && g2 == 1) || (g1 == 1 && g2 == 0)))
      return fail(ZB_EMODEL, "the sole pair collides the two soles, geoms 0 and 1 (ngeom=%d, pair %d-%d)",
                  m->ngeom, g1, g2);
    if (m->geom_type[0] != ZB_GEOM_BOX || m->geom_type[1] != ZB_GEOM_BOX)
      return fail(ZB_EMODEL, "the sole pair collides two boxes (box-box)");
    int head[2];
    for (int k = 0; k < 2; k++) {
      int d = m->body_lastdof[m->geom_body[k]];
      if (d < 6) return fail(ZB_EMODEL, "sole %d hangs off the base: the pair needs both on limbs", k);
      while (m->dof_parent[d] >= 6) d = m->dof_parent[d];
      head[k] = d;
    }
    if (head[0] == head[1]) return fail(ZB_EMODEL, "the two soles of the pair are on one limb");
    if (!(m->pair_friction[0] >= 0.f) || !(m->pair_solref[0] > 0.f) || !(m->pair_solimp[1] > 0.f))
      return fail(ZB_EMODEL, "the sole pair's friction / solref / solimp are invalid");
  }
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
  /* the depths the engine is compiled for (zb_engine.hip MAXBD, MAXDD / NLIMBLV): the pointer-jumping
     passes cover bodies up to depth 8 and limb chains up to 6 dofs below the 6 root dofs */
  if (maxbd > TOPO_MAXBD || m->max_depth > 12 || m->nlevel > 12)
    return fail(ZB_EMODEL, "body depth %d (max %d), dof depth %d (max 12), %d levels (max 12)", maxbd, TOPO_MAXBD,
                m->max_depth, m->nlevel);
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

int needs_xg(const ZbModel* m) {
  /* the sole pair: alone with the soles (XG 3, the second bank holds the pair's rows), or beside other
     floor colliders (XG 4: the floor bank and a third bank for the pair's rows) */
  if (m->npair > 0) return m->ngeom > 2 ? 4 : 3;
  /* ZB_FORCE_XG=1 (profiling only): the two-sole model on the general-collider instantiation, whose
     second bank then stays empty, to time that kernel's overhead on the headline's work */
  const char* fx = getenv("ZB_FORCE_XG");
  if (m->ngeom == 2 && m->geom_type[0] == ZB_GEOM_BOX && m->geom_type[1] == ZB_GEOM_BOX)
    return (fx && fx[0] == '1') ? 1 : 0;
  /* more than two colliders beyond the soles: the second and third banks both hold floor colliders,
     the first four within reach of the floor each substep (XG 5, every collider type compiled) */
  if (m->ngeom > 4) return 5;
  for (int g = 0; g < m->ngeom; g++)
    if (m->geom_type[g] == ZB_GEOM_CYLINDER || m->geom_type[g] == ZB_GEOM_ELLIPSOID || m->geom_type[g] == ZB_GEOM_MESH)
      return 2;
  return 1;
}

int check_cfg(const ZbEnvConfig* c) {
  if (c->struct_bytes != (int32_t)sizeof(ZbEnvConfig))
    return fail(ZB_EARG, "config struct_bytes %d != %zu", c->struct_bytes, sizeof(ZbEnvConfig));
  if (c->n_substeps < 1 || c->iterations < 0 || c->ls_iterations < 0 || !(c->dt > 0.f))
    return fail(ZB_EARG, "invalid solver/timestep configuration");
  if (c->solver != (int32_t)ZB_SOLVER_NEWTON && c->solver != (int32_t)ZB_SOLVER_CG)
    return fail(ZB_EARG, "unknown solver %d", c->solver);
  return ZB_OK;
}

/* The per-lane roles of a 32-lane team (body lane, dof lane, limb-chain position, contact
   rows holding the dof, actuator), computed once here instead of by every wave at the top
   of every launch. Field-major [TP_NF][32]; the checks of check_model hold. */
void build_topology(const ZbModel* m, int32_t t[zb::TP_NF][zb::TOPO_LANES]) {
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
    /* contact rows of geom g: bank g / 2, lanes 16 (g % 2) .. + 15 */
    uint32_t rm[2] = {0u, 0u};
    for (int g = 0; g < m->ngeom && g < 2 * TOPO_NGEOM; g++) {
      const int kd = m->body_lastdof[m->geom_body[g]];
      if (isd && kd >= 0 && (kd == l || ((desc >> kd) & 1u))) rm[g / 2] |= 0xFFFFu << (16 * (g % 2));
    }
    uint32_t rp = 0u;
    if (m->npair > 0) {
      /* the sole pair's rows (the second bank with the soles alone, XG 3; a third bank beside other
         floor colliders, XG 4): lanes 0-15 the half rows on geom2's limb (+J), lanes 16-31 those on
         geom1's limb (-J); the root dofs' columns cancel, so a limb dof only */
      for (int h = 0; h < 2; h++) {
        const int kd = m->body_lastdof[m->geom_body[m->pair_geom[1 - h]]];
        if (isd && l >= 6 && kd >= 0 && (kd == l || ((desc >> kd) & 1u))) rp |= 0xFFFFu << (16 * h);
      }
      if (m->ngeom == 2) {
        rm[1] = rp;
        rp = 0u;
      }
    }
    t[TP_ROWMASK][l] = (int32_t)rm[0];
    t[TP_ROWMASK2][l] = (int32_t)rm[1];
    t[TP_ROWMASK3][l] = (int32_t)rp;
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

}  // namespace zb

using zb::fail;

extern "C" {

const char* zb_last_error(void) { return zb::g_err.c_str(); }

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
  c->solver = (int32_t)ZB_SOLVER_CG; /* MJX's CG, as ksim's model setup selects it [U] */
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

}  // extern "C"
