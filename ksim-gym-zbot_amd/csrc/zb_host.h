/*
 * zb_host.h — host-only pieces of the C ABI (zb_host.cpp): model / config validation, the
 * per-lane team topology zb_create uploads, the thread-local error string. No HIP here, so the
 * same source builds under the host sanitizers (csrc/sanitize.mk, tests/test_sanitizers.py).
 * Not part of the public ABI.
 */
#ifndef ZB_HOST_H
#define ZB_HOST_H

#include <stdint.h>

#include "zbot.h"

namespace zb {

/* per-lane topology of a team (32 lanes), built once by zb_create from the model
   (zb_capi.cpp build_topology) and read by the kernels' make_ctx: field-major
   [TP_NF][32] int32 */
enum {
  TP_BPAR, TP_BDEP, TP_BJT, TP_BDOFADR, TP_BLAST, TP_NCH, TP_CH0, TP_CH1, TP_LVL_LO, TP_LVL_HI,
  TP_DDEP, TP_DBODY, TP_QADR, TP_ACT, TP_ROWMASK, TP_ROWMASK2, TP_ROWMASK3, TP_DK0, TP_DFREE, TP_CHD, TP_CPS, TP_CLN, TP_NF
};
constexpr int TOPO_LANES = 32;
constexpr int TOPO_NROOT = 6;  /* root dof chain (the free joint), zb_engine.hip NROOT */
constexpr int TOPO_NGEOM = 2;  /* geoms per contact-row bank, zb_engine.hip NGEOM */
constexpr int TOPO_MAXBD = 8;  /* deepest body, zb_engine.hip MAXBD */

/* fail(): record the message for zb_last_error() and return `code` */
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
/* ZB_OK, or ZB_EARG / ZB_EMODEL with the reason in zb_last_error() */
int check_model(const ZbModel* m);
int check_cfg(const ZbEnvConfig* c);
/* the model needs the general-collider kernels (anything but exactly two box soles) */
int needs_xg(const ZbModel* m); /* 0 two-sole, 1 general colliders, 2 with cylinders / ellipsoids / meshes, 3 the sole pair alone, 4 the sole pair beside other colliders, 5 more than two colliders beyond the soles (two floor banks) */
/* requires check_model(m) == ZB_OK */
void build_topology(const ZbModel* m, int32_t t[TP_NF][TOPO_LANES]);

}  // namespace zb

#endif
