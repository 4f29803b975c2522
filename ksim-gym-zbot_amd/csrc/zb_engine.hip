/*
 * zb_engine.hip — MI355X (gfx950) batched Z-Bot env.step()/reset() engine.
 *
 * Replaces, per environment, ksim's step_engine over MuJoCo-MJX:
 *   20 x [FeetechActuators.get_stateful_ctrl (train.py:1242-1280) -> mj_step]
 *   -> terminations (train.py:1588-1593) -> reward terms (train.py:1546-1586)
 *   -> observations (train.py:1478-1537, 1624-1679) -> auto-reset (train.py:1471-1476)
 *
 * Execution model:
 *   - one TEAM of 32 lanes simulates one environment; a 64-lane wavefront
 *     holds two teams; a workgroup is exactly one wavefront, so "team sync"
 *     is a single-wave barrier (LDS ordering only, no cross-wave traffic);
 *   - lane l plays three roles: body l (kinematics, inertias, velocities),
 *     dof l (mass-matrix row, factor row, accelerations) and constraint row l
 *     (the 32 pyramid edges of the 8 sole/floor contacts);
 *   - the dof tree is stored "depth-indexed": row j of M / L holds the
 *     entries (j, anc_e(j)) for e = 0..depth(j) (MuJoCo's sparse tree layout,
 *     mj_factorM), so every row fits 12 registers/LDS words;
 *   - all 20 substeps of a control step, the Newton solve, sensors, rewards,
 *     observations and auto-reset run inside ONE launch; HBM traffic is one
 *     read and one write of the env's state row plus its outputs.
 *
 * Numerics: fp32 like the reference (JAX x64 off). Team reductions are xor
 * butterflies, so every lane of a team holds the bit-identical sum and all
 * team-uniform decisions agree. Results are deterministic run to run and
 * independent of how envs are sharded (RNG keyed by global env id).
 */
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <type_traits>

#include "zb_internal.h"

/* The product library compiles this file twice (Makefile): once for the collider sets (XG) whose step
   kernels run fastest under the iterative-ILP machine scheduler, once, with ZB_ENGINE_TU_B, for the
   others under the default one (the scheduler is chosen per compilation unit). ZB_XG_MASK: the XG
   values whose kernels this unit compiles; the entry points of the first unit hand the others' to the
   second unit's (*_tu_b). Without the defines (diagnostic builds) one unit holds every XG. */
#ifndef ZB_XG_MASK
#define ZB_XG_MASK 0x3F
#endif
#ifdef ZB_ENGINE_TU_B
#define ZB_EP(f) f##_tu_b
#else
#define ZB_EP(f) f
#endif

namespace zb {
constexpr int XG_MASK = ZB_XG_MASK;
__host__ __device__ constexpr bool xg_here(int xg) { return ((XG_MASK >> xg) & 1) != 0; }
#if !defined(ZB_ENGINE_TU_B) && ZB_XG_MASK != 0x3F
int step_resident_blocks_tu_b(int device, int xg, int solver, int ed);
hipError_t launch_step_tu_b(const StepArgs& a, hipStream_t s);
hipError_t launch_reset_tu_b(const StepArgs& a, hipStream_t s);
hipError_t launch_debug_forward_tu_b(const StepArgs& a, hipStream_t s);
#define ZB_HANDOFF(xg, fn, ...)                 \
  do {                                          \
    if (!xg_here(xg)) return fn##_tu_b(__VA_ARGS__); \
  } while (0)
#else
/* an XG this unit does not hold never reaches it (the first unit hands it off): fail loudly */
template <typename T>
constexpr T not_here() {
  if constexpr (std::is_same<T, hipError_t>::value) return hipErrorInvalidValue;
  else return T{};
}
#define ZB_HANDOFF(xg, fn, ...)                                          \
  do {                                                                   \
    if (!xg_here(xg)) return not_here<decltype(ZB_EP(fn)(__VA_ARGS__))>(); \
  } while (0)
#endif

constexpr int TEAM = 32;
constexpr int NTEAM = 64 / TEAM;
constexpr int CAP = ZB_MAX_DEPTH; /* 12 */
constexpr float MINVAL = 1e-15f;
constexpr float MINIMP = 0.0001f;
constexpr float MAXIMP = 0.9999f;
constexpr float DEADBAND = (float)(2.0 * 0.087 * 3.14159265358979323846 / 180.0); /* train.py:1113-1116 */

enum { V_QVEL = 0, V_TMP = 1, V_TMP2 = 2, NVEC = 3 };
constexpr int RMAX = 6;  /* root dof chain factored as one dense block: the free joint */
/* task topology, fixed by the C-ABI (zb_create checks the model against it):
   26 bodies, nv = 6 (free joint) + 20 hinges, root dof chain of length 6 */
constexpr int NB = ZB_NBODY_TASK;
constexpr int NV = 6 + ZB_NJ;
constexpr int NROOT = RMAX;
constexpr int NGEOM = 2;      /* geoms per contact-row bank (bank 0: the two foot soles) */
constexpr int MAXBD = 8;      /* deepest body (world 0, base 1, ..., foot 8) */
constexpr int MAXDD = 12;     /* dof chain depth: 6 root + 6 leg */
constexpr int NLIMBLV = 6;    /* elimination levels inside the limbs (longest limb) */
enum { P_Q0 = 0, P_ARM = 1, P_DAMP = 2, P_FLOSS = 3, P_MSCALE = 4 };
/* stamp slots: STAMP(i) closes phase i (time since the previous stamp) */
enum {
  S_FEETECH, S_KIN, S_CRB, S_FACM, S_RNE, S_SOLVES, S_CON, S_WARM, S_UPD0, S_HESS0, S_SOLVE0, S_LS, S_UPD,
  S_HESS, S_SOLVE, S_CHECK, S_SENS, S_INT, S_STEPEND, S_ENTRY, NSTAMP
};
static_assert(NSTAMP == ZB_NSTAMP, "stamp slots");

/* per-env scalars: one copy per team in LDS, read by every lane (broadcast) and
   written by every lane with the bit-identical value it computed */
struct EnvS {
  float bp[3], bq[4];
  float ema[4], lag, air[2], push_timer, touch[2], feet_dist, ep_ret, prev_cont[2];
  uint32_t ep_steps, rng_step, episode, nanflag;
  float floor_mu, imu_q[4], imu_p[3];
  /* the team's RNG identity (global env id, seed): read only at draw sites (observation noise,
     pushes, resets), so kept here rather than in registers across the substep loop */
  uint32_t env, seed_lo, seed_hi;
  /* XG kernels: the env's block of second-bank Jacobian rows in global scratch (xrows) */
  uint32_t xj_lo, xj_hi;
  /* XG 1 / 2: the geoms in the second contact-row bank this substep (half 0, half 1; -1: none):
     the first two of geoms 2.. within reach of the floor (select_bank2) */
  int32_t xsel[2];
};
struct Sensors {
  float fq[4], gyro[3], acc[3], touch[2], force[6];
};
/* per-environment LDS working set */
struct __align__(16) EnvL {
  float cdof[32][6];
  float M[32][CAP];
  float L[32][CAP];
  struct {
    float J[32][CAP];     /* contact-row Jacobians (constraint phase) */
  } u;
  union {
    float sub[32][10];      /* subtree sums (smooth phase, sensors) */
    struct {
      float Hs[32][CAP]; /* unfactored Newton Hessian rows (16-byte aligned for ld_row) */
      float Hsd[32];     /* and their diagonals */
    };
  };
  float vec[NVEC][32];
  float rowDA[32];
  float rowF[32];
  float Dk[32];
  float Di[32];      /* 1 / pivot of the root-chain block */
  float ci[32][10];  /* body cinert (lane b), kept for RNE / sensors / observations */
  float par[5][32];  /* effective dof / body parameters (lane), see P_* */
  float tgt[32];     /* general-collider kernels: the action target of the actuated dof lanes (held in a
                        VGPR, the register allocator of those kernels spilled it and reloaded it from
                        scratch at the head of every substep) */
  EnvS s;
  Sensors sen;
  /* XG 5: the third bank's geoms this substep (the third and fourth within reach; -1: none). Kept
     behind the sensors rather than in EnvS so every field the other kernels address keeps its offset
     and alignment (it fills the struct's tail padding) */
  int32_t ysel[2];
#ifdef ZB_STAMPS
  unsigned long long stamp[NSTAMP];
  unsigned long long stamp_last;
#endif
};


/* the block's two team working sets (one wave = two teams) */
__shared__ EnvL g_lds[NTEAM];


/* ----------------------------- team primitives ----------------------------- */
__device__ __forceinline__ float tsh(float v, int src) { return __shfl(v, src, TEAM); }
__device__ __forceinline__ int tshi(int v, int src) { return __shfl(v, src, TEAM); }
/* value of v in lane k (team-relative, uniform k) of this lane's team: two
   readlanes and a select, no LDS */
__device__ __forceinline__ float team_lane(float v, int k) {
  const int a = __builtin_amdgcn_readlane(__float_as_int(v), k);
  const int b = __builtin_amdgcn_readlane(__float_as_int(v), k + TEAM);
  return __int_as_float((threadIdx.x & TEAM) ? b : a);
}
/* DPP butterfly within 16-lane rows (quad xor 1, xor 2, half-row mirror, row
   mirror), then one cross-row exchange (xor 16). Every pairing is symmetric,
   so all lanes of a team end with the bit-identical result. */
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dppi(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
/* value of lane l ^ 16 (the other 16-lane row of the team) without LDS:
   v_permlane16_swap exchanges rows 0<->1 and 2<->3 of two copies */
__device__ __forceinline__ uint32_t xor16(uint32_t v) {
  auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  return (threadIdx.x & 16) ? r[0] : r[1];
}
__device__ __forceinline__ float xor16f(float v) { return __uint_as_float(xor16(__float_as_uint(v))); }
/* the two 16-lane rows of each team, broadcast: r[0] = row 0's value, r[1] =
   row 1's, in every lane. A symmetric combine of the pair needs no select. */
__device__ __forceinline__ void rows2(float v, float& a, float& b) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}
__device__ __forceinline__ int rows2max(int v) {
  auto r = __builtin_amdgcn_permlane16_swap((uint32_t)v, (uint32_t)v, false, false);
  return max((int)r[0], (int)r[1]);
}
__device__ __forceinline__ float tsum(float v) {
  v += dppf<0xB1>(v);
  v += dppf<0x4E>(v);
  v += dppf<0x141>(v);
  v += dppf<0x140>(v);
  float a, b;
  rows2(v, a, b);
  return a + b;
}
/* N independent team sums, stage by stage so the DPP/permlane steps of
   different values interleave (bit-identical to N separate tsum calls) */
template <int N>
__device__ __forceinline__ void tsum_n(float v[N]) {
#pragma unroll
  for (int i = 0; i < N; i++) v[i] += dppf<0xB1>(v[i]);
#pragma unroll
  for (int i = 0; i < N; i++) v[i] += dppf<0x4E>(v[i]);
#pragma unroll
  for (int i = 0; i < N; i++) v[i] += dppf<0x141>(v[i]);
#pragma unroll
  for (int i = 0; i < N; i++) v[i] += dppf<0x140>(v[i]);
  /* the row exchange two values at a time: one swap of (v[i], v[i + 1]) puts value i's two row sums
     side by side in rows 0 / 2 and value i + 1's in rows 1 / 3; their sum, swapped with itself, sends
     each value's team total to all 32 lanes. The same additions in the same order as rows2 + add */
#pragma unroll
  for (int i = 0; i + 1 < N; i += 2) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[i]), __float_as_uint(v[i + 1]), false, false);
    const float t = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    auto q = __builtin_amdgcn_permlane16_swap(__float_as_uint(t), __float_as_uint(t), false, false);
    v[i] = __uint_as_float(q[0]);
    v[i + 1] = __uint_as_float(q[1]);
  }
  if constexpr ((N & 1) != 0) {
    float a, b;
    rows2(v[N - 1], a, b);
    v[N - 1] = a + b;
  }
}
/* 21 team sums (the root Schur complement), written to out[0..20] in LDS: a
 * transposing butterfly instead of 21 all-lane reductions. Rows 0/1 of the team
 * first exchange halves with v_permlane16_swap (value i stays in row 0, value
 * 11 + i in row 1), then four DPP stages inside each 16-lane row each keep the
 * half of the slots on the lane's side and add the partner's copy of them, so
 * lane 16r + c ends with the full sum of value 11r + c (67 VALU instructions
 * instead of 126). The caller syncs before reading out[]. */
__device__ __forceinline__ void reduce21_to(const float v[21], float* out) {
  float w[16];
#pragma unroll
  for (int i = 0; i < 11; i++) {
    const float hi = i + 11 < 21 ? v[i + 11] : 0.f;
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[i]), __float_as_uint(hi), false, false);
    w[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
#pragma unroll
  for (int i = 11; i < 16; i++) w[i] = 0.f;
  const int li = threadIdx.x & 15;
  float u8[8], u4[4], u2[2];
  const bool s1 = li >= 8;
#pragma unroll
  for (int k = 0; k < 8; k++) u8[k] = (s1 ? w[8 + k] : w[k]) + dppf<0x140>(s1 ? w[k] : w[8 + k]);
  const bool s2 = (li & 4) != 0;
#pragma unroll
  for (int k = 0; k < 4; k++) u4[k] = (s2 ? u8[4 + k] : u8[k]) + dppf<0x141>(s2 ? u8[k] : u8[4 + k]);
  const bool s3 = (li & 2) != 0;
#pragma unroll
  for (int k = 0; k < 2; k++) u2[k] = (s3 ? u4[2 + k] : u4[k]) + dppf<0x4E>(s3 ? u4[k] : u4[2 + k]);
  const bool s4 = (li & 1) != 0;
  const float sum = (s4 ? u2[1] : u2[0]) + dppf<0xB1>(s4 ? u2[0] : u2[1]);
  const int idx = ((threadIdx.x & 16) ? 11 : 0) + li;
  if (li < 11 && idx < 21) out[idx] = sum;
}
/* six team sums, lane i (< 6) receiving sum i: a transposing butterfly (plain pair add
 * with the row mirror, then three stages that each keep the half of the slots selected by
 * one lane bit: slot = lane & 7), then the two 16-lane rows added. 29 VALU instructions
 * instead of tsum_n<6>'s 42. */
__device__ __forceinline__ float reduce6_lane(const float v[6]) {
  const int li = threadIdx.x & 15;
  float q[8];
#pragma unroll
  for (int k = 0; k < 6; k++) q[k] = v[k] + dppf<0x140>(v[k]);
  q[6] = q[7] = 0.f;
  const bool s2 = (li & 4) != 0;
  float u4[4];
#pragma unroll
  for (int k = 0; k < 4; k++) u4[k] = (s2 ? q[4 + k] : q[k]) + dppf<0x141>(s2 ? q[k] : q[4 + k]);
  const bool s1 = (li & 2) != 0;
  float u2[2];
#pragma unroll
  for (int k = 0; k < 2; k++) u2[k] = (s1 ? u4[2 + k] : u4[k]) + dppf<0x4E>(s1 ? u4[k] : u4[2 + k]);
  const bool s0 = (li & 1) != 0;
  const float r = (s0 ? u2[1] : u2[0]) + dppf<0xB1>(s0 ? u2[0] : u2[1]);
  float a, b;
  rows2(r, a, b);
  return a + b;
}
/* K team sums written to out[0..K-1] in LDS by a transposing butterfly (the K <= 16
 * generalisation of reduce21_to): the two 16-lane rows exchange halves (value i stays in
 * row 0, value H + i goes to row 1), then the four DPP pairings inside a row either add
 * (while there are fewer slots than lanes to spread them over) or keep the half of the
 * slots selected by one lane bit, so that lane 16r + s ends with value rH + s. The caller
 * syncs before reading out[]. */
template <int K>
__device__ __forceinline__ void reduce_to_lds(const float v[K], float* out) {
  constexpr int H = (K + 1) / 2;
  constexpr int S = H <= 2 ? 2 : (H <= 4 ? 4 : (H <= 8 ? 8 : 16));
  static_assert(K <= 32 && H <= 16, "two rows of 16 slots");
  float w[16];
#pragma unroll
  for (int i = 0; i < H; i++) {
    const float hi = i + H < K ? v[i + H] : 0.f;
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[i]), __float_as_uint(hi), false, false);
    w[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
#pragma unroll
  for (int i = H; i < 16; i++) w[i] = 0.f;
  const int li = threadIdx.x & 15;
  /* stage 1: row mirror (lane ^ 15); selects on bit 3 when there are 16 slots */
  if constexpr (S == 16) {
    const bool s3 = li >= 8;
#pragma unroll
    for (int k = 0; k < 8; k++) w[k] = (s3 ? w[8 + k] : w[k]) + dppf<0x140>(s3 ? w[k] : w[8 + k]);
  } else {
#pragma unroll
    for (int k = 0; k < H; k++) w[k] += dppf<0x140>(w[k]);
  }
  /* stage 2: half-row mirror (lane ^ 7); bit 2 when there are 8 or more slots */
  if constexpr (S >= 8) {
    const bool s2 = (li & 4) != 0;
#pragma unroll
    for (int k = 0; k < 4; k++) w[k] = (s2 ? w[4 + k] : w[k]) + dppf<0x141>(s2 ? w[k] : w[4 + k]);
  } else {
#pragma unroll
    for (int k = 0; k < (H < 4 ? H : 4); k++) w[k] += dppf<0x141>(w[k]);
  }
  /* stage 3: lane ^ 2, bit 1 (S >= 4) */
  if constexpr (S >= 4) {
    const bool s1 = (li & 2) != 0;
#pragma unroll
    for (int k = 0; k < 2; k++) w[k] = (s1 ? w[2 + k] : w[k]) + dppf<0x4E>(s1 ? w[k] : w[2 + k]);
  } else {
#pragma unroll
    for (int k = 0; k < 2; k++) w[k] += dppf<0x4E>(w[k]);
  }
  /* stage 4: lane ^ 1, bit 0 */
  const bool s0 = (li & 1) != 0;
  const float sum = (s0 ? w[1] : w[0]) + dppf<0xB1>(s0 ? w[0] : w[1]);
  const int slot = li & (S - 1);
  const int idx = ((threadIdx.x & 16) ? H : 0) + slot;
  if (li < S && slot < H && idx < K) out[idx] = sum;
}
/* the largest v over the lane's 16-lane row (every lane of the row ends with it) */
__device__ __forceinline__ float rowmax16(float v) {
  v = fmaxf(v, dppf<0xB1>(v));
  v = fmaxf(v, dppf<0x4E>(v));
  v = fmaxf(v, dppf<0x141>(v));
  v = fmaxf(v, dppf<0x140>(v));
  return v;
}
/* (w, i) with the row's largest w, the smallest i among equal w (jnp.argmax's first maximum) */
__device__ __forceinline__ void rowargmax16(float& w, int& i) {
  auto take = [&](float w2, int i2) {
    const bool t = w2 > w || (w2 == w && i2 < i);
    w = t ? w2 : w;
    i = t ? i2 : i;
  };
  take(dppf<0xB1>(w), dppi<0xB1>(i));
  take(dppf<0x4E>(w), dppi<0x4E>(i));
  take(dppf<0x141>(w), dppi<0x141>(i));
  take(dppf<0x140>(w), dppi<0x140>(i));
}
__device__ __forceinline__ float tmaxf(float v) {
  v = fmaxf(v, dppf<0xB1>(v));
  v = fmaxf(v, dppf<0x4E>(v));
  v = fmaxf(v, dppf<0x141>(v));
  v = fmaxf(v, dppf<0x140>(v));
  float a, b;
  rows2(v, a, b);
  return fmaxf(a, b);
}
__device__ __forceinline__ int tmaxi(int v) {
  v = max(v, dppi<0xB1>(v));
  v = max(v, dppi<0x4E>(v));
  v = max(v, dppi<0x141>(v));
  v = max(v, dppi<0x140>(v));
  return rows2max(v);
}
/* The team exchange point. A workgroup is one wave, and the LDS unit executes one wave's
   DS instructions in issue order, so a lane's ds_write is seen by any later ds_read or
   ds_bpermute of the wave: no s_barrier and no lgkmcnt drain are needed, only a point the
   compiler cannot move LDS accesses across. */
__device__ __forceinline__ void tsync() {
  static_assert(NTEAM * TEAM == 64, "one wave per workgroup");
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}
/* a loaded value pinned in place: `t = keepf(load); p ? t : k` stays a load and a select. Without
   it the compiler sinks the load into a branch of its own, with a full LDS round trip
   (s_waitcnt lgkmcnt(0)) per element instead of all loads in flight. */
__device__ __forceinline__ float keepf(float v) {
  asm volatile("" : "+v"(v));
  return v;
}
/* bitmask over the team's lanes of predicate p */
__device__ __forceinline__ uint32_t team_ballot(bool p) { return (uint32_t)(__ballot(p) >> (threadIdx.x & 32)); }
/* An opaque copy of a per-lane constant: stops the compiler from hoisting
   compares against it (e.g. the 12 `e < depth` lane masks) out of the step
   loops, where they would pin SGPR pairs for the whole launch. */
__device__ __forceinline__ int vopq(int x) {
  asm volatile("" : "+v"(x));
  return x;
}
/* a compile-time bool as a value (a generic lambda's argument picks its instantiation) */
template <bool B>
struct BoolC {
  static constexpr bool value = B;
};
template <int N>
struct IntC {
  static constexpr int value = N;
};

/* Diagnostic phase stamps (separate build, -DZB_STAMPS): cycles per phase of the
   step, accumulated per env; never compiled into the product library. */
#ifdef ZB_STAMPS
__device__ __forceinline__ void zb_stamp(EnvL* L, int i) {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  if ((threadIdx.x & (TEAM - 1)) == 0) {
    L->stamp[i] += (t - L->stamp_last) + (1ull << 44); /* cycles (low 44 bits) + call count */
    L->stamp_last = t;
  }
}
#define STAMP(i) zb_stamp(c.L, i)
#else
#define STAMP(i) ((void)0)
#endif

/* ------------------------------- small math -------------------------------- */
__device__ __forceinline__ void cross3(float r[3], const float a[3], const float b[3]) {
  float t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
__device__ __forceinline__ float dot3(const float a[3], const float b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
__device__ __forceinline__ void quat_mul(float r[4], const float a[4], const float b[4]) {
  float w = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  float x = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  float y = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  float z = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  r[0] = w; r[1] = x; r[2] = y; r[3] = z;
}
__device__ __forceinline__ void quat_normalize(float q[4]) {
  float n = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < MINVAL) { q[0] = 1; q[1] = q[2] = q[3] = 0; return; }
  float s = 1.0f / n;
  q[0] *= s; q[1] *= s; q[2] *= s; q[3] *= s;
}
__device__ __forceinline__ void quat2mat(float m[9], const float q[4]) {
  float w = q[0], x = q[1], y = q[2], z = q[3];
  m[0] = 1 - 2 * (y * y + z * z); m[1] = 2 * (x * y - w * z); m[2] = 2 * (x * z + w * y);
  m[3] = 2 * (x * y + w * z); m[4] = 1 - 2 * (x * x + z * z); m[5] = 2 * (y * z - w * x);
  m[6] = 2 * (x * z - w * y); m[7] = 2 * (y * z + w * x); m[8] = 1 - 2 * (x * x + y * y);
}
/* r = q v q* for a unit quaternion q = (w, u): v + w t + u x t with t = 2 u x v
   (21 VALU instead of quat2mat + mulmv3's 30) */
__device__ __forceinline__ void quat_rotate(float r[3], const float q[4], const float v[3]) {
  const float u[3] = {q[1], q[2], q[3]};
  float t[3], c2[3];
  cross3(t, u, v);
  t[0] += t[0]; t[1] += t[1]; t[2] += t[2];
  cross3(c2, u, t);
  r[0] = v[0] + q[0] * t[0] + c2[0];
  r[1] = v[1] + q[0] * t[1] + c2[1];
  r[2] = v[2] + q[0] * t[2] + c2[2];
}
__device__ __forceinline__ void mulmv3(float r[3], const float m[9], const float v[3]) {
  float t0 = m[0] * v[0] + m[1] * v[1] + m[2] * v[2];
  float t1 = m[3] * v[0] + m[4] * v[1] + m[5] * v[2];
  float t2 = m[6] * v[0] + m[7] * v[1] + m[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
__device__ __forceinline__ void mulmtv3(float r[3], const float m[9], const float v[3]) {
  float t0 = m[0] * v[0] + m[3] * v[1] + m[6] * v[2];
  float t1 = m[1] * v[0] + m[4] * v[1] + m[7] * v[2];
  float t2 = m[2] * v[0] + m[5] * v[1] + m[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
__device__ __forceinline__ void mulmm3(float r[9], const float a[9], const float b[9]) {
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) r[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
}
/* sin / cos for |x| <= pi/2 by their Taylor series through x^11 / x^12 (truncation below
   6e-8, the fp32 epsilon; ~14 VALU instead of sincosf's range reduction); larger arguments
   (a joint more than pi from its reference) take sincosf */
__device__ __forceinline__ void sincos_small(float x, float* s, float* c) {
  if (fabsf(x) <= 1.5707964f) {
    const float x2 = x * x;
    float ps = -2.5052108e-8f;                  /* -1/11! */
    ps = fmaf(ps, x2, 2.7557319e-6f);           /* 1/9! */
    ps = fmaf(ps, x2, -1.9841270e-4f);          /* -1/7! */
    ps = fmaf(ps, x2, 8.3333333e-3f);           /* 1/5! */
    ps = fmaf(ps, x2, -1.6666667e-1f);          /* -1/3! */
    *s = fmaf(ps * x2, x, x);
    float pc = 2.0876757e-9f;                   /* 1/12! */
    pc = fmaf(pc, x2, -2.7557319e-7f);          /* -1/10! */
    pc = fmaf(pc, x2, 2.4801587e-5f);           /* 1/8! */
    pc = fmaf(pc, x2, -1.3888889e-3f);          /* -1/6! */
    pc = fmaf(pc, x2, 4.1666667e-2f);           /* 1/4! */
    pc = fmaf(pc, x2, -0.5f);
    *c = fmaf(pc, x2, 1.f);
  } else {
    sincosf(x, s, c);
  }
}
__device__ __forceinline__ void axis_angle_quat(float q[4], const float ax[3], float angle) {
  float s, c;
  sincos_small(0.5f * angle, &s, &c);
  q[0] = c; q[1] = ax[0] * s; q[2] = ax[1] * s; q[3] = ax[2] * s;
}
__device__ __forceinline__ void cross_motion(float r[6], const float v[6], const float u[6]) {
  float a[3], b[3], c[3];
  cross3(a, v, u);
  cross3(b, v, u + 3);
  cross3(c, v + 3, u);
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2];
  r[3] = b[0] + c[0]; r[4] = b[1] + c[1]; r[5] = b[2] + c[2];
}
__device__ __forceinline__ void cross_force(float r[6], const float v[6], const float f[6]) {
  float a[3], b[3], c[3];
  cross3(a, v, f);
  cross3(b, v + 3, f + 3);
  cross3(c, v, f + 3);
  r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2];
  r[3] = c[0]; r[4] = c[1]; r[5] = c[2];
}
__device__ __forceinline__ void mul_inert_vec(float r[6], const float i[10], const float v[6]) {
  r[0] = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  r[1] = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  r[2] = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  r[3] = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  r[4] = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  r[5] = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
}
__device__ __forceinline__ float dot6(const float a[6], const float b[6]) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}
__device__ __forceinline__ uint32_t fbits(float f) { return __float_as_uint(f); }
__device__ __forceinline__ float bitsf(uint32_t u) { return __uint_as_float(u); }

/* State-row words handed from one workgroup to another inside a launch (the chunked step,
   step_kernel): agent-scope relaxed atomics lower to global_load / global_store with sc1, which
   bypass the CU's L1. Every load and store of those words uses them, the storing wave waits for
   its stores (vmcnt(0)) before one lane publishes the progress flag with an sc1 store, and the
   consumer polls that flag with sc1 loads: the sc1 hand-off of MI355X_MICROARCH.md (inter-
   workgroup visibility, first row of its hand-off table). */
typedef __attribute__((address_space(1))) float gfloat_t;
typedef __attribute__((address_space(1))) uint32_t guint_t;
typedef float xv4f __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) xv4f gfloat4_t;

/* The second contact-row bank of the general-collider kernels (XG: geoms 2-3, or any model that
   is not exactly two box soles) keeps its Jacobian rows in global scratch (StepArgs::xj, one
   [32][CAP] block per env): 1.5 KB per env in LDS would take those kernels from 8 workgroups per
   CU to 6. They are written and read only while the bank has rows in the wave (shins or hands on
   the floor), through the CU's L1; its J'DJ blocks and row scratch reuse the first bank's LDS. */
__device__ __forceinline__ gfloat_t* xrows(const EnvL* L) {
  return (gfloat_t*)(((uint64_t)L->s.xj_hi << 32) | (uint64_t)L->s.xj_lo);
}
/* XG 4 / 5: the third bank's rows follow the second bank's in the env's block */
__device__ __forceinline__ gfloat_t* yrows(const EnvL* L) { return xrows(L) + 32 * CAP; }
/* floats of StepArgs::xj per env: one [32][CAP] block per extra bank */
template <int XG>
constexpr int XJ_STRIDE = ZB_XJ_STRIDE * (XG == 4 || XG == 5 ? 2 : 1);
__device__ __forceinline__ void set_xrows(EnvL* L, float* base) {
  L->s.xj_lo = (uint32_t)(uint64_t)base;
  L->s.xj_hi = (uint32_t)((uint64_t)base >> 32);
}
template <bool CG = true>
__device__ __forceinline__ float ld_cg(const float* p) {
  if constexpr (CG) return __hip_atomic_load((gfloat_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}
template <bool CG = true>
__device__ __forceinline__ void st_cg(float* p, float v) {
  if constexpr (CG) __hip_atomic_store((gfloat_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
__device__ __forceinline__ uint32_t ldu_cg(const uint32_t* p) {
  return __hip_atomic_load((guint_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void stu_cg(uint32_t* p, uint32_t v) {
  __hip_atomic_store((guint_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t addu_cg(uint32_t* p, uint32_t v) {
  return __hip_atomic_fetch_add((guint_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void maxu_cg(uint32_t* p, uint32_t v) {
  (void)__hip_atomic_fetch_max((guint_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

/* ------------------------ RNG: threefry2x32-20 (Random123) ------------------ */
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ void threefry2x32(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1, uint32_t& o0,
                                             uint32_t& o1) {
  const uint32_t ks2 = 0x1BD11BDAu ^ k0 ^ k1;
  uint32_t x0 = c0 + k0, x1 = c1 + k1;
#define TF_R(r) { x0 += x1; x1 = rotl32(x1, r); x1 ^= x0; }
  TF_R(13) TF_R(15) TF_R(26) TF_R(6)  x0 += k1;  x1 += ks2 + 1u;
  TF_R(17) TF_R(29) TF_R(16) TF_R(24) x0 += ks2; x1 += k0 + 2u;
  TF_R(13) TF_R(15) TF_R(26) TF_R(6)  x0 += k0;  x1 += k1 + 3u;
  TF_R(17) TF_R(29) TF_R(16) TF_R(24) x0 += k1;  x1 += ks2 + 4u;
  TF_R(13) TF_R(15) TF_R(26) TF_R(6)  x0 += ks2; x1 += k0 + 5u;
#undef TF_R
  o0 = x0; o1 = x1;
}
#define P_OBS 1u
#define P_PUSH 2u
#define P_RESET 3u
#define P_RAND 4u
__device__ __forceinline__ void rng_bits(uint64_t seed, uint32_t purpose, uint32_t k, uint32_t env, uint32_t ctr,
                                         uint32_t& a, uint32_t& b) {
  /* the key is re-derived at every draw site (opaque seed) so its round-key
     schedule is not hoisted into SGPRs for the whole launch */
  uint32_t slo = (uint32_t)seed, shi = (uint32_t)(seed >> 32);
  asm volatile("" : "+v"(slo), "+v"(shi));
  slo = __builtin_amdgcn_readfirstlane(slo);
  shi = __builtin_amdgcn_readfirstlane(shi);
  threefry2x32(slo ^ (purpose * 0x9E3779B9u), shi ^ (k * 0x85EBCA6Bu), env, ctr, a, b);
}
__device__ __forceinline__ float u01(uint32_t b) { return (float)(b >> 8) * (1.0f / 16777216.0f); }
__device__ __forceinline__ void uniform2(uint64_t seed, uint32_t p, uint32_t k, uint32_t env, uint32_t ctr, float& u0,
                                         float& u1) {
  uint32_t a, b;
  rng_bits(seed, p, k, env, ctr, a, b);
  u0 = u01(a);
  u1 = u01(b);
}
__device__ __forceinline__ void normal2(uint64_t seed, uint32_t p, uint32_t k, uint32_t env, uint32_t ctr, float& z0,
                                        float& z1) {
  uint32_t a, b;
  rng_bits(seed, p, k, env, ctr, a, b);
  float u1 = 1.0f - u01(a), u2 = u01(b);
  float r = sqrtf(-2.0f * logf(u1));
  float s, c;
  sincosf(6.283185307179586f * u2, &s, &c);
  z0 = r * c;
  z1 = r * s;
}

/* --------------------------------- contexts -------------------------------- */
/* The model and config are device buffers never written by a kernel, so they
   are read through the constant address space (scalar loads for uniform
   fields). `opaque` re-derives the pointers at the top of every substep: the
   compiler cannot hoist the uniform loads out of the substep loop, so they
   are re-issued from the scalar cache instead of pinning ~300 SGPRs (which
   spilled into VGPR lanes) across the whole launch. */
typedef const __attribute__((address_space(4))) ZbModel* MP;
typedef const __attribute__((address_space(4))) ZbEnvConfig* CP;
template <typename P>
__device__ __forceinline__ P opaque(P p) {
  uint64_t v = (uint64_t)p;
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  asm volatile("" : "+v"(lo), "+v"(hi));
  lo = __builtin_amdgcn_readfirstlane(lo);
  hi = __builtin_amdgcn_readfirstlane(hi);
  return (P)(((uint64_t)hi << 32) | lo);
}
struct Ctx {
  MP m;
  CP cfg;
  EnvL* L;
  int l;
  int nu;
  /* lane as a limb-chain dof (dofs >= nroot; each limb is an unbranched chain of
     consecutive dofs hanging off dof nroot-1, checked by zb_create) */
  int chd, cps, cln; /* chain head dof, position in the chain, chain length (chd = -1: not a chain dof) */
  /* lane as body */
  int bpar, bdep, bjt, bdofadr, blast, nch;
  uint32_t ch0, ch1;
  uint64_t lvlch; /* per body depth: max #children among bodies at that depth (4 bits each) */
  /* lane as dof */
  int ddep, dbody, qadr, act;
  /* contact rows whose Jacobian chain contains dof l, by 16-row half: bits 0-1 the first bank's
     (geoms 0, 1), bits 2-3 the second bank's (XG); one register instead of two masks */
  uint32_t rmb;
  int dk0;          /* index of dof l within its body's joint (free joint: 0..5) */
  int dfree;        /* dof l belongs to a free joint */
};


/* a 2-bit half mask of Ctx::rmb as the 32-row mask */
__device__ __forceinline__ uint32_t rm_rows(uint32_t b) {
  return ((b & 1u) ? 0xFFFFu : 0u) | ((b & 2u) ? 0xFFFF0000u : 0u);
}

/* the team's RNG identity (EnvS.env / seed, written by make_ctx) */
__device__ __forceinline__ uint64_t cseed(const Ctx& c) {
  return (uint64_t)c.L->s.seed_lo | ((uint64_t)c.L->s.seed_hi << 32);
}
__device__ __forceinline__ uint32_t cenv(const Ctx& c) { return c.L->s.env; }

/* ancestor dof at depth e of a dof whose limb chain starts at dof `head`
   (root dofs: head < 0): the tree shape makes ancestors dofs 0..NROOT-1
   followed by a contiguous run of the limb (e past the depth: a valid dummy) */
__device__ __forceinline__ int anc_lin(int head, int e) { return e < NROOT ? e : (head < 0 ? 0 : head) + e - NROOT; }
__device__ __forceinline__ int childof(const Ctx& c, int k) {
  uint32_t w = k < 4 ? c.ch0 : c.ch1;
  return (int)((w >> ((k & 3) * 8)) & 0xffu);
}

/* per-lane persistent registers */
struct LaneS {
  float q, v, w;        /* dof lane: hinge angle, qvel, qacc_warmstart */
  float pp, pv, ptau;   /* planner (actuated dof lane) */
  float tgt;            /* action target */
  float ctrl;           /* actuator ctrl of this dof lane */
  float qacc;           /* last constrained qacc */
  float actforce;       /* actuator force (gear*clamped ctrl) */
  float fq;             /* qfrc_smooth + qfrc_constraint of the last solve (implicit damping only) */
};
/* per-substep body outputs */
struct BodyK {
  float xp[3], xq[4]; /* rotation matrices are recomputed from xq where needed */
  float cv[6];
};
/* a contact row of the second bank (XG), held by the lane like Rows' own */
struct XRow {
  bool any; /* wave-uniform: some row of the bank exists in either env of the wave */
  bool ex;
  int chd; int kdep;
  uint32_t rowmask; /* XG 1 / 2: the bank's rows whose chain holds dof l (its geoms change per substep) */
  float aref, D, jar, Jv, f;
  int act;
  int nrow;
  uint32_t exmask;
};
/* constraint rows held by the lane */
struct Rows {
  /* contact row (lane = row) */
  bool ex;
  int chd; int kdep; /* limb chain head and depth of the row's last dof */
  float aref, D, jar, Jv, f;
  int act;
  /* dof rows: frictionloss, lower, upper limit */
  bool hf, hl;
  float af, Df, Rf, fl, jf, ff; int actf;
  /* the joint-limit row (exists only past a limit, at most one side per dof):
     Jacobian sl * e_dof (sl = +1 lower, -1 upper), jl = sl * qacc - al */
  float sl, al, Dl, jl, flim; int actl;
  /* wave-uniform: some joint-limit row exists in either env of the wave. While none does (the
     usual case: no C2 substep has a dof past a limit) the solvers skip the limit row's terms,
     which would all be exact zeros, so the results are the same bits */
  bool anyl;
  int nrow;
  uint32_t exmask; /* team-uniform: existing contact rows */
  XRow x;          /* second bank (XG kernels only) */
  XRow y;          /* third bank: the sole pair beside floor colliders (XG 4 only) */
};

/* 16-byte LDS row access (rows are 12 floats = 48 B, 16-B aligned) */
__device__ __forceinline__ void ld_row(const float* p, float v[CAP]) {
  const float4* q = reinterpret_cast<const float4*>(p);
  float4 a = q[0], b = q[1], c4 = q[2];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  v[8] = c4.x; v[9] = c4.y; v[10] = c4.z; v[11] = c4.w;
}
__device__ __forceinline__ void st_row(float* p, const float v[CAP]) {
  float4* q = reinterpret_cast<float4*>(p);
  q[0] = make_float4(v[0], v[1], v[2], v[3]);
  q[1] = make_float4(v[4], v[5], v[6], v[7]);
  q[2] = make_float4(v[8], v[9], v[10], v[11]);
}
/* the same for a row of the second bank's global scratch (xrows) */
__device__ __forceinline__ void ld_row(const gfloat_t* p, float v[CAP]) {
  const gfloat4_t* q = reinterpret_cast<const gfloat4_t*>(p);
  const xv4f a = q[0], b = q[1], c4 = q[2];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  v[8] = c4.x; v[9] = c4.y; v[10] = c4.z; v[11] = c4.w;
}
__device__ __forceinline__ void st_row(gfloat_t* p, const float v[CAP]) {
  gfloat4_t* q = reinterpret_cast<gfloat4_t*>(p);
  q[0] = xv4f{v[0], v[1], v[2], v[3]};
  q[1] = xv4f{v[4], v[5], v[6], v[7]};
  q[2] = xv4f{v[8], v[9], v[10], v[11]};
}

/* ------------------------------- kinematics -------------------------------- */
/* mj_kinematics by pointer jumping: each body lane first builds its frame
 * relative to its parent (for a hinge: rotate about the anchor, the local form
 * of MuJoCo's anchor -> rotate -> un-anchor update), then composes with the
 * frame of the ancestor its transform is currently relative to, doubling the
 * covered depth each round: ceil(log2(depth)) rounds instead of one pass per
 * tree level. The floating base is absolute from the start. */
__device__ __forceinline__ void kinematics(const Ctx& c, const EnvS& s, const LaneS& ls, BodyK& B) {
  MP m = c.m;
  const int b = c.l;
  const bool isb = b >= 1 && b < NB;
  /* relative hinge angle of this body's joint, from its dof lane */
  float qrel_dof = ls.q - c.L->par[P_Q0][c.l];
  float ang = tsh(qrel_dof, c.bdofadr < 0 ? 0 : c.bdofadr);
  float p[3] = {0.f, 0.f, 0.f}, q[4] = {1.f, 0.f, 0.f, 0.f};
  int anc = 0; /* frame the transform is relative to (0: world) */
  if (isb) {
    if (c.bjt == ZB_JNT_FREE) {
#pragma unroll
      for (int k = 0; k < 3; k++) p[k] = s.bp[k];
#pragma unroll
      for (int k = 0; k < 4; k++) q[k] = s.bq[k];
      quat_normalize(q);
    } else {
#pragma unroll
      for (int k = 0; k < 3; k++) p[k] = m->body_pos[b][k];
#pragma unroll
      for (int k = 0; k < 4; k++) q[k] = m->body_quat[b][k];
      if (c.bjt == ZB_JNT_HINGE) {
        float jp[3] = {m->jnt_pos[b][0], m->jnt_pos[b][1], m->jnt_pos[b][2]};
        float ax[3] = {m->jnt_axis[b][0], m->jnt_axis[b][1], m->jnt_axis[b][2]};
        float t1[3], t2[3], ql[4], qn[4];
        quat_rotate(t1, q, jp);
        axis_angle_quat(ql, ax, ang);
        quat_mul(qn, q, ql);
        quat_normalize(qn);
        quat_rotate(t2, qn, jp);
#pragma unroll
        for (int k = 0; k < 3; k++) p[k] += t1[k] - t2[k];
#pragma unroll
        for (int k = 0; k < 4; k++) q[k] = qn[k];
      }
      anc = c.bpar;
    }
  }
  for (int span = 1; span < MAXBD; span <<= 1) {
    float ap[3], aq[4];
#pragma unroll
    for (int k = 0; k < 3; k++) ap[k] = tsh(p[k], anc);
#pragma unroll
    for (int k = 0; k < 4; k++) aq[k] = tsh(q[k], anc);
    const int aa = tshi(anc, anc);
    if (anc != 0) {
      float t[3], qq[4];
      quat_rotate(t, aq, p);
#pragma unroll
      for (int k = 0; k < 3; k++) p[k] = ap[k] + t[k];
      quat_mul(qq, aq, q);
#pragma unroll
      for (int k = 0; k < 4; k++) q[k] = qq[k];
      anc = aa;
    }
  }
  if (isb && c.bjt != ZB_JNT_FREE) quat_normalize(q);
#pragma unroll
  for (int k = 0; k < 3; k++) B.xp[k] = p[k];
#pragma unroll
  for (int k = 0; k < 4; k++) B.xq[k] = q[k];
}

/* subtree sum of K-vectors over the body tree: out (lane b) = sum over subtree(b).
 * Uses c.L->sub as the exchange buffer; result also left in sub[b]. */
/* subtree sums of K-vectors over the body tree: out (lane b) = sum over
 * subtree(b), left in registers and in LDS sub[b]. The model has a single
 * branching body (the floating base, body 1; checked by zb_create), so below
 * it every subtree is a chain suffix: pointer jumping along the child links
 * sums the chains in log2(length) rounds, then the base gathers its children. */
template <int K>
__device__ __forceinline__ void subtree_sum(const Ctx& c, float v[K]) {
  EnvL* L = c.L;
  const bool chain = c.l >= 2 && c.l < NB && c.nch == 1;
  int nxt = chain ? childof(c, 0) : c.l;
  bool live = chain;
  for (int span = 1; span < MAXBD - 1; span <<= 1) {
    float w[K];
#pragma unroll
    for (int i = 0; i < K; i++) w[i] = tsh(v[i], nxt);
    const int nn = tshi(nxt, nxt);
    const bool nl = tshi(live ? 1 : 0, nxt) != 0;
    if (live) {
#pragma unroll
      for (int i = 0; i < K; i++) v[i] += w[i];
      nxt = nn;
      live = nl;
    }
  }
#pragma unroll
  for (int i = 0; i < K; i++) L->sub[c.l][i] = v[i];
  /* the base (the one branching body): its own value plus its children's chain sums,
     one transposing team reduction straight into its row sub[1] (written after the
     plain stores above, in program order). Callers read the sums from sub[]. */
  {
    const bool bchild = c.l >= 2 && c.l < NB && c.bpar == 1;
    const bool take = bchild || c.l == 1;
    float w[K];
#pragma unroll
    for (int i = 0; i < K; i++) w[i] = take ? v[i] : 0.f;
    reduce_to_lds<K>(w, &L->sub[1][0]);
  }
  tsync();
}

/* ------------------------------ mass matrix -------------------------------- */
/* com, cinert (lane b), cdof (lane j -> LDS), crb, M rows (LDS + return) */
__device__ __forceinline__ void com_crb_m(const Ctx& c, const EnvS& s, const LaneS& ls, BodyK& B, float cm[3]) {
  const int ddep = vopq(c.ddep);
  MP m = c.m;
  EnvL* L = c.L;
  const int b = c.l;
  const bool isbody = b >= 1 && b < NB;
  const int bb = isbody ? b : 0;
  const float mscale = keepf(c.L->par[P_MSCALE][c.l]);
  const float bmass = keepf(m->body_mass[bb][0]);
  float mass = isbody ? bmass * mscale : 0.f;
  float xipos[3], Ri[9];
  {
    float ip[3] = {m->body_ipos[isbody ? b : 0][0], m->body_ipos[isbody ? b : 0][1], m->body_ipos[isbody ? b : 0][2]}, t[3];
    quat_rotate(t, B.xq, ip); /* xmat * ipos */
#pragma unroll
    for (int k = 0; k < 3; k++) xipos[k] = B.xp[k] + t[k];
    float iq[4] = {m->body_iquat[isbody ? b : 0][0], m->body_iquat[isbody ? b : 0][1],
                   m->body_iquat[isbody ? b : 0][2], m->body_iquat[isbody ? b : 0][3]}, xi[4];
    quat_mul(xi, B.xq, iq); /* ximat = frame of xquat * body_iquat (mj_local2Global) */
    quat2mat(Ri, xi);
  }
  float ms[4] = {mass, mass * xipos[0], mass * xipos[1], mass * xipos[2]};
  tsum_n<4>(ms);
  const float mt = ms[0];
#pragma unroll
  for (int k = 0; k < 3; k++) cm[k] = ms[1 + k] / mt;
  /* cinert: inertia about cm in world orientation (mju_inertCom) */
  float ci[10];
  {
    float in[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const float bi = keepf(m->body_inertia[bb][k]);
      in[k] = isbody ? bi * mscale : 0.f;
    }
    float dif[3] = {xipos[0] - cm[0], xipos[1] - cm[1], xipos[2] - cm[2]};
    float I[9];
#pragma unroll
    for (int a = 0; a < 3; a++)
#pragma unroll
      for (int bb = 0; bb < 3; bb++)
        I[3 * a + bb] = Ri[3 * a] * in[0] * Ri[3 * bb] + Ri[3 * a + 1] * in[1] * Ri[3 * bb + 1] +
                        Ri[3 * a + 2] * in[2] * Ri[3 * bb + 2];
    float dd = dot3(dif, dif);
    ci[0] = I[0] + mass * (dd - dif[0] * dif[0]);
    ci[1] = I[4] + mass * (dd - dif[1] * dif[1]);
    ci[2] = I[8] + mass * (dd - dif[2] * dif[2]);
    ci[3] = I[1] - mass * dif[0] * dif[1];
    ci[4] = I[2] - mass * dif[0] * dif[2];
    ci[5] = I[5] - mass * dif[1] * dif[2];
    ci[6] = mass * dif[0];
    ci[7] = mass * dif[1];
    ci[8] = mass * dif[2];
    ci[9] = mass;
#pragma unroll
    for (int k = 0; k < 10; k++) L->ci[b][k] = ci[k];
  }
  /* cdof (lane j): fetch body frame of dof's body */
  {
    const int j = c.l;
    int bj = c.dbody < 0 ? 0 : c.dbody;
    float R[9], xp[3], xqs[4];
#pragma unroll
    for (int k = 0; k < 4; k++) xqs[k] = tsh(B.xq[k], bj);
    quat2mat(R, xqs);
#pragma unroll
    for (int k = 0; k < 3; k++) xp[k] = tsh(B.xp[k], bj);
    /* every lane, the non-dof ones storing zero rows (read as zero by com_vel / com_acc) */
    {
      /* branch-free over the dof kinds (the task's dofs are the free joint's 6 and
         hinges): the motion axis in the body frame is jnt_axis for a hinge and unit
         axis k-3 for a free-joint rotation, anchored at jnt_pos / the body origin;
         a free-joint translation k < 3 is the pure linear motion e_k */
      const bool isfree = c.dfree;
      const int k = c.dk0;
      const bool trans = isfree && k < 3;
      float ja[3], jp[3], t[3], ax[3];
#pragma unroll
      for (int i = 0; i < 3; i++) {
        ja[i] = isfree ? (k - 3 == i ? 1.f : 0.f) : m->jnt_axis[bj][i];
        jp[i] = isfree ? 0.f : m->jnt_pos[bj][i];
      }
      mulmv3(t, R, jp);
      mulmv3(ax, R, ja);
      float off[3] = {cm[0] - (xp[0] + t[0]), cm[1] - (xp[1] + t[1]), cm[2] - (xp[2] + t[2])}, cr[3];
      cross3(cr, ax, off);
      float cd[6];
#pragma unroll
      for (int i = 0; i < 3; i++) {
        cd[i] = trans ? 0.f : ax[i];
        cd[3 + i] = trans ? (k == i ? 1.f : 0.f) : cr[i];
      }
      const bool isd = j < NV;
#pragma unroll
      for (int i = 0; i < 6; i++) L->cdof[j][i] = isd ? cd[i] : 0.f;
    }
  }
  /* crb = subtree sums of cinert */
  float crb[10];
#pragma unroll
  for (int k = 0; k < 10; k++) crb[k] = ci[k];
  tsync();
  subtree_sum<10>(c, crb);
  /* M rows: M(j, anc_e(j)) = cdof_anc . (crb_body(j) * cdof_j), packed storage */
  {
    const int j = c.l;
    if (j < NV) {
      float cr[10], cd[6], F[6], mr[CAP];
#pragma unroll
      for (int k = 0; k < 10; k++) cr[k] = L->sub[c.dbody][k];
#pragma unroll
      for (int k = 0; k < 6; k++) cd[k] = L->cdof[j][k];
      mul_inert_vec(F, cr, cd);
      const float arm = c.L->par[P_ARM][c.l];
      /* branch-free gather, four ancestor rows in flight per chunk (rows past
         the lane's depth read ancestor slot 0 and are masked) */
#pragma unroll
      for (int e0 = 0; e0 < CAP; e0 += 4) {
        float ca[4][6];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const int a = anc_lin(c.chd, e0 + i);
          if (e0 + i >= 3) {
#pragma unroll
            for (int k = 0; k < 6; k++) ca[i][k] = L->cdof[a][k];
          }
        }
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const int e = e0 + i;
          /* ancestors 0..2 are the free joint's world-frame translations, cdof = (0, e_k):
             their products are components of F (body 1 carries the free joint, zb_create) */
          const float v = e < 3 ? F[3 + e] : dot6(ca[i], F);
          mr[e] = e <= ddep ? v : 0.f;
        }
      }
      st_row(&L->M[j][0], mr);
      /* the diagonal (ancestor slot ddep = the dof itself) with the armature */
      L->M[j][ddep] = dot6(cd, F) + arm;
    } /* non-dof lanes keep the zero rows make_ctx stored, so M x needs no lane mask */
  }
  tsync();
  /* The transposed entries in the row padding: slot ddep + q of row j holds M(j + q, j) for
   * the q-th deeper dof of j's chain (the root chain for a root dof), zero past it. The
   * ancestor gather of mul_m reads slot e > ddep at dof anc_lin(chd, e) = j + (e - ddep), so
   * one 12-entry row product gives M(j, anc) x_anc + M(j, j) x_j + sum_q M(j + q, j) x_{j+q}.
   * Nothing else reads past the diagonal (the factorizations take off-diagonals below it). */
  {
    const int j = c.l;
    const bool isd = j < NV;
    const int nd = vopq(isd ? (j < NROOT ? NROOT - 1 - j : c.cln - c.cps - 1) : 0);
    const int jb = isd ? j : 0;
    float t[NLIMBLV - 1];
#pragma unroll
    for (int q = 1; q < NLIMBLV; q++) {
      const float v = L->M[jb + q][ddep];
      t[q - 1] = q <= nd ? v : 0.f;
    }
#pragma unroll
    for (int q = 1; q < NLIMBLV; q++) {
      /* past the chain the (zero) value goes to row 31, which stays the zero row */
      float* dst = q <= nd ? &L->M[j][ddep + q] : &L->M[31][0];
      *dst = t[q - 1];
    }
  }
  tsync();
}

typedef float v4f __attribute__((ext_vector_type(4)));

/* Root Schur complement of the limb elimination on the matrix cores, for both
 * envs of the wave: G[i][e] = sum_k D_k L(k,i) L(k,e), i,e < NROOT, k over the
 * limb dofs NROOT..NV-1 (their eliminated rows are in LDS L[][] / Dk[]). Per
 * env five v_mfma_f32_16x16x4_f32 (K = 4 limb dofs each; lane l supplies row
 * NROOT + 4*chunk + l/16, entry l%16 < NROOT), accumulating from the parked root
 * block. Lane l ends with (A_root - G)[4*(l/16) + v][l%16]; the lower triangle (21
 * values, packed i(i+1)/2 + e) is left in the env's vec[V_TMP2], free during every
 * factorization. Replaces 21 team reductions (126 DPP/permlane VALU instructions per
 * factor) and the 21 subtractions from the parked block.
 * Wave-uniform: call with every lane active (the MFMA reads all 64 lanes). */
__device__ __forceinline__ void root_schur_mfma() {
  static_assert(NV - NROOT == 20, "five K=4 chunks cover the 20 limb dofs");
  const int l = vopq(threadIdx.x & 63); /* opaque: the store masks below are rebuilt per call */
  const int i = l & 15, kk = l >> 4;
  const int ic = i < RMAX ? i : 0;
  /* the accumulators start from the parked root block (its diagonal parked in L[r][r] too),
     so the result is A_root - G; entries above the diagonal or outside the 6 x 6 block are
     never stored */
  v4f acc[NTEAM];
#pragma unroll
  for (int t = 0; t < NTEAM; t++)
#pragma unroll
    for (int v = 0; v < 4; v++) {
      const int row = 4 * kk + v;
      acc[t][v] = g_lds[t].L[row < RMAX ? row : 0][ic];
    }
#pragma unroll
  for (int ch = 0; ch < (NV - NROOT) / 4; ch++)
#pragma unroll
    for (int t = 0; t < NTEAM; t++) {
      const int k = NROOT + 4 * ch + kk;
      const float lv = g_lds[t].L[k][ic];
      const float dv = g_lds[t].Dk[k];
      /* no masks: lanes i >= RMAX feed rows / columns of G that are never stored */
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(-(dv * lv), lv, acc[t], 0, 0, 0);
    }
#pragma unroll
  for (int t = 0; t < NTEAM; t++)
#pragma unroll
    for (int v = 0; v < 4; v++) {
      const int row = 4 * kk + v;
      if (row < RMAX && i <= row) g_lds[t].vec[V_TMP2][row * (row + 1) / 2 + i] = acc[t][v];
    }
}

/* ---------------------- sparse L'DL factor + solves ------------------------ */
/* Sparse L'DL of depth-indexed rows (mj_factorM order: leaves first) for the
 * dof tree the engine accepts (zb_create): a root chain 0..nroot-1 and
 * unbranched limb chains hanging off dof nroot-1. Lane j holds the
 * off-diagonal entries X[e] = A(j, anc_e(j)), e < depth(j), and the diagonal
 * Xd. Limbs are eliminated level by level (height inside the chain) with the
 * pivot rows pulled through ds_bpermute; their Schur complement on the root
 * block is a set of team reductions; the root block is eliminated densely in
 * registers. On return the L rows are in LDS L[][] (L(k, anc_e(k))), pivots in
 * Dk[] (root: also 1/D in Di[]); returns 1/D_j. */
template <bool MFMA_SCHUR>
__device__ __forceinline__ float factor_ldl(const Ctx& c, float X[CAP], float Xd, const float (*S)[CAP]) {
  const int ddep = vopq(c.ddep);
  EnvL* L = c.L;
  const int nroot = NROOT;
  const bool isroot = c.l < nroot;
  const bool ischain = c.chd >= 0;
  /* root rows are only touched by the dense block at the end: park them */
  if (isroot) {
    st_row(&L->L[c.l][0], X);
    L->L[c.l][c.l] = Xd; /* the diagonal in place too (root_schur_mfma starts from the block) */
    L->Dk[c.l] = Xd;
  }
  /* limb levels by chain position q = NLIMBLV-1 .. 1 (leaves first; chains
     shorter than q+1 idle): every shallower lane of a chain pulls the pivot's
     unscaled row with ds_bpermute (only the NROOT+q entries a receiver uses),
     scales by 1/D_k itself (mj_factorI order: update with A(k,j)/D_k, divide
     the pivot row afterwards) and applies its Schur update. Position 0 has no
     receivers inside the chain. */
  const int cps = vopq(c.cps);
  const int clnv = vopq(c.cln); /* opaque per call: the level masks are recomputed, not kept live */
  const int chdv = ischain ? c.chd : 0;
  /* Alongside, each chain lane p builds row p of W = (I + Lt)^-1, the inverse of
     its chain's unit triangular block (Lt(p, k) = L(k, p), k deeper in the chain),
     by absolute chain position: W(p, k) = -sum_{m > p} L(m, p) W(m, k), W(m, m) = 1.
     At level q the receiver already holds L(q, p) (sc) and pulls the pivot's
     finished accumulators, so W costs no extra round trip here; solve_ldl then
     applies each chain's triangular solve as one gather instead of a chain of
     dependent ones. wacc[k] = -W(p, k) (zero for k <= p and past the chain). */
  float wacc[NLIMBLV];
#pragma unroll
  for (int k = 0; k < NLIMBLV; k++) wacc[k] = 0.f;
#pragma unroll
  for (int q = NLIMBLV - 1; q >= 1; q--) {
    const bool has = cps < q && q < clnv; /* clnv = 0 off the chains */
    /* lanes without a pivot at this level pull from any lane of a valid index and
       discard it (sc = 0 below; every pulled value is finite) */
    const int src = chdv + q;
    /* only the chain entries travel: the root columns follow from W below */
    float r[NROOT + NLIMBLV], wq[NLIMBLV];
#pragma unroll
    for (int e = NROOT; e < NROOT + q; e++) r[e] = tsh(X[e], src);
    const float dk = tsh(Xd, src);
#pragma unroll
    for (int k = q + 1; k < NLIMBLV; k++) wq[k] = tsh(wacc[k], src);
    /* A(q, p) from the lane's own row: slot NROOT + pos holds A(p, pos) for every chain
       position, ancestors below the diagonal and deeper dofs in the padding (the rows
       carry their transposed entries there, com_crb_m / hessian_factor), and the update
       below keeps the padding current, so the entry sits at a fixed slot */
    const float t = X[NROOT + q];
    const float sc = has ? t / fmaxf(dk, MINVAL) : 0.f;
    Xd -= sc * t;
    /* every position below the pivot: the ancestors (read by later pivots' receivers)
       and the padding up to q - 1 (the next levels' t); the slot of the lane's own
       position is junk, never read (Xd is the diagonal) */
#pragma unroll
    for (int e = NROOT; e < NROOT + q; e++) X[e] -= sc * r[e];
    wacc[q] += sc;
#pragma unroll
    for (int k = q + 1; k < NLIMBLV; k++) wacc[k] -= sc * wq[k];
  }
  if (ischain) {
    /* root columns of the eliminated chain row: the level updates on them compose to
       B(p, :) + sum_{k > p} W(p, k) B(k, :), B the chain rows' root entries as passed
       in (rows S[] in LDS; wacc[k] = -W(p, k) is zero for k <= p and past the chain) */
    const int chd = c.chd;
#pragma unroll
    for (int k = 1; k < NLIMBLV; k++) {
      float b[NROOT];
#pragma unroll
      for (int e = 0; e < NROOT; e++) b[e] = S[chd + k][e];
#pragma unroll
      for (int e = 0; e < NROOT; e++) X[e] -= wacc[k] * b[e];
    }
    const float Dkv = fmaxf(Xd, MINVAL);
    const float inv = 1.0f / Dkv;
#pragma unroll
    for (int e = 0; e < NROOT; e++) X[e] = X[e] * inv;
    /* stored row: L(j, root i) in slots 0..NROOT-1, W(p, k) in slots NROOT + k (the
       chain-ancestor entries of L are not needed once W is known) */
#pragma unroll
    for (int k = 0; k < NLIMBLV; k++) X[NROOT + k] = -wacc[k];
    Xd = Dkv;
    st_row(&L->L[c.l][0], X);
    L->Dk[c.l] = Xd;
  }
  if (nroot > 0) {
    /* root block: parked rows minus the limbs' Schur complement
       G[i][e] = sum_k D_k L(k,i) L(k,e) (team reductions), then the dense
       elimination k = nroot-1 .. 0, redundantly in every lane */
    tsync();
    constexpr int NG = RMAX * (RMAX + 1) / 2;
    float g[NG];
    if constexpr (MFMA_SCHUR) {
      /* wave-uniform call sites: the matrix cores sum over the limb rows in LDS */
      root_schur_mfma();
      tsync();
#pragma unroll
      for (int t = 0; t < NG; t++) g[t] = L->vec[V_TMP2][t];
    } else {
      static_assert(NG == 21, "reduce21_to");
      int t = 0;
#pragma unroll
      for (int i = 0; i < RMAX; i++) {
        const float wi = ischain ? Xd * X[i] : 0.f;
#pragma unroll
        for (int j = 0; j <= i; j++) g[t++] = wi * X[j];
      }
      reduce21_to(g, &L->vec[V_TMP2][0]);
      tsync();
#pragma unroll
      for (int t2 = 0; t2 < NG; t2++) g[t2] = L->vec[V_TMP2][t2];
    }
    float A[RMAX][RMAX], D[RMAX];
    {
      int t = 0;
#pragma unroll
      for (int i = 0; i < RMAX; i++) {
#pragma unroll
        for (int j = 0; j < RMAX; j++) A[i][j] = 0.f;
        if constexpr (MFMA_SCHUR) {
          /* the matrix cores already subtracted the Schur complement from the parked block */
#pragma unroll
          for (int j = 0; j < i; j++) A[i][j] = i < nroot ? g[t + j] : 0.f;
          D[i] = i < nroot ? g[t + i] : 1.f;
        } else {
#pragma unroll
          for (int j = 0; j < i; j++) A[i][j] = i < nroot ? L->L[i][j] - g[t + j] : 0.f;
          D[i] = i < nroot ? L->Dk[i] - g[t + i] : 1.f;
        }
        t += i + 1;
      }
    }
    tsync();
#pragma unroll
    for (int k = RMAX - 1; k >= 0; k--) {
      if (k < nroot) {
        const float Dkv = fmaxf(D[k], MINVAL);
        const float inv = 1.0f / Dkv;
        D[k] = Dkv;
        float tk[RMAX]; /* the unscaled row: the update multiplier A(k,i) = L(k,i) D_k */
#pragma unroll
        for (int i = 0; i < k; i++) {
          tk[i] = A[k][i];
          A[k][i] = A[k][i] * inv;
        }
#pragma unroll
        for (int i = 0; i < k; i++) {
          const float t = tk[i];
          D[i] -= t * A[k][i];
#pragma unroll
          for (int e = 0; e < i; e++) A[i][e] -= t * A[k][e];
        }
        if (c.l == 0) {
#pragma unroll
          for (int i = 0; i < k; i++) L->L[k][i] = A[k][i];
          L->Dk[k] = Dkv;
          L->Di[k] = inv;
        }
      }
    }
    tsync();
    const float di = keepf(L->Di[c.l & 31]);
    if (isroot) return di;
  }
  tsync();
  return 1.0f / fmaxf(Xd, MINVAL);
}

/* load a depth-indexed M row into off-diagonal X[] (masked) and diagonal */
__device__ __forceinline__ float load_mrow(const Ctx& c, float X[CAP]) {
  const int ddep = vopq(c.ddep);
  const int j = c.l & 31;
  /* no mask: entries at or past the depth (the diagonal, the transposed entries) are never read
     as off-diagonals by the factorization, and non-dof rows are zero */
  ld_row(&c.L->M[j][0], X);
  /* non-dof rows are zero: their diagonal becomes 1 without a select around the load */
  return c.L->M[j][ddep] + (c.l < NV ? 0.f : 1.f);
}

/* x <- (L'DL)^-1 x, x held by dof lanes (mj_solveM order: L' pass from the
 * leaves, diagonal, L pass from the root). Inside each limb chain both
 * triangular passes are one gather with the chain's W = (I + Lt)^-1 from
 * factor_ldl (slots NROOT.. of the stored rows): forward z_p = b_p +
 * sum_{k > p} W(p, k) b_k, backward x_p = v_p + sum_{a < p} W(a, p) v_a. The
 * root chain is dense and redundant in every lane. */
/* Per-lane solve data for solve_pre (CG: M's factor is fixed for the substep's ~10 solves).
 * With W = (I + Lt)^-1 the chain inverses of factor_ldl (Wf: W with its unit diagonal), Lr the limb
 * rows' root entries L(j, root), D the pivots and R^-1 = L_r^-1 D_r^-1 L_r^-T the inverse of the
 * factored 6 x 6 root block, the tree solve x = L^-1 D^-1 L^-T b is, for limb dof p of a chain,
 *   x_p = sum_k Q(p, k) b_k + sum_e U(p, e) sr_e,   sr_e = b_e(root) - sum_j g_j[e] b_j,
 *   Q = Wf' D^-1 Wf (the chain block), U(p, .) = sum_{m <= p} Wf(m, p) u_m, g_j[e] = sum_{m <= j} Lr(m, e) Wf(m, j),
 * u_m = -R^-1 Lr(m, .)' (a root lane e: u = R^-1 e_e, x_e = sum u sr; Q = g = 0). So a solve is one
 * gather of the lane's chain values and one team reduction, both of b, in flight together, then 12
 * products: the limb passes' two dependent exchange rounds and the root block's dense passes leave
 * the solve (the same arithmetic, another order). Stored after the last reader of the factor's rows:
 * Q, g in L[lane][0..11] (CG reads no factor row past this point), U in Hs[lane][0..5] (CG builds no
 * Hessian; Hs shares memory with sub[], so the caller runs this after the smooth phase's last subtree
 * sum, rne_project, and the sensors' first one comes after the solver). */
__device__ __forceinline__ void solve_prep(const Ctx& c) {
  EnvL* L = c.L;
  const bool isroot = c.l < NROOT, ischain = c.chd >= 0;
  const int lr = c.l & 31;
  /* u: this lane's row of the root coupling (the dense passes of solve_ldl on e_l or -Lr(l, .)) */
  float w[CAP];
  ld_row(&L->L[lr][0], w);
  float xr[RMAX];
#pragma unroll
  for (int k = 0; k < RMAX; k++) xr[k] = isroot ? (c.l == k ? 1.f : 0.f) : (ischain ? -w[k] : 0.f);
#pragma unroll
  for (int k = RMAX - 1; k >= 1; k--)
#pragma unroll
    for (int i = 0; i < k; i++) xr[i] -= L->L[k][i] * xr[k];
#pragma unroll
  for (int k = 0; k < RMAX; k++) xr[k] *= L->Di[k];
#pragma unroll
  for (int k = 1; k < RMAX; k++)
#pragma unroll
    for (int a = 0; a < k; a++) xr[k] -= L->L[k][a] * xr[a];
  tsync(); /* sub[] (same memory as Hs) is read by other lanes up to here */
  static_assert(RMAX == 6 && NLIMBLV == 6, "six-entry rows");
  *reinterpret_cast<v4f*>(&L->Hs[lr][0]) = v4f{xr[0], xr[1], xr[2], xr[3]};
  L->Hs[lr][4] = xr[4];
  L->Hs[lr][5] = xr[5];
  tsync();
  /* the chain sums over the shallower-or-equal chain positions m <= p */
  const int p = ischain ? vopq(c.cps) : -1;
  const int chd = ischain ? c.chd : 0;
  float Q[NLIMBLV], U[RMAX], g[RMAX];
#pragma unroll
  for (int k = 0; k < NLIMBLV; k++) Q[k] = 0.f;
#pragma unroll
  for (int e = 0; e < RMAX; e++) {
    U[e] = isroot ? xr[e] : 0.f;
    g[e] = 0.f;
  }
#pragma unroll
  for (int m = 0; m < NLIMBLV; m++) {
    const int lm = chd + m; /* a valid lane for every lane (chd + 5 <= 31) */
    float wm[CAP];
    ld_row(&L->L[lm][0], wm); /* Lr(m, .) in 0..5, W(m, k) in NROOT + k (zero for k <= m) */
    const v4f um4 = *reinterpret_cast<const v4f*>(&L->Hs[lm][0]);
    const float um[RMAX] = {um4[0], um4[1], um4[2], um4[3], L->Hs[lm][4], L->Hs[lm][5]};
    const float dinv = 1.f / fmaxf(L->Dk[lm], MINVAL);
    /* Wf(m, p): 1 on the diagonal, the stored entry past it, 0 for m > p (and off the chains) */
    float wmp = 0.f;
#pragma unroll
    for (int k = 0; k < NLIMBLV; k++) wmp = (p == k) ? wm[NROOT + k] : wmp;
    wmp = m == p ? 1.f : (m < p ? wmp : 0.f);
    const float wd = wmp * dinv;
#pragma unroll
    for (int k = 0; k < NLIMBLV; k++) Q[k] += wd * (k == m ? 1.f : wm[NROOT + k]);
#pragma unroll
    for (int e = 0; e < RMAX; e++) {
      U[e] += wmp * um[e];
      g[e] += wm[e] * wmp;
    }
  }
  tsync(); /* every lane's reads of the factor rows and of u are done */
  *reinterpret_cast<v4f*>(&L->L[lr][0]) = v4f{Q[0], Q[1], Q[2], Q[3]};
  *reinterpret_cast<v4f*>(&L->L[lr][4]) = v4f{Q[4], Q[5], g[0], g[1]};
  *reinterpret_cast<v4f*>(&L->L[lr][8]) = v4f{g[2], g[3], g[4], g[5]};
  *reinterpret_cast<v4f*>(&L->Hs[lr][0]) = v4f{U[0], U[1], U[2], U[3]};
  L->Hs[lr][4] = U[4];
  L->Hs[lr][5] = U[5];
  tsync();
}

/* x <- M^-1 x with solve_prep's per-lane data (CG): the chain gather and the root sums of b in
   flight together, then x_p = sum_k Q(p, k) b_k + sum_e U(p, e) sr_e (solve_prep) */
__device__ __forceinline__ float solve_pre(const Ctx& c, float x) {
  EnvL* L = c.L;
  const int lr = c.l & 31;
  const bool ischain = c.chd >= 0;
  const int chd = ischain ? c.chd : 0;
  float qg[CAP];
  ld_row(&L->L[lr][0], qg); /* Q[0..5], g[0..5] */
  const v4f u4 = *reinterpret_cast<const v4f*>(&L->Hs[lr][0]);
  const float U[RMAX] = {u4[0], u4[1], u4[2], u4[3], L->Hs[lr][4], L->Hs[lr][5]};
  float bk[NLIMBLV];
#pragma unroll
  for (int k = 0; k < NLIMBLV; k++) bk[k] = tsh(x, chd + k);
  float sr[RMAX];
#pragma unroll
  for (int e = 0; e < RMAX; e++) sr[e] = (c.l == e ? x : 0.f) - qg[NLIMBLV + e] * x;
  tsum_n<RMAX>(sr);
  float y = 0.f;
#pragma unroll
  for (int k = 0; k < NLIMBLV; k++) y += qg[k] * bk[k];
#pragma unroll
  for (int e = 0; e < RMAX; e++) y += U[e] * sr[e];
  return y;
}

__device__ __forceinline__ float solve_ldl(const Ctx& c, float x, float Dinv) {
  EnvL* L = c.L;
  const int nroot = NROOT;
  const bool ischain = c.chd >= 0;
  const int cps = vopq(c.cps), cln = vopq(c.cln), chd = ischain ? c.chd : 0;
  /* the lane's stored row: W(p, k) in slots NROOT + k (chain lanes), L(j, root i) in 0..NROOT-1 */
  float w[CAP];
  ld_row(&L->L[c.l & 31][0], w);
  /* forward pass along the limbs: the chain's deeper right-hand sides, all in flight */
  {
    /* W(p, k) is zero for k <= p and past the chain, so only non-chain lanes mask it */
    float bk[NLIMBLV];
#pragma unroll
    for (int k = 1; k < NLIMBLV; k++) bk[k] = tsh(x, chd + k);
    float z = x;
#pragma unroll
    for (int k = 1; k < NLIMBLV; k++) z += (ischain ? w[NROOT + k] : 0.f) * bk[k];
    x = z;
  }
  /* root chain, dense and redundant in every lane */
  float xr[RMAX];
#pragma unroll
  for (int k = 0; k < RMAX; k++) xr[k] = 0.f;
  if (nroot > 0) {
    /* xr[k] = x_k - sum_{limb j} L(j, k) x_j: root lane k adds its own value into the
       same team reduction (no separate broadcast of x_k); w[] of a root or non-dof lane
       meets a zero (xs), and non-dof rows are zero */
    const float xs = ischain ? x : 0.f;
    float sr[RMAX];
#pragma unroll
    for (int k = 0; k < RMAX; k++) sr[k] = c.l == k ? x : -w[k] * xs;
    tsum_n<RMAX>(sr);
#pragma unroll
    for (int k = 0; k < RMAX; k++)
      if (k < nroot) xr[k] = sr[k];
#pragma unroll
    for (int k = RMAX - 1; k >= 1; k--)
      if (k < nroot)
#pragma unroll
        for (int i = 0; i < k; i++) xr[i] -= L->L[k][i] * xr[k];
#pragma unroll
    for (int k = 0; k < RMAX; k++)
      if (k < nroot) xr[k] *= L->Di[k];
#pragma unroll
    for (int k = 1; k < RMAX; k++)
      if (k < nroot)
#pragma unroll
        for (int a = 0; a < k; a++) xr[k] -= L->L[k][a] * xr[a];
    x *= Dinv;
    /* limb lanes; a root lane's x is replaced below, a non-dof row is zero */
#pragma unroll
    for (int e = 0; e < RMAX; e++)
      if (e < nroot) x -= w[e] * xr[e];
#pragma unroll
    for (int k = 0; k < RMAX; k++)
      if (c.l == k && k < nroot) x = xr[k];
  } else {
    x *= Dinv;
  }
  /* backward pass down the limbs: the shallower chain values and W(a, p), all in flight */
  {
    /* W(a, p) for chain position a: zero for a >= p (stored W rows are zero at and before
       their own position), so no mask inside the chain; positions past the chain read its
       last row (zero there too), and a non-chain lane reads the zero rows 26.. */
    float va[NLIMBLV - 1], wa[NLIMBLV - 1];
    static_assert(NV + NLIMBLV - 1 <= 31, "zero rows NV .. NV + 4");
    const int chz = vopq(ischain ? c.chd : NV);
    const int alast = vopq(ischain ? c.cln - 1 : NLIMBLV - 2);
#pragma unroll
    for (int a = 0; a < NLIMBLV - 1; a++) wa[a] = L->L[chz + min(a, alast)][NROOT + cps];
#pragma unroll
    for (int a = 0; a < NLIMBLV - 1; a++) va[a] = tsh(x, chz + a);
    float y = x;
#pragma unroll
    for (int a = 0; a < NLIMBLV - 1; a++) y += wa[a] * va[a];
    x = y;
  }
  return x;
}

/* y = M x (M rows in LDS), x in dof lanes; uses vec[slot] */
__device__ __forceinline__ float mul_m(const Ctx& c, float x, int slot) {
  EnvL* L = c.L;
  const int j = c.l;
  const bool ischain = c.chd >= 0;
  const int nroot = NROOT;
  if (j < 32) L->vec[slot][j] = x;
  tsync();
  /* M(j, anc) x_anc, the diagonal and the deeper dofs of j's chain (their entries sit in
     the row padding, com_crb_m): one row load + all ancestor values in flight */
  float mrow[CAP], vv[CAP];
  ld_row(&L->M[j & 31][0], mrow);
#pragma unroll
  for (int e = 0; e < CAP; e++) vv[e] = L->vec[slot][anc_lin(c.chd, e)];
  float y = 0.f;
#pragma unroll
  for (int e = 0; e < CAP; e++) y += mrow[e] * vv[e]; /* zero past the chain */
  if (nroot > 0) {
    /* root lanes: the limb dofs' M(k, root i) = mrow[i], one transposing reduction
       (the deeper root dofs come with the row product, from the row padding) */
    static_assert(RMAX == 6, "reduce6_lane");
    float si[RMAX];
#pragma unroll
    for (int i = 0; i < RMAX; i++) si[i] = (ischain && i < nroot) ? mrow[i] * x : 0.f;
    const float sr = reduce6_lane(si); /* root lane j: sum j */
    if (j < nroot) y += sr;
  }
  tsync();
  return y;
}

/* chain gather: sum_e Jc[e] * vec[slot][anc_e] for a contact row (Jrow: the row in bank 0's or
   bank 1's J, chd: the row's chain head) */
template <typename JP>
__device__ __forceinline__ float row_dot(const Ctx& c, JP Jrow, int chd, int slot) {
  float jr[CAP], vv[CAP];
  ld_row(Jrow, jr);
#pragma unroll
  for (int e = 0; e < CAP; e++) vv[e] = c.L->vec[slot][anc_lin(chd, e)];
  float v = 0.f;
#pragma unroll
  for (int e = 0; e < CAP; e++) v += jr[e] * vv[e]; /* zero past the row's depth */
  return v;
}
__device__ __forceinline__ float row_dot(const Ctx& c, const Rows& r, int slot) {
  return row_dot(c, &c.L->u.J[c.l][0], r.chd, slot);
}
__device__ __forceinline__ float row_dot_x(const Ctx& c, const Rows& r, int slot) {
  return row_dot(c, (const gfloat_t*)xrows(c.L) + c.l * CAP, r.x.chd, slot);
}
__device__ __forceinline__ float row_dot_y(const Ctx& c, const Rows& r, int slot) {
  return row_dot(c, (const gfloat_t*)yrows(c.L) + c.l * CAP, r.y.chd, slot);
}

/* row_dot with the lane's row already in registers (jr) */
__device__ __forceinline__ float row_dot_pre(const Ctx& c, const float jr[CAP], int chd, int slot) {
  float vv[CAP];
#pragma unroll
  for (int e = 0; e < CAP; e++) vv[e] = c.L->vec[slot][anc_lin(chd, e)];
  float v = 0.f;
#pragma unroll
  for (int e = 0; e < CAP; e++) v += jr[e] * vv[e];
  return v;
}
/* y = M x (mul_m) and, in the same LDS round trip, the lane's contact-row products with x
 * (jv, row_dot over vec[slot]) and, when slot2 >= 0, with vec[slot2] (jv2, published before the
 * call): the row loads go out with mul_m's ancestor gather instead of after its reduction and
 * exchange point. jr: the lane's contact-row Jacobian, loaded once per solve. Bit-identical to
 * mul_m followed by row_dot. */
__device__ __forceinline__ float mul_m_dot(const Ctx& c, const Rows& r, const float jr[CAP], float x, int slot, float& jv,
                                           int slot2, float& jv2) {
  EnvL* L = c.L;
  const int j = c.l;
  const bool ischain = c.chd >= 0;
  const int nroot = NROOT;
  if (j < 32) L->vec[slot][j] = x;
  tsync();
  float mrow[CAP], vv[CAP];
  ld_row(&L->M[j & 31][0], mrow);
#pragma unroll
  for (int e = 0; e < CAP; e++) vv[e] = L->vec[slot][anc_lin(c.chd, e)];
  jv = row_dot_pre(c, jr, r.chd, slot);
  jv2 = slot2 >= 0 ? row_dot_pre(c, jr, r.chd, slot2) : 0.f;
  float y = 0.f;
#pragma unroll
  for (int e = 0; e < CAP; e++) y += mrow[e] * vv[e];
  if (nroot > 0) {
    static_assert(RMAX == 6, "reduce6_lane");
    float si[RMAX];
#pragma unroll
    for (int i = 0; i < RMAX; i++) si[i] = (ischain && i < nroot) ? mrow[i] * x : 0.f;
    const float sr = reduce6_lane(si);
    if (j < nroot) y += sr;
  }
  tsync();
  return y;
}

/* ----------------------------------- RNE ----------------------------------- */
/* inclusive prefix sums of per-dof 6-vectors along the dof tree (root ->
 * dof), by pointer jumping over the parent links: ceil(log2(depth)) rounds of
 * cross-lane pulls instead of one ancestor gather per depth */
__device__ __forceinline__ void dof_prefix6(const Ctx& c, float P[6]) {
  const int ddep = vopq(c.ddep);
  bool live = c.l < NV && ddep > 0;
  int ptr = live ? anc_lin(c.chd, ddep - 1) : c.l;
  for (int span = 1; span < MAXDD; span <<= 1) {
    float w[6];
#pragma unroll
    for (int k = 0; k < 6; k++) w[k] = tsh(P[k], ptr);
    const int nptr = tshi(ptr, ptr);
    const bool nlive = tshi(live ? 1 : 0, ptr) != 0;
    if (live) {
#pragma unroll
      for (int k = 0; k < 6; k++) P[k] += w[k];
      ptr = nptr;
      live = nlive;
    }
  }
}

/* mj_comVel: cvel (lane b, in B.cv) and cdof_dot (lane j, returned).
   Requires the dof lanes' qvel in ls_v. */
__device__ __forceinline__ void com_vel(const Ctx& c, BodyK& B, float qv, float cdd[6]) {
  const int ddep = vopq(c.ddep);
  EnvL* L = c.L;
  const int j = c.l;
  const bool isd = j < NV;
  /* non-dof rows of cdof are zero (com_crb_m) and so is their qv */
  float cd[6];
#pragma unroll
  for (int k = 0; k < 6; k++) cd[k] = L->cdof[j][k];
  float P[6];
#pragma unroll
  for (int k = 0; k < 6; k++) P[k] = cd[k] * qv;
  dof_prefix6(c, P);
  /* velocity before this dof's own contribution: the parent's prefix for a
     hinge, the translational part (dof 2) for the free joint's rotations */
  const bool isfree = c.dfree;
  const int k0 = c.dk0;
  const int par = (isd && ddep > 0) ? anc_lin(c.chd, ddep - 1) : j;
  const int src = (isfree && k0 >= 3) ? 2 : par; /* one pull per component */
  float before[6];
#pragma unroll
  for (int k = 0; k < 6; k++) {
    const float pp = tsh(P[k], src);
    before[k] = ddep > 0 ? pp : 0.f;
  }
#pragma unroll
  for (int k = 0; k < 6; k++) cdd[k] = 0.f;
  if (isd && !(isfree && k0 < 3)) cross_motion(cdd, before, cd);
  /* body velocity = prefix at the body's deepest dof */
  const int bl = (c.l < NB && c.blast >= 0) ? c.blast : 0;
#pragma unroll
  for (int k = 0; k < 6; k++) {
    const float v = tsh(P[k], bl);
    B.cv[k] = (c.l < NB && c.blast >= 0) ? v : 0.f;
  }
}

/* cacc per body (lane b): -g + prefix of cdof_dot*qvel (+ cdof*qacc) */
__device__ __forceinline__ void com_acc(const Ctx& c, const float cdd[6], float qv, float qa, float ca[6],
                                        bool with_acc) {
  MP m = c.m;
  EnvL* L = c.L;
  const int j = c.l;
  const bool isd = j < NV;
  float P[6];
#pragma unroll
  for (int k = 0; k < 6; k++) P[k] = isd ? cdd[k] * qv : 0.f;
  if (with_acc) {
#pragma unroll
    for (int k = 0; k < 6; k++) P[k] += L->cdof[j][k] * qa; /* zero rows past the dofs */
  }
  dof_prefix6(c, P);
  const float g[6] = {0.f, 0.f, 0.f, -m->gravity[0], -m->gravity[1], -m->gravity[2]};
  const int bl = (c.l < NB && c.blast >= 0) ? c.blast : 0;
#pragma unroll
  for (int k = 0; k < 6; k++) {
    const float v = tsh(P[k], bl);
    ca[k] = g[k] + ((c.l < NB && c.blast >= 0) ? v : 0.f);
  }
}

/* body force cfrc (lane b) -> subtree sums in sub[] ; returns dof projection cdof_j . sub[body(j)] */
__device__ __forceinline__ float rne_project(const Ctx& c, const BodyK& B, const float ca[6], const float fext[6]) {
  EnvL* L = c.L;
  float f[6];
  if (c.l >= 1 && c.l < NB) {
    float f1[6], t[6], f2[6], ci[10];
#pragma unroll
    for (int k = 0; k < 10; k++) ci[k] = L->ci[c.l][k];
    mul_inert_vec(f1, ci, ca);
    mul_inert_vec(t, ci, B.cv);
    cross_force(f2, B.cv, t);
#pragma unroll
    for (int k = 0; k < 6; k++) f[k] = f1[k] + f2[k] - fext[k];
  } else {
#pragma unroll
    for (int k = 0; k < 6; k++) f[k] = 0.f;
  }
  subtree_sum<6>(c, f);
  float r = 0.f;
  if (c.l < NV) {
    float cd[6], fs[6];
#pragma unroll
    for (int k = 0; k < 6; k++) {
      cd[k] = L->cdof[c.l][k];
      fs[k] = L->sub[c.dbody][k];
    }
    r = dot6(cd, fs);
  }
  tsync();
  return r;
}

/* --------------------------- constraint model ------------------------------ */
template <typename PS>
__device__ __forceinline__ float impedance(PS si, float xabs) {
  const float dmin = si[0], dmax = si[1], width = si[2], mid = si[3], power = si[4];
  /* mj_makeImpedance; branch-free in the per-lane distance, the power is a
     model constant (uniform branch; 2 is MuJoCo's default, without powf) */
  const bool sat = width <= MINVAL || xabs >= width;
  const float x = sat ? 0.f : xabs / width;
  float y;
  if (power == 1.f) {
    y = x;
  } else if (power == 2.f) {
    const float ylo = x * x / mid, yhi = 1.f - (1.f - x) * (1.f - x) / (1.f - mid);
    y = x <= mid ? ylo : yhi;
  } else {
    y = x <= mid ? powf(x, power) / powf(mid, power - 1.f) : 1.f - powf(1.f - x, power) / powf(1.f - mid, power - 1.f);
  }
  const float imp = sat ? dmax : dmin + y * (dmax - dmin);
  return fminf(fmaxf(imp, MINIMP), MAXIMP);
}
template <typename PR, typename PS>
__device__ __forceinline__ void row_params(PR solref, PS solimp, float pos, float dA, float vel,
                                           float dt, float& D, float& R, float& aref) {
  float tc = fmaxf(solref[0], 2.f * dt), dr = solref[1], dmax = solimp[1];
  float bb = 2.f / (dmax * tc);
  float kk = 1.f / (dmax * dmax * tc * tc * dr * dr);
  float imp = impedance(solimp, fabsf(pos));
  R = fmaxf((1.f - imp) / imp * dA, MINVAL);
  D = 1.f / R;
  aref = -bb * vel - kk * imp * pos;
}

/* The extra contact-row banks by kernel instantiation (zb_host.cpp needs_xg): XG 1 / 2 the second bank
   (Rows::x) holds the general floor colliders (the first two beyond the soles within reach, select_bank2;
   XG 2 compiles cylinders, ellipsoids and meshes), XG 3 the sole pair (the two box soles against each
   other, pair_rows), XG 4 both: the floor colliders in the second bank and the sole pair in a third
   (Rows::y, round 6), XG 5 (models with more than two colliders beyond the soles) floor colliders in
   the second and third banks: the first four within reach of the floor each substep. XG 0: the two
   soles alone. */
template <int XG>
constexpr bool XFLOOR = XG == 1 || XG == 2 || XG == 4 || XG == 5;
template <int XG>
constexpr bool XPAIR = XG == 3; /* the pair in the second bank */
template <int XG>
constexpr bool YPAIR = XG == 4; /* the pair in the third bank */
template <int XG>
constexpr bool YFLOOR = XG == 5; /* floor colliders in the third bank too */
template <int XG>
constexpr bool YBANK = YPAIR<XG> || YFLOOR<XG>; /* the third bank exists */
template <int XG>
constexpr bool XRICH = XG == 2 || XG == 4 || XG == 5; /* cylinder / ellipsoid / mesh rules compiled */
template <int XG>
constexpr bool ANYPAIR = XPAIR<XG> || YPAIR<XG>;

/* The collider of team lane l in contact-row bank `bank`: geom 2 bank + l / 16 (general colliders), or
   sole l / 16 (the two-sole and sole-pair kernels). gb: its body; false when the model has no such geom. */
template <int XG>
__device__ __forceinline__ bool lane_geom(const Ctx& c, int bank, int& g, int& gb) {
  MP m = c.m;
  const int gl = c.l >> 4;
  if (XFLOOR<XG> && bank >= 1) {
    /* the second (third: XG 5) bank's geoms of this substep (select_bank2) */
    const int sg = bank == 1 ? c.L->s.xsel[gl] : c.L->ysel[gl];
    const bool sv = sg >= 0;
    g = sv ? sg : 0;
    gb = sv ? m->geom_body[g] : 0;
    return sv;
  }
  g = XFLOOR<XG> ? 2 * bank + gl : gl;
  const bool gvalid = XFLOOR<XG> ? g < m->ngeom : gl < NGEOM;
  if (!gvalid) g = 0;
  gb = gvalid ? m->geom_body[g] : 0;
  return gvalid;
}

/* Floor contact of team lane l = 16*geom + 4*slot + edge (MuJoCo's primitive colliders,
 * engine_collision_primitive.c; oracle collision()):
 *   box (mjc_PlaneBox): contact slot k holds the corner of the pair (k, 7-k) that lies below the
 *     box centre along the normal: corner k = (+-x, +-y, -z) by the bits of k, or its mirror
 *     7-k = -corner k. Exactly those four corners pass MuJoCo's "offset along the normal <= 0"
 *     test (an offset of exactly zero aside), so the set is MuJoCo's; only the row order differs.
 *   capsule (mjc_PlaneCapsule, XG): slots 0 / 1 = the sphere at the +/- half-length end, tangent
 *     frame along the axis projected on the plane (mjx plane_capsule: +y when that projection is
 *     shorter than 0.5);
 *   sphere (mjc_PlaneSphere, XG): slot 0;
 *   ellipsoid (mjc_PlaneEllipsoid, XG): slot 0, the support point along -n;
 *   cylinder (mjc_PlaneCylinder, XG): slots 0-3 (below).
 * Sets the contact point (the deepest point moved back by half the distance), the pyramid edge
 * direction n +- mu t (t1 = +y, t2 = n x t1 = -x for boxes and spheres: mju_makeFrame(+z)) and the
 * friction; returns the signed distance, 1e30 where the slot holds no contact. Recomputed by the
 * sensors instead of being held in registers through the solver. */
template <int XG>
__device__ __forceinline__ float contact_point(const Ctx& c, const EnvS& s, const BodyK& B, int bank, float pos[3],
                                               float dir[3], float& mu) {
  MP m = c.m;
  const int l = c.l;
  const int slot = (l >> 2) & 3, edge = l & 3;
  int g, gb;
  const bool gvalid = lane_geom<XG>(c, bank, g, gb);
  float xp[3], xqs[4];
#pragma unroll
  for (int k = 0; k < 4; k++) xqs[k] = tsh(B.xq[k], gb);
#pragma unroll
  for (int k = 0; k < 3; k++) xp[k] = tsh(B.xp[k], gb);
  const int ty = XFLOOR<XG> ? m->geom_type[g] : ZB_GEOM_BOX;
  /* XG 2: the instantiation for models with cylinders or ellipsoids (zb_host.cpp needs_xg), so that
     the others carry no code for them */
  const bool box = !XFLOOR<XG> || ty == ZB_GEOM_BOX, cap = XFLOOR<XG> && ty == ZB_GEOM_CAPSULE,
             cyl = XRICH<XG> && ty == ZB_GEOM_CYLINDER, ell = XRICH<XG> && ty == ZB_GEOM_ELLIPSOID,
             msh = XRICH<XG> && ty == ZB_GEOM_MESH;
  /* the lane's point relative to the geom centre, geom frame -> body frame -> world */
  float gq[4] = {m->geom_quat[g][0], m->geom_quat[g][1], m->geom_quat[g][2], m->geom_quat[g][3]};
  float gp[3] = {m->geom_pos[g][0], m->geom_pos[g][1], m->geom_pos[g][2]};
  const float s0 = m->geom_size[g][0], s1 = m->geom_size[g][1], s2 = m->geom_size[g][2];
  float p[3], dist;
  bool slot_ok;
  float t1x = 0.f, t1y = 1.f;
  if (cyl || ell || msh) {
    /* the geom's world rotation R from one quaternion product (body then geom), and its centre */
    const float qw0 = xqs[0] * gq[0] - xqs[1] * gq[1] - xqs[2] * gq[2] - xqs[3] * gq[3];
    const float qw1 = xqs[0] * gq[1] + xqs[1] * gq[0] + xqs[2] * gq[3] - xqs[3] * gq[2];
    const float qw2 = xqs[0] * gq[2] - xqs[1] * gq[3] + xqs[2] * gq[0] + xqs[3] * gq[1];
    const float qw3 = xqs[0] * gq[3] + xqs[1] * gq[2] - xqs[2] * gq[1] + xqs[3] * gq[0];
    const float R00 = 1.f - 2.f * (qw2 * qw2 + qw3 * qw3), R01 = 2.f * (qw1 * qw2 - qw0 * qw3), R02 = 2.f * (qw1 * qw3 + qw0 * qw2);
    const float R10 = 2.f * (qw1 * qw2 + qw0 * qw3), R11 = 1.f - 2.f * (qw1 * qw1 + qw3 * qw3), R12 = 2.f * (qw2 * qw3 - qw0 * qw1);
    const float R20 = 2.f * (qw1 * qw3 - qw0 * qw2), R21 = 2.f * (qw2 * qw3 + qw0 * qw1), R22 = 1.f - 2.f * (qw1 * qw1 + qw2 * qw2);
    float cw[3];
    quat_rotate(cw, xqs, gp);
    const float c0 = xp[0] + cw[0], c1 = xp[1] + cw[1], c2 = xp[2] + cw[2];
    if (msh) {
      /* MJX plane_convex (oracle plane_mesh, which states the rule): the 16 lanes of the geom's half
         scan the hull's vertices (lane li: vertices li + 16 j), every argmax a row reduction; the
         lane's slot then takes manifold point a, b, c or d */
      const int adr = m->geom_vertadr[g], nvt = m->geom_vertnum[g];
      const int li = l & 15;
      const float n[3] = {R20, R21, R22}; /* the plane normal in the geom frame, R' e_z */
      const float pp[3] = {-(R00 * c0 + R10 * c1 + R20 * c2), -(R01 * c0 + R11 * c1 + R21 * c2),
                           -(R02 * c0 + R12 * c1 + R22 * c2)}; /* the plane's origin, R' (0 - c) */
      /* NJ vertices per lane: one for a hull of at most 16 (a box's 8 corners), four otherwise */
      auto manifold = [&](auto njc) {
      constexpr int NJ = decltype(njc)::value;
      float v[NJ][3], sup[NJ], dm[NJ];
      bool ok[NJ];
      float smax = -3.0e38f;
#pragma unroll
      for (int j = 0; j < NJ; j++) {
        const int i = li + 16 * j;
        ok[j] = i < nvt;
        const int ii = adr + (ok[j] ? i : 0);
#pragma unroll
        for (int k = 0; k < 3; k++) v[j][k] = m->mesh_vert[ii][k];
        sup[j] = (pp[0] - v[j][0]) * n[0] + (pp[1] - v[j][1]) * n[1] + (pp[2] - v[j][2]) * n[2];
        smax = ok[j] ? fmaxf(smax, sup[j]) : smax;
      }
      smax = rowmax16(smax);
      const float thr = fmaxf(smax - 1e-3f, 0.f);
#pragma unroll
      for (int j = 0; j < NJ; j++) dm[j] = sup[j] > thr ? 0.f : -1e6f;
      /* argmax over the lane's vertices (in index order), then over the row; absent vertices never win */
      auto argmax = [&](auto value) {
        float bw = -3.0e38f;
        int bi = 0x7fffffff;
#pragma unroll
        for (int j = 0; j < NJ; j++) {
          const float w = value(j) + dm[j];
          if (ok[j] && w > bw) { bw = w; bi = li + 16 * j; }
        }
        rowargmax16(bw, bi);
        return bi;
      };
      const int ia = argmax([&](int) { return 0.f; });
      float A[3], Bv[3], Cv[3];
#pragma unroll
      for (int k = 0; k < 3; k++) A[k] = m->mesh_vert[adr + ia][k];
      const int ib = argmax([&](int j) {
        const float e0 = A[0] - v[j][0], e1 = A[1] - v[j][1], e2 = A[2] - v[j][2];
        return e0 * e0 + e1 * e1 + e2 * e2;
      });
#pragma unroll
      for (int k = 0; k < 3; k++) Bv[k] = m->mesh_vert[adr + ib][k];
      float ab[3];
      {
        const float amb[3] = {A[0] - Bv[0], A[1] - Bv[1], A[2] - Bv[2]};
        cross3(ab, n, amb);
      }
      const int ic = argmax([&](int j) {
        const float ap[3] = {A[0] - v[j][0], A[1] - v[j][1], A[2] - v[j][2]};
        return fabsf(dot3(ap, ab));
      });
#pragma unroll
      for (int k = 0; k < 3; k++) Cv[k] = m->mesh_vert[adr + ic][k];
      float ac[3], bc[3];
      {
        const float amc[3] = {A[0] - Cv[0], A[1] - Cv[1], A[2] - Cv[2]};
        const float bmc[3] = {Bv[0] - Cv[0], Bv[1] - Cv[1], Bv[2] - Cv[2]};
        cross3(ac, n, amc);
        cross3(bc, n, bmc);
      }
      /* d: the first maximum over the concatenation [|(b - v) . bc| ..., |(a - v) . ac| ...] (key i, then
         nvt + i) */
      int id;
      {
        float bw = -3.0e38f;
        int bk = 0x7fffffff;
#pragma unroll
        for (int h = 0; h < 2; h++)
#pragma unroll
          for (int j = 0; j < NJ; j++) {
            const float* o = h == 0 ? Bv : A;
            const float* ax = h == 0 ? bc : ac;
            const float op[3] = {o[0] - v[j][0], o[1] - v[j][1], o[2] - v[j][2]};
            const float w = fabsf(dot3(op, ax)) + dm[j];
            const int key = (h == 0 ? 0 : nvt) + li + 16 * j;
            if (ok[j] && (w > bw || (w == bw && key < bk))) { bw = w; bk = key; }
          }
        rowargmax16(bw, bk);
        id = bk < nvt ? bk : bk - nvt;
      }
      /* the lane's manifold point (slot 0..3: a, b, c, d); a repeat of an earlier one has dist 1 */
      const int iq = slot == 0 ? ia : (slot == 1 ? ib : (slot == 2 ? ic : id));
      const bool uniq = slot == 0 || (slot == 1 && ib != ia) || (slot == 2 && ic != ia && ic != ib) ||
                        (slot == 3 && id != ia && id != ib && id != ic);
      float V[3];
#pragma unroll
      for (int k = 0; k < 3; k++) V[k] = m->mesh_vert[adr + iq][k];
      const float sq = (pp[0] - V[0]) * n[0] + (pp[1] - V[1]) * n[1] + (pp[2] - V[2]) * n[2];
      p[0] = c0 + (R00 * V[0] + R01 * V[1] + R02 * V[2]);
      p[1] = c1 + (R10 * V[0] + R11 * V[1] + R12 * V[2]);
      p[2] = c2 + (R20 * V[0] + R21 * V[1] + R22 * V[2]);
      dist = uniq ? -sq : 1.f;
      slot_ok = true;
      };
      if (nvt <= 16) manifold(IntC<1>{});
      else manifold(IntC<ZB_MAX_MESHV / 16>{});
    } else if (cyl) {
      /* mjc_PlaneCylinder (oracle collision()): the axis a (R's z column) turned toward the plane,
         v the radius vector in the disk planes toward it; slot 0 the near disk's deepest point
         c + v + a, 1 the far disk's c + v - a, 2 / 3 the near disk's points 120 degrees away,
         c + a - v / 2 +- v1; none unless slot 0 is within the margin */
      const float sg = R22 > 0.f ? -1.f : 1.f;
      float a[3] = {sg * R02, sg * R12, sg * R22};
      float prja = a[2];
      float v[3] = {a[0] * prja, a[1] * prja, a[2] * prja - 1.f};
      const float len = sqrtf(dot3(v, v));
      const bool par = !(len >= MINVAL); /* the disks parallel to the plane: the geom's x axis */
      const float sv = par ? s0 : s0 / len;
      v[0] = (par ? R00 : v[0]) * sv;
      v[1] = (par ? R10 : v[1]) * sv;
      v[2] = (par ? R20 : v[2]) * sv;
      const float prjv = v[2];
#pragma unroll
      for (int k = 0; k < 3; k++) a[k] *= s1;
      prja *= s1;
      const float d1 = c2 + prja + prjv;
      float v1[3];
      cross3(v1, v, a);
      const float n1 = sqrtf(dot3(v1, v1));
      const float sc = n1 > 0.f ? s0 * 0.8660254037844386f / n1 : 0.f;
      const float sa = slot == 1 ? -1.f : 1.f;                    /* +a, except the far disk */
      const float svv = slot >= 2 ? -0.5f : 1.f;                  /* +v, -v / 2 on the triangle */
      const float s1v = slot == 2 ? sc : (slot == 3 ? -sc : 0.f); /* +- v1 on the triangle */
      p[0] = c0 + svv * v[0] + sa * a[0] + s1v * v1[0];
      p[1] = c1 + svv * v[1] + sa * a[1] + s1v * v1[1];
      p[2] = c2 + svv * v[2] + sa * a[2] + s1v * v1[2];
      dist = slot == 0 ? d1 : (slot == 1 ? c2 - prja + prjv : c2 + prja - 0.5f * prjv);
      slot_ok = d1 <= m->floor_margin;
    } else {
      /* mjc_PlaneEllipsoid (oracle collision()): sn = s .* (R' n) (R's z row), the support point
         R (-s .* sn / |sn|) from the centre */
      const float sn0 = s0 * R20, sn1 = s1 * R21, sn2 = s2 * R22;
      const float inv = 1.f / sqrtf(sn0 * sn0 + sn1 * sn1 + sn2 * sn2);
      const float l0 = -s0 * sn0 * inv, l1 = -s1 * sn1 * inv, l2 = -s2 * sn2 * inv;
      p[0] = c0 + R00 * l0 + R01 * l1 + R02 * l2;
      p[1] = c1 + R10 * l0 + R11 * l1 + R12 * l2;
      p[2] = c2 + R20 * l0 + R21 * l1 + R22 * l2;
      dist = p[2];
      slot_ok = slot == 0;
    }
  } else {
    float v[3];
    if (box) {
      v[0] = (slot & 1) ? s0 : -s0;
      v[1] = (slot & 2) ? s1 : -s1;
      v[2] = -s2;
    } else {
      v[0] = 0.f;
      v[1] = 0.f;
      v[2] = cap ? (slot == 0 ? s1 : -s1) : 0.f;
    }
    float w[3], t[3];
    quat_rotate(w, gq, v);
    if (box) {
      /* the corner's offset along the normal: the z row of the body rotation times w */
      const float rz0 = 2.f * (xqs[1] * xqs[3] - xqs[0] * xqs[2]), rz1 = 2.f * (xqs[2] * xqs[3] + xqs[0] * xqs[1]);
      const float rz2 = 1.f - 2.f * (xqs[1] * xqs[1] + xqs[2] * xqs[2]);
      if (rz0 * w[0] + rz1 * w[1] + rz2 * w[2] > 0.f) {
        /* corner k lies above the centre: its mirror 7-k is the one MuJoCo keeps */
#pragma unroll
        for (int k = 0; k < 3; k++) w[k] = -w[k];
      }
    }
    float gl[3] = {gp[0] + w[0], gp[1] + w[1], gp[2] + w[2]};
    quat_rotate(t, xqs, gl);
    const float rad = box ? 0.f : s0;
    p[0] = xp[0] + t[0];
    p[1] = xp[1] + t[1];
    p[2] = xp[2] + t[2] - rad;
    dist = p[2];
    if (cap) {
      /* the +z axis of the capsule in the world: the rotated offset / half-length, sign of the +end */
      float u[3];
      quat_rotate(u, xqs, w);
      const float ax = slot == 0 ? u[0] : -u[0], ay = slot == 0 ? u[1] : -u[1];
      const float bn = sqrtf(ax * ax + ay * ay) / s1;
      const bool dflt = bn < 0.5f;
      const float inv = dflt ? 0.f : 1.f / (bn * s1);
      t1x = dflt ? 0.f : ax * inv;
      t1y = dflt ? 1.f : ay * inv;
    }
    slot_ok = box || (cap ? slot < 2 : slot == 0);
  }
  pos[0] = p[0]; pos[1] = p[1]; pos[2] = p[2] - 0.5f * dist;
  mu = m->floor_friction[0] * s.floor_mu;
  const float sg = (edge & 1) ? -mu : mu;
  /* edges 0/1: n +- mu t1; 2/3: n +- mu t2, t2 = n x t1 = (-t1y, t1x, 0) */
  dir[0] = edge < 2 ? sg * t1x : -sg * t1y;
  dir[1] = edge < 2 ? sg * t1y : sg * t1x;
  dir[2] = 1.f;
  return (gvalid && slot_ok) ? dist : 1e30f;
}

/* the contact rows of one bank: collision, then the row of lane l (J at Jrow) */
template <int XG, typename CR, typename JP>
__device__ __forceinline__ void contact_rows(const Ctx& c, const EnvS& s, const BodyK& B, const float cm[3], int bank,
                                             CR& r, JP Jrow) {
  MP m = c.m;
  CP cfg = c.cfg;
  EnvL* L = c.L;
  int g, gb;
  const bool gvalid = lane_geom<XG>(c, bank, g, gb);
  r.ex = false;
  r.act = 0;
  r.f = 0.f;
  r.jar = 0.f;
  r.Jv = 0.f;
  r.D = 0.f;
  r.aref = 0.f;
  if (XFLOOR<XG> && bank >= 1 && __ballot(gvalid) == 0ull) {
    /* no geom of the second bank within reach of the floor in either env of the wave (select_bank2):
       no row, the same state as the full test finds, without its shuffles and rotations (the row's
       chain is read only while the bank has a row: r.x.any) */
    r.chd = -1;
    r.kdep = 0;
    r.nrow = 0;
    r.exmask = 0u;
    return;
  }
  int kd = gvalid ? m->body_lastdof[gb] : 0;
  if (kd < 0) kd = 0;
  r.chd = tshi(c.chd, kd);
  r.kdep = tshi(c.ddep, kd);
  float Jc[CAP];
#pragma unroll
  for (int e = 0; e < CAP; e++) Jc[e] = 0.f;
  float pos[3], dir[3], mu;
  const float dist = contact_point<XG>(c, s, B, bank, pos, dir, mu);
  if (dist <= m->floor_margin) {
    r.ex = true;
    float off[3] = {pos[0] - cm[0], pos[1] - cm[1], pos[2] - cm[2]}, sa[3];
    cross3(sa, off, dir);
    float vel = 0.f;
#pragma unroll
    for (int e = 0; e < CAP; e++) {
      /* every entry computed (anc_lin past the depth is a valid dummy dof), kept up to the
         row's depth: all loads in flight */
      const int a = anc_lin(r.chd, e);
      /* free-joint translations (ancestors 0..2): cdof = (0, e_k), J = dir_k */
      float v = e < 3 ? dir[e]
                      : sa[0] * L->cdof[a][0] + sa[1] * L->cdof[a][1] + sa[2] * L->cdof[a][2] +
                            dir[0] * L->cdof[a][3] + dir[1] * L->cdof[a][4] + dir[2] * L->cdof[a][5];
      v = e <= r.kdep ? v : 0.f;
      Jc[e] = v;
      vel += v * L->vec[V_QVEL][a];
    }
    float dA = m->body_invweight0[gb][0] * (1.f + mu * mu);
    float Rr;
    row_params(m->floor_solref, m->floor_solimp, dist, dA, vel, cfg->dt, r.D, Rr, r.aref);
  }
  /* compaction list of existing contact rows */
  uint64_t bal = __ballot(r.ex);
  uint32_t tb = (uint32_t)(bal >> ((threadIdx.x & 63) & ~(TEAM - 1)));
  if (TEAM < 64) tb &= 0xffffffffu;
  r.nrow = __popc(tb);
  r.exmask = tb;
  /* every row is stored, zero where there is no contact (and past the row's depth), so the row
     products below need no per-entry masks; the global second bank only while the wave uses it */
  if (bank == 0 || bal != 0ull) st_row(Jrow, Jc);
}

/* the world frame of geom g (body frame then geom frame): centre cw, rotation R (row-major) */
__device__ __forceinline__ void geom_world(const Ctx& c, const BodyK& B, int g, float cw[3], float R[9]) {
  MP m = c.m;
  const int gb = m->geom_body[g];
  float xq[4], xp[3];
#pragma unroll
  for (int k = 0; k < 4; k++) xq[k] = tsh(B.xq[k], gb);
#pragma unroll
  for (int k = 0; k < 3; k++) xp[k] = tsh(B.xp[k], gb);
  const float gq[4] = {m->geom_quat[g][0], m->geom_quat[g][1], m->geom_quat[g][2], m->geom_quat[g][3]};
  const float gp[3] = {m->geom_pos[g][0], m->geom_pos[g][1], m->geom_pos[g][2]};
  float q[4], t[3];
  quat_mul(q, xq, gq);
  quat2mat(R, q);
  quat_rotate(t, xq, gp);
#pragma unroll
  for (int k = 0; k < 3; k++) cw[k] = xp[k] + t[k];
}

/* The sole pair's box-box contacts (ZbModel.npair; the oracle's box_box / pair_collision, whose
   comment states the method): every lane runs the separating-axis test on team-uniform values; for a
   face contact lane i < 24 holds candidate i of the clip in the oracle's order ((a) incident vertices
   0-3, (b) edge crossings 4 + 4 edge + side, (c) rectangle corners 20-23), duplicates and the four-point
   selection are team ballots and reductions. Lane l's contact is q = (l & 15) >> 2: its point, distance
   (1e30 past the count) and the contact frame (n from geom1 to geom2, t1, t2 = n x t1: mju_makeFrame). */
__device__ __forceinline__ float pair_contact(const Ctx& c, const BodyK& B, float pos[3], float n[3], float t1[3],
                                              float t2[3]) {
  MP m = c.m;
  const int q = (c.l & 15) >> 2;
  float c1[3], c2[3], R1[9], R2[9];
  geom_world(c, B, m->pair_geom[0], c1, R1);
  geom_world(c, B, m->pair_geom[1], c2, R2);
  const float a[3] = {m->geom_size[m->pair_geom[0]][0], m->geom_size[m->pair_geom[0]][1], m->geom_size[m->pair_geom[0]][2]};
  const float b[3] = {m->geom_size[m->pair_geom[1]][0], m->geom_size[m->pair_geom[1]][1], m->geom_size[m->pair_geom[1]][2]};
  const float margin = m->pair_margin;
  const float dv[3] = {c2[0] - c1[0], c2[1] - c1[1], c2[2] - c1[2]};
  n[0] = 0.f; n[1] = 0.f; n[2] = 1.f;
  t1[0] = 0.f; t1[1] = 1.f; t1[2] = 0.f;
  t2[0] = -1.f; t2[1] = 0.f; t2[2] = 0.f;
  pos[0] = pos[1] = pos[2] = 0.f;
  /* the bounding spheres first (the soles are usually far apart): wave-uniform skip */
  const float ra = sqrtf(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]), rb = sqrtf(b[0] * b[0] + b[1] * b[1] + b[2] * b[2]);
  const bool near = sqrtf(dot3(dv, dv)) <= ra + rb + margin;
  if (__ballot(near) == 0ull) return 1e30f;
  /* the boxes' axes in the world: columns of the rotations */
  float A[3][3], Bx[3][3];
#pragma unroll
  for (int k = 0; k < 3; k++)
#pragma unroll
    for (int r = 0; r < 3; r++) {
      A[k][r] = R1[3 * r + k];
      Bx[k][r] = R2[3 * r + k];
    }
  float best = -1e30f, L[3] = {0.f, 0.f, 1.f};
  int code = -1;
  bool sep_found = false;
#pragma unroll
  for (int ax = 0; ax < 15; ax++) {
    float l[3];
    bool ok = true;
    if (ax < 3) {
      l[0] = A[ax][0]; l[1] = A[ax][1]; l[2] = A[ax][2];
    } else if (ax < 6) {
      l[0] = Bx[ax - 3][0]; l[1] = Bx[ax - 3][1]; l[2] = Bx[ax - 3][2];
    } else {
      const int i = (ax - 6) / 3, j = (ax - 6) % 3;
      cross3(l, A[i], Bx[j]);
      const float ln = sqrtf(dot3(l, l));
      ok = ln >= 1e-6f;
      const float inv = ok ? 1.f / ln : 0.f;
      l[0] *= inv; l[1] *= inv; l[2] *= inv;
    }
    float rsum = 0.f;
#pragma unroll
    for (int k = 0; k < 3; k++) rsum += a[k] * fabsf(dot3(A[k], l)) + b[k] * fabsf(dot3(Bx[k], l));
    const float dl = dot3(dv, l);
    const float sep = fabsf(dl) - rsum;
    if (ok && sep > margin) sep_found = true;
    const bool better = ok && (ax < 6 ? sep > best : sep > best + 0.05f * fabsf(best));
    if (better) {
      best = sep;
      code = ax;
      const float sg = dl < 0.f ? -1.f : 1.f;
      L[0] = sg * l[0]; L[1] = sg * l[1]; L[2] = sg * l[2];
    }
  }
  const bool contact = near && !sep_found;
  n[0] = L[0]; n[1] = L[1]; n[2] = L[2];
  {
    /* mju_makeFrame(n) */
    float y[3] = {0.f, 1.f, 0.f};
    if (!(fabsf(n[1]) < 0.5f)) { y[1] = 0.f; y[2] = 1.f; }
    const float d = dot3(n, y);
#pragma unroll
    for (int k = 0; k < 3; k++) t1[k] = y[k] - d * n[k];
    const float inv = 1.f / sqrtf(dot3(t1, t1));
#pragma unroll
    for (int k = 0; k < 3; k++) t1[k] *= inv;
    cross3(t2, n, t1);
  }
  float dist = 1e30f;
  if (code >= 6) {
    /* edge-edge: one contact */
    const int i = (code - 6) / 3, j = (code - 6) % 3;
    float p1[3] = {c1[0], c1[1], c1[2]}, p2[3] = {c2[0], c2[1], c2[2]};
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const float s1 = dot3(A[k], L) > 0.f ? a[k] : -a[k], s2 = dot3(Bx[k], L) > 0.f ? -b[k] : b[k];
#pragma unroll
      for (int r = 0; r < 3; r++) {
        p1[r] += k != i ? s1 * A[k][r] : 0.f;
        p2[r] += k != j ? s2 * Bx[k][r] : 0.f;
      }
    }
    const float w[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]};
    const float ab = dot3(A[i], Bx[j]), d1 = dot3(A[i], w), d2 = dot3(Bx[j], w);
    const float den = 1.f - ab * ab;
    float t = den > 1e-12f ? (ab * d2 - d1) / den : 0.f;
    t = fminf(fmaxf(t, -a[i]), a[i]);
    float u = d2 + t * ab;
    u = fminf(fmaxf(u, -b[j]), b[j]);
#pragma unroll
    for (int r = 0; r < 3; r++) pos[r] = 0.5f * (p1[r] + t * A[i][r] + p2[r] + u * Bx[j][r]);
    dist = (contact && q == 0) ? best : 1e30f;
    return dist;
  }
  /* face contact: reference box R (the axis's box), incident box I */
  const bool ref2 = code >= 3;
  const int k = ref2 ? code - 3 : (code < 0 ? 0 : code);
  const int ku = (k + 1) % 3, kv = (k + 2) % 3;
  float nr[3], o[3], u3[3], v3[3], I[3][3], is[3], cI[3];
#pragma unroll
  for (int r = 0; r < 3; r++) {
    nr[r] = ref2 ? -L[r] : L[r];
    o[r] = (ref2 ? c2[r] : c1[r]) + (ref2 ? b[k] : a[k]) * nr[r];
    u3[r] = ref2 ? Bx[ku][r] : A[ku][r];
    v3[r] = ref2 ? Bx[kv][r] : A[kv][r];
    cI[r] = ref2 ? c1[r] : c2[r];
  }
#pragma unroll
  for (int e = 0; e < 3; e++) {
    is[e] = ref2 ? a[e] : b[e];
#pragma unroll
    for (int r = 0; r < 3; r++) I[e][r] = ref2 ? A[e][r] : Bx[e][r];
  }
  const float hu = ref2 ? b[ku] : a[ku], hv = ref2 ? b[kv] : a[kv];
  int jj = 0;
  {
    float bd = -1.f;
#pragma unroll
    for (int e = 0; e < 3; e++) {
      const float v = fabsf(dot3(I[e], nr));
      if (v > bd) { bd = v; jj = e; }
    }
  }
  float Ij[3], Ia[3], Ib[3];
  const int ja = (jj + 1) % 3, jb = (jj + 2) % 3;
#pragma unroll
  for (int r = 0; r < 3; r++) { Ij[r] = I[jj][r]; Ia[r] = I[ja][r]; Ib[r] = I[jb][r]; }
  const float sIj = is[jj], sIa = is[ja], sIb = is[jb];
  const float sgi = dot3(Ij, nr) > 0.f ? -1.f : 1.f;
  float px[4], py[4], pz[4];
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const float va = (e == 0 || e == 3) ? 1.f : -1.f, vb = e < 2 ? 1.f : -1.f;
    float V[3];
#pragma unroll
    for (int r = 0; r < 3; r++) V[r] = cI[r] + sgi * sIj * Ij[r] + va * sIa * Ia[r] + vb * sIb * Ib[r] - o[r];
    px[e] = dot3(V, u3);
    py[e] = dot3(V, v3);
    pz[e] = dot3(V, nr);
  }
  /* this lane's candidate */
  const int i = c.l;
  float cx = 0.f, cy = 0.f, cz = 0.f;
  bool valid = false;
  if (i < 4) {
    const float x0 = i == 0 ? px[0] : i == 1 ? px[1] : i == 2 ? px[2] : px[3];
    const float y0 = i == 0 ? py[0] : i == 1 ? py[1] : i == 2 ? py[2] : py[3];
    const float z0 = i == 0 ? pz[0] : i == 1 ? pz[1] : i == 2 ? pz[2] : pz[3];
    valid = fabsf(x0) <= hu && fabsf(y0) <= hv;
    cx = x0; cy = y0; cz = z0;
  } else if (i < 20) {
    const int e = (i - 4) >> 2, sd = (i - 4) & 3, e1 = (e + 1) & 3;
    const float xa = e == 0 ? px[0] : e == 1 ? px[1] : e == 2 ? px[2] : px[3];
    const float ya = e == 0 ? py[0] : e == 1 ? py[1] : e == 2 ? py[2] : py[3];
    const float za = e == 0 ? pz[0] : e == 1 ? pz[1] : e == 2 ? pz[2] : pz[3];
    const float xb = e1 == 0 ? px[0] : e1 == 1 ? px[1] : e1 == 2 ? px[2] : px[3];
    const float yb = e1 == 0 ? py[0] : e1 == 1 ? py[1] : e1 == 2 ? py[2] : py[3];
    const float zb = e1 == 0 ? pz[0] : e1 == 1 ? pz[1] : e1 == 2 ? pz[2] : pz[3];
    const bool isx = sd < 2;
    const float X = (sd & 1) ? (isx ? hu : hv) : (isx ? -hu : -hv);
    const float e0 = isx ? xa : ya, ee1 = isx ? xb : yb;
    if ((e0 - X) * (ee1 - X) < 0.f) {
      const float t = (X - e0) / (ee1 - e0);
      const float oth = isx ? ya + t * (yb - ya) : xa + t * (xb - xa);
      valid = fabsf(oth) <= (isx ? hv : hu);
      cx = isx ? X : oth;
      cy = isx ? oth : X;
      cz = za + t * (zb - za);
    }
  } else if (i < 24) {
    const int e = i - 20;
    const float X = (e == 1 || e == 2) ? hu : -hu, Y = e >= 2 ? hv : -hv;
    int pos_ = 0, neg_ = 0;
#pragma unroll
    for (int f = 0; f < 4; f++) {
      const int f1 = (f + 1) & 3;
      const float cr = (px[f1] - px[f]) * (Y - py[f]) - (py[f1] - py[f]) * (X - px[f]);
      pos_ += cr >= 0.f;
      neg_ += cr <= 0.f;
    }
    valid = pos_ == 4 || neg_ == 4;
    float ni[3];
#pragma unroll
    for (int r = 0; r < 3; r++) ni[r] = sgi * Ij[r];
    const float nx = dot3(ni, u3), ny = dot3(ni, v3), nz = dot3(ni, nr);
    cx = X;
    cy = Y;
    cz = pz[0] - (nx * (X - px[0]) + ny * (Y - py[0])) / nz;
  }
  const bool inm = contact && valid && cz <= margin;
  /* duplicates: within 1e-6 in x and y of an earlier candidate within the margin */
  bool dup = false;
  for (int j = 0; j < 24; j++) {
    const float xj = tsh(cx, j), yj = tsh(cy, j);
    const int mj = tshi(inm ? 1 : 0, j);
    dup = dup || (j < i && mj && fabsf(cx - xj) <= 1e-6f && fabsf(cy - yj) <= 1e-6f);
  }
  const bool keep = inm && !dup;
  const uint32_t km = team_ballot(keep);
  const int nk = __popc(km);
  int sel[4] = {0, 0, 0, 0}, ns;
  if (nk <= 4) {
    uint32_t mm = km;
#pragma unroll
    for (int t = 0; t < 4; t++) {
      sel[t] = mm ? __ffs(mm) - 1 : 0;
      mm &= mm - 1u;
    }
    ns = nk;
  } else {
    /* MJX's manifold points from the deepest: first lane at each extreme (team-uniform indices) */
    auto first_of = [&](float v, bool on) {
      const float mx = tmaxf(on ? v : -1e30f);
      return __ffs(team_ballot(on && v == mx)) - 1;
    };
    const int ia = first_of(-cz, keep);
    const float xa = tsh(cx, ia), ya = tsh(cy, ia);
    const int ib = first_of((cx - xa) * (cx - xa) + (cy - ya) * (cy - ya), keep);
    const float xb = tsh(cx, ib), yb = tsh(cy, ib);
    const int ic = first_of(fabsf((xb - xa) * (cy - ya) - (yb - ya) * (cx - xa)), keep);
    const float xc = tsh(cx, ic), yc = tsh(cy, ic);
    const float v1 = fabsf((xb - xc) * (yb - cy) - (yb - yc) * (xb - cx));
    const float v2 = fabsf((xa - xc) * (ya - cy) - (ya - yc) * (xa - cx));
    const float m1 = tmaxf(keep ? v1 : -1e30f), m2 = tmaxf(keep ? v2 : -1e30f);
    const int id = m1 >= m2 ? __ffs(team_ballot(keep && v1 == m1)) - 1 : __ffs(team_ballot(keep && v2 == m2)) - 1;
    const int cand[4] = {ia, ib, ic, id};
    ns = 0;
#pragma unroll
    for (int t = 0; t < 4; t++) {
      bool d = false;
#pragma unroll
      for (int e = 0; e < t; e++) d = d || cand[e] == cand[t];
      if (!d) {
        sel[ns] = cand[t];
        ns++;
      }
    }
  }
  const int mine = q == 0 ? sel[0] : q == 1 ? sel[1] : q == 2 ? sel[2] : sel[3];
  const float x = tsh(cx, mine), y = tsh(cy, mine), z = tsh(cz, mine);
#pragma unroll
  for (int r = 0; r < 3; r++) pos[r] = o[r] + x * u3[r] + y * v3[r] + 0.5f * z * nr[r];
  return (contact && q < ns) ? z : 1e30f;
}

/* The sole pair's contact rows (second bank of the XG 3 kernels): lane l = 16 h + 4 q + edge holds the
   pyramid row (n +- mu t1, n +- mu t2) of contact q, half h: h = 0 the row's entries on geom2's limb
   (+J of its body), h = 1 those on geom1's limb (-J of its body). The root dofs' columns of
   J(body2) - J(body1) cancel exactly (mj_jacDifPair), so each half is a one-chain row of the limb dofs;
   both halves carry the row's scalars (aref, D, jar, Jv, f), the cost counts them once (h = 0). */
template <typename JP>
__device__ __forceinline__ void pair_rows(const Ctx& c, const EnvS& s, const BodyK& B, const float cm[3], XRow& r,
                                          JP Jrow) {
  MP m = c.m;
  CP cfg = c.cfg;
  EnvL* L = c.L;
  const int h = c.l >> 4, edge = c.l & 3;
  const int g = m->pair_geom[1 - h];
  const int gb = m->geom_body[g];
  int kd = m->body_lastdof[gb];
  if (kd < 0) kd = 0;
  r.chd = tshi(c.chd, kd);
  r.kdep = tshi(c.ddep, kd);
  r.ex = false;
  r.act = 0;
  r.f = 0.f;
  r.jar = 0.f;
  r.Jv = 0.f;
  r.D = 0.f;
  r.aref = 0.f;
  float pos[3], n[3], t1[3], t2[3];
  const float dist = pair_contact(c, B, pos, n, t1, t2);
  const float mu = m->pair_friction[0];
  const float sg = (edge & 1) ? -mu : mu;
  float dir[3];
#pragma unroll
  for (int k = 0; k < 3; k++) dir[k] = n[k] + sg * (edge < 2 ? t1[k] : t2[k]);
  const float hs = h ? -1.f : 1.f;
  float off[3] = {pos[0] - cm[0], pos[1] - cm[1], pos[2] - cm[2]}, sa[3];
  cross3(sa, off, dir);
  float Jc[CAP];
  float vel = 0.f;
#pragma unroll
  for (int e = 0; e < CAP; e++) {
    const int a = anc_lin(r.chd, e);
    float v = sa[0] * L->cdof[a][0] + sa[1] * L->cdof[a][1] + sa[2] * L->cdof[a][2] + dir[0] * L->cdof[a][3] +
              dir[1] * L->cdof[a][4] + dir[2] * L->cdof[a][5];
    v = (e >= NROOT && e <= r.kdep) ? hs * v : 0.f;
    Jc[e] = v;
    vel += v * L->vec[V_QVEL][a];
  }
  vel += xor16f(vel); /* the row's velocity: both halves */
  const bool ex = dist <= m->pair_margin;
  if (ex) {
    r.ex = true;
    const int b1 = m->geom_body[m->pair_geom[0]], b2 = m->geom_body[m->pair_geom[1]];
    const float dA = (m->body_invweight0[b1][0] + m->body_invweight0[b2][0]) * (1.f + mu * mu);
    float Rr;
    row_params(m->pair_solref, m->pair_solimp, dist, dA, vel, cfg->dt, r.D, Rr, r.aref);
  }
  const uint64_t bal = __ballot(r.ex);
  const uint32_t tb = (uint32_t)(bal >> ((threadIdx.x & 63) & ~(TEAM - 1)));
  r.nrow = __popc(tb);
  r.exmask = tb;
  if (bal != 0ull) st_row(Jrow, Jc);
}

/* collision + contact rows (lane r; XG: both banks) + dof rows (lane j) */
/* The second contact-row bank's geoms for this substep (XG 1 / 2; model v9: up to ZB_MAX_GEOM floor
   colliders). Lane l tests geom 2 + l by a bound: no point of a geom lies lower than its body origin
   minus |geom_pos| minus the geom's bounding radius (box half-diagonal; capsule radius + half-length;
   cylinder sqrt(r^2 + h^2); ellipsoid largest semi-axis; sphere radius; mesh the largest vertex
   distance, geom_size[0]); the first two within reach of the margin (+1 mm against rounding), in
   geom order, take the bank's halves (EnvS.xsel, -1: none). Any other geom is then off the floor, so
   the contacts are MuJoCo's, except when more than two such geoms are within reach in one substep:
   their contacts beyond the first two are not simulated, and the state's flag word records it
   (EnvS.nanflag, ZB_S_NAN: bit 1 sticky, bit 2 for the current control step, so a caller can tell a
   step that overflowed, the step that ends an episode included). */
template <int XG>
__device__ __forceinline__ void select_bank2(const Ctx& c, const BodyK& B) {
  MP m = c.m;
  const int ng = m->ngeom;
  const int g = 2 + c.l;
  const bool valid = g < ng;
  const int gg = valid ? g : 0;
  const float zb = tsh(B.xp[2], m->geom_body[gg]);
  const float gx = m->geom_pos[gg][0], gy = m->geom_pos[gg][1], gz = m->geom_pos[gg][2];
  const float s0 = m->geom_size[gg][0], s1 = m->geom_size[gg][1], s2 = m->geom_size[gg][2];
  const int ty = m->geom_type[gg];
  const float rb = ty == ZB_GEOM_BOX ? sqrtf(s0 * s0 + s1 * s1 + s2 * s2)
                   : ty == ZB_GEOM_CAPSULE ? s0 + s1
                   : ty == ZB_GEOM_CYLINDER ? sqrtf(s0 * s0 + s1 * s1)
                   : ty == ZB_GEOM_ELLIPSOID ? fmaxf(s0, fmaxf(s1, s2)) : s0;
  const bool reach = valid && zb - sqrtf(gx * gx + gy * gy + gz * gz) - rb <= m->floor_margin + 1e-3f;
  uint32_t mk = team_ballot(reach);
  int sel0, sel1;
  if (ng <= 2 + NGEOM) {
    /* at most two other geoms: each keeps its own half (geom 2 lanes 0-15, geom 3 lanes 16-31), the
       row layout of the static bank */
    sel0 = (mk & 1u) ? 2 : -1;
    sel1 = (mk & 2u) ? 3 : -1;
    mk = 0u;
  } else {
    sel0 = mk ? 1 + __ffs(mk) : -1; /* 2 + (ffs - 1) */
    mk &= mk - 1u;
    sel1 = mk ? 1 + __ffs(mk) : -1;
    mk &= mk - 1u;
  }
  if constexpr (YFLOOR<XG>) {
    /* XG 5: the third and fourth geoms within reach take the third bank's halves */
    const int sel2 = mk ? 1 + __ffs(mk) : -1;
    mk &= mk - 1u;
    const int sel3 = mk ? 1 + __ffs(mk) : -1;
    mk &= mk - 1u;
    c.L->ysel[0] = sel2;
    c.L->ysel[1] = sel3;
  }
  /* team-uniform values, written by every lane of the team */
  c.L->s.xsel[0] = sel0;
  c.L->s.xsel[1] = sel1;
  if (mk) c.L->s.nanflag |= 2u | 4u; /* sticky, and this control step's (cleared at its start) */
  tsync();
}

template <int XG>
__device__ __forceinline__ void make_constraints(const Ctx& c, const EnvS& s, const LaneS& ls, const BodyK& B, const float cm[3],
                                 Rows& r) {
  MP m = c.m;
  CP cfg = c.cfg;
  const int l = c.l;
  contact_rows<XG>(c, s, B, cm, 0, r, &c.L->u.J[l][0]);
  if constexpr (XG) {
    if constexpr (XPAIR<XG>) {
      pair_rows(c, s, B, cm, r.x, xrows(c.L) + l * CAP);
    } else {
      select_bank2<XG>(c, B);
      contact_rows<XG>(c, s, B, cm, 1, r.x, xrows(c.L) + l * CAP);
      /* the bank's rows on dof l's chain: dof l is an ancestor of (or is) the geom's last dof kd, a
         root dof or one of kd's own limb chain at or above it */
      uint32_t rm = rm_rows(c.rmb >> 2); /* at most two other geoms: zb_create's static mask (geoms 2, 3) */
      if (m->ngeom > 2 + NGEOM) {
        rm = 0u;
#pragma unroll
        for (int h = 0; h < 2; h++) {
          const int sg = c.L->s.xsel[h];
          const int kd = sg >= 0 ? m->body_lastdof[m->geom_body[sg]] : -1;
          const int kdc = kd >= 0 ? kd : 0;
          const int hkd = tshi(c.chd, kdc);
          const bool on = l < NV && kd >= 0 && l <= kd && (l < NROOT || c.chd == hkd);
          rm |= on ? (0xFFFFu << (16 * h)) : 0u;
        }
      }
      r.x.rowmask = rm;
    }
    /* the second bank's work is skipped, bit for bit, while no row of it exists in the wave (the
       usual case: shins and hands off the floor) */
    r.x.any = __ballot(r.x.ex) != 0ull;
    bool yany = false;
    if constexpr (YPAIR<XG>) {
      pair_rows(c, s, B, cm, r.y, yrows(c.L) + l * CAP);
      r.y.any = yany = __ballot(r.y.ex) != 0ull;
    }
    if constexpr (YFLOOR<XG>) {
      /* XG 5: the third and fourth geoms within reach in the third bank, row masks as the second's */
      contact_rows<XG>(c, s, B, cm, 2, r.y, yrows(c.L) + l * CAP);
      uint32_t rm = 0u;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int sg = c.L->ysel[h];
        const int kd = sg >= 0 ? m->body_lastdof[m->geom_body[sg]] : -1;
        const int kdc = kd >= 0 ? kd : 0;
        const int hkd = tshi(c.chd, kdc);
        const bool on = l < NV && kd >= 0 && l <= kd && (l < NROOT || c.chd == hkd);
        rm |= on ? (0xFFFFu << (16 * h)) : 0u;
      }
      r.y.rowmask = rm;
      r.y.any = yany = __ballot(r.y.ex) != 0ull;
    }
    if (r.x.any || yany) {
      /* the rows just stored are read by other lanes from here on */
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
  }
  /* ---- dof rows (lane j) ---- */
  r.hf = r.hl = false;
  r.actf = r.actl = 0;
  r.ff = r.flim = 0.f;
  r.jf = r.jl = 0.f;
  r.Df = r.Dl = 0.f;
  r.af = r.al = 0.f;
  r.sl = 1.f;
  r.Rf = 0.f;
  r.fl = 0.f;
  if (l < NV) {
    /* frictionloss and both joint-limit rows evaluated for every dof lane,
       kept where they exist (no per-lane branches) */
    const float v = ls.v;
    const float dA = m->dof_invweight0[l];
    const float floss = c.L->par[P_FLOSS][c.l];
    const bool lim = m->dof_limited[l] != 0;
    const float dlo = ls.q - m->dof_range[l][0], dhi = m->dof_range[l][1] - ls.q;
    /* frictionloss row: pos = 0, so the impedance is solimp's dmin (dmax when the
       width is zero) and aref = -b v (mj_makeImpedance at distance 0) */
    float D0, R0, a0;
    {
      const auto si = m->dof_solimp;
      const float tc = fmaxf(m->dof_solref[0], 2.f * cfg->dt), dmax = si[1];
      const float imp = fminf(fmaxf(si[2] <= MINVAL ? dmax : si[0], MINIMP), MAXIMP);
      R0 = fmaxf((1.f - imp) / imp * dA, MINVAL);
      D0 = 1.f / R0;
      a0 = -(2.f / (dmax * tc)) * v;
    }
    r.hf = floss > 0.f;
    r.fl = r.hf ? floss : 0.f;
    r.Df = r.hf ? D0 : 0.f;
    r.Rf = r.hf ? R0 : 0.f;
    r.af = r.hf ? a0 : 0.f;
    const bool hlo = lim && dlo < 0.f, hhi = lim && dhi < 0.f;
    r.hl = hlo || hhi;
    r.sl = hhi ? -1.f : 1.f;
    /* joint-limit rows exist only past a limit (at most one side per dof): one row
       evaluation, and none at all when no dof of the wave is past a limit */
    if (__ballot(r.hl) != 0ull) {
      float D1, R1, a1;
      row_params(m->dof_solref, m->dof_solimp, hlo ? dlo : dhi, dA, r.sl * v, cfg->dt, D1, R1, a1);
      r.Dl = r.hl ? D1 : 0.f;
      r.al = r.hl ? a1 : 0.f;
    }
  }
  /* taken with every lane active, so the flag is one wave-uniform (scalar) value */
  r.anyl = __ballot(r.hl) != 0ull;
  tsync();
}

/* Wave priority of the constraint solvers (s_setprio). The two waves of a SIMD run independent envs
   and their VALU issue is arbitrated by priority, then age. The solver is a chain of short dependent
   steps (line-search evaluations, exchanges, pivots), the smooth phase around it is denser in
   independent instructions: a wave inside its solver takes precedence over a partner outside it,
   whose work absorbs the delay (C2: +3 % on one stream, +0.6 % with two env groups; DESIGN.md §4d
   round 3). Results are unchanged. */
#ifndef ZB_SOLVER_PRIO
#define ZB_SOLVER_PRIO 1
#endif

/* ------------------------------ Newton solver ------------------------------ */
/* row cost / force / activity (mj_constraintUpdate), branch-free selects */
__device__ __forceinline__ float eval_fric(float jar, float D, float R, float fl, float& force, int& act) {
  const float Rf = R * fl;
  const bool lo = jar <= -Rf, hi = jar >= Rf;
  force = lo ? fl : (hi ? -fl : -D * jar);
  act = (lo || hi) ? 0 : 1;
  return lo ? -fl * (0.5f * Rf + jar) : (hi ? fl * (jar - 0.5f * Rf) : 0.5f * D * jar * jar);
}
__device__ __forceinline__ float eval_one(float jar, float D, float& force, int& act) {
  const bool on = jar < 0.f;
  force = on ? -D * jar : 0.f;
  act = on ? 1 : 0;
  return on ? 0.5f * D * jar * jar : 0.f;
}

/* row costs at given jar values (no state change); jx: the second bank's contact row (XG) */
template <int XG, bool XA = true>
__device__ __forceinline__ float rows_cost(const Ctx& c, const Rows& r, float jc, float jf_, float jl_, float jx,
                                           float jy = 0.f) {
  float f;
  int a;
  const float k0 = eval_one(jc, r.D, f, a);
  const float k1 = eval_fric(jf_, r.Df, r.Rf, r.fl, f, a);
  float cost = 0.f;
  cost += r.ex ? k0 : 0.f;
  cost += r.hf ? k1 : 0.f;
  if (r.anyl) {
    const float k2 = eval_one(jl_, r.Dl, f, a);
    cost += r.hl ? k2 : 0.f;
  }
  if constexpr (XG && XA) {
    const float k3 = eval_one(jx, r.x.D, f, a);
    /* the sole pair's row is held by two lanes (its halves): counted once */
    cost += (r.x.ex && (!XPAIR<XG> || c.l < 16)) ? k3 : 0.f;
  }
  if constexpr (YBANK<XG> && XA) {
    const float k4 = eval_one(jy, r.y.D, f, a);
    cost += (r.y.ex && (YFLOOR<XG> || c.l < 16)) ? k4 : 0.f; /* the pair's halves: once */
  }
  return cost;
}

/* sum_r J_r[e] f_r over the 16 contact rows of a geom (one 16-lane DPP row; they share the geom's
   dof chain): a transposing butterfly over the rows (pairings: row mirror, half-row mirror, quad
   xor 2, quad xor 1). At each stage a lane keeps the half of its column sums on its side and adds
   its partner's copy of them, so lane 16 f + e ends with the geom-f sum of column e (45 instead of
   108 VALU instructions). */
__device__ __forceinline__ float colsum16_pre(const float jr[CAP], float fr) {
  float q[16];
  {
#pragma unroll
    for (int e = 0; e < CAP; e++) q[e] = jr[e] * fr; /* J rows are zero where no contact */
#pragma unroll
    for (int e = CAP; e < 16; e++) q[e] = 0.f;
  }
  const int li = threadIdx.x & 15;
  float u8[8], u4[4], u2[2];
  {
    const bool s1 = li >= 8;
#pragma unroll
    for (int k = 0; k < 8; k++) u8[k] = (s1 ? q[8 + k] : q[k]) + dppf<0x140>(s1 ? q[k] : q[8 + k]);
    const bool s2 = (li & 4) != 0;
#pragma unroll
    for (int k = 0; k < 4; k++) u4[k] = (s2 ? u8[4 + k] : u8[k]) + dppf<0x141>(s2 ? u8[k] : u8[4 + k]);
    const bool s3 = (li & 2) != 0;
#pragma unroll
    for (int k = 0; k < 2; k++) u2[k] = (s3 ? u4[2 + k] : u4[k]) + dppf<0x4E>(s3 ? u4[k] : u4[2 + k]);
  }
  const bool s4 = (li & 1) != 0;
  return (s4 ? u2[1] : u2[0]) + dppf<0xB1>(s4 ? u2[0] : u2[1]);
}
template <typename JP>
__device__ __forceinline__ float colsum16(JP Jrow, float fr) {
  float jr[CAP];
  ld_row(Jrow, jr);
  return colsum16_pre(jr, fr);
}

/* forces/activity at current jar, qfrc_constraint, grad, total cost */
/* returns this lane's cost share; the caller reduces it over the team (alone, or together with
   the Newton loop's other per-iteration sums in one tsum_n) */
/* HS: the rows' force and active D are also stored in LDS for the Newton Hessian (hessian_factor,
   jdj_mfma); CG builds no Hessian and skips the stores */
template <int XG, bool XA = true, bool HS = true>
__device__ __forceinline__ float update_constraint_lane(const Ctx& c, Rows& r, const float jr[CAP], float qacc,
                                                       float qs, float fs, float Ma, float& grad) {
  const int ddep = vopq(c.ddep);
  EnvL* L = c.L;
  float cost = 0.f;
  if (c.l < NV) cost += 0.5f * (Ma - fs) * (qacc - qs);
  {
    /* all four row kinds evaluated, results kept only for rows that exist */
    float f0, f1;
    int a0, a1;
    const float k0 = eval_one(r.jar, r.D, f0, a0);
    const float k1 = eval_fric(r.jf, r.Df, r.Rf, r.fl, f1, a1);
    cost += r.ex ? k0 : 0.f;
    cost += r.hf ? k1 : 0.f;
    r.f = r.ex ? f0 : r.f;
    r.act = r.ex ? a0 : r.act;
    r.ff = r.hf ? f1 : r.ff;
    r.actf = r.hf ? a1 : r.actf;
    if (r.anyl) {
      float f2;
      int a2;
      const float k2 = eval_one(r.jl, r.Dl, f2, a2);
      cost += r.hl ? k2 : 0.f;
      r.flim = r.hl ? f2 : r.flim;
      r.actl = r.hl ? a2 : r.actl;
    }
  }
  if constexpr (HS) {
    if (r.ex) L->rowF[c.l] = r.f;
    L->rowDA[c.l] = (r.ex && r.act) ? r.D : 0.f; /* every row: read by jdj_mfma */
  }
  float sx0 = 0.f, sx1 = 0.f;
  if (XG && XA && r.x.any) {
    float f3;
    int a3;
    const float k3 = eval_one(r.x.jar, r.x.D, f3, a3);
    cost += (r.x.ex && (!XPAIR<XG> || c.l < 16)) ? k3 : 0.f; /* the pair's halves: once */
    r.x.f = r.x.ex ? f3 : r.x.f;
    r.x.act = r.x.ex ? a3 : r.x.act;
    const float cx = colsum16((const gfloat_t*)xrows(c.L) + c.l * CAP, r.x.ex ? r.x.f : 0.f);
    sx0 = tsh(cx, ddep);
    sx1 = tsh(cx, 16 + ddep);
  }
  float sy0 = 0.f, sy1 = 0.f;
  if constexpr (YBANK<XG> && XA) {
    if (r.y.any) {
      float f4;
      int a4;
      const float k4 = eval_one(r.y.jar, r.y.D, f4, a4);
      cost += (r.y.ex && (YFLOOR<XG> || c.l < 16)) ? k4 : 0.f; /* the pair's halves: once */
      r.y.f = r.y.ex ? f4 : r.y.f;
      r.y.act = r.y.ex ? a4 : r.y.act;
      const float cy = colsum16((const gfloat_t*)yrows(c.L) + c.l * CAP, r.y.ex ? r.y.f : 0.f);
      sy0 = tsh(cy, ddep);
      sy1 = tsh(cy, 16 + ddep);
    }
  }
  /* J'f per dof: a dof adds the column sum at its depth of every geom whose chain holds it */
  const float colsum = colsum16_pre(jr, r.ex ? r.f : 0.f);
  const float so = tsh(colsum, ddep), sx = tsh(colsum, 16 + ddep);
  tsync();
  float qc = 0.f;
  if (c.l < NV) {
    const bool f0 = (c.rmb & 1u) != 0u, f1 = (c.rmb & 2u) != 0u;
    qc = (f0 ? so : 0.f) + (f1 ? sx : 0.f);
    if constexpr (XG && XA) {
      const uint32_t rm2 = XPAIR<XG> ? rm_rows(c.rmb >> 2) : r.x.rowmask;
      const bool f2 = (rm2 & 0xFFFFu) != 0u, f3 = (rm2 >> 16) != 0u;
      qc += (f2 ? sx0 : 0.f) + (f3 ? sx1 : 0.f);
    }
    if constexpr (YBANK<XG> && XA) {
      /* the pair's static row masks (XG 4), the third floor bank's of this substep (XG 5) */
      const bool f4 = YFLOOR<XG> ? (r.y.rowmask & 0xFFFFu) != 0u : (c.rmb & 16u) != 0u;
      const bool f5 = YFLOOR<XG> ? (r.y.rowmask >> 16) != 0u : (c.rmb & 32u) != 0u;
      qc += (f4 ? sy0 : 0.f) + (f5 ? sy1 : 0.f);
    }
    if (r.hf) qc += r.ff;
    if (r.anyl && r.hl) qc += r.sl * r.flim;
  }
  grad = Ma - fs - qc;
  return cost;
}
template <int XG, bool XA = true, bool HS = true>
__device__ __forceinline__ float update_constraint(const Ctx& c, Rows& r, const float jr[CAP], float qacc, float qs,
                                                  float fs, float Ma, float& grad) {
  return tsum(update_constraint_lane<XG, XA, HS>(c, r, jr, qacc, qs, fs, Ma, grad));
}

/* G_f = sum_{r in foot f} D_r J_r J_r' (depth-indexed 12x12) for both feet of
 * both envs of the wave on the matrix cores: per (env, foot) four
 * v_mfma_f32_16x16x4_f32 over the foot's 16 contact rows (K = 4 rows each;
 * lane l supplies row 4*chunk + l/16, entry l%16). Staged in the env's L[][]
 * as [foot][12][12]; L[][] is free until factor_ldl writes it. D is rowDA
 * (0 for absent / inactive rows). Wave-uniform: call with every lane active.
 * BANK 1 / 2: the same for the second / third bank's geoms (xrows / yrows J, rowDA holding that bank's
 * D), staged in the Hessian rows Hs[][], free until hessian_factor stores the assembled rows. */
template <int BANK>
__device__ __forceinline__ void jdj_mfma() {
  const int l = threadIdx.x & 63;
  const int e = l & 15, k = l >> 4;
  const int ec = e < CAP ? e : CAP - 1;
  v4f acc[NTEAM][NGEOM];
#pragma unroll
  for (int t = 0; t < NTEAM; t++)
#pragma unroll
    for (int f = 0; f < NGEOM; f++) acc[t][f] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ch = 0; ch < 4; ch++)
#pragma unroll
    for (int t = 0; t < NTEAM; t++)
#pragma unroll
      for (int f = 0; f < NGEOM; f++) {
        const int r = 16 * f + 4 * ch + k;
        /* no masks: rowDA is zero for absent / inactive rows, and output rows or
           columns e >= CAP (lanes reading entry CAP-1) are never stored */
        const float jv = BANK == 2   ? yrows(&g_lds[t])[r * CAP + ec]
                         : BANK == 1 ? xrows(&g_lds[t])[r * CAP + ec]
                                     : g_lds[t].u.J[r][ec];
        const float dv = g_lds[t].rowDA[r]; /* BANK >= 1: that bank's, written by hessian_factor */
        acc[t][f] = __builtin_amdgcn_mfma_f32_16x16x4f32(dv * jv, jv, acc[t][f], 0, 0, 0);
      }
  /* lane l holds G[4*(l/16) + v][l%16], v = 0..3: G is symmetric (to rounding), so the
     four go to row l%16, columns 4*(l/16) + v, as one 16-byte store */
  static_assert(CAP % 4 == 0, "16-byte G rows");
  if (k < CAP / 4 && e < CAP)
#pragma unroll
    for (int t = 0; t < NTEAM; t++)
#pragma unroll
      for (int f = 0; f < NGEOM; f++)
        *reinterpret_cast<v4f*>((BANK ? &g_lds[t].Hs[0][0] : &g_lds[t].L[0][0]) + f * CAP * CAP + e * CAP + 4 * k) =
            acc[t][f];
}

/* H[e] += D_r J_r[e] J_r' over the rows of bitmask tb (pairs of rows per pass; da: the rows' D) */
template <typename JP>
__device__ __forceinline__ void add_rows(uint32_t tb, JP J, const float* da, int ddep, float H[CAP], float& Hd) {
  while (tb) {
    const int k0 = __ffs(tb) - 1;
    tb &= tb - 1u;
    const bool h1 = tb != 0u;
    const int k1 = h1 ? __ffs(tb) - 1 : k0;
    tb &= tb - 1u;
    float j0[CAP], j1[CAP];
    ld_row(J + k0 * CAP, j0);
    ld_row(J + k1 * CAP, j1);
    const float jd0 = J[k0 * CAP + ddep], jd1 = J[k1 * CAP + ddep];
    const float jj0 = da[k0] * jd0;
    const float jj1 = (da[k1] * jd1) * (h1 ? 1.f : 0.f); /* a weight, not a select (loads) */
    Hd += jj0 * jd0;
    Hd += jj1 * jd1;
#pragma unroll
    for (int e = 0; e < CAP; e++) {
      H[e] += jj0 * j0[e]; /* entries at or past the depth are never read */
      H[e] += jj1 * j1[e];
    }
  }
}

/* H = M + J' D_active J (depth-indexed rows), then factor -> 1/D_j.
 * full: from M and every active contact row. Otherwise the stored unfactored
 * H of the previous build is updated with the rows whose activity changed
 * (+-D_r J_r J_r') -- MuJoCo's Newton also only re-assembles on a change of
 * the active set, and the change is usually a handful of rows. XG: both banks. */
template <int XG, bool XA = true>
__device__ __forceinline__ float hessian_factor(const Ctx& c, const Rows& r, bool full, int pa, int pf, int plo,
                                                int pa2, int pa3) {
  const int ddep = vopq(c.ddep);
  EnvL* L = c.L;
  float H[CAP], Hd;
  uint32_t tb, tb2 = 0u, ch2 = 0u, tb3 = 0u, ch3 = 0u;
  float dl2 = 0.f, dl3 = 0.f;
  if (full) {
    Hd = load_mrow(c, H);
    tb = 0u;
    jdj_mfma<0>();
    if (XFLOOR<XG> && XA && r.x.any) {
      /* the second bank's D (rowDA is free once the first bank's J'DJ has read it) */
      tsync();
      L->rowDA[c.l] = (r.x.ex && r.x.act) ? r.x.D : 0.f;
      tsync();
      jdj_mfma<1>();
    }
    tsync();
    if (c.l < NV) {
      /* the G row of each foot whose chain holds the dof, else the zero row 31 of L
         (G occupies rows 0..23): no per-entry selects */
      const float* G = &L->L[0][0] + ddep * CAP;
      const bool f0 = (c.rmb & 1u) != 0u, f1 = (c.rmb & 2u) != 0u;
      static_assert(NGEOM * CAP * CAP <= 31 * CAP, "G staged below the zero row 31");
      const float* G0 = f0 ? G : &L->L[31][0];
      const float* G1 = f1 ? G + CAP * CAP : &L->L[31][0];
      float g0[CAP], g1[CAP];
      ld_row(G0, g0);
      ld_row(G1, g1);
      const float d0 = G0[f0 ? ddep : 0], d1 = G1[f1 ? ddep : 0];
#pragma unroll
      /* entries at or past the lane's depth are never read by the factorization,
         so they need no mask */
      for (int e = 0; e < CAP; e++) H[e] += g0[e] + g1[e];
      Hd += d0 + d1;
      if (XFLOOR<XG> && XA && r.x.any) {
        const float* GX = &L->Hs[0][0] + ddep * CAP;
        const bool f2 = (r.x.rowmask & 0xFFFFu) != 0u, f3 = (r.x.rowmask >> 16) != 0u;
        const float* G2 = f2 ? GX : &L->L[31][0];
        const float* G3 = f3 ? GX + CAP * CAP : &L->L[31][0];
        ld_row(G2, g0);
        ld_row(G3, g1);
        const float d2 = G2[f2 ? ddep : 0], d3 = G3[f3 ? ddep : 0];
#pragma unroll
        for (int e = 0; e < CAP; e++) H[e] += g0[e] + g1[e];
        Hd += d2 + d3;
      }
    }
    if (YFLOOR<XG> && XA && r.y.any) {
      /* XG 5: the third bank's J'DJ through the same staging rows, once the second's are read */
      tsync();
      L->rowDA[c.l] = (r.y.ex && r.y.act) ? r.y.D : 0.f;
      tsync();
      jdj_mfma<2>();
      tsync();
      if (c.l < NV) {
        const float* GY = &L->Hs[0][0] + ddep * CAP;
        const bool f4 = (r.y.rowmask & 0xFFFFu) != 0u, f5 = (r.y.rowmask >> 16) != 0u;
        const float* G4 = f4 ? GY : &L->L[31][0];
        const float* G5 = f5 ? GY + CAP * CAP : &L->L[31][0];
        float g4[CAP], g5[CAP];
        ld_row(G4, g4);
        ld_row(G5, g5);
        const float d4 = G4[f4 ? ddep : 0], d5 = G5[f5 ? ddep : 0];
#pragma unroll
        for (int e = 0; e < CAP; e++) H[e] += g4[e] + g5[e];
        Hd += d4 + d5;
      }
    }
  } else {
    ld_row(&L->Hs[c.l][0], H);
    Hd = L->Hsd[c.l];
    const float dl = r.ex ? ((r.act ? r.D : 0.f) - (pa ? r.D : 0.f)) : 0.f;
    L->rowF[c.l] = dl; /* rowF is free until the next update_constraint */
    tb = team_ballot(dl != 0.f) & rm_rows(c.rmb);
    if (XFLOOR<XG> && XA && r.x.any) {
      dl2 = r.x.ex ? ((r.x.act ? r.x.D : 0.f) - (pa2 ? r.x.D : 0.f)) : 0.f;
      ch2 = team_ballot(dl2 != 0.f); /* team-uniform: some row of the bank changed */
      tb2 = ch2 & r.x.rowmask;       /* per dof lane: the changed rows on its chain */
    }
    if (YFLOOR<XG> && XA && r.y.any) {
      dl3 = r.y.ex ? ((r.y.act ? r.y.D : 0.f) - (pa3 ? r.y.D : 0.f)) : 0.f;
      ch3 = team_ballot(dl3 != 0.f);
      tb3 = ch3 & r.y.rowmask;
    }
    tsync();
  }
  if (c.l < NV) {
    add_rows(tb, (const float*)&L->u.J[0][0], full ? L->rowDA : L->rowF, ddep, H, Hd);
    float dd = 0.f;
    if (full) {
      if (r.hf && r.actf) dd += r.Df;
      if (r.anyl && r.hl && r.actl) dd += r.Dl;
    } else {
      if (r.hf) dd += (float)(r.actf - pf) * r.Df;
      if (r.anyl && r.hl) dd += (float)(r.actl - plo) * r.Dl;
    }
    Hd += dd;
  }
  if (XFLOOR<XG> && ch2 != 0u) {
    /* the second bank's changed rows, their D through rowF after the first bank's: every lane of the
       team writes its row (team-uniform branch), a dof lane then adds the rows on its chain */
    tsync();
    L->rowF[c.l] = dl2;
    tsync();
    if (c.l < NV) add_rows(tb2, (const gfloat_t*)xrows(L), L->rowF, ddep, H, Hd);
  }
  if (YFLOOR<XG> && ch3 != 0u) {
    /* XG 5: the third bank's changed rows, the same way after the second's */
    tsync();
    L->rowF[c.l] = dl3;
    tsync();
    if (c.l < NV) add_rows(tb3, (const gfloat_t*)yrows(L), L->rowF, ddep, H, Hd);
  }
  /* the second / third bank's G rows in Hs[] are read before H is stored there */
  if (XA && full && ((XFLOOR<XG> && r.x.any) || (YFLOOR<XG> && r.y.any))) tsync();
  st_row(&L->Hs[c.l][0], H);
  L->Hsd[c.l] = Hd;
  tsync();
  /* the full build runs with the whole wave (matrix-core Schur complement); a
     refactor inside the Newton loop may run for one team only (team reductions) */
  return full ? factor_ldl<true>(c, H, Hd, L->Hs) : factor_ldl<false>(c, H, Hd, L->Hs);
}

/* exact line search along `search`; returns alpha (team-uniform) and Mv/Jv */
template <int XG, bool XA = true>
__device__ __forceinline__ float line_search(const Ctx& c, Rows& r, const float jr[CAP], float search, float Ma, float fs,
                                             float grad, float& Mv) {
  CP cfg = c.cfg;
  EnvL* L = c.L;
  /* leaves search in vec[V_TMP]; J rows are zero where no contact: no branch around the loads */
  float unused_;
  Mv = mul_m_dot(c, r, jr, search, V_TMP, r.Jv, -1, unused_);
  if constexpr (XG && XA) {
    float jx = r.x.any ? row_dot_x(c, r, V_TMP) : 0.f;
    if constexpr (XPAIR<XG>) jx += xor16f(jx); /* the pair's row: both halves */
    r.x.Jv = jx;
  }
  if constexpr (YBANK<XG> && XA) {
    float jy = r.y.any ? row_dot_y(c, r, V_TMP) : 0.f;
    if constexpr (YPAIR<XG>) jy += xor16f(jy); /* the pair's row: both halves */
    r.y.Jv = jy;
  }
  tsync();
  /* the quadratic's coefficients and the slope/curvature at alpha = 0 in one reduction:
     d1(0) = search . grad (the gradient update_constraint left for the current active
     set), d2(0) = c2 + sum of D (J search)^2 over the rows active now */
  const bool isd = c.l < NV;
  const float jv0 = isd ? search : 0.f;
  float g20 = (r.ex && r.act) ? r.D * r.Jv * r.Jv : 0.f;
  g20 += (r.hf && r.actf) ? r.Df * jv0 * jv0 : 0.f;
  if (r.anyl) g20 += (r.hl && r.actl) ? r.Dl * jv0 * jv0 : 0.f;
  const bool xprim = !XPAIR<XG> || c.l < 16; /* the lane that counts the second bank's row (pair: half 0) */
  /* XA: the second bank has rows in the wave; without, its terms are exact zeros and its row state is
     not carried through the loop (fewer live registers in the common copy) */
  if constexpr (XG && XA) g20 += (r.x.ex && r.x.act && xprim) ? r.x.D * r.x.Jv * r.x.Jv : 0.f;
  if constexpr (YBANK<XG> && XA)
    g20 += (r.y.ex && r.y.act && (YFLOOR<XG> || c.l < 16)) ? r.y.D * r.y.Jv * r.y.Jv : 0.f;
  float cc[4] = {isd ? search * (Ma - fs) : 0.f, isd ? search * Mv : 0.f, isd ? search * grad : 0.f, g20};
  tsum_n<4>(cc);
  const float c1 = cc[0], c2 = cc[1];
  /* per-row constants of the piecewise quadratic along the search direction (the
     two joint-limit rows of a dof are folded into one: at most one side exists) */
  /* row existence folded into the constants (zero for a row that does not exist) */
  const float DJ = r.ex ? r.D * r.Jv : 0.f, DJ2 = DJ * r.Jv;
  const float Rf = r.Rf * r.fl, DfJ = r.hf ? r.Df * jv0 : 0.f, DfJ2 = DfJ * jv0;
  float sv = 0.f, jl0 = 0.f, DlJ = 0.f, DlJ2 = 0.f;
  if (r.anyl) {
    sv = r.sl * jv0;
    jl0 = r.jl;
    DlJ = r.hl ? r.Dl * sv : 0.f;
    DlJ2 = DlJ * sv;
  }
  const float DXJ = (XG && XA && r.x.ex && xprim) ? r.x.D * r.x.Jv : 0.f, DXJ2 = (XG && XA) ? DXJ * r.x.Jv : 0.f;
  const float DYJ = (YBANK<XG> && XA && r.y.ex && (YFLOOR<XG> || c.l < 16)) ? r.y.D * r.y.Jv : 0.f,
              DYJ2 = (YBANK<XG> && XA) ? DYJ * r.y.Jv : 0.f;
  float d1 = cc[2], d2 = c2 + cc[3];
  if (!(d1 < 0.f) || !(d2 > 0.f)) return 0.f;
  const float gtol = cfg->ls_tolerance * (-d1);
  /* the iteration loop in two copies, with and without the joint-limit row (LIM): a branch on
     r.anyl inside the evaluation is if-converted by the compiler into selects around the row's
     arithmetic, which then runs in every evaluation */
  auto iterate = [&](auto lim, auto xany) -> float {
    constexpr bool LIM = decltype(lim)::value;
    constexpr bool XANY = decltype(xany)::value; /* XG: the second bank has rows in the wave */
    auto eval = [&](float alpha, float& e1, float& e2) {
      /* branch-free; rows that do not exist or are inactive add exact zeros */
      float g1, g2;
      {
        /* contact: active below zero */
        const float x = r.jar + alpha * r.Jv;
        g1 = DJ * fminf(x, 0.f);
        g2 = x < 0.f ? DJ2 : 0.f;
      }
      {
        /* frictionloss: linear zone |x| < R fl, saturated at -+fl outside (the force
           D x clamped to the saturation: D x = fl at x = R fl) */
        const float x = r.jf + alpha * jv0;
        g1 += DfJ * __builtin_amdgcn_fmed3f(x, -Rf, Rf);
        g2 += fabsf(x) < Rf ? DfJ2 : 0.f;
      }
      if constexpr (LIM) {
        /* joint limit: active below zero (the copy without it runs while no row of the wave
           exists, whose terms here would be exact zeros) */
        const float x = jl0 + alpha * sv;
        g1 += DlJ * fminf(x, 0.f);
        g2 += x < 0.f ? DlJ2 : 0.f;
      }
      if constexpr (XANY) {
        /* second-bank contact row (the copy without it runs while the bank has no row in the wave;
           a branch on r.x.any here was if-converted as the joint-limit one was) */
        const float x = r.x.jar + alpha * r.x.Jv;
        g1 += DXJ * fminf(x, 0.f);
        g2 += x < 0.f ? DXJ2 : 0.f;
        if constexpr (YBANK<XG>) {
          const float xy = r.y.jar + alpha * r.y.Jv;
          g1 += DYJ * fminf(xy, 0.f);
          g2 += xy < 0.f ? DYJ2 : 0.f;
        }
      }
      float gg[2] = {g1, g2};
      tsum_n<2>(gg);
      e1 = c1 + alpha * c2 + gg[0];
      e2 = c2 + gg[1];
    };
    float lo = 0.f, hi = -1.f;
    float alpha = -d1 / d2;
    for (int it = 0; it < cfg->ls_iterations; it++) {
      eval(alpha, d1, d2);
      if (fabsf(d1) <= gtol) break;
      if (d1 < 0.f) lo = alpha; else hi = alpha;
      float an = alpha - d1 / d2;
      if (!(an > lo) || (hi >= 0.f && !(an < hi))) an = 0.5f * (lo + (hi >= 0.f ? hi : 2.f * alpha));
      alpha = an;
    }
    return alpha;
  };
  /* XA: the caller's instantiation for a wave whose second bank has rows (solve_newton / solve_cg) */
  return r.anyl ? iterate(BoolC<true>{}, BoolC<XG != 0 && XA>{}) : iterate(BoolC<false>{}, BoolC<XG != 0 && XA>{});
}

/* H p for the sole-pair kernels' Newton direction (hsolve_pair): M p, the floor rows' and dof rows'
   D J J' p over the current active set (the terms of the factored tree Hessian H_t, hessian_factor:
   the soles' bank and, XG 4, the floor colliders' bank), plus the pair's active rows' D u u' p (u: the
   row over both limbs, held as two half rows: the second bank in XG 3, the third in XG 4). */
template <int XG>
__device__ __forceinline__ float hmul_pair(const Ctx& c, const Rows& r, const float jr[CAP], float p) {
  const int ddep = vopq(c.ddep);
  float jv, unused_;
  const float Mp = mul_m_dot(c, r, jr, p, V_TMP, jv, -1, unused_);
  const XRow& pr = YPAIR<XG> ? r.y : r.x;
  float jp = row_dot(c, (const gfloat_t*)(YPAIR<XG> ? yrows(c.L) : xrows(c.L)) + c.l * CAP, pr.chd, V_TMP);
  jp += xor16f(jp);
  const float w0 = (r.ex && r.act) ? r.D * jv : 0.f;
  const float wp = (pr.ex && pr.act) ? pr.D * jp : 0.f;
  const float cs0 = colsum16_pre(jr, w0);
  const float cs1 = colsum16((const gfloat_t*)(YPAIR<XG> ? yrows(c.L) : xrows(c.L)) + c.l * CAP, wp);
  const float so = tsh(cs0, ddep), sx = tsh(cs0, 16 + ddep), s2 = tsh(cs1, ddep), s3 = tsh(cs1, 16 + ddep);
  float s4 = 0.f, s5 = 0.f;
  if constexpr (YPAIR<XG>) {
    /* XG 4: the floor colliders' bank is part of H_t */
    if (r.x.any) {
      const float jf = row_dot_x(c, r, V_TMP);
      const float wf = (r.x.ex && r.x.act) ? r.x.D * jf : 0.f;
      const float cs2 = colsum16((const gfloat_t*)xrows(c.L) + c.l * CAP, wf);
      s4 = tsh(cs2, ddep);
      s5 = tsh(cs2, 16 + ddep);
    }
  }
  float y = 0.f;
  if (c.l < NV) {
    const bool f0 = (c.rmb & 1u) != 0u, f1 = (c.rmb & 2u) != 0u;
    /* the pair's static row masks: rmb bits 2-3 (XG 3) or 4-5 (XG 4) */
    const uint32_t pb = YPAIR<XG> ? (c.rmb >> 4) : (c.rmb >> 2);
    const bool f2 = (pb & 1u) != 0u, f3 = (pb & 2u) != 0u;
    y = Mp + (f0 ? so : 0.f) + (f1 ? sx : 0.f) + (f2 ? s2 : 0.f) + (f3 ? s3 : 0.f);
    if constexpr (YPAIR<XG>) {
      const bool f4 = (r.x.rowmask & 0xFFFFu) != 0u, f5 = (r.x.rowmask >> 16) != 0u;
      y += (f4 ? s4 : 0.f) + (f5 ? s5 : 0.f);
    }
    if (r.hf && r.actf) y += r.Df * p;
    if (r.anyl && r.hl && r.actl) y += r.Dl * p;
  }
  return y;
}

/* Newton direction H^-1 g of the sole-pair kernels. H = H_t + sum over the pair's active rows of
   D u u': the pair's rows couple the two legs, which the tree factorization of H_t (hessian_factor)
   cannot hold, so while any of them is active the system is solved by conjugate gradients
   preconditioned with H_t. H_t^-1 H = I + H_t^-1 U D U' has at most 1 + rank(U) <= 13 distinct
   eigenvalues (U spans the two limbs' dofs), so the iteration is exact in at most 13 steps in exact
   arithmetic; it stops at a relative residual |r|^2 <= 1e-12 |g|^2 or after 16. Without an active pair
   row it is the tree solve. [The oracle factors the dense H, mju_cholFactor; the two agree to the
   residual.] Team-uniform loop (no matrix cores inside). */
template <int XG>
__device__ __forceinline__ float hsolve_pair(const Ctx& c, const Rows& r, const float jr[CAP], float g, float Dinv) {
  const bool isd = c.l < NV;
  float z = solve_ldl(c, g, Dinv);
  const XRow& pr = YPAIR<XG> ? r.y : r.x;
  if (team_ballot(pr.ex && pr.act) == 0u) return z;
  float x = 0.f, rr = isd ? g : 0.f, p = isd ? z : 0.f;
  float dd[2] = {isd ? rr * z : 0.f, isd ? g * g : 0.f};
  tsum_n<2>(dd);
  float rz = dd[0];
  const float g2 = dd[1];
  for (int it = 0; it < 16; it++) {
    const float Hp = hmul_pair<XG>(c, r, jr, p);
    const float pHp = tsum(isd ? p * Hp : 0.f);
    if (!(pHp > 0.f)) break;
    const float alpha = rz / pHp;
    x += alpha * p;
    rr -= alpha * Hp;
    const float rn = tsum(isd ? rr * rr : 0.f);
    if (!(rn > 1e-12f * g2)) break;
    z = solve_ldl(c, rr, Dinv);
    const float rzn = tsum(isd ? rr * z : 0.f);
    const float beta = rzn / rz;
    rz = rzn;
    p = isd ? z + beta * p : 0.f;
  }
  return x;
}

/* constrained acceleration (mj_solNewton, primal). Returns qacc (dof lane). */
template <int XG, bool XA = true>
__device__ __forceinline__ float solve_newton(const Ctx& c, Rows& r, float qs, float fs, float w, int& iters,
                                              bool live, float& ftot) {
  CP cfg = c.cfg;
  MP m = c.m;
  EnvL* L = c.L;
  __builtin_amdgcn_s_setprio(ZB_SOLVER_PRIO);
  /* warmstart selection */
  float x = w;
  if (c.l < 32) L->vec[V_TMP2][c.l] = qs; /* mul_m's barrier publishes it with x in vec[V_TMP] */
  /* rows that do not exist have zero J and zero aref: no mask */
  float jw, js;
  /* the lane's contact-row Jacobian: constant through the solve, kept in registers */
  float jr[CAP];
  ld_row(&L->u.J[c.l][0], jr);
  float Ma = mul_m_dot(c, r, jr, x, V_TMP, jw, V_TMP2, js);
  jw -= r.aref;
  js -= r.aref;
  float jwx = 0.f, jsx = 0.f;
  if (XG && XA && r.x.any) {
    jwx = row_dot_x(c, r, V_TMP);
    jsx = row_dot_x(c, r, V_TMP2);
    if constexpr (XPAIR<XG>) {
      jwx += xor16f(jwx);
      jsx += xor16f(jsx);
    }
    jwx -= r.x.aref;
    jsx -= r.x.aref;
  }
  float jwy = 0.f, jsy = 0.f;
  if constexpr (YBANK<XG> && XA) {
    if (r.y.any) {
      jwy = row_dot_y(c, r, V_TMP);
      jsy = row_dot_y(c, r, V_TMP2);
      if constexpr (YPAIR<XG>) {
        jwy += xor16f(jwy);
        jsy += xor16f(jsy);
      }
      jwy -= r.y.aref;
      jsy -= r.y.aref;
    }
  }
  tsync();
  float cws[2] = {(c.l < NV ? 0.5f * (Ma - fs) * (x - qs) : 0.f) + rows_cost<XG, XA>(c, r, jw, x - r.af, r.sl * x - r.al, jwx, jwy),
                  rows_cost<XG, XA>(c, r, js, qs - r.af, r.sl * qs - r.al, jsx, jsy)};
  tsum_n<2>(cws);
  const float cw = cws[0], cs = cws[1];
  if (cw > cs) {
    x = qs;
    Ma = mul_m(c, x, V_TMP);
    r.jar = js;
    r.x.jar = jsx;
    r.y.jar = jsy;
  } else {
    r.jar = jw;
    r.x.jar = jwx;
    r.y.jar = jwy;
  }
  STAMP(S_WARM);
  r.jf = x - r.af;
  r.jl = r.sl * x - r.al;
  float scale = 1.0f / (m->meaninertia * (float)(NV > 1 ? NV : 1));
  float grad;
  float cost = update_constraint<XG, XA>(c, r, jr, x, qs, fs, Ma, grad);
  STAMP(S_UPD0);
  float Dinv = hessian_factor<XG, XA>(c, r, true, 0, 0, 0, 0, 0);
  STAMP(S_HESS0);
  float search;
  if constexpr (ANYPAIR<XG> && XA) search = -hsolve_pair<XG>(c, r, jr, grad, Dinv);
  else search = -solve_ldl(c, grad, Dinv);
  STAMP(S_SOLVE0);
  int it = 0;
  while (live && it < cfg->iterations) {
    float Mv;
    STAMP(S_CHECK);
    float alpha = line_search<XG, XA>(c, r, jr, search, Ma, fs, grad, Mv);
    STAMP(S_LS);
    if (alpha == 0.f) break;
    x += alpha * search;
    Ma += alpha * Mv;
    r.jar += alpha * r.Jv;
    if constexpr (XG && XA) r.x.jar += alpha * r.x.Jv;
    if constexpr (YBANK<XG> && XA) r.y.jar += alpha * r.y.Jv;
    r.jf += alpha * search;
    if (r.anyl) r.jl += alpha * (r.sl * search);
    float oldcost = cost;
    const int pa = r.act, pf = r.actf, plo = r.actl, pa2 = (XG && XA) ? r.x.act : 0,
              pa3 = (YFLOOR<XG> && XA) ? r.y.act : 0;
    /* the iteration's three team sums in one interleaved reduction (the same DPP sequence per
       value, so the bits of separate tsum calls): cost, |grad|^2 and the active-set change */
    float red[3];
    red[0] = update_constraint_lane<XG, XA>(c, r, jr, x, qs, fs, Ma, grad);
    red[1] = c.l < NV ? grad * grad : 0.f;
    red[2] = (r.act != pa || r.actf != pf || (XFLOOR<XG> && XA && r.x.act != pa2) ||
              (YFLOOR<XG> && XA && r.y.act != pa3)) ? 1.f : 0.f;
    if (r.anyl && r.actl != plo) red[2] = 1.f;
    tsum_n<3>(red);
    cost = red[0];
    STAMP(S_UPD);
    it++;
    /* mj_solNewton's termination test. MuJoCo runs it after the Hessian update and the new
       search direction; both only feed the next iteration, so a terminating iteration skips
       them here (qacc, forces and costs are the same bits either way). */
    const float improvement = scale * (oldcost - cost);
    const float gradient = scale * sqrtf(red[1]);
    if (improvement < cfg->tolerance || gradient < cfg->tolerance || it >= cfg->iterations) break;
    /* H depends only on the active set (M, D fixed within a substep):
       refactor only when it changed (MuJoCo's Newton does the same) */
    const bool changed = red[2] > 0.f;
    if (changed) Dinv = hessian_factor<XG, XA>(c, r, false, pa, pf, plo, pa2, pa3);
    STAMP(S_HESS);
    float mg;
    if constexpr (ANYPAIR<XG> && XA) mg = hsolve_pair<XG>(c, r, jr, grad, Dinv);
    else mg = solve_ldl(c, grad, Dinv);
    STAMP(S_SOLVE);
    search = -mg;
  }
  iters += it;
  /* qfrc_smooth + qfrc_constraint at the returned qacc (grad = Ma - qfrc_smooth - J'f), for
     mj_Euler's implicit damping */
  ftot = Ma - grad;
  __builtin_amdgcn_s_setprio(0);
  return x;
}

/* constrained acceleration by the primal nonlinear conjugate gradient (mj_solCG; MJX solver.py
   with SolverType.CG; oracle solve_cg). The same warmstart, cost, exact line search and
   termination test as solve_newton; the direction is the M^-1-preconditioned gradient, solved with
   the smooth factor of M that forward() left in L[] / Dk / Di (DinvM: this lane's 1/D), with
   Polak-Ribiere beta = max(0, g . (Mg - Mg_prev) / max(MINVAL, g_prev . Mg_prev)). No Hessian is
   built or factored. Returns qacc (dof lane). */
template <int XG, bool XA = true>
__device__ __forceinline__ float solve_cg(const Ctx& c, Rows& r, float qs, float fs, float w, int& iters, bool live,
                                          float DinvM, float& ftot) {
  CP cfg = c.cfg;
  MP m = c.m;
  EnvL* L = c.L;
  __builtin_amdgcn_s_setprio(ZB_SOLVER_PRIO);
  float x = w;
  if (c.l < 32) L->vec[V_TMP2][c.l] = qs;
  float jw, js;
  /* the lane's contact-row Jacobian: constant through the solve, kept in registers */
  float jr[CAP];
  ld_row(&L->u.J[c.l][0], jr);
  float Ma = mul_m_dot(c, r, jr, x, V_TMP, jw, V_TMP2, js);
  jw -= r.aref;
  js -= r.aref;
  float jwx = 0.f, jsx = 0.f;
  if (XG && XA && r.x.any) {
    jwx = row_dot_x(c, r, V_TMP);
    jsx = row_dot_x(c, r, V_TMP2);
    if constexpr (XPAIR<XG>) {
      jwx += xor16f(jwx);
      jsx += xor16f(jsx);
    }
    jwx -= r.x.aref;
    jsx -= r.x.aref;
  }
  float jwy = 0.f, jsy = 0.f;
  if constexpr (YBANK<XG> && XA) {
    if (r.y.any) {
      jwy = row_dot_y(c, r, V_TMP);
      jsy = row_dot_y(c, r, V_TMP2);
      if constexpr (YPAIR<XG>) {
        jwy += xor16f(jwy);
        jsy += xor16f(jsy);
      }
      jwy -= r.y.aref;
      jsy -= r.y.aref;
    }
  }
  tsync();
  float cws[2] = {(c.l < NV ? 0.5f * (Ma - fs) * (x - qs) : 0.f) + rows_cost<XG, XA>(c, r, jw, x - r.af, r.sl * x - r.al, jwx, jwy),
                  rows_cost<XG, XA>(c, r, js, qs - r.af, r.sl * qs - r.al, jsx, jsy)};
  tsum_n<2>(cws);
  if (cws[0] > cws[1]) {
    x = qs;
    Ma = mul_m(c, x, V_TMP);
    r.jar = js;
    r.x.jar = jsx;
    r.y.jar = jsy;
  } else {
    r.jar = jw;
    r.x.jar = jwx;
    r.y.jar = jwy;
  }
  STAMP(S_WARM);
  r.jf = x - r.af;
  r.jl = r.sl * x - r.al;
  const float scale = 1.0f / (m->meaninertia * (float)(NV > 1 ? NV : 1));
  float grad;
  float cost = update_constraint<XG, XA, false>(c, r, jr, x, qs, fs, Ma, grad);
  STAMP(S_UPD0);
  float mg = solve_pre(c, grad);
  STAMP(S_SOLVE0);
  float search = -mg;
  int it = 0;
  const int itmax = cfg->iterations;
  while (live && it < itmax) {
    float Mv;
    STAMP(S_CHECK);
    const float alpha = line_search<XG, XA>(c, r, jr, search, Ma, fs, grad, Mv);
    STAMP(S_LS);
    if (alpha == 0.f) break;
    x += alpha * search;
    Ma += alpha * Mv;
    r.jar += alpha * r.Jv;
    if constexpr (XG && XA) r.x.jar += alpha * r.x.Jv;
    if constexpr (YBANK<XG> && XA) r.y.jar += alpha * r.y.Jv;
    r.jf += alpha * search;
    if (r.anyl) r.jl += alpha * (r.sl * search);
    const float oldcost = cost, gold = grad, mgold = mg;
    const float cl = update_constraint_lane<XG, XA, false>(c, r, jr, x, qs, fs, Ma, grad);
    STAMP(S_UPD);
    it++;
    /* MJX's order (solver.py: _update_gradient, then the Polak-Ribiere beta, then the termination
       test): the next direction M^-1 grad is solved before the test, so that the iteration's four
       team sums (cost, |grad|^2 and beta's numerator and denominator) are one interleaved reduction
       (the same DPP sequence per value: the bits of separate sums). An iteration at the cap skips the
       solve and the beta sums, which only feed the next iteration. */
    if (it < itmax) {
      mg = solve_pre(c, grad);
      STAMP(S_SOLVE);
      float red[4] = {cl, c.l < NV ? grad * grad : 0.f, c.l < NV ? grad * (mg - mgold) : 0.f,
                      c.l < NV ? gold * mgold : 0.f};
      tsum_n<4>(red);
      cost = red[0];
      const float improvement = scale * (oldcost - cost);
      const float gradient = scale * sqrtf(red[1]);
      if (improvement < cfg->tolerance || gradient < cfg->tolerance) break;
      const float beta = fmaxf(red[2] / fmaxf(red[3], MINVAL), 0.f);
      search = -mg + beta * search;
    } else {
      (void)cl; /* the cap: the cost and |grad| feed only a test whose outcome is known */
      break;
    }
  }
  iters += it;
  ftot = Ma - grad; /* as solve_newton */
  __builtin_amdgcn_s_setprio(0);
  return x;
}

/* ----------------------------- Feetech actuator ---------------------------- */
/* trapezoidal_step (train.py:1137-1196) + duty/torque (train.py:1260-1269) */
template <int XG>
constexpr bool TGT_LDS = XG != 0; /* the action target in EnvL.tgt, not in LaneS.tgt */
template <int XG>
__device__ __forceinline__ void feetech(const Ctx& c, LaneS& ls) {
  MP m = c.m;
  if (c.act < 0) { ls.ctrl = 0.f; return; }
  const int a = c.act;
  const float dt = c.cfg->dt;
  float pos = ls.pp, vel = ls.pv, tgt = TGT_LDS<XG> ? c.L->tgt[c.l] : ls.tgt;
  float err = tgt - pos;
  bool in_db = fabsf(err) <= DEADBAND;
  float db_vel = vel * 0.8f;
  float db_pos = pos + db_vel * dt;
  float tdir = (float)((err > 0.f) - (err < 0.f));
  float amax = m->fe_amax[a], vmax = m->fe_vmax[a];
  float stop = fabsf(vel * vel) / (2.f * amax);
  float vdir = (float)((vel > 0.f) - (vel < 0.f));
  bool towards = vdir * tdir >= 0.f;
  bool accel = towards && fabsf(err) > stop;
  float acc = accel ? tdir * amax : -vdir * amax;
  if (fabsf(vel) < 1e-6f) acc = tdir * amax;
  float pv = vel + acc * dt;
  pv = fminf(fmaxf(pv, -vmax), vmax);
  float pp = pos + pv * dt;
  float npos = in_db ? db_pos : pp, nvel = in_db ? db_vel : pv;
  float perr = npos - ls.q, verr = nvel - ls.v;
  float duty = m->fe_kp[a] * m->fe_error_gain[a] * perr + m->fe_kd[a] * verr;
  duty = fminf(fmaxf(duty, -m->fe_max_pwm[a]), m->fe_max_pwm[a]);
  float tau = duty * m->fe_vin[a] * m->fe_kt[a] / m->fe_R[a];
  ls.pp = npos;
  ls.pv = nvel;
  ls.ptau = tau;
  ls.ctrl = tau;
}

/* ------------------------------- full forward ------------------------------ */
/* mj_forward (+ sensors if requested). Leaves qacc in ls.qacc, kinematics in B. */
template <int SOLVER, int XG>
__device__ __forceinline__ void forward(const Ctx& c, const EnvS& s, LaneS& ls, BodyK& B, Rows& r, bool with_sensors,
                                        Sensors& sen, int& iters) {
  MP m = c.m;
  EnvL* L = c.L;
  STAMP(S_ENTRY);
  kinematics(c, s, ls, B);
  STAMP(S_KIN);
  float cm[3];
  com_crb_m(c, s, ls, B, cm);
  STAMP(S_CRB);
  /* factor M (copy of rows) */
  float X[CAP];
  float Xd = load_mrow(c, X);
  float DinvM = factor_ldl<true>(c, X, Xd, L->M);
  STAMP(S_FACM);
  /* velocities */
  if (c.l < 32) L->vec[V_QVEL][c.l] = c.l < NV ? ls.v : 0.f;
  tsync();
  const float qv = c.l < NV ? ls.v : 0.f;
  float cdd[6];
  com_vel(c, B, qv, cdd);
  float ca[6], zero6[6] = {0, 0, 0, 0, 0, 0};
  com_acc(c, cdd, qv, 0.f, ca, false);
  float bias = rne_project(c, B, ca, zero6);
  /* actuation + passive -> qfrc_smooth, qacc_smooth */
  float act = 0.f;
  if (c.act >= 0) {
    float ct = fminf(fmaxf(ls.ctrl, m->act_ctrlrange[c.act][0]), m->act_ctrlrange[c.act][1]);
    ls.actforce = m->act_gear[c.act] * ct;
    act = m->act_gear[c.act] * ls.actforce;
  } else {
    ls.actforce = 0.f;
  }
  const float damp = keepf(c.L->par[P_DAMP][c.l & 31]);
  float fs = (c.l < NV) ? (-damp * ls.v - bias + act) : 0.f;
  STAMP(S_RNE);
  constexpr bool PRE = SOLVER == ZB_SOLVER_CG; /* CG's ~10 solves with M's factor per substep */
  if constexpr (PRE) solve_prep(c);
  float qs = PRE ? solve_pre(c, fs) : solve_ldl(c, fs, DinvM);
  STAMP(S_SOLVES);
  /* constraints */
  make_constraints<XG>(c, s, ls, B, cm, r);
  STAMP(S_CON);
  int nrows = tmaxi(r.nrow + (XG ? r.x.nrow : 0) + (YBANK<XG> ? r.y.nrow : 0) + (r.hf || r.hl ? 1 : 0));
  float qacc;
  /* entered by the whole wave when either env has rows (the full Hessian
     build runs on the matrix cores and needs every lane); an env without
     rows leaves the Newton loop at once and keeps qacc_smooth */
  qacc = qs;
  float ftot = fs; /* qfrc_smooth (+ qfrc_constraint below) */
  if (__ballot(nrows > 0) != 0ull) {
    int it2 = 0;
    float ft = 0.f;
    /* XG: the solver in two copies, with and without the second bank's terms (wave-uniform
       r.x.any; branches on it inside the loops were if-converted into every evaluation) */
    auto solve = [&](auto xa) -> float {
      constexpr bool XA = decltype(xa)::value;
      return SOLVER == ZB_SOLVER_CG ? solve_cg<XG, XA>(c, r, qs, fs, ls.w, it2, nrows > 0, DinvM, ft)
                                    : solve_newton<XG, XA>(c, r, qs, fs, ls.w, it2, nrows > 0, ft);
    };
    const bool xa = XG != 0 && (r.x.any || (YBANK<XG> && r.y.any)); /* wave-uniform */
    const float qn = xa ? solve(BoolC<true>{}) : solve(BoolC<false>{});
    if (nrows > 0) {
      qacc = qn;
      ftot = ft;
      iters += it2;
    }
  }
  ls.qacc = (c.l < NV) ? qacc : 0.f;
  ls.fq = (c.l < NV) ? ftot : 0.f;
  STAMP(S_CHECK);
  if (!with_sensors) return;
  /* ------------------- sensors (mj_rnePostConstraint etc.) ------------------ */
  tsync();
  /* contact forces per geom -> cfrc_ext on the geom body, touch */
  float fext[6] = {0, 0, 0, 0, 0, 0};
  float cpos[3], cdir[3], cmu;
  (void)contact_point<XG>(c, s, B, 0, cpos, cdir, cmu);
  float xpos[3], xdir[3], ypos[3], ydir[3];
  /* the pair's row direction n +- mu t; the half on geom1's limb (lanes 16-31) takes -F */
  auto pair_dir = [&](float* pos, float* dir) {
    float n[3], t1[3], t2[3];
    (void)pair_contact(c, B, pos, n, t1, t2);
    const int edge = c.l & 3;
    const float sg = (edge & 1) ? -m->pair_friction[0] : m->pair_friction[0];
    const float hs = (c.l >> 4) ? -1.f : 1.f;
#pragma unroll
    for (int k = 0; k < 3; k++) dir[k] = hs * (n[k] + sg * (edge < 2 ? t1[k] : t2[k]));
  };
  if constexpr (XPAIR<XG>) {
    if (r.x.any) pair_dir(xpos, xdir);
  } else if (XG && r.x.any) {
    (void)contact_point<XG>(c, s, B, 1, xpos, xdir, cmu);
  }
  if constexpr (YPAIR<XG>) {
    if (r.y.any) pair_dir(ypos, ydir);
  } else if (YFLOOR<XG> && r.y.any) {
    (void)contact_point<XG>(c, s, B, 2, ypos, ydir, cmu);
  }
  const int rgeom = c.l >> 4;
  float tch0 = 0.f, tch1 = 0.f;
  for (int g = 0; g < (YBANK<XG> ? 3 * NGEOM : XG ? 2 * NGEOM : NGEOM); g++) {
    /* geom g: bank g / 2, lanes 16 (g % 2) .. + 15 (XG 4: bank 2 = the pair's halves) */
    const bool b1 = XG && g >= NGEOM && g < 2 * NGEOM, b2 = YBANK<XG> && g >= 2 * NGEOM;
    if (b1 && !r.x.any) continue; /* wave-uniform */
    if (b2 && !r.y.any) continue;
    const bool mine = (b2 ? r.y.ex : b1 ? r.x.ex : r.ex) && rgeom == (g & 1);
    const float rf = b2 ? r.y.f : b1 ? r.x.f : r.f;
    const float* pp = b2 ? ypos : b1 ? xpos : cpos;
    const float* dd = b2 ? ydir : b1 ? xdir : cdir;
    float F[3] = {0, 0, 0}, tq[3] = {0, 0, 0};
    float fn = 0.f;
    if (mine) {
      F[0] = rf * dd[0]; F[1] = rf * dd[1]; F[2] = rf * dd[2];
      float off[3] = {pp[0] - cm[0], pp[1] - cm[1], pp[2] - cm[2]};
      cross3(tq, off, F);
      fn = rf;
    }
    float ex7[7] = {tq[0], tq[1], tq[2], F[0], F[1], F[2], fn};
    tsum_n<7>(ex7);
    float ext[6] = {ex7[0], ex7[1], ex7[2], ex7[3], ex7[4], ex7[5]};
    float fnt = ex7[6];
    /* the pair's halves: g = 2 geom2's body (+F), g = 3 geom1's (-F, in xdir); each foot's touch
       sensor takes the pair's normal force (its geom is in the contact) */
    const int gg = (YFLOOR<XG> && b2) ? c.L->ysel[g - 2 * NGEOM]
                   : b2 ? m->pair_geom[g == 2 * NGEOM ? 1 : 0]
                   : (XPAIR<XG> && b1) ? m->pair_geom[g == NGEOM ? 1 : 0]
                   : (XFLOOR<XG> && b1) ? c.L->s.xsel[g - NGEOM] : g;
    if (gg >= 0 && gg < m->ngeom && c.l == m->geom_body[gg]) {
#pragma unroll
      for (int k = 0; k < 6; k++) fext[k] += ext[k];
    }
    if (gg == m->geom_left_foot) tch0 += fnt;
    if (gg == m->geom_right_foot) tch1 += fnt;
  }
  sen.touch[0] = tch0;
  sen.touch[1] = tch1;
  float cacc[6];
  {
    BodyK B2 = B; /* cdof_dot again (not kept in registers through the solver) */
    float cdd2[6];
    com_vel(c, B2, qv, cdd2);
    com_acc(c, cdd2, qv, ls.qacc, cacc, true);
  }
  /* cfrc_int subtree sums (in sub[]) */
  (void)rne_project(c, B, cacc, fext);
  /* imu site: framequat, gyro, accelerometer */
  {
    int sb = m->site_body[m->site_imu];
    float xq[4], xp[3], R[9], cv[6], cc[6];
#pragma unroll
    for (int k = 0; k < 4; k++) xq[k] = tsh(B.xq[k], sb);
#pragma unroll
    for (int k = 0; k < 3; k++) xp[k] = tsh(B.xp[k], sb);
    quat2mat(R, xq);
#pragma unroll
    for (int k = 0; k < 6; k++) { cv[k] = tsh(B.cv[k], sb); cc[k] = tsh(cacc[k], sb); }
    float sq[4];
    quat_mul(sq, xq, s.imu_q);
#pragma unroll
    for (int k = 0; k < 4; k++) sen.fq[k] = sq[k];
    float sR[9], t[3];
    quat2mat(sR, sq);
    mulmv3(t, R, s.imu_p);
    float sp[3] = {xp[0] + t[0], xp[1] + t[1], xp[2] + t[2]};
    float dif[3] = {sp[0] - cm[0], sp[1] - cm[1], sp[2] - cm[2]};
    mulmtv3(sen.gyro, sR, cv);
    float v[3], a[3];
    cross3(t, cv, dif);
    for (int k = 0; k < 3; k++) v[k] = cv[3 + k] + t[k];
    cross3(t, cc, dif);
    for (int k = 0; k < 3; k++) a[k] = cc[3 + k] + t[k];
    cross3(t, cv, v);
    for (int k = 0; k < 3; k++) a[k] += t[k];
    mulmtv3(sen.acc, sR, a);
  }
  /* foot force sensors: cfrc_int of the site body, site frame */
  {
    int fs_[2] = {m->site_left_foot, m->site_right_foot};
    for (int side = 0; side < 2; side++) {
      int ss = fs_[side], sb = m->site_body[ss];
      float F[3] = {L->sub[sb][3], L->sub[sb][4], L->sub[sb][5]};
      float xq[4], sq[4], sR[9];
#pragma unroll
      for (int k = 0; k < 4; k++) xq[k] = tsh(B.xq[k], sb);
      float sqm[4] = {m->site_quat[ss][0], m->site_quat[ss][1], m->site_quat[ss][2], m->site_quat[ss][3]};
      quat_mul(sq, xq, sqm);
      quat2mat(sR, sq);
      mulmtv3(&sen.force[3 * side], sR, F);
    }
  }
  tsync();
  STAMP(S_SENS);
}

/* ------------------------- implicit damping (EULERDAMP) --------------------- */
/* mj_Euler with EULERDAMP enabled (MuJoCo's default; MJX forward.euler): the joint damping is
   integrated implicitly, qacc_e = (M + dt diag(B))^-1 (qfrc_smooth + qfrc_constraint), and qvel
   advances with qacc_e; qacc itself (sensors, qacc_warmstart) stays the solver's. M's rows are
   still in L->M (the solvers only read them); the factor lands in L[] / Dk / Di, which the next
   forward() rewrites. Wave-uniform: factor_ldl's Schur complement runs on the matrix cores. */
__device__ __forceinline__ float implicit_damping(const Ctx& c, const LaneS& ls) {
  tsync(); /* the solve's last reads of L[] are done before the factor overwrites it */
  float X[CAP];
  float Xd = load_mrow(c, X);
  const float damp = keepf(c.L->par[P_DAMP][c.l & 31]);
  Xd += (c.l < NV) ? c.cfg->dt * damp : 0.f;
  const float Dinv = factor_ldl<true>(c, X, Xd, c.L->M);
  return solve_ldl(c, ls.fq, Dinv);
}

/* ------------------------------ Euler integrate ----------------------------- */
/* mj_Euler / mj_advance. ED: qvel advances with the implicit-damping qacc_e (implicit_damping). */
template <bool ED>
__device__ __forceinline__ void integrate(const Ctx& c, EnvS& s, LaneS& ls, float qacc_e) {
  const float dt = c.cfg->dt;
  float vn = ls.v + dt * (ED ? qacc_e : ls.qacc);
  float v0 = tsh(vn, 0), v1 = tsh(vn, 1), v2 = tsh(vn, 2), w0 = tsh(vn, 3), w1 = tsh(vn, 4), w2 = tsh(vn, 5);
  if (c.l < NV) {
    ls.w = ls.qacc; /* mj_advance: qacc_warmstart */
    ls.v = vn;
    if (c.qadr >= 0) ls.q += dt * vn;
  }
  /* free joint (root): world-frame translation, body-frame rotation */
  if (c.m->body_jnttype[1] == ZB_JNT_FREE) {
    s.bp[0] += dt * v0; s.bp[1] += dt * v1; s.bp[2] += dt * v2;
    float w[3] = {w0, w1, w2};
    float nw = sqrtf(dot3(w, w));
    if (nw > MINVAL) {
      float ax[3] = {w[0] / nw, w[1] / nw, w[2] / nw}, qr[4], qn[4];
      axis_angle_quat(qr, ax, nw * dt);
      quat_mul(qn, s.bq, qr);
#pragma unroll
      for (int k = 0; k < 4; k++) s.bq[k] = qn[k];
    }
    quat_normalize(s.bq);
  }
}

/* --------------------------- env-level (ksim) logic ------------------------- */
__device__ __forceinline__ void load_params(const Ctx& c, EnvS& s, LaneS& ls, const float* rnd) {
  MP m = c.m;
  const bool rz = (c.cfg->flags & ZB_F_RANDOMIZE) && rnd;
  const int l = c.l;
  float arm = 0.f, damp = 0.f, floss = 0.f, q0 = 0.f;
  if (l < NV) {
    arm = m->dof_armature[l] * (rz ? rnd[ZB_R_ARMATURE + l] : 1.f);
    damp = m->dof_damping[l] * (rz ? rnd[ZB_R_DAMPING + l] : 1.f);
    floss = m->dof_frictionloss[l] * (rz ? rnd[ZB_R_FRICTION + l] : 1.f);
    if (c.qadr >= 0) q0 = m->qpos0[c.qadr] + ((rz && c.act >= 0) ? rnd[ZB_R_QPOS0 + c.act] : 0.f);
  }
  c.L->par[P_MSCALE][l] = (rz && l < NB) ? rnd[ZB_R_MASS + l] : 1.f;
  c.L->par[P_ARM][l] = arm;
  c.L->par[P_DAMP][l] = damp;
  c.L->par[P_FLOSS][l] = floss;
  c.L->par[P_Q0][l] = q0;
  s.floor_mu = rz ? rnd[ZB_R_FLOOR_MU] : 1.f;
  int si = m->site_imu;
  float sq[4] = {m->site_quat[si][0], m->site_quat[si][1], m->site_quat[si][2], m->site_quat[si][3]};
#pragma unroll
  for (int k = 0; k < 3; k++) s.imu_p[k] = m->site_pos[si][k] + (rz ? rnd[ZB_R_IMU_POS + k] : 0.f);
  if (rz) {
    float rq[4] = {rnd[ZB_R_IMU_QUAT], rnd[ZB_R_IMU_QUAT + 1], rnd[ZB_R_IMU_QUAT + 2], rnd[ZB_R_IMU_QUAT + 3]}, o[4];
    quat_mul(o, sq, rq);
#pragma unroll
    for (int k = 0; k < 4; k++) sq[k] = o[k];
  }
#pragma unroll
  for (int k = 0; k < 4; k++) s.imu_q[k] = sq[k];
}

/* randomizer sampling (must match oracle/zb_oracle.c sample_rand) */
__device__ __forceinline__ void sample_rand(const Ctx& c, uint32_t episode, float* rnd) {
  /* re-derived here: hoisted out of the substep loop, the per-k field addresses were live for the
     whole launch and spilled to scratch (only this rare path reads them) */
  CP cfg = opaque(c.cfg);
  /* opaque lane id: the per-k selections and keys below depend on the lane only, and hoisted to the
     kernel entry they were live (spilled) for the whole launch though only this rare path reads them */
  const int l = vopq(c.l);
  for (int k = l; k < 75; k += TEAM) {
    float u0, u1;
    uniform2(cseed(c), P_RAND, (uint32_t)k, cenv(c), episode, u0, u1);
    float lo, hi;
    int base;
    if (k < 16) { lo = cfg->rand_mass[0]; hi = cfg->rand_mass[1]; base = ZB_R_MASS + 2 * k; }
    else if (k < 32) { lo = cfg->rand_armature[0]; hi = cfg->rand_armature[1]; base = ZB_R_ARMATURE + 2 * (k - 16); }
    else if (k < 48) { lo = cfg->rand_damping[0]; hi = cfg->rand_damping[1]; base = ZB_R_DAMPING + 2 * (k - 32); }
    else if (k < 64) { lo = cfg->rand_friction[0]; hi = cfg->rand_friction[1]; base = ZB_R_FRICTION + 2 * (k - 48); }
    else if (k < 74) { lo = cfg->rand_qpos0[0]; hi = cfg->rand_qpos0[1]; base = ZB_R_QPOS0 + 2 * (k - 64); }
    else { lo = cfg->rand_floor_mu[0]; hi = cfg->rand_floor_mu[1]; base = ZB_R_FLOOR_MU; }
    rnd[base] = lo + (hi - lo) * u0;
    if (k < 74) rnd[base + 1] = lo + (hi - lo) * u1;
  }
  if (l == 0) {
    float z00, z01, z10, z11, z20, z21;
    normal2(cseed(c), P_RAND, 75u, cenv(c), episode, z00, z01);
    normal2(cseed(c), P_RAND, 76u, cenv(c), episode, z10, z11);
    normal2(cseed(c), P_RAND, 77u, cenv(c), episode, z20, z21);
    float rv[3] = {cfg->rand_imu_tilt_std * z00, cfg->rand_imu_tilt_std * z01, cfg->rand_imu_yaw_std * z10};
    float ang = sqrtf(dot3(rv, rv)), q[4] = {1.f, 0.f, 0.f, 0.f};
    if (ang > MINVAL) {
      float ax[3] = {rv[0] / ang, rv[1] / ang, rv[2] / ang};
      axis_angle_quat(q, ax, ang);
    }
    for (int k = 0; k < 4; k++) rnd[ZB_R_IMU_QUAT + k] = q[k];
    rnd[ZB_R_IMU_POS + 0] = cfg->rand_imu_pos_std * z11;
    rnd[ZB_R_IMU_POS + 1] = cfg->rand_imu_pos_std * z20;
    rnd[ZB_R_IMU_POS + 2] = cfg->rand_imu_pos_std * z21;
  }
  for (int k = ZB_R_END + l; k < ZB_RAND_STRIDE; k += TEAM) rnd[k] = 0.f;
}

/* rotate_quat_by_quat (train.py:751-787) */
__device__ __forceinline__ void rotate_quat_by_quat(const float q_[4], const float r_[4], bool inverse, float out[4]) {
  const float eps = 1e-6f;
  float n1 = sqrtf(q_[0] * q_[0] + q_[1] * q_[1] + q_[2] * q_[2] + q_[3] * q_[3]) + eps;
  float n2 = sqrtf(r_[0] * r_[0] + r_[1] * r_[1] + r_[2] * r_[2] + r_[3] * r_[3]) + eps;
  float a[4] = {r_[0] / n2, r_[1] / n2, r_[2] / n2, r_[3] / n2};
  float b[4] = {q_[0] / n1, q_[1] / n1, q_[2] / n1, q_[3] / n1};
  if (inverse) { a[1] = -a[1]; a[2] = -a[2]; a[3] = -a[3]; }
  float r[4];
  quat_mul(r, a, b);
  float n = sqrtf(r[0] * r[0] + r[1] * r[1] + r[2] * r[2] + r[3] * r[3]) + eps;
  for (int k = 0; k < 4; k++) out[k] = r[k] / n;
}

/* observation assembly + obs-derived carries (train.py:1478-1537, 1624-1679) */
__device__ __forceinline__ void observe(const Ctx& c, EnvS& s, const LaneS& ls, const BodyK& B, const Sensors& sen, float* oa,
                        float* oc, float* ox) {
  MP m = c.m;
  CP cfg = c.cfg;
  const int l = c.l;
  /* ImuOrientationObservation (heading command 0) */
  float hq[4] = {1.f, 0.f, 0.f, 0.f}, bq[4];
  rotate_quat_by_quat(sen.fq, hq, true, bq);
  if (bq[0] < 0.f) for (int k = 0; k < 4; k++) bq[k] = -bq[k];
  float imu[4];
  for (int k = 0; k < 4; k++) {
    float x = s.ema[k] * s.lag + bq[k] * (1.f - s.lag);
    s.ema[k] = x;
    imu[k] = x;
  }
  float acc[3] = {sen.acc[0], sen.acc[1], sen.acc[2]};
  if (cfg->flags & ZB_F_OBS_NOISE) {
    float z0 = 0.f, z1 = 0.f;
    if (l < 4) normal2(cseed(c), P_OBS, (uint32_t)l, cenv(c), s.rng_step, z0, z1);
    float a0 = tsh(z0, 0), a1 = tsh(z1, 0), b0 = tsh(z0, 1), b1 = tsh(z1, 1);
    float c0 = tsh(z0, 2), c1 = tsh(z1, 2), d0 = tsh(z0, 3);
    imu[0] += cfg->imu_noise_std * a0; imu[1] += cfg->imu_noise_std * a1;
    imu[2] += cfg->imu_noise_std * b0; imu[3] += cfg->imu_noise_std * b1;
    acc[0] += cfg->acc_noise_std * c0; acc[1] += cfg->acc_noise_std * c1; acc[2] += cfg->acc_noise_std * d0;
  }
  /* feet positions in the robot frame (train.py:451-465) */
  float bqn[4] = {s.bq[0], s.bq[1], s.bq[2], s.bq[3]}, bm[9];
  quat_normalize(bqn);
  quat2mat(bm, bqn);
  float fpos[2][3];
  {
    int sides[2] = {m->site_left_foot, m->site_right_foot};
    for (int sd = 0; sd < 2; sd++) {
      int ss = sides[sd], sb = m->site_body[ss];
      float xp[3], R[9], t[3], xqs[4];
      for (int k = 0; k < 3; k++) xp[k] = tsh(B.xp[k], sb);
      for (int k = 0; k < 4; k++) xqs[k] = tsh(B.xq[k], sb);
      quat2mat(R, xqs);
      float sp[3] = {m->site_pos[ss][0], m->site_pos[ss][1], m->site_pos[ss][2]};
      mulmv3(t, R, sp);
      float w[3] = {xp[0] + t[0], xp[1] + t[1], xp[2] + t[2]};
      mulmtv3(fpos[sd], bm, w);
    }
  }
  float dfx = fpos[0][0] - fpos[1][0], dfy = fpos[0][1] - fpos[1][1], dfz = fpos[0][2] - fpos[1][2];
  s.feet_dist = sqrtf(dfx * dfx + dfy * dfy + dfz * dfz);
  s.touch[0] = sen.touch[0];
  s.touch[1] = sen.touch[1];
  /* joint-space values of actuated dof lanes, fetched by output index */
  const int jl = l < ZB_NJ ? m->act_dof[l] : 0;
  const float qa = tsh(ls.q, jl), va = tsh(ls.v, jl), fa = tsh(ls.actforce, jl), ta = tsh(ls.ptau, jl);
  const float acca = tsh(ls.qacc, jl);
  float xb = tsh(B.xp[2], 1);
  if (oa) {
    if (l < ZB_NJ) {
      oa[l] = qa;
      oa[ZB_NJ + l] = va;
    }
    if (l < 4) oa[40 + l] = imu[l];
    if (l >= 4 && l < 10) oa[40 + l] = 0.f;
  }
  if (oc) {
    if (l < ZB_NJ) {
      oc[l] = qa;
      oc[ZB_NJ + l] = va / 10.f;
      oc[457 + l] = fa / 100.f;
    }
    if (l >= 1 && l < NB) {
      for (int k = 0; k < 10; k++) oc[40 + (l - 1) * 10 + k] = c.L->ci[l][k];
      for (int k = 0; k < 6; k++) oc[290 + (l - 1) * 6 + k] = B.cv[k];
    }
    if (l < 3) oc[440 + l] = acc[l];
    if (l < 3) oc[443 + l] = sen.gyro[l];
    if (l < 4) oc[446 + l] = imu[l];
    if (l < ZB_NUM_CMD) oc[450 + l] = 0.f;
    if (l < 3) oc[477 + l] = s.bp[l];
    if (l < 4) oc[480 + l] = s.bq[l];
  }
  if (ox) {
    if (l < 6) {
      ox[ZB_X_BASE_LINVEL + l] = ls.v;   /* qvel[0:6] (lin then ang) */
      ox[ZB_X_BASE_LINACC + l] = ls.qacc; /* qacc[0:6] (lin then ang) */
    }
    if (l == 0) {
      ox[ZB_X_BASE_HEIGHT] = xb;
      ox[ZB_X_TOUCH] = sen.touch[0];
      ox[ZB_X_TOUCH + 1] = sen.touch[1];
#pragma unroll
      for (int k = 0; k < 6; k++) ox[ZB_X_FORCE + k] = sen.force[k];
#pragma unroll
      for (int k = 0; k < 3; k++) {
        ox[ZB_X_FEET_POS + k] = fpos[0][k];
        ox[ZB_X_FEET_POS + 3 + k] = fpos[1][k];
      }
    }
    if (l < ZB_NJ) {
      ox[ZB_X_FEETECH_TAU + l] = ta;
      ox[ZB_X_ACT_ACC + l] = acca;
    }
    for (int i = ZB_X_END + l; i < ZB_OBS_EXTRA; i += TEAM) ox[i] = 0.f;
  }
}

/* xax.quat_to_euler roll & pitch */
__device__ __forceinline__ void quat_roll_pitch(const float q_[4], float& roll, float& pitch) {
  float q[4] = {q_[0], q_[1], q_[2], q_[3]};
  quat_normalize(q);
  float w = q[0], x = q[1], y = q[2], z = q[3];
  roll = atan2f(2.f * (w * x + y * z), 1.f - 2.f * (x * x + y * y));
  float sp = fminf(fmaxf(2.f * (w * y - z * x), -1.f), 1.f);
  pitch = asinf(sp);
}

/* terminations + reward terms (train.py:1546-1593) ; returns done */
__device__ __forceinline__ bool rewards(const Ctx& c, EnvS& s, const LaneS& ls, const BodyK& B, float cur, float* terms_out,
                        float& total, bool& fail, float& airtime_term) {
  MP m = c.m;
  CP cfg = c.cfg;
  const int l = c.l;
  float z = s.bp[2];
  float bq[4] = {s.bq[0], s.bq[1], s.bq[2], s.bq[3]};
  quat_normalize(bq);
  float upz = 1.f - 2.f * (bq[1] * bq[1] + bq[2] * bq[2]);
  uint32_t steps = s.ep_steps + 1u;
  fail = (z < cfg->bad_z[0]) || (z > cfg->bad_z[1]) || (upz < cosf(cfg->max_tilt_rad)) || !(z == z);
  bool trunc = (float)steps * cfg->ctrl_dt >= cfg->max_episode_sec;
  bool done = fail || trunc;
  float t[ZB_NUM_TERMS];
  t[ZB_T_STAY_ALIVE] = fail ? -1.f : 1.f / cfg->stay_alive_balance;
  float xq1[4];
  for (int k = 0; k < 4; k++) xq1[k] = tsh(B.xq[k], 1);
  t[ZB_T_UPRIGHT] = 1.f - 2.f * (xq1[1] * xq1[1] + xq1[2] * xq1[2]);
  float v0 = tsh(ls.v, 0), v1 = tsh(ls.v, 1), v2 = tsh(ls.v, 2);
  t[ZB_T_NAIVE_FORWARD] = fminf(v0, cfg->naive_forward_clip_max);
  t[ZB_T_FWD_ORIENT] = 1.f - 2.f * (xq1[2] * xq1[2] + xq1[3] * xq1[3]);
  {
    float bm[9], vb[3], vw[3] = {v0, v1, v2};
    quat2mat(bm, bq);
    mulmtv3(vb, bm, vw);
    t[ZB_T_LINVEL_Y] = fabsf(vb[1]);
  }
  bool lc = s.touch[0] > cfg->touch_threshold, rc = s.touch[1] > cfg->touch_threshold;
  t[ZB_T_SINGLE_FOOT] = (lc != rc) ? 1.f : 0.f;
  {
    bool cont[2] = {lc, rc};
    float rr = 0.f;
    for (int sd = 0; sd < 2; sd++) {
      float air_prev = s.air[sd];
      bool prev = s.prev_cont[sd] > 0.5f;
      bool td = cont[sd] && !prev;
      rr += (air_prev - cfg->feet_airtime_touchdown_penalty) * (td ? 1.f : 0.f);
      s.air[sd] = (cont[sd] || done) ? 0.f : air_prev + cfg->ctrl_dt;
      s.prev_cont[sd] = cont[sd] ? 1.f : 0.f;
    }
    t[ZB_T_FEET_AIRTIME] = rr;
    airtime_term = rr;
  }
  {
    float ql[4], qr[4];
    for (int k = 0; k < 4; k++) {
      ql[k] = tsh(B.xq[k], m->body_left_foot);
      qr[k] = tsh(B.xq[k], m->body_right_foot);
    }
    float rl, pl, rrr, pr;
    quat_roll_pitch(ql, rl, pl);
    quat_roll_pitch(qr, rrr, pr);
    float err = fabsf(rl) + fabsf(pl) + fabsf(rrr) + fabsf(pr);
    t[ZB_T_FEET_ORIENT] = expf(-err / cfg->feet_orient_error_scale);
  }
  t[ZB_T_FEET_TOO_CLOSE] = s.feet_dist < cfg->feet_too_close_threshold ? 1.f : 0.f;
  {
    /* joint deviation penalties; group masks over ctrl index (train.py:584-640) */
    const uint32_t straight = (1u << 7) | (1u << 6) | (1u << 1) | (1u << 0);
    const uint32_t ankle = (1u << 9) | (1u << 10) | (1u << 11) | (1u << 3) | (1u << 4) | (1u << 5);
    const uint32_t arm = 0xFF000u;
    float p1 = 0.f, p2 = 0.f, p3 = 0.f;
    if (c.act >= 0) {
      float e = ls.q - m->joint_bias[c.act];
      float w = m->joint_weight[c.act] * e * e;
      if ((straight >> c.act) & 1u) p1 = w;
      if ((ankle >> c.act) & 1u) p2 = w;
      if ((arm >> c.act) & 1u) p3 = w;
    }
    float pp[3] = {p1, p2, p3};
    tsum_n<3>(pp);
    t[ZB_T_STRAIGHT_LEG] = pp[0];
    t[ZB_T_ANKLE_KNEE] = pp[1];
    t[ZB_T_ARM_POSE] = pp[2];
  }
  total = 0.f;
  for (int i = 0; i < ZB_NUM_TERMS; i++) {
    float sc = cfg->reward_scale[i] * (cfg->reward_by_curriculum[i] ? cur : 1.f);
    total += sc * t[i];
  }
  if (terms_out && l < ZB_NUM_TERMS) {
    float v = 0.f;
    for (int i = 0; i < ZB_NUM_TERMS; i++)
      if (i == l) v = t[i];
    terms_out[l] = v;
  }
  s.ep_steps = steps;
  s.ep_ret += total;
  return done;
}

/* ------------------------------ state I/O ---------------------------------- */
/* CG: sc1 accesses (the chunked step hands state rows between workgroups); plain otherwise */
template <bool CG = false>
__device__ __forceinline__ void load_state(const Ctx& c, EnvS& s, LaneS& ls, const float* st) {
  const int l = c.l;
  for (int k = 0; k < 3; k++) s.bp[k] = ld_cg<CG>(st + ZB_S_QPOS + k);
  for (int k = 0; k < 4; k++) s.bq[k] = ld_cg<CG>(st + ZB_S_QPOS + 3 + k);
  for (int k = 0; k < 4; k++) s.ema[k] = ld_cg<CG>(st + ZB_S_IMU_EMA + k);
  s.lag = ld_cg<CG>(st + ZB_S_IMU_LAG);
  s.air[0] = ld_cg<CG>(st + ZB_S_AIRTIME); s.air[1] = ld_cg<CG>(st + ZB_S_AIRTIME + 1);
  s.push_timer = ld_cg<CG>(st + ZB_S_PUSH_TIMER);
  s.touch[0] = ld_cg<CG>(st + ZB_S_TOUCH); s.touch[1] = ld_cg<CG>(st + ZB_S_TOUCH + 1);
  s.feet_dist = ld_cg<CG>(st + ZB_S_FEET_DIST);
  s.ep_ret = ld_cg<CG>(st + ZB_S_EP_RETURN);
  s.ep_steps = fbits(ld_cg<CG>(st + ZB_S_EP_STEPS));
  s.rng_step = fbits(ld_cg<CG>(st + ZB_S_RNG_STEP));
  s.prev_cont[0] = ld_cg<CG>(st + ZB_S_PREV_CONT); s.prev_cont[1] = ld_cg<CG>(st + ZB_S_PREV_CONT + 1);
  s.episode = fbits(ld_cg<CG>(st + ZB_S_EPISODE));
  s.nanflag = fbits(ld_cg<CG>(st + ZB_S_NAN));
  ls.q = ls.v = ls.w = 0.f;
  ls.pp = ls.pv = ls.ptau = 0.f;
  if (l < NV) {
    ls.v = ld_cg<CG>(st + ZB_S_QVEL + l);
    ls.w = ld_cg<CG>(st + ZB_S_QACCW + l);
    if (c.qadr >= 0) ls.q = ld_cg<CG>(st + ZB_S_QPOS + c.qadr);
  }
  if (c.act >= 0) {
    ls.pp = ld_cg<CG>(st + ZB_S_PLAN_POS + c.act);
    ls.pv = ld_cg<CG>(st + ZB_S_PLAN_VEL + c.act);
    ls.ptau = ld_cg<CG>(st + ZB_S_PLAN_TAU + c.act);
  }
  ls.ctrl = 0.f;
  ls.qacc = 0.f;
  ls.actforce = 0.f;
}

template <bool CG = false>
__device__ __forceinline__ void store_state(const Ctx& c, const EnvS& s, const LaneS& ls, float* st) {
  const int l = c.l;
  if (l < NV) {
    st_cg<CG>(st + ZB_S_QVEL + l, ls.v);
    st_cg<CG>(st + ZB_S_QACCW + l, ls.w);
    if (c.qadr >= 0) st_cg<CG>(st + ZB_S_QPOS + c.qadr, ls.q);
  }
  if (c.act >= 0) {
    st_cg<CG>(st + ZB_S_PLAN_POS + c.act, ls.pp);
    st_cg<CG>(st + ZB_S_PLAN_VEL + c.act, ls.pv);
    st_cg<CG>(st + ZB_S_PLAN_TAU + c.act, ls.ptau);
  }
  if (l == 0) {
    for (int k = 0; k < 3; k++) st_cg<CG>(st + ZB_S_QPOS + k, s.bp[k]);
    for (int k = 0; k < 4; k++) st_cg<CG>(st + ZB_S_QPOS + 3 + k, s.bq[k]);
    for (int k = 0; k < 4; k++) st_cg<CG>(st + ZB_S_IMU_EMA + k, s.ema[k]);
    st_cg<CG>(st + ZB_S_IMU_LAG, s.lag);
    st_cg<CG>(st + ZB_S_AIRTIME, s.air[0]); st_cg<CG>(st + ZB_S_AIRTIME + 1, s.air[1]);
    st_cg<CG>(st + ZB_S_PUSH_TIMER, s.push_timer);
    st_cg<CG>(st + ZB_S_TOUCH, s.touch[0]); st_cg<CG>(st + ZB_S_TOUCH + 1, s.touch[1]);
    st_cg<CG>(st + ZB_S_FEET_DIST, s.feet_dist);
    st_cg<CG>(st + ZB_S_EP_RETURN, s.ep_ret);
    st_cg<CG>(st + ZB_S_EP_STEPS, bitsf(s.ep_steps));
    st_cg<CG>(st + ZB_S_RNG_STEP, bitsf(s.rng_step));
    st_cg<CG>(st + ZB_S_PREV_CONT, s.prev_cont[0]); st_cg<CG>(st + ZB_S_PREV_CONT + 1, s.prev_cont[1]);
    st_cg<CG>(st + ZB_S_EPISODE, bitsf(s.episode));
    st_cg<CG>(st + ZB_S_NAN, bitsf(s.nanflag));
  }
}

/* ksim reset (train.py:1471-1476); the caller then runs mjx.forward (forward()) */
__device__ __forceinline__ void reset_prepare(const Ctx& c, EnvS& s, LaneS& ls, float* rnd) {
  MP m = c.m;
  CP cfg = c.cfg;
  const int l = c.l;
  uint32_t episode = s.episode;
  if ((cfg->flags & ZB_F_RANDOMIZE) && rnd) {
    sample_rand(c, episode, rnd);
    tsync();
    __threadfence_block();
  }
  load_params(c, s, ls, rnd);
  for (int k = 0; k < 3; k++) s.bp[k] = m->qpos0[k];
  for (int k = 0; k < 4; k++) s.bq[k] = m->qpos0[3 + k];
  ls.v = 0.f;
  ls.w = 0.f;
  if (c.act >= 0) {
    int qa = c.qadr;
    ls.q = m->joint_bias[c.act] + (c.L->par[P_Q0][c.l] - m->qpos0[qa]);
    float u0, u1;
    uniform2(cseed(c), P_RESET, (uint32_t)(vopq(c.act) / 2), cenv(c), episode, u0, u1);
    float u = (c.act & 1) ? u1 : u0;
    ls.v = cfg->reset_qvel_scale * (2.f * u - 1.f);
  } else if (l < NV && c.qadr >= 0) {
    ls.q = m->qpos0[c.qadr];
  }
  {
    float u0, u1;
    uniform2(cseed(c), P_RESET, 15u, cenv(c), episode, u0, u1);
    s.lag = cfg->lag_range[0] + (cfg->lag_range[1] - cfg->lag_range[0]) * u0;
    s.push_timer = cfg->push_interval[0] + (cfg->push_interval[1] - cfg->push_interval[0]) * u1;
  }
  for (int k = 0; k < 4; k++) s.ema[k] = 0.f;
  ls.pp = ls.q;
  ls.pv = ls.v;
  ls.ptau = 0.f;
  ls.ctrl = 0.f;
  s.ep_ret = 0.f;
  s.ep_steps = 0u;
  s.episode = episode + 1u;
}

/* push event (train.py:1459-1468) */
__device__ __forceinline__ void push_event(const Ctx& c, EnvS& s, LaneS& ls, float cur) {
  CP cfg = c.cfg;
  float timer = s.push_timer - cfg->ctrl_dt;
  if (timer <= 0.f) {
    float u0, u1, w0, w1;
    uniform2(cseed(c), P_PUSH, 0u, cenv(c), s.rng_step, u0, u1);
    uniform2(cseed(c), P_PUSH, 1u, cenv(c), s.rng_step, w0, w1);
    float mag = (cfg->push_vel_range[0] + (cfg->push_vel_range[1] - cfg->push_vel_range[0]) * w1) / cfg->push_vel_range[1];
    if (c.l == 0) ls.v += cur * mag * cfg->push_linvel[0] * (2.f * u0 - 1.f);
    if (c.l == 1) ls.v += cur * mag * cfg->push_linvel[1] * (2.f * u1 - 1.f);
    if (c.l == 2) ls.v += cur * mag * cfg->push_linvel[2] * (2.f * w0 - 1.f);
    timer = cfg->push_interval[0] + (cfg->push_interval[1] - cfg->push_interval[0]) * w1;
  }
  s.push_timer = timer;
}

/* ---------------------------- per-team context ------------------------------ */
__device__ __forceinline__ void make_ctx(Ctx& c, const ZbModel* m, const ZbEnvConfig* cfg, const int32_t* topo,
                                         EnvL* L, uint64_t seed, uint32_t env) {
  static_assert(TOPO_NROOT == NROOT && TOPO_NGEOM == NGEOM && TOPO_MAXBD == MAXBD && TOPO_LANES == TEAM,
                "topology table built for this kernel's constants");
  c.m = (MP)m;
  c.cfg = (CP)cfg;
  c.L = L;
  L->s.env = env;
  L->s.seed_lo = (uint32_t)seed;
  L->s.seed_hi = (uint32_t)(seed >> 32);
  const int l = threadIdx.x & (TEAM - 1);
  c.l = l;
  c.nu = m->nu;
  /* the lane's roles, from the table zb_create built (all loads in flight) */
  const int32_t* t = topo + l;
  c.bpar = t[TP_BPAR * TEAM];
  c.bdep = t[TP_BDEP * TEAM];
  c.bjt = t[TP_BJT * TEAM];
  c.bdofadr = t[TP_BDOFADR * TEAM];
  c.blast = t[TP_BLAST * TEAM];
  c.nch = t[TP_NCH * TEAM];
  c.ch0 = (uint32_t)t[TP_CH0 * TEAM];
  c.ch1 = (uint32_t)t[TP_CH1 * TEAM];
  c.lvlch = (uint64_t)(uint32_t)t[TP_LVL_LO * TEAM] | ((uint64_t)(uint32_t)t[TP_LVL_HI * TEAM] << 32);
  c.ddep = t[TP_DDEP * TEAM];
  c.dbody = t[TP_DBODY * TEAM];
  c.qadr = t[TP_QADR * TEAM];
  c.act = t[TP_ACT * TEAM];
  {
    const uint32_t r0 = (uint32_t)t[TP_ROWMASK * TEAM], r1 = (uint32_t)t[TP_ROWMASK2 * TEAM];
    const uint32_t r2 = (uint32_t)t[TP_ROWMASK3 * TEAM]; /* the sole pair's rows beside the floor bank (XG 4) */
    c.rmb = (r0 & 1u) | ((r0 >> 15) & 2u) | ((r1 & 1u) << 2) | ((r1 >> 13) & 8u) | ((r2 & 1u) << 4) | ((r2 >> 11) & 32u);
  }
  c.dk0 = t[TP_DK0 * TEAM];
  c.dfree = t[TP_DFREE * TEAM];
  c.chd = t[TP_CHD * TEAM];
  c.cps = t[TP_CPS * TEAM];
  c.cln = t[TP_CLN * TEAM];
  if (l >= NV) {
    /* non-dof lanes: zero factor and mass rows (row 31 is the zero row that masked
       gathers point at; kernels never write these rows afterwards) */
    float z[CAP];
#pragma unroll
    for (int e = 0; e < CAP; e++) z[e] = 0.f;
    st_row(&L->L[l][0], z);
    st_row(&L->M[l][0], z);
  }
}

/* ---------------------------------- kernels --------------------------------- */

/* 2 waves per SIMD: the register allocator spills ~1 KB/lane of cold state to
   scratch (L1/L2-resident) instead of holding ~440 registers at 1 wave/SIMD;
   measured 1.6x faster (tests/diag_variants.py). */
#ifndef ZB_WAVES_PER_EU
#define ZB_WAVES_PER_EU 2
#endif
template <int SOLVER, int XG, int ED>
__global__ __launch_bounds__(64, ZB_WAVES_PER_EU) void step_kernel(StepArgs a) {
  const int team = threadIdx.x / TEAM;
  /* Chunked step (a.nchunk > 1, one control step): the launch has npair * nchunk workgroups, each
     running n_substeps / nchunk substeps of one pair of envs. A workgroup takes the next unit from
     the counter sched[0] in chunk-major order (every pair's chunk 0, then every pair's chunk 1,
     ...) and waits until the pair's previous chunk has published its state. Taking units in
     order means a unit's predecessor was taken by a running workgroup, so every wait ends. The
     slow pairs of the last round of waves then hold up the launch by a chunk, not by a whole
     control step. The state passes between chunks through the state row exactly
     as it passes between control steps, so the results do not depend on the chunking. */
  const int K = a.nchunk;
  const int npair = (a.n_envs + NTEAM - 1) / NTEAM;
  int pair = blockIdx.x, ch = 0;
  bool timed_out = false;
  if (K > 1) {
    uint32_t u = 0;
    if (threadIdx.x == 0) u = addu_cg(a.sched, 1u);
    u = __builtin_amdgcn_readfirstlane(u);
    ch = (int)(u / (uint32_t)npair);
    pair = (int)(u - (uint32_t)ch * (uint32_t)npair);
    if (ch > 0) {
      /* bounded: a wait that outlives ~2 s gives up. That is fatal for the launch: the sticky
         error word sched[2 + npair] is raised (zb_check reports it to the host), the env's
         iteration count is marked, and this unit stores no state (it would have run on the
         predecessor's unpublished row) */
      for (uint32_t spins = 0; ldu_cg(a.sched + 2 + pair) < (uint32_t)ch; spins++) {
        if (spins > (1u << 23)) {
          timed_out = true;
          break;
        }
        __builtin_amdgcn_s_sleep(4);
      }
      if (timed_out) {
        if (threadIdx.x == 0) stu_cg(a.sched + 2 + npair, 1u);
      } else {
        /* the predecessor's state stores happen-before the loads below */
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      }
    }
  }
  const int e = pair * NTEAM + team;
#ifdef ZB_WAVETIME
  /* diagnostic build: the pair's start / end on the 100 MHz constant clock and its CU */
  const unsigned long long wt0 = __builtin_amdgcn_s_memrealtime();
#endif
  /* Both teams of a wave stay live to the end: forward()'s J'DJ runs on the
     matrix cores with operands from all 64 lanes (jdj_mfma). A team past the
     last env (odd n) runs as a ghost copy of env n-1 that stores nothing. */
  const bool live = e < a.n_envs;
  const int ee = live ? e : a.n_envs - 1;
  const ZbModel* m = a.model;
  const ZbEnvConfig* cfg = a.cfg;
  Ctx c;
  make_ctx(c, m, cfg, a.topo, &g_lds[team], a.seed, (uint32_t)(a.env_offset + ee));
  /* the env's second-bank rows (a team past n: the spare block n) */
  if constexpr (XG) set_xrows(c.L, a.xj + (size_t)(live ? e : a.n_envs) * XJ_STRIDE<XG>);
  /* per-env row addresses are formed where they are used, from an opaque copy of the env
     index: held across the substep loop they were 64-bit values spilled to scratch */
  auto state_row = [&]() { return a.state + (size_t)vopq(ee) * ZB_STATE_STRIDE; };
  auto rand_row = [&]() {
    return live && (cfg->flags & ZB_F_RANDOMIZE) && a.rnd ? a.rnd + (size_t)vopq(ee) * ZB_RAND_STRIDE : nullptr;
  };
#ifdef ZB_STAMPS
  if (c.l < NSTAMP) c.L->stamp[c.l] = 0;
  if (c.l == 0) c.L->stamp_last = __builtin_amdgcn_s_memtime();
  tsync();
#endif
  EnvS& s = c.L->s;
  LaneS ls;
  if (K > 1) load_state<true>(c, s, ls, state_row());
  else load_state<false>(c, s, ls, state_row());
  load_params(c, s, ls, rand_row());
  BodyK B;
  Rows r;
  Sensors& sen = c.L->sen;
  int iters = (K > 1 && ch > 0) ? (int)ldu_cg((const uint32_t*)a.itpart + ee) : 0;
  if (timed_out) iters -= 1 << 24;
  float rsum = 0.f;
  bool done = false;
  bool success = false; /* done by the time limit alone (ksim successful termination) */
  const int nsteps = a.nsteps;
  const bool rollout = nsteps > 1;
  const int ss_end = (ch + 1) * cfg->n_substeps / K; /* this unit's substeps: [ss0, ss_end) */
  bool partial = false;                               /* a chunk before the last one */
  for (int t = 0; t < nsteps; t++) {
    const bool last_t = t == nsteps - 1;
    if (c.act >= 0) {
      const float at = a.action[((size_t)t * a.n_envs + vopq(ee)) * ZB_NJ + vopq(c.act)];
      if constexpr (TGT_LDS<XG>) c.L->tgt[c.l] = at;
      else ls.tgt = at;
    }
    if (ch == 0) s.nanflag &= ~4u; /* bit 2: a bank-2 overflow in this control step (select_bank2) */
    if (ch == 0 && (cfg->flags & ZB_F_PUSH)) push_event(c, s, ls, a.curriculum);
    float total = 0.f;
    int ss = ch * cfg->n_substeps / K;
    bool resetting = false; /* this team re-enters forward() for its reset state */
    bool ghost = false;     /* the other team resets: a discarded forward() pass */
    bool done_reset = false;
    /* 20 substeps; a terminated env then runs one more pass of the same code
       path for the reset forward (mjx.forward after MjxEngine.reset). That pass
       is wave-uniform: when one team resets, the other takes its observation
       first and then runs the same forward() on its state, discarded. */
    while (true) {
      c.m = opaque((MP)m);
      c.cfg = opaque((CP)cfg);
      STAMP(S_STEPEND);
      if (!resetting && !ghost) feetech<XG>(c, ls);
      STAMP(S_FEETECH);
      int it_pass = 0;
      forward<SOLVER, XG>(c, s, ls, B, r, resetting || ss == cfg->n_substeps - 1, sen, it_pass);
      if (!ghost) iters += it_pass;
      if (!resetting && !ghost) {
        /* wave-uniform: both teams integrate, or both run the reset / ghost pass */
        float qacc_e = 0.f;
        if constexpr (ED != 0) qacc_e = implicit_damping(c, ls);
        integrate<ED != 0>(c, s, ls, qacc_e);
        STAMP(S_INT);
        if (++ss < cfg->n_substeps) {
          if (ss < ss_end) continue;
          partial = true; /* wave-uniform: no team resets before the last substep */
          break;
        }
        {
          bool bad = (c.l < NV) && !(isfinite(ls.q) && isfinite(ls.v));
          if (tmaxi(bad ? 1 : 0)) s.nanflag |= 1u; /* keeps bit 1 (select_bank2) */
        }
        bool fail;
        float* terms = (live && a.reward_terms && !rollout) ? a.reward_terms + (size_t)vopq(e) * ZB_NUM_TERMS : nullptr;
        float air_term;
        done = rewards(c, s, ls, B, a.curriculum, terms, total, fail, air_term);
        success = done && !fail;
        if (a.air_mark && t == 0 && live && c.l == 0) {
          /* first step of a rollout: its contact flags and causal FeetAirtime term, for the
             exact ksim form patched in after the rollout (airtime_exact_kernel) */
          float* st = state_row();
          const uint32_t bits = (s.prev_cont[0] > 0.5f ? 1u : 0u) | (s.prev_cont[1] > 0.5f ? 2u : 0u);
          st_cg<true>(st + ZB_S_AIR0_CONT, bitsf(bits));
          st_cg<true>(st + ZB_S_AIR0_TERM, air_term);
        }
        rsum += total;
        if (live && a.stats && c.l == 0) {
          float* sp = a.stats + (size_t)vopq(e) * ZB_NUM_STATS;
          sp[ZB_ST_REWARD] += total;
          if (done) {
            sp[ZB_ST_RETURN] += s.ep_ret;
            sp[ZB_ST_LENGTH] += (float)s.ep_steps;
            sp[ZB_ST_DONE] += 1.f;
          }
        }
        done_reset = done && (cfg->flags & ZB_F_AUTORESET);
      }
      /* observation point: the stepped state, or the reset state */
      c.m = opaque((MP)m);
      c.cfg = opaque((CP)cfg);
      if (!ghost && (resetting || !done_reset)) {
        const bool out = live && last_t;
        const size_t eo = (size_t)vopq(e);
        observe(c, s, ls, B, sen, (out && a.obs_actor) ? a.obs_actor + eo * ZB_OBS_ACTOR : nullptr,
                (out && a.obs_critic) ? a.obs_critic + eo * ZB_OBS_CRITIC : nullptr,
                (out && a.obs_extra) ? a.obs_extra + eo * ZB_OBS_EXTRA : nullptr);
      }
      if (resetting || ghost) break;
      if (__ballot(done_reset) == 0ull) break;
      if (done_reset) {
        reset_prepare(c, s, ls, rand_row());
        resetting = true;
      } else {
        ghost = true;
      }
    }
    if (partial) break;
    s.rng_step += 1u;
    if (live && c.l == 0 && last_t) {
      const int eo = vopq(e);
      if (a.reward) a.reward[eo] = rollout ? rsum : total;
      if (a.done) a.done[eo] = done ? 1 : 0;
      if (a.success) a.success[eo] = success ? 1 : 0;
    }
  }
  if (partial) {
    if (live && c.l == 0) stu_cg((uint32_t*)a.itpart + vopq(e), (uint32_t)iters);
  } else if (live && a.iters && c.l == 0) {
    a.iters[vopq(e)] = iters;
  }
  if (live && !timed_out) {
    if (K > 1) store_state<true>(c, s, ls, state_row());
    else store_state<false>(c, s, ls, state_row());
  }
  if (K > 1) {
    /* publish: every state store of this wave happens-before lane 0's flag store */
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    if (threadIdx.x == 0) {
      if (partial) {
        /* atomic max: a late publish never lowers a flag a later chunk already advanced */
        maxu_cg(a.sched + 2 + pair, (uint32_t)(ch + 1));
      } else {
        /* last chunk: leave the pair's flag and (after the last pair's last chunk, when every
           unit has been taken) both counters at zero for the next launch */
        stu_cg(a.sched + 2 + pair, 0u);
        if (addu_cg(a.sched + 1, 1u) == (uint32_t)npair - 1u) {
          stu_cg(a.sched, 0u);
          stu_cg(a.sched + 1, 0u);
        }
      }
    }
  }
#ifdef ZB_WAVETIME
  if (threadIdx.x == 0 && a.dbg) {
    unsigned long long* w = reinterpret_cast<unsigned long long*>(a.dbg) + ((size_t)ch * npair + pair) * 4;
    w[0] = wt0;
    w[1] = __builtin_amdgcn_s_memrealtime();
    w[2] = (unsigned long long)__smid();
    w[3] = (unsigned long long)iters;
  }
#endif
#ifdef ZB_STAMPS
  STAMP(S_STEPEND);
  if (live && a.dbg && c.l == 0)
    for (int i = 0; i < NSTAMP; i++) reinterpret_cast<unsigned long long*>(a.dbg)[(size_t)e * NSTAMP + i] = c.L->stamp[i];
#endif
}

template <int SOLVER, int XG>
__global__ __launch_bounds__(64) void reset_kernel(StepArgs a) {
  const int team = threadIdx.x / TEAM;
  const int e = blockIdx.x * NTEAM + team;
  /* a team that is masked out (or past n) runs a discarded forward() on its
     current state: the matrix-core J'DJ needs all 64 lanes of the wave */
  const bool inb = e < a.n_envs;
  const bool live = inb && !(a.reset_mask && !a.reset_mask[e]);
  if (__ballot(live) == 0ull) return;
  const int ee = inb ? e : a.n_envs - 1;
  const ZbModel* m = a.model;
  const ZbEnvConfig* cfg = a.cfg;
  Ctx c;
  make_ctx(c, m, cfg, a.topo, &g_lds[team], a.seed, (uint32_t)(a.env_offset + ee));
  /* the env's second-bank rows (a team past n: the spare block n) */
  if constexpr (XG) set_xrows(c.L, a.xj + (size_t)(inb ? e : a.n_envs) * XJ_STRIDE<XG>);
  float* st = a.state + (size_t)ee * ZB_STATE_STRIDE;
  float* rnd = live && (cfg->flags & ZB_F_RANDOMIZE) && a.rnd ? a.rnd + (size_t)ee * ZB_RAND_STRIDE : nullptr;
  EnvS& s = c.L->s;
  LaneS ls;
  load_state(c, s, ls, st);
  BodyK B;
  Rows r;
  Sensors& sen = c.L->sen;
  int it = 0;
  if (live) reset_prepare(c, s, ls, rnd);
  else load_params(c, s, ls, nullptr);
  forward<SOLVER, XG>(c, s, ls, B, r, live, sen, it);
  if (!live) return;
  observe(c, s, ls, B, sen, a.obs_actor ? a.obs_actor + (size_t)e * ZB_OBS_ACTOR : nullptr,
          a.obs_critic ? a.obs_critic + (size_t)e * ZB_OBS_CRITIC : nullptr,
          a.obs_extra ? a.obs_extra + (size_t)e * ZB_OBS_EXTRA : nullptr);
  store_state(c, s, ls, st);
}

/* single forward on the stored (qpos, qvel), ctrl = action row; dumps internals */
template <int SOLVER, int XG>
__global__ __launch_bounds__(64) void debug_forward_kernel(StepArgs a) {
  const int team = threadIdx.x / TEAM;
  const int e = blockIdx.x * NTEAM + team;
  const bool live = e < a.n_envs; /* a ghost team (odd n) keeps the wave whole through forward() */
  const int ee = live ? e : a.n_envs - 1;
  const ZbModel* m = a.model;
  const ZbEnvConfig* cfg = a.cfg;
  Ctx c;
  make_ctx(c, m, cfg, a.topo, &g_lds[team], a.seed, (uint32_t)(a.env_offset + ee));
  /* the env's second-bank rows (a team past n: the spare block n) */
  if constexpr (XG) set_xrows(c.L, a.xj + (size_t)(live ? e : a.n_envs) * XJ_STRIDE<XG>);
  float* st = a.state + (size_t)ee * ZB_STATE_STRIDE;
  EnvS& s = c.L->s;
  LaneS ls;
  load_state(c, s, ls, st);
  load_params(c, s, ls, nullptr);
  ls.ctrl = (c.act >= 0 && a.action) ? a.action[(size_t)ee * ZB_NJ + c.act] : 0.f;
  BodyK B;
  Rows r;
  Sensors& sen = c.L->sen;
  int it = 0;
  forward<SOLVER, XG>(c, s, ls, B, r, true, sen, it);
  if (!live) return;
  float* d = a.dbg + (size_t)e * ZB_DBG_STRIDE;
  const int l = c.l;
  EnvL* L = c.L;
  /* dense M from depth-indexed rows */
  for (int i = l; i < NV * NV; i += TEAM) d[ZB_DBG_QM + i] = 0.f;
  __threadfence_block();
  tsync();
  if (l < NV) {
    for (int ee = 0; ee <= c.ddep; ee++) {
      int aa = anc_lin(c.chd, ee);
      float v = L->M[l][ee];
      d[ZB_DBG_QM + l * NV + aa] = v;
      d[ZB_DBG_QM + aa * NV + l] = v;
    }
    d[ZB_DBG_QACC + l] = ls.qacc;
  }
  /* recompute smooth quantities for the dump is avoided: store qacc only; the
     bias/qacc_smooth slots are filled by a second, constraint-free pass below */
  if (l < NB) {
    for (int k = 0; k < 3; k++) d[ZB_DBG_XPOS + 3 * l + k] = B.xp[k];
    for (int k = 0; k < 10; k++) d[ZB_DBG_CINERT + 10 * l + k] = c.L->ci[l][k];
    for (int k = 0; k < 6; k++) d[ZB_DBG_CVEL + 6 * l + k] = B.cv[k];
  }
  int nefc = (int)tsum((float)((r.ex ? 1 : 0) + (XG && r.x.ex && (!XPAIR<XG> || l < 16) ? 1 : 0) +
                               (YBANK<XG> && r.y.ex && (YFLOOR<XG> || l < 16) ? 1 : 0) + (r.hf ? 1 : 0) +
                               (r.hl ? 1 : 0)));
  if (l == 0) {
    d[ZB_DBG_MISC + 0] = (float)nefc;
    d[ZB_DBG_MISC + 1] = (float)((r.nrow + (XG ? r.x.nrow / (XPAIR<XG> ? 2 : 1) : 0) + (YBANK<XG> ? r.y.nrow / (YPAIR<XG> ? 2 : 1) : 0)) / 4);
    d[ZB_DBG_MISC + 2] = sen.touch[0];
    d[ZB_DBG_MISC + 3] = sen.touch[1];
    for (int k = 0; k < 4; k++) d[ZB_DBG_MISC + 4 + k] = sen.fq[k];
    for (int k = 0; k < 3; k++) d[ZB_DBG_MISC + 8 + k] = sen.gyro[k];
    for (int k = 0; k < 3; k++) d[ZB_DBG_MISC + 11 + k] = sen.acc[k];
  }
  /* smooth dynamics: qfrc_bias and qacc_smooth recomputed on the same state */
  {
    float X[CAP];
    float Xd = load_mrow(c, X);
    float Dinv = factor_ldl<true>(c, X, Xd, L->M);
    if (l < 32) L->vec[V_QVEL][l] = l < NV ? ls.v : 0.f;
    tsync();
    const float qv = l < NV ? ls.v : 0.f;
    float cdd[6];
    com_vel(c, B, qv, cdd);
    float ca[6], z6[6] = {0, 0, 0, 0, 0, 0};
    com_acc(c, cdd, qv, 0.f, ca, false);
    float bias = rne_project(c, B, ca, z6);
    float act = c.act >= 0 ? m->act_gear[c.act] * ls.actforce : 0.f;
    float fs = (l < NV) ? (-c.L->par[P_DAMP][c.l] * ls.v - bias + act) : 0.f;
    float qs = solve_ldl(c, fs, Dinv);
    if (l < NV) {
      d[ZB_DBG_BIAS + l] = bias;
      d[ZB_DBG_QACCS + l] = qs;
    }
  }
}

/* the kernel instantiation for a handle: solver x collider set (zb_host.cpp needs_xg: 0 two soles,
   1 / 2 general floor colliders, 3 the sole pair, 4 both) x implicit damping (ZB_F_EULERDAMP, step kernel
   only). f(S, X, D) is called with std::integral_constant values. */
template <typename F>
__host__ void with_variant(int solver, int xg, int ed, F&& f) {
  using std::integral_constant;
  auto by_xg = [&](auto S, auto D) {
    switch (xg) {
      /* only this unit's XG values are instantiated (ZB_XG_MASK); the entry points hand the others off */
      case 5: if constexpr (xg_here(5)) f(S, integral_constant<int, 5>{}, D); break;
      case 4: if constexpr (xg_here(4)) f(S, integral_constant<int, 4>{}, D); break;
      case 3: if constexpr (xg_here(3)) f(S, integral_constant<int, 3>{}, D); break;
      case 2: if constexpr (xg_here(2)) f(S, integral_constant<int, 2>{}, D); break;
      case 1: if constexpr (xg_here(1)) f(S, integral_constant<int, 1>{}, D); break;
      default: if constexpr (xg_here(0)) f(S, integral_constant<int, 0>{}, D); break;
    }
  };
  auto by_ed = [&](auto S) {
    if (ed) by_xg(S, integral_constant<int, 1>{});
    else by_xg(S, integral_constant<int, 0>{});
  };
  if (solver == ZB_SOLVER_CG) by_ed(integral_constant<int, ZB_SOLVER_CG>{});
  else by_ed(integral_constant<int, ZB_SOLVER_NEWTON>{});
}

int ZB_EP(step_resident_blocks)(int device, int xg, int solver, int ed) {
  ZB_HANDOFF(xg, step_resident_blocks, device, xg, solver, ed);
  int per_cu = 0, cus = 0;
  /* the instantiation the handle launches: CG and Newton differ in registers and LDS */
  hipError_t e = hipSuccess;
  with_variant(solver, xg, ed, [&](auto S, auto X, auto D) {
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, step_kernel<decltype(S)::value, decltype(X)::value,
                                                                          decltype(D)::value>, 64, 0);
  });
  if (e != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return 0;
  return per_cu * cus;
}

hipError_t ZB_EP(launch_step)(const StepArgs& a, hipStream_t s) {
  if (a.n_envs <= 0) return hipSuccess;
  ZB_HANDOFF(a.xg, launch_step, a, s);
  if (a.nchunk < 1 || (a.nchunk > 1 && (a.nsteps != 1 || !a.sched || !a.itpart))) return hipErrorInvalidValue;
#ifdef ZB_STAMPS
  StepArgs b = a;
  b.nchunk = 1; /* the phase stamps are per env-step */
#else
  const StepArgs& b = a;
#endif
  dim3 grid((unsigned)((b.n_envs + NTEAM - 1) / NTEAM * b.nchunk)), block(64);
  with_variant(b.solver, b.xg, b.ed, [&](auto S, auto X, auto D) {
    hipLaunchKernelGGL((step_kernel<decltype(S)::value, decltype(X)::value, decltype(D)::value>), grid, block, 0, s, b);
  });
  return hipGetLastError();
}
/* ksim's FeetAirtimeReward over one trajectory (train.py:503-546), row 0. The fused step
   computes the causal form, Σ_feet (air[t-1] - penalty) · [c_t ∧ ¬c_{t-1}], which is ksim's term
   for every t ≥ 1: the airtime scan (contact-or-done zeroes it, else + ctrl_dt) and the touchdown
   test are the same recurrences. Row 0 differs: ksim's touchdown takes prev = False at t = 0
   (`concatenate([False], c[:-1])`) and its airtime is `roll(air, 1)`, which reads air[T-1], the
   airtime after the trajectory's last step. The first step of a marked rollout saved c_0 and its
   causal term in the state row (ZB_S_AIR0_*); the state row now holds air[T-1]. One lane per env:
   term0 = Σ_feet c_0 · (air[T-1] - penalty), added to reward0 as scale · (term0 - causal0) and
   written over reward_terms0's FeetAirtime slot. The episode statistics' reward sum (ZB_ST_REWARD)
   gets the same delta, so it stays the sum of the rollout's patched rows; episode returns
   (ZB_ST_RETURN, the state row's running return) keep the causal row 0 (include/zbot.h). */
#ifndef ZB_ENGINE_TU_B
__global__ __launch_bounds__(256) void airtime_exact_kernel(const float* __restrict__ state, const ZbEnvConfig* cfg,
                                                            int n, float curriculum, float* reward0, float* terms0,
                                                            float* stats) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const float* st = state + (size_t)e * ZB_STATE_STRIDE;
  const uint32_t bits = fbits(st[ZB_S_AIR0_CONT]);
  const float causal = st[ZB_S_AIR0_TERM];
  const float pen = cfg->feet_airtime_touchdown_penalty;
  float term = 0.f;
  term += (st[ZB_S_AIRTIME] - pen) * ((bits & 1u) ? 1.f : 0.f);
  term += (st[ZB_S_AIRTIME + 1] - pen) * ((bits & 2u) ? 1.f : 0.f);
  const float sc = cfg->reward_scale[ZB_T_FEET_AIRTIME] * (cfg->reward_by_curriculum[ZB_T_FEET_AIRTIME] ? curriculum : 1.f);
  const float delta = sc * (term - causal);
  if (reward0) reward0[e] += delta;
  if (terms0) terms0[(size_t)e * ZB_NUM_TERMS + ZB_T_FEET_AIRTIME] = term;
  if (stats) stats[(size_t)e * ZB_NUM_STATS + ZB_ST_REWARD] += delta;
}

hipError_t launch_airtime_exact(const StepArgs& a, hipStream_t s) {
  if (a.n_envs <= 0) return hipSuccess;
  dim3 grid((unsigned)((a.n_envs + 255) / 256)), block(256);
  hipLaunchKernelGGL(airtime_exact_kernel, grid, block, 0, s, (const float*)a.state, a.cfg, a.n_envs, a.curriculum,
                     a.reward, a.reward_terms, a.stats);
  return hipGetLastError();
}
#endif

hipError_t ZB_EP(launch_reset)(const StepArgs& a, hipStream_t s) {
  if (a.n_envs <= 0) return hipSuccess;
  ZB_HANDOFF(a.xg, launch_reset, a, s);
  dim3 grid((a.n_envs + NTEAM - 1) / NTEAM), block(64);
  with_variant(a.solver, a.xg, 0, [&](auto S, auto X, auto) {
    hipLaunchKernelGGL((reset_kernel<decltype(S)::value, decltype(X)::value>), grid, block, 0, s, a);
  });
  return hipGetLastError();
}
hipError_t ZB_EP(launch_debug_forward)(const StepArgs& a, hipStream_t s) {
  if (a.n_envs <= 0) return hipSuccess;
  ZB_HANDOFF(a.xg, launch_debug_forward, a, s);
  dim3 grid((a.n_envs + NTEAM - 1) / NTEAM), block(64);
  with_variant(a.solver, a.xg, 0, [&](auto S, auto X, auto) {
    hipLaunchKernelGGL((debug_forward_kernel<decltype(S)::value, decltype(X)::value>), grid, block, 0, s, a);
  });
  return hipGetLastError();
}

}  // namespace zb
