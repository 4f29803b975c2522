/*
 * zb_policy.hip — the ZbotWalkingTask GRU actor / critic on the MI355X matrix
 * cores, one control step per launch. C ABI:
 * include/zbot_policy.h; CPU restatement: oracle/zb_oracle_policy.c.
 *
 * Reference: train.py Actor (:885-967), Critic (:970-1023), run_actor /
 * run_critic (:1616-1681), sample_action (:1737-1763); equinox GRUCell and
 * ksim MixtureOfGaussians [U].
 *
 * Layout of one launch (n envs, one step):
 *   workgroup = 32 envs x 8 waves; the 32 envs are two row tiles of
 *   v_mfma_f32_16x16x4_f32 (M = 16), and wave w owns the 16-unit tile w of
 *   every layer for both row tiles, so each weight fragment a wave loads
 *   feeds two MFMAs (the weight stream per env of a 32-env tile) while every
 *   SIMD holds two waves: one wave's GRU epilogue, LDS traffic and barriers run
 *   under the other's MFMAs. The r / z / n gates of a unit land in the same
 *   lane and the GRU update happens in registers: per layer 12 accumulators
 *   (W_ih x and W_hh h for r, z, n, two row tiles), K = 128 in 32 MFMA steps.
 *   A operands (activations) live in LDS k-major, [k][env] with a 33-float
 *   row stride: one ds_read_b32 per operand per step.
 *   B operands (weights) are pre-packed on the host in fragment order —
 *   [16-unit tile][group of 4 k-steps][lane][4] — so each lane streams one 16-B
 *   load per 4 MFMA steps per matrix tile; every workgroup reads the whole
 *   weight set (2.0 MB actor, 2.2 MB critic), which stays L2-resident.
 *   The carry of layer l + 1 is loaded from HBM into registers while layer l
 *   runs (its latency hides behind the MFMAs) and layer l's new carry is
 *   written at its end ([n][5][128] fp32, 2.5 KB per env per step).
 *
 * Numerics (bit-identical to the oracle): every product is the matrix core's
 * k-ordered fp32 fmaf chain from 0, biases are added afterwards, elementwise
 * code runs without contraction and the transcendental functions and RNG
 * come from include/zbot_fmath.h.
 *
 * Roofline: 2 x (50x128 + 5 x 6 x 128 x 128 + 128 x 300) = 1.07 MFLOP per env
 * per actor step (critic 1.11 MFLOP) on the f32 matrix cores (157.3 TF/s).
 */
#include <hip/hip_runtime.h>

#include "zb_internal.h"
#include "zbot_fmath.h"

namespace zb {
namespace pol {

constexpr int H = ZB_POL_HIDDEN;
constexpr int D = ZB_POL_DEPTH;
#ifndef ZB_POL_NET
#define ZB_POL_NET 2
#endif
constexpr int MT = 16;                   /* envs per MFMA row tile */
constexpr int M = MT * ZB_POL_NET;       /* envs per workgroup */
constexpr int NET = M / MT;              /* row tiles per workgroup */
constexpr int NWAVE = H / 16;            /* one wave per 16-unit tile */
constexpr int NTHR = 64 * NWAVE;
#ifndef ZB_POL_LDA
#define ZB_POL_LDA (M + 1)
#endif
constexpr int LDA = ZB_POL_LDA;  /* row stride of the [unit][env] layer tiles */
constexpr int LDU = M + 1;       /* row stride of the [k][env] observation tile */
constexpr int GH = H / 16;  /* 4-step (16-k) groups over K = H */
constexpr int NJ = ZB_POL_JOINTS;
constexpr int NMIX = ZB_POL_MIX;
#if ZB_POL_NET == 1
#define ZB_POL_OCC __attribute__((amdgpu_waves_per_eu(4, 4))) /* two workgroups per CU */
#else
#define ZB_POL_OCC
#endif
static_assert(NET == 1 || NET == 2, "one or two 16-env row tiles of v_mfma_f32_16x16x4_f32");

typedef float f32x4 __attribute__((ext_vector_type(4)));

/* env of accumulator register v in lane l of row tile et (16x16 f32 MFMA C/D map) */
__device__ __forceinline__ int crow(int et, int v, int l) { return MT * et + 4 * (l >> 4) + v; }

__device__ __forceinline__ f32x4 mma(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float q4(const float4& v, int u) {
  return u == 0 ? v.x : (u == 1 ? v.y : (u == 2 ? v.z : v.w));
}

/* one output tile (16 columns) of X[32][K] W^T over K = 16 * G for both row tiles, A from
   LDS; each weight fragment feeds both row tiles */
template <int LD>
__device__ __forceinline__ void tile_gemm(const float* xs, const float4* wp, int G, int lane, f32x4 acc[NET]) {
  const int c16 = lane & 15, k4 = lane >> 4;
#pragma unroll
  for (int et = 0; et < NET; ++et) acc[et] = f32x4{0.f, 0.f, 0.f, 0.f};
  float4 b = wp[0];
  for (int g = 0; g < G; ++g) {
    const float4 bn = wp[(size_t)(g + 1 < G ? g + 1 : g) * 64];
    __builtin_amdgcn_sched_barrier(0); /* next group's load stays a group ahead */
    const float* xp = xs + (16 * g + k4) * LD + c16;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int et = 0; et < NET; ++et) acc[et] = mma(xp[4 * u * LD + MT * et], q4(b, u), acc[et]);
    b = bn;
  }
}

/* PERSIST: the persistent T-step form (a0.T > 1), whose carries stay in registers between steps. The
   one-step form (T = 1) is its own instantiation, so it keeps no such registers: round 5's one kernel
   for both spilled in the one-step launches too (the critic 121 VGPRs; actor 19), round 6 splits it
   (one-step actor 0.111 -> 0.107 ms, critic 0.134 -> 0.111 ms at 8192 envs, no spills, the same bits;
   profiles/r06_p11_policy_ab.log). */
template <int KIN, int NOUT, bool ACTOR, bool PERSIST>
__global__ __launch_bounds__(NTHR) ZB_POL_OCC void policy_kernel(PolicyArgs a0) {
#pragma clang fp contract(off)
  constexpr int KPAD = (KIN + 15) / 16 * 16;
  constexpr int GIN = KPAD / 16;
  constexpr int NTO = (NOUT + 15) / 16;
  constexpr int OUTS = NOUT + 1;
  constexpr int XIN = KPAD * LDU;
  constexpr int OUTW = ACTOR ? M * OUTS : 1;
  constexpr int UW = XIN > OUTW ? XIN : OUTW;
  __shared__ float su[UW];          /* observation tile [k][env]; then the actor output [env][c] */
  __shared__ float sx[2][H * LDA];  /* layer input / output [unit][env], ping-pong */
  __shared__ float sh[H * LDA];     /* carry of the current layer [unit][env] */

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c16 = lane & 15, k4 = lane >> 4;
  const int e0 = blockIdx.x * M;
  const float4* wp4 = reinterpret_cast<const float4*>(a0.wpack);

  /* Persistent mode (a0.T > 1): one launch runs T steps of the recurrence. The
     carry of every layer stays in this thread's registers between steps, as the 8 (unit, env) pairs
     its GRU update writes (unit 16 w + c16, env crow(et, v, lane)); HBM sees the carry once on entry
     and once after the last step. Every product is the same k-ordered chain as one launch per step,
     so the results are the same bits. */
  const int TT = PERSIST && a0.T > 1 ? a0.T : 1;
  float hreg[D][NET][4];
#pragma unroll
  for (int l = 0; l < D; ++l)
#pragma unroll
    for (int et = 0; et < NET; ++et)
#pragma unroll
      for (int v = 0; v < 4; ++v) hreg[l][et][v] = 0.f;
  for (int t = 0; t < TT; ++t) {
  PolicyArgs a = a0;
  a.obs = a0.obs + (size_t)t * a0.n * KIN;
  a.reset = a0.reset ? a0.reset + (size_t)t * a0.n : nullptr;
  a.step = a0.step + (uint32_t)t;
  if (a0.actions) a.actions = a0.actions + (size_t)t * a0.n * NJ;
  if (a0.log_prob) a.log_prob = a0.log_prob + (size_t)t * a0.n * NJ;
  if (a0.value) a.value = a0.value + (size_t)t * a0.n;
  const bool last = t == TT - 1;

  constexpr int CPT = M * (H / 4) / NTHR;
  static_assert(CPT * NTHR == M * (H / 4), "carry float4s per thread");
  float4 cr[CPT];
  auto load_carry = [&](int l) {
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int i = tid + j * NTHR;
      const int e = i / (H / 4), q = i - e * (H / 4);
      const int ge = e0 + e;
      cr[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (ge < a.n && !(a.reset && a.reset[ge]))
        cr[j] = *reinterpret_cast<const float4*>(a.carry + ((size_t)ge * D + l) * H + 4 * q);
    }
  };
  if (t == 0) load_carry(0); /* layer 0's carry loads overlap the observation tile and input projection */

  /* 1. observation tile [k][env], zero-padded to KPAD. The block's 32 observation rows are one
        contiguous chunk of M * KIN floats: stream it with 16-B loads, all issued before the
        first LDS store (a load-then-store loop would wait out one HBM round trip per pass). */
  {
    constexpr int FL = M * KIN, NV4 = (FL + 3) / 4, PASSES = (NV4 + NTHR - 1) / NTHR;
    const int lim = (a.n - e0 < M ? a.n - e0 : M) * KIN; /* valid floats of this block */
    const float* src = a.obs + (size_t)e0 * KIN;
    if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) {
      float4 v[PASSES];
#pragma unroll
      for (int p = 0; p < PASSES; ++p) {
        const int i4 = tid + p * NTHR;
        v[p] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (4 * i4 + 3 < lim) {
          v[p] = reinterpret_cast<const float4*>(src)[i4];
        } else if (4 * i4 < lim) {
          v[p].x = src[4 * i4];
          if (4 * i4 + 1 < lim) v[p].y = src[4 * i4 + 1];
          if (4 * i4 + 2 < lim) v[p].z = src[4 * i4 + 2];
        }
      }
#pragma unroll
      for (int p = 0; p < PASSES; ++p) {
        const int i4 = tid + p * NTHR;
        const float c4[4] = {v[p].x, v[p].y, v[p].z, v[p].w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int f = 4 * i4 + c;
          if (f < FL) {
            const int e = f / KIN, k = f - e * KIN;
            su[k * LDU + e] = c4[c]; /* zero past the last env */
          }
        }
      }
    } else {
      for (int i = tid; i < FL; i += NTHR) {
        const int e = i / KIN, k = i - e * KIN;
        su[k * LDU + e] = i < lim ? src[i] : 0.f;
      }
    }
    for (int i = tid; i < M * (KPAD - KIN); i += NTHR) { /* padding rows k = KIN .. KPAD - 1 */
      const int k = KIN + i / M, e = i - (i / M) * M;
      su[k * LDU + e] = 0.f;
    }
  }
  __syncthreads();

  /* 2. input projection (no activation: train.py:944): the wave's unit tile */
  {
    const int unit = 16 * w + c16;
    f32x4 acc[NET];
    tile_gemm<LDU>(su, wp4 + (size_t)w * GIN * 64 + lane, GIN, lane, acc);
    const float bu = a.bias[unit];
#pragma unroll
    for (int et = 0; et < NET; ++et)
#pragma unroll
      for (int v = 0; v < 4; ++v) sx[0][unit * LDA + crow(et, v, lane)] = acc[et][v] + bu;
  }

  /* 3. GRU stack (train.py:945-948) */
  const size_t off_gru = (size_t)(H / 16) * GIN * 64;  /* float4 offset of layer 0's W_ih pack */
  constexpr size_t MAT = (size_t)(3 * H / 16) * GH * 64; /* one packed [3H][H] matrix, float4 */
  int cur = 0;
  for (int l = 0; l < D; ++l) {
    if (t == 0) {
      /* carry of layer l (prefetched during layer l - 1) -> sh */
#pragma unroll
      for (int j = 0; j < CPT; ++j) {
        const int i = tid + j * NTHR;
        const int e = i / (H / 4), q = i - e * (H / 4);
        sh[(4 * q) * LDA + e] = cr[j].x;
        sh[(4 * q + 1) * LDA + e] = cr[j].y;
        sh[(4 * q + 2) * LDA + e] = cr[j].z;
        sh[(4 * q + 3) * LDA + e] = cr[j].w;
      }
    } else {
      /* persistent: the previous step's carry from registers (zero where the episode restarts) */
      const int unit = 16 * w + c16;
#pragma unroll
      for (int et = 0; et < NET; ++et)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int e = crow(et, v, lane), ge = e0 + e;
          float hv = hreg[0][et][v];
#pragma unroll
          for (int k = 1; k < D; ++k) hv = l == k ? hreg[k][et][v] : hv;
          const bool rs = ge >= a.n || (a.reset && a.reset[ge]);
          sh[unit * LDA + e] = rs ? 0.f : hv;
        }
    }
    __syncthreads();
    if (t == 0 && l + 1 < D) load_carry(l + 1);

    const float4* wih = wp4 + off_gru + (size_t)l * 2 * MAT + lane;
    const float4* whh = wih + MAT;
    const float* xs = sx[cur];
    /* gate tiles of this wave's units: r = w, z = 8 + w, n = 16 + w */
    size_t to[3];
#pragma unroll
    for (int gt = 0; gt < 3; ++gt) to[gt] = (size_t)(8 * gt + w) * GH * 64;
    /* accumulators [gate][row tile] */
    f32x4 ia[3][NET], ha[3][NET];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int et = 0; et < NET; ++et) ia[i][et] = ha[i][et] = f32x4{0.f, 0.f, 0.f, 0.f};
    float4 bi[3], bh[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      bi[i] = wih[to[i]];
      bh[i] = whh[to[i]];
    }
    for (int g = 0; g < GH; ++g) {
      const size_t gn = (size_t)(g + 1 < GH ? g + 1 : g) * 64;
      float4 ni[3], nh[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        ni[i] = wih[to[i] + gn];
        nh[i] = whh[to[i] + gn];
      }
      /* keep the next group's loads here, a whole group (48 MFMAs) ahead of their use */
      __builtin_amdgcn_sched_barrier(0);
      const float* xp = xs + (16 * g + k4) * LDA + c16;
      const float* hp = sh + (16 * g + k4) * LDA + c16;
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int et = 0; et < NET; ++et) {
          const float ax = xp[4 * u * LDA + MT * et], ah = hp[4 * u * LDA + MT * et];
#pragma unroll
          for (int i = 0; i < 3; ++i) ia[i][et] = mma(ax, q4(bi[i], u), ia[i][et]);
#pragma unroll
          for (int i = 0; i < 3; ++i) ha[i][et] = mma(ah, q4(bh[i], u), ha[i][et]);
        }
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        bi[i] = ni[i];
        bh[i] = nh[i];
      }
    }
    /* equinox GRUCell: r, z, n gates; h' = n + z (h - n) */
    const float* bl = a.bias + H + (size_t)l * 4 * H;
    float* xo = sx[cur ^ 1];
    {
      const int unit = 16 * w + c16;
      const float br = bl[unit], bz = bl[H + unit], bni = bl[2 * H + unit], bnh = bl[3 * H + unit];
#pragma unroll
      for (int et = 0; et < NET; ++et)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int e = crow(et, v, lane);
        const float r = zbf_sigmoid((ia[0][et][v] + br) + ha[0][et][v]);
        const float z = zbf_sigmoid((ia[1][et][v] + bz) + ha[1][et][v]);
        const float nn = zbf_tanh((ia[2][et][v] + bni) + r * (ha[2][et][v] + bnh));
        const float ho = sh[unit * LDA + e];
        const float hv = nn + z * (ho - nn);
        xo[unit * LDA + e] = hv;
        if (last && e0 + e < a.n) a.carry[((size_t)(e0 + e) * D + l) * H + unit] = hv;
        if (TT > 1) {
#pragma unroll
          for (int k = 0; k < D; ++k) hreg[k][et][v] = l == k ? hv : hreg[k][et][v];
        }
      }
    }
    __syncthreads();
    cur ^= 1;
  }

  /* 4. heads */
  const float* xs = sx[cur];
  const float* tail = a.bias + H + (size_t)D * 4 * H; /* output bias [NOUT], then head constants */
  if constexpr (ACTOR) {
    /* output projection (train.py:950) into su[env][c] */
    const float4* wo = wp4 + off_gru + (size_t)D * 2 * MAT + lane;
    for (int nt = w; nt < NTO; nt += NWAVE) {
      f32x4 acc[NET];
      tile_gemm<LDA>(xs, wo + (size_t)nt * GH * 64, GH, lane, acc);
      const int c = nt * 16 + c16;
      if (c < NOUT) {
        const float bc = tail[c];
#pragma unroll
        for (int et = 0; et < NET; ++et)
#pragma unroll
          for (int v = 0; v < 4; ++v) su[crow(et, v, lane) * OUTS + c] = acc[et][v] + bc;
      }
    }
    __syncthreads();
    /* mixture head per (env, joint) (train.py:952-965) */
    const float* mean_bias = tail + NOUT;
    for (int it = tid; it < M * NJ; it += NTHR) {
      const int e = it / NJ, j = it - e * NJ, ge = e0 + e;
      if (ge >= a.n) continue;
      const float* o = su + e * OUTS;
      float mu[NMIX], sd[NMIX], lg[NMIX];
#pragma unroll
      for (int m = 0; m < NMIX; ++m) {
        mu[m] = o[j * NMIX + m] + mean_bias[j];
        const float s = (zbf_softplus(o[NJ * NMIX + j * NMIX + m]) + 0.01f) * 1.0f;
        sd[m] = s < 1.0f ? s : 1.0f;
        lg[m] = o[2 * NJ * NMIX + j * NMIX + m];
      }
      const size_t ai = (size_t)ge * NJ + j;
      float act;
      if (a.mode == ZB_POL_EVAL) {
        act = a.actions[ai];
      } else {
        act = zbf_mix_sample(mu, sd, lg, a.mode == ZB_POL_MODE, a.seed, ZB_RNG_POLICY, (uint32_t)j,
                             (uint32_t)(NJ + j), (uint32_t)(a.env_offset + ge), a.step);
        a.actions[ai] = act;
      }
      if (a.log_prob) a.log_prob[ai] = zbf_mix_log_prob(mu, sd, lg, act);
    }
  } else {
    /* value head (train.py:1017): one fmaf chain per env, natural-layout W_out */
    if (tid < M && e0 + tid < a.n) {
      const float* wo = tail + NOUT;
      float acc = 0.f;
      for (int k = 0; k < H; ++k) acc = fmaf(xs[k * LDA + tid], wo[k], acc);
      a.value[e0 + tid] = acc + tail[0];
    }
  }
  __syncthreads(); /* the heads' LDS reads are done before the next step's tiles overwrite them */
  }  /* t */
}

/* ---------------------------------------------------------------------------------------------
 * One-wave layout (policy_wave_kernel): a workgroup is ONE wave over 16 envs (one row tile) that
 * runs every unit tile of every layer itself. It is sized to take the slot of one step-kernel wave
 * (<= 256 VGPRs, <= 20 KB of LDS), so its waves can start in the slots a step launch frees as it
 * drains instead of waiting for whole CUs. The A operands of a layer (its input
 * and the carry) are held in registers in the MFMA A layout, 32 values a lane for K = 128; the
 * layer's outputs go through one [unit][env] LDS tile back into that layout. Every product is the
 * same k-ordered chain from 0 as in policy_kernel, and the epilogue and heads are the same code, so
 * the two layouts are bit-identical.
 * ------------------------------------------------------------------------------------------- */
constexpr int WM = 16;       /* envs per one-wave workgroup */
constexpr int WLDA = WM + 1; /* row stride of the [unit][env] tile */

/* wave priority of the slot-sized kernels, which share CUs with step waves in an actor-in-the-loop
   rollout (diagnostic knob; 0 = the hardware default) */
#ifndef ZB_POLWAVE_PRIO
#define ZB_POLWAVE_PRIO 0
#endif
template <int KIN, int NOUT, bool ACTOR, int NWV>
__global__ __launch_bounds__(64 * NWV, 2) void policy_wave_kernel(PolicyArgs a) {
#pragma clang fp contract(off)
  if constexpr (ZB_POLWAVE_PRIO > 0) __builtin_amdgcn_s_setprio(ZB_POLWAVE_PRIO);
  constexpr int KPAD = (KIN + 15) / 16 * 16;
  constexpr int GIN = KPAD / 16;
  constexpr int NTO = (NOUT + 15) / 16;
  constexpr int OUTS = NOUT + 1;
  constexpr int TW = H * WLDA;                          /* [unit][env] tile */
  constexpr int OW = ACTOR ? WM * OUTS : 1;             /* actor output [env][c] */
  constexpr int SW = 2 * TW > OW ? 2 * TW : OW;
  __shared__ float st[SW]; /* layer output tile, then the old carry tile; the actor output after */
  static_assert(SW * 4 <= 20 * 1024, "one step-wave slot of LDS");
  float* const so = st + TW;

  /* NWV waves (1 or 2) share the 16 envs: wave v takes the unit tiles v, v + NWV, ... */
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, c16 = lane & 15, k4 = lane >> 4;
  const int e0 = blockIdx.x * WM;
  const int ge_a = e0 + c16; /* env of this lane's A operands */
  const bool va = ge_a < a.n;
  const float4* wp4 = reinterpret_cast<const float4*>(a.wpack);

  /* 1. input projection: A = observation values k = 16 g + 4 u + k4 of env c16, in registers */
  float xa[4 * GIN];
  {
    const float* src = a.obs + (size_t)ge_a * KIN;
#pragma unroll
    for (int i = 0; i < 4 * GIN; ++i) {
      const int k = 4 * i + k4; /* i = 4 g + u */
      xa[i] = (va && k < KIN) ? src[k] : 0.f;
    }
  }
  float xr[4 * GH]; /* the current layer's input in A layout */
  for (int w = wv; w < NWAVE; w += NWV) {
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    const float4* wp = wp4 + (size_t)w * GIN * 64 + lane;
    float4 b = wp[0];
#pragma unroll
    for (int g = 0; g < GIN; ++g) {
      const float4 bn = wp[(size_t)(g + 1 < GIN ? g + 1 : g) * 64];
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc = mma(xa[4 * g + u], q4(b, u), acc);
      b = bn;
    }
    const int unit = 16 * w + c16;
    const float bu = a.bias[unit];
#pragma unroll
    for (int v = 0; v < 4; ++v) st[unit * WLDA + crow(0, v, lane)] = acc[v] + bu;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4 * GH; ++i) xr[i] = st[(4 * i + k4) * WLDA + c16];
  __syncthreads();

  /* 2. GRU stack */
  const size_t off_gru = (size_t)(H / 16) * GIN * 64;
  constexpr size_t MAT = (size_t)(3 * H / 16) * GH * 64;
  for (int l = 0; l < D; ++l) {
    float hr[4 * GH]; /* carry of layer l in A layout */
    {
      const bool live = va && !(a.reset && a.reset[ge_a]);
      const float* cp = a.carry + ((size_t)ge_a * D + l) * H;
#pragma unroll
      for (int i = 0; i < 4 * GH; ++i) hr[i] = live ? cp[4 * i + k4] : 0.f;
      /* and in [unit][env] for the GRU update's old carry */
#pragma unroll
      for (int i = 0; i < 4 * GH; ++i)
        if (wv == 0) so[(4 * i + k4) * WLDA + c16] = hr[i];
      __syncthreads();
    }
    const float4* wih = wp4 + off_gru + (size_t)l * 2 * MAT + lane;
    const float4* whh = wih + MAT;
    const float* bl = a.bias + H + (size_t)l * 4 * H;
    for (int w = wv; w < NWAVE; w += NWV) {
      size_t to[3];
#pragma unroll
      for (int gt = 0; gt < 3; ++gt) to[gt] = (size_t)(8 * gt + w) * GH * 64;
      f32x4 ia[3], ha[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) ia[i] = ha[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      float4 bi[3], bh[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        bi[i] = wih[to[i]];
        bh[i] = whh[to[i]];
      }
#pragma unroll
      for (int g = 0; g < GH; ++g) {
        /* the next group's fragments are loaded a whole group (24 MFMAs) ahead of their use */
        float4 ni[3], nh[3];
        const size_t gn = (size_t)(g + 1 < GH ? g + 1 : g) * 64;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          ni[i] = wih[to[i] + gn];
          nh[i] = whh[to[i] + gn];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
          for (int i = 0; i < 3; ++i) ia[i] = mma(xr[4 * g + u], q4(bi[i], u), ia[i]);
#pragma unroll
          for (int i = 0; i < 3; ++i) ha[i] = mma(hr[4 * g + u], q4(bh[i], u), ha[i]);
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          bi[i] = ni[i];
          bh[i] = nh[i];
        }
      }
      const int unit = 16 * w + c16;
      const float br = bl[unit], bz = bl[H + unit], bni = bl[2 * H + unit], bnh = bl[3 * H + unit];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int e = crow(0, v, lane), ge = e0 + e;
        const float r = zbf_sigmoid((ia[0][v] + br) + ha[0][v]);
        const float z = zbf_sigmoid((ia[1][v] + bz) + ha[1][v]);
        const float nn = zbf_tanh((ia[2][v] + bni) + r * (ha[2][v] + bnh));
        const float ho = so[unit * WLDA + e]; /* the old carry of (env e, unit) */
        const float hv = nn + z * (ho - nn);
        st[unit * WLDA + e] = hv;
        if (ge < a.n) a.carry[((size_t)ge * D + l) * H + unit] = hv;
      }
    }
    __syncthreads();
    if (l + 1 < D || ACTOR) {
#pragma unroll
      for (int i = 0; i < 4 * GH; ++i) xr[i] = st[(4 * i + k4) * WLDA + c16];
      __syncthreads();
    }
  }

  /* 3. heads */
  const float* tail = a.bias + H + (size_t)D * 4 * H;
  if constexpr (ACTOR) {
    const float4* wo = wp4 + off_gru + (size_t)D * 2 * MAT + lane;
    for (int nt = wv; nt < NTO; nt += NWV) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
      const float4* wt = wo + (size_t)nt * GH * 64;
      float4 b = wt[0];
#pragma unroll
      for (int g = 0; g < GH; ++g) {
        const float4 bn = wt[(size_t)(g + 1 < GH ? g + 1 : g) * 64];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc = mma(xr[4 * g + u], q4(b, u), acc);
        b = bn;
      }
      const int c = nt * 16 + c16;
      if (c < NOUT) {
        const float bc = tail[c];
#pragma unroll
        for (int v = 0; v < 4; ++v) st[crow(0, v, lane) * OUTS + c] = acc[v] + bc;
      }
    }
    __syncthreads();
    const float* mean_bias = tail + NOUT;
    for (int it = tid; it < WM * NJ; it += 64 * NWV) {
      const int e = it / NJ, j = it - e * NJ, ge = e0 + e;
      if (ge >= a.n) continue;
      const float* o = st + e * OUTS;
      float mu[NMIX], sd[NMIX], lg[NMIX];
#pragma unroll
      for (int m = 0; m < NMIX; ++m) {
        mu[m] = o[j * NMIX + m] + mean_bias[j];
        const float s = (zbf_softplus(o[NJ * NMIX + j * NMIX + m]) + 0.01f) * 1.0f;
        sd[m] = s < 1.0f ? s : 1.0f;
        lg[m] = o[2 * NJ * NMIX + j * NMIX + m];
      }
      const size_t ai = (size_t)ge * NJ + j;
      float act;
      if (a.mode == ZB_POL_EVAL) {
        act = a.actions[ai];
      } else {
        act = zbf_mix_sample(mu, sd, lg, a.mode == ZB_POL_MODE, a.seed, ZB_RNG_POLICY, (uint32_t)j,
                             (uint32_t)(NJ + j), (uint32_t)(a.env_offset + ge), a.step);
        a.actions[ai] = act;
      }
      if (a.log_prob) a.log_prob[ai] = zbf_mix_log_prob(mu, sd, lg, act);
    }
  } else {
    /* value head: one fmaf chain per env over the [unit][env] tile of the last layer */
    if (tid < WM && e0 + tid < a.n) {
      const float* wo = tail + NOUT;
      float acc = 0.f;
      for (int k = 0; k < H; ++k) acc = fmaf(st[k * WLDA + tid], wo[k], acc);
      a.value[e0 + tid] = acc + tail[0];
    }
  }
}

}  // namespace pol

hipError_t launch_policy(int kind, const PolicyArgs& a, hipStream_t s) {
  if (a.n <= 0) return hipSuccess;
  if (a.layout == ZB_POL_LAYOUT_WAVE || a.layout == ZB_POL_LAYOUT_WAVE2 || a.layout == ZB_POL_LAYOUT_WAVE4) {
    const int nw = (a.n + pol::WM - 1) / pol::WM;
    if (a.layout == ZB_POL_LAYOUT_WAVE4) {
      if (kind == ZB_POL_ACTOR)
        hipLaunchKernelGGL((pol::policy_wave_kernel<ZB_POL_ACTOR_IN, ZB_POL_ACTOR_OUT, true, 4>), dim3(nw), dim3(256),
                           0, s, a);
      else
        hipLaunchKernelGGL((pol::policy_wave_kernel<ZB_POL_CRITIC_IN, 1, false, 4>), dim3(nw), dim3(256), 0, s, a);
    } else if (a.layout == ZB_POL_LAYOUT_WAVE) {
      if (kind == ZB_POL_ACTOR)
        hipLaunchKernelGGL((pol::policy_wave_kernel<ZB_POL_ACTOR_IN, ZB_POL_ACTOR_OUT, true, 1>), dim3(nw), dim3(64), 0,
                           s, a);
      else
        hipLaunchKernelGGL((pol::policy_wave_kernel<ZB_POL_CRITIC_IN, 1, false, 1>), dim3(nw), dim3(64), 0, s, a);
    } else {
      if (kind == ZB_POL_ACTOR)
        hipLaunchKernelGGL((pol::policy_wave_kernel<ZB_POL_ACTOR_IN, ZB_POL_ACTOR_OUT, true, 2>), dim3(nw), dim3(128),
                           0, s, a);
      else
        hipLaunchKernelGGL((pol::policy_wave_kernel<ZB_POL_CRITIC_IN, 1, false, 2>), dim3(nw), dim3(128), 0, s, a);
    }
    return hipGetLastError();
  }
  const int nblk = (a.n + pol::M - 1) / pol::M;
  const bool persist = a.T > 1;
  if (kind == ZB_POL_ACTOR) {
    if (persist)
      hipLaunchKernelGGL((pol::policy_kernel<ZB_POL_ACTOR_IN, ZB_POL_ACTOR_OUT, true, true>), dim3(nblk),
                         dim3(pol::NTHR), 0, s, a);
    else
      hipLaunchKernelGGL((pol::policy_kernel<ZB_POL_ACTOR_IN, ZB_POL_ACTOR_OUT, true, false>), dim3(nblk),
                         dim3(pol::NTHR), 0, s, a);
  } else {
    if (persist)
      hipLaunchKernelGGL((pol::policy_kernel<ZB_POL_CRITIC_IN, 1, false, true>), dim3(nblk), dim3(pol::NTHR), 0, s, a);
    else
      hipLaunchKernelGGL((pol::policy_kernel<ZB_POL_CRITIC_IN, 1, false, false>), dim3(nblk), dim3(pol::NTHR), 0, s,
                         a);
  }
  return hipGetLastError();
}

}  // namespace zb
