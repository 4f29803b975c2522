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
 *   workgroup = 32 envs (the M = 32 tile of v_mfma_f32_32x32x2_f32) x 4 waves;
 *   wave w owns hidden units 32w .. 32w+31 of every layer, so the r / z / n
 *   gates of a unit land in the same lane and the GRU update happens in
 *   registers: per layer 6 accumulators (W_ih x and W_hh h for r, z, n),
 *   K = 128 in 64 MFMA steps each.
 *   A operands (activations) live in LDS k-major, [k][env] with a 33-float
 *   row stride: one ds_read_b32 per operand per step, conflict-free.
 *   B operands (weights) are pre-packed on the host in fragment order —
 *   [tile][group of 4 k-steps][lane][4] — so each lane streams one 16-B load
 *   per 4 MFMA steps per matrix; every workgroup reads the whole weight set
 *   (2.0 MB actor, 2.2 MB critic), which stays L2-resident across the chip.
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
constexpr int M = ZB_POL_ENVS_PER_BLOCK; /* envs per workgroup: the MFMA M tile */
constexpr int NWAVE = H / 32;            /* one wave per 32 hidden units */
constexpr int NTHR = 64 * NWAVE;
constexpr int LDA = M + 1;  /* row stride of the [k][env] activation tiles */
constexpr int GH = H / 8;   /* 4-step (8-k) groups over K = H */
constexpr int NJ = ZB_POL_JOINTS;
constexpr int NMIX = ZB_POL_MIX;

typedef float f32x16 __attribute__((ext_vector_type(16)));

/* env row of accumulator register i in lane l (32x32 f32 MFMA C/D map) */
__device__ __forceinline__ int crow(int i, int l) { return (i & 3) + 8 * (i >> 2) + 4 * (l >> 5); }

__device__ __forceinline__ f32x16 mma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float q4(const float4& v, int u) {
  return u == 0 ? v.x : (u == 1 ? v.y : (u == 2 ? v.z : v.w));
}

/* one output tile (32 columns) of X[32][K] W^T over K = 8 * G, A from LDS */
__device__ __forceinline__ f32x16 tile_gemm(const float* xs, const float4* wp, int G, int lane) {
  const int c32 = lane & 31, h2 = lane >> 5;
  f32x16 acc = {};
  float4 b = wp[0];
  for (int g = 0; g < G; ++g) {
    const float4 bn = wp[(size_t)(g + 1 < G ? g + 1 : g) * 64];
    __builtin_amdgcn_sched_barrier(0); /* next group's load stays a group ahead */
    const float* xp = xs + (8 * g + h2) * LDA + c32;
#pragma unroll
    for (int u = 0; u < 4; ++u) acc = mma(xp[2 * u * LDA], q4(b, u), acc);
    b = bn;
  }
  return acc;
}

template <int KIN, int NOUT, bool ACTOR>
__global__ __launch_bounds__(NTHR) void policy_kernel(PolicyArgs a) {
#pragma clang fp contract(off)
  constexpr int KPAD = (KIN + 7) / 8 * 8;
  constexpr int GIN = KPAD / 8;
  constexpr int NTO = (NOUT + 31) / 32;
  constexpr int OUTS = NOUT + 1;
  constexpr int XIN = KPAD * LDA;
  constexpr int OUTW = ACTOR ? M * OUTS : 1;
  constexpr int UW = XIN > OUTW ? XIN : OUTW;
  __shared__ float su[UW];          /* observation tile [k][env]; then the actor output [env][c] */
  __shared__ float sx[2][H * LDA];  /* layer input / output [unit][env], ping-pong */
  __shared__ float sh[H * LDA];     /* carry of the current layer [unit][env] */

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c32 = lane & 31, h2 = lane >> 5;
  const int e0 = blockIdx.x * M;
  const int unit = 32 * w + c32;
  const float4* wp4 = reinterpret_cast<const float4*>(a.wpack);

  constexpr int CPT = M * (H / 4) / NTHR;
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
  load_carry(0); /* layer 0's carry loads overlap the observation tile and input projection */

  /* 1. observation tile [k][env], zero-padded to KPAD. The block's 32 observation rows are one
        contiguous chunk of M * KIN floats: stream it with 16-B loads, all issued before the
        first LDS store (a load-then-store loop would wait out one HBM round trip per pass:
        61 passes for the critic's 484 features). */
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
            su[k * LDA + e] = c4[c]; /* zero past the last env */
          }
        }
      }
    } else {
      for (int i = tid; i < FL; i += NTHR) {
        const int e = i / KIN, k = i - e * KIN;
        su[k * LDA + e] = i < lim ? src[i] : 0.f;
      }
    }
    for (int i = tid; i < M * (KPAD - KIN); i += NTHR) { /* padding rows k = KIN .. KPAD - 1 */
      const int k = KIN + i / M, e = i - (i / M) * M;
      su[k * LDA + e] = 0.f;
    }
  }
  __syncthreads();

  /* 2. input projection (no activation: train.py:944) */
  {
    const f32x16 acc = tile_gemm(su, wp4 + (size_t)w * GIN * 64 + lane, GIN, lane);
    const float bu = a.bias[unit];
#pragma unroll
    for (int i = 0; i < 16; ++i) sx[0][unit * LDA + crow(i, lane)] = acc[i] + bu;
  }

  /* 3. GRU stack (train.py:945-948) */
  const size_t off_gru = (size_t)(H / 32) * GIN * 64;  /* float4 offset of layer 0's W_ih pack */
  constexpr size_t MAT = (size_t)12 * GH * 64;         /* one packed [3H][H] matrix, float4 */
  int cur = 0;
  for (int l = 0; l < D; ++l) {
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
    __syncthreads();
    if (l + 1 < D) load_carry(l + 1);

    const float4* wih = wp4 + off_gru + (size_t)l * 2 * MAT + lane;
    const float4* whh = wih + MAT;
    const float* xs = sx[cur];
    /* gate tiles of this wave's units: r = w, z = 4 + w, n = 8 + w */
    const size_t tr = (size_t)w * GH * 64, tz = (size_t)(4 + w) * GH * 64, tn = (size_t)(8 + w) * GH * 64;
    f32x16 ir = {}, iz = {}, in = {}, hr = {}, hz = {}, hn = {};
    float4 b0 = wih[tr], b1 = wih[tz], b2 = wih[tn], b3 = whh[tr], b4 = whh[tz], b5 = whh[tn];
    for (int g = 0; g < GH; ++g) {
      const size_t gn = (size_t)(g + 1 < GH ? g + 1 : g) * 64;
      const float4 n0 = wih[tr + gn], n1 = wih[tz + gn], n2 = wih[tn + gn];
      const float4 n3 = whh[tr + gn], n4 = whh[tz + gn], n5 = whh[tn + gn];
      /* keep the next group's loads here, a whole group (24 MFMAs) ahead of their use: the
         fully unrolled loop otherwise lets the scheduler sink them next to their first MFMA */
      __builtin_amdgcn_sched_barrier(0);
      const float* xp = xs + (8 * g + h2) * LDA + c32;
      const float* hp = sh + (8 * g + h2) * LDA + c32;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float ax = xp[2 * u * LDA], ah = hp[2 * u * LDA];
        ir = mma(ax, q4(b0, u), ir);
        iz = mma(ax, q4(b1, u), iz);
        in = mma(ax, q4(b2, u), in);
        hr = mma(ah, q4(b3, u), hr);
        hz = mma(ah, q4(b4, u), hz);
        hn = mma(ah, q4(b5, u), hn);
      }
      b0 = n0; b1 = n1; b2 = n2; b3 = n3; b4 = n4; b5 = n5;
    }
    /* equinox GRUCell: r, z, n gates; h' = n + z (h - n) */
    const float* bl = a.bias + H + (size_t)l * 4 * H;
    const float br = bl[unit], bz = bl[H + unit], bni = bl[2 * H + unit], bnh = bl[3 * H + unit];
    float* xo = sx[cur ^ 1];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int e = crow(i, lane);
      const float r = zbf_sigmoid((ir[i] + br) + hr[i]);
      const float z = zbf_sigmoid((iz[i] + bz) + hz[i]);
      const float nn = zbf_tanh((in[i] + bni) + r * (hn[i] + bnh));
      const float ho = sh[unit * LDA + e];
      const float hv = nn + z * (ho - nn);
      xo[unit * LDA + e] = hv;
      if (e0 + e < a.n) a.carry[((size_t)(e0 + e) * D + l) * H + unit] = hv;
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
      const f32x16 acc = tile_gemm(xs, wo + (size_t)nt * GH * 64, GH, lane);
      const int c = nt * 32 + c32;
      if (c < NOUT) {
        const float bc = tail[c];
#pragma unroll
        for (int i = 0; i < 16; ++i) su[crow(i, lane) * OUTS + c] = acc[i] + bc;
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
}

}  // namespace pol

hipError_t launch_policy(int kind, const PolicyArgs& a, hipStream_t s) {
  if (a.n <= 0) return hipSuccess;
  const int nblk = (a.n + pol::M - 1) / pol::M;
  if (kind == ZB_POL_ACTOR)
    hipLaunchKernelGGL((pol::policy_kernel<ZB_POL_ACTOR_IN, ZB_POL_ACTOR_OUT, true>), dim3(nblk), dim3(pol::NTHR), 0,
                       s, a);
  else
    hipLaunchKernelGGL((pol::policy_kernel<ZB_POL_CRITIC_IN, 1, false>), dim3(nblk), dim3(pol::NTHR), 0, s, a);
  return hipGetLastError();
}

}  // namespace zb
