/*
 * zb_ppo.hip — post-rollout PPO inputs on MI355X:
 * GAE reverse scan, value targets, batch moments and advantage
 * normalization over a [T, n] rollout. C ABI: include/zbot_ppo.h.
 *
 * Reference: ksim 0.1.99 PPOTask's `compute_ppo_inputs` (un-vendored
 * ksim/task/ppo.py [U]) over the rewards/dones of the rollout and the critic
 * values of get_ppo_variables (train.py:1683-1729). The CPU restatement is
 * oracle/zb_oracle_ppo.c; results are bit-identical to it.
 *
 * The path is HBM-bound (9 B read + 8 B written per (t, env), no reuse):
 *
 *   gae_kernel   one workgroup = 32 envs (one 128-B row) x 64 rows in flight
 *                (512 threads). For each 256-step segment, latest first:
 *                  1. every thread streams in 4 rows x 4 envs with 16-B loads
 *                     (reward, value; done/success as one 4-byte word),
 *                     values go to LDS;
 *                  2. delta_t and c_t = gamma*lam*mask_t are formed in
 *                     parallel (next value from the LDS row below) into LDS;
 *                  3. one lane per env runs the exact serial recurrence
 *                     gae_t = fma(c_t, gae_{t+1}, delta_t) out of LDS — one
 *                     FMA on the dependency chain per step, the same
 *                     operation order as the reference scan, hence bit-exact;
 *                  4. all threads stream gae and value targets back out with
 *                     16-B stores and form fp64 moment partials: per thread
 *                     over its 4 rows, a pairwise tree over the 8 row groups
 *                     of a wave (lane shuffles), summed per wave over
 *                     segments; at the end a pairwise tree over the 8 waves.
 *   moments      per-env (sum, sum^2) -> pairwise tree over the 32 envs of a
 *                block -> per-block partials -> pairwise tree over blocks
 *                (zb_moments_combine / the tail of zb_gae). Zero padding to a
 *                power of two keeps every level a perfect binary tree, so
 *                rank-order combining reproduces the one-GPU bits.
 *   normalize    grid-stride float4 stream, IEEE division.
 */
#include <hip/hip_runtime.h>

#include "zb_internal.h"

namespace zb {

constexpr int GE = ZB_GAE_ENVS_PER_BLOCK; /* envs per workgroup (32: a 128-B row) */
constexpr int GQ = GE / 4;                /* 16-B env quads per row */
constexpr int GR = 64;                    /* rows in flight per pass */
constexpr int GJ = 4;                     /* passes per segment */
constexpr int GSEG = GR * GJ;             /* rows (time steps) per segment: 256 */
constexpr int GTHREADS = GR * GQ;         /* 512 */
constexpr int MTREE = 1024;               /* leaves per level of the moment tree */


/* Pairwise sum over a power-of-two LDS array of (s1, s2) pairs, in place;
   the root lands in element 0. Threads: blockDim.x, all participate. */
template <int N>
__device__ inline void tree_pairs(double* s1, double* s2) {
#pragma unroll
  for (int s = 1; s < N; s <<= 1) {
    __syncthreads();
    for (int i = threadIdx.x * 2 * s; i < N; i += blockDim.x * 2 * s) {
      s1[i] = s1[i] + s1[i + s];
      s2[i] = s2[i] + s2[i + s];
    }
  }
  __syncthreads();
}

/* 4 consecutive envs of one row: a float4 when the row is 16-B aligned and all
   4 envs exist (VEC instantiation), scalar loads otherwise */
template <bool VEC>
__device__ inline void ld4(const float* p, size_t i, int nv, float o[4]) {
  if (VEC) {
    const float4 v = *reinterpret_cast<const float4*>(p + i);
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = k < nv ? p[i + k] : 0.f;
  }
}
template <bool VEC>
__device__ inline uint32_t ld4u8(const uint8_t* p, size_t i, int nv) {
  if (!p) return 0u;
  if (VEC) return *reinterpret_cast<const uint32_t*>(p + i);
  uint32_t w = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) w |= (k < nv ? (uint32_t)p[i + k] : 0u) << (8 * k);
  return w;
}
template <bool VEC>
__device__ inline void st4(float* p, size_t i, int nv, const float o[4]) {
  if (VEC) {
    *reinterpret_cast<float4*>(p + i) = make_float4(o[0], o[1], o[2], o[3]);
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < nv) p[i + k] = o[k];
  }
}

template <bool VEC>
__global__ __launch_bounds__(GTHREADS) void gae_kernel(GaeArgs a) {
#pragma clang fp contract(off)
  __shared__ float2 sdc[GSEG][GE];   /* (delta_t, c_t); then the fp64 moment exchange */
  __shared__ float sv[GSEG + 1][GE]; /* values_t (+ next-segment value row); then gae_t */

  const int tid = threadIdx.x;
  const int q = tid % GQ;  /* env quad of this thread */
  const int r0 = tid / GQ; /* first row of this thread (rows r0 + GR*j) */
  const int e0 = blockIdx.x * GE;
  const int eq = e0 + 4 * q;
  const int nvq = min(4, a.n - eq); /* VEC: n % 4 == 0, so 4 or <= 0 */
  const size_t n = (size_t)a.n;
  const int nseg = (a.T + GSEG - 1) / GSEG;

  float carry = 0.f;  /* gae at the first row of the later segment (scan lanes) */
  float vcarry = 0.f; /* value at the first row of the later segment (scan lanes) */
  double S1[4] = {0.0, 0.0, 0.0, 0.0}, S2[4] = {0.0, 0.0, 0.0, 0.0}; /* per-env moments (r0 == 0) */

  for (int sg = nseg - 1; sg >= 0; --sg) {
    const int tbase = sg * GSEG;
    const int tl = min(GSEG, a.T - tbase);

    /* 1. stream this thread's rows in: 16-B loads of 4 envs, all independent */
    float rr[GJ][4], vv[GJ][4];
    uint32_t dn[GJ], sc[GJ];
#pragma unroll
    for (int j = 0; j < GJ; ++j) {
      const int row = r0 + GR * j;
      if (row < tl && nvq > 0) {
        const size_t i = (size_t)(tbase + row) * n + eq;
        ld4<VEC>(a.reward, i, nvq, rr[j]);
        ld4<VEC>(a.values, i, nvq, vv[j]);
        dn[j] = ld4u8<VEC>(a.done, i, nvq);
        sc[j] = ld4u8<VEC>(a.success, i, nvq);
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) rr[j][k] = vv[j][k] = 0.f;
        dn[j] = sc[j] = 0u;
      }
    }
#pragma unroll
    for (int j = 0; j < GJ; ++j) {
      const int row = r0 + GR * j;
      if (row < tl) {
#pragma unroll
        for (int k = 0; k < 4; ++k) sv[row][4 * q + k] = vv[j][k];
      }
    }
    if (tid < GE) {
      /* next value of the segment's last row: the bootstrap (or the last value) at the
         end of the rollout, else the first value of the later segment */
      float vn = vcarry;
      const int e = e0 + tid;
      if (sg == nseg - 1)
        vn = e < a.n ? (a.bootstrap ? a.bootstrap[e] : a.values[(size_t)(a.T - 1) * n + e]) : 0.f;
      sv[tl][tid] = vn;
    }
    __syncthreads();

    /* 2. delta_t and c_t = gamma*lam*mask_t, fully parallel */
#pragma unroll
    for (int j = 0; j < GJ; ++j) {
      const int row = r0 + GR * j;
      if (row < tl) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float mask = ((dn[j] >> (8 * k)) & 0xffu) ? 0.f : 1.f;
          const float vs = sv[row + 1][4 * q + k];
          const float nxt = ((sc[j] >> (8 * k)) & 0xffu) ? vv[j][k] : vs * mask;
          const float gn = a.gamma * nxt;
          sdc[row][4 * q + k] = make_float2((rr[j][k] + gn) - vv[j][k], a.gl * mask);
        }
      }
    }
    __syncthreads();

    /* 3. the exact serial reverse scan, one lane per env: one FMA per step on the
          chain (the unrolled loop keeps 8 steps of LDS reads in flight; a deeper
          software pipeline measured 6 us slower, scripts/gae_variants.py) */
    if (tid < GE) {
      vcarry = sv[0][tid];
      float g = carry;
#pragma unroll 8
      for (int k = tl - 1; k >= 0; --k) {
        const float2 dc = sdc[k][tid];
        g = __builtin_fmaf(dc.y, g, dc.x);
        sv[k][tid] = g;
      }
      carry = g;
    }
    __syncthreads();

    /* 4. stream gae and value targets out; moment partials over this thread's rows */
    double p1[4] = {0.0, 0.0, 0.0, 0.0}, p2[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int j = GJ - 1; j >= 0; --j) {
      const int row = r0 + GR * j;
      if (row < tl && nvq > 0) {
        float g4[4], t4[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          g4[k] = sv[row][4 * q + k];
          t4[k] = g4[k] + vv[j][k];
          if (VEC || k < nvq) {
            const double gd = (double)g4[k];
            p1[k] = p1[k] + gd;
            p2[k] = p2[k] + gd * gd;
          }
        }
        const size_t i = (size_t)(tbase + row) * n + eq;
        st4<VEC>(a.gae, i, nvq, g4);
        if (a.vtarget) st4<VEC>(a.vtarget, i, nvq, t4);
      }
    }

    /* 5. per-env segment moments: pairwise tree over the 8 row groups of this wave
          (lanes 8 / 16 / 32 apart, no barrier), accumulated per wave over segments */
    if (a.partials) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
#pragma unroll
        for (int d = GQ; d < 64; d <<= 1) {
          p1[k] = p1[k] + __shfl_down(p1[k], d);
          p2[k] = p2[k] + __shfl_down(p2[k], d);
        }
        S1[k] = S1[k] + p1[k]; /* meaningful in lanes 0..7 of each wave */
        S2[k] = S2[k] + p2[k];
      }
    }
    __syncthreads(); /* sdc / sv are rewritten by the next segment */
  }

  if (a.partials) {
    /* per env: pairwise tree over the 8 waves' sums; then over the 32 envs */
    constexpr int NW = GTHREADS / 64;
    double* w1 = reinterpret_cast<double*>(&sdc[0][0]); /* [NW][GE] */
    double* w2 = w1 + NW * GE;
    double* m1 = w2 + NW * GE; /* [GE] */
    double* m2 = m1 + GE;
    const int lane = tid % 64, w = tid / 64;
    if (lane < GQ) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        w1[w * GE + 4 * lane + k] = S1[k];
        w2[w * GE + 4 * lane + k] = S2[k];
      }
    }
    __syncthreads();
    if (tid < GE) {
      double x1[NW], x2[NW];
#pragma unroll
      for (int i = 0; i < NW; ++i) {
        x1[i] = w1[i * GE + tid];
        x2[i] = w2[i * GE + tid];
      }
#pragma unroll
      for (int st = 1; st < NW; st <<= 1)
#pragma unroll
        for (int i = 0; i + st < NW; i += 2 * st) {
          x1[i] = x1[i] + x1[i + st];
          x2[i] = x2[i] + x2[i + st];
        }
      const bool live = e0 + tid < a.n;
      m1[tid] = live ? x1[0] : 0.0;
      m2[tid] = live ? x2[0] : 0.0;
    }
    tree_pairs<GE>(m1, m2);
    if (tid == 0) {
      a.partials[2 * blockIdx.x] = m1[0];
      a.partials[2 * blockIdx.x + 1] = m2[0];
    }
  }
}

/* One workgroup: pairwise tree over k pairs, zero-padded; groups of MTREE
   leaves are reduced first, then the group roots (k <= MTREE*MTREE). */
__global__ __launch_bounds__(MTREE) void moments_kernel(const double* in, int k, double* out) {
  __shared__ double a1[MTREE], a2[MTREE];
  __shared__ double g1[MTREE], g2[MTREE];
  const int ngroups = (k + MTREE - 1) / MTREE;
  for (int g = 0; g < ngroups; ++g) {
    const int i = g * MTREE + threadIdx.x;
    a1[threadIdx.x] = i < k ? in[2 * i] : 0.0;
    a2[threadIdx.x] = i < k ? in[2 * i + 1] : 0.0;
    tree_pairs<MTREE>(a1, a2);
    if (threadIdx.x == 0) {
      g1[g] = a1[0];
      g2[g] = a2[0];
    }
    __syncthreads();
  }
  if (ngroups == 1) {
    if (threadIdx.x == 0) {
      out[0] = g1[0];
      out[1] = g2[0];
    }
    return;
  }
  if ((int)threadIdx.x >= ngroups) {
    g1[threadIdx.x] = 0.0;
    g2[threadIdx.x] = 0.0;
  }
  tree_pairs<MTREE>(g1, g2);
  if (threadIdx.x == 0) {
    out[0] = g1[0];
    out[1] = g2[0];
  }
}

__global__ __launch_bounds__(256) void normalize_kernel(const float* gae, float* adv, long long count,
                                                        const double* mom, double total, float eps, bool vec) {
#pragma clang fp contract(off)
  const double mean = mom[0] / total;
  const double var = fmax(mom[1] / total - mean * mean, 0.0);
  const float mean_f = (float)mean;
  const float denom = (float)sqrt(var) + eps;
  const long long n4 = vec ? count / 4 : 0;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const float4* g4 = reinterpret_cast<const float4*>(gae);
  float4* a4 = reinterpret_cast<float4*>(adv);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = g4[i];
    v.x = (v.x - mean_f) / denom;
    v.y = (v.y - mean_f) / denom;
    v.z = (v.z - mean_f) / denom;
    v.w = (v.w - mean_f) / denom;
    a4[i] = v;
  }
  for (long long i = n4 * 4 + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride)
    adv[i] = (gae[i] - mean_f) / denom;
}

hipError_t launch_gae(const GaeArgs& a, double* moments_out, hipStream_t s) {
  const int nblk = (a.n + GE - 1) / GE;
  const auto al = [](const void* p, uintptr_t m) { return p == nullptr || ((uintptr_t)p % m) == 0; };
  const bool vec = (a.n % 4 == 0) && al(a.reward, 16) && al(a.values, 16) && al(a.gae, 16) && al(a.vtarget, 16) &&
                   al(a.done, 4) && al(a.success, 4);
  if (vec)
    hipLaunchKernelGGL(gae_kernel<true>, dim3(nblk), dim3(GTHREADS), 0, s, a);
  else
    hipLaunchKernelGGL(gae_kernel<false>, dim3(nblk), dim3(GTHREADS), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !moments_out) return e;
  hipLaunchKernelGGL(moments_kernel, dim3(1), dim3(MTREE), 0, s, a.partials, nblk, moments_out);
  return hipGetLastError();
}

hipError_t launch_moments(const double* in, int k, double* out, hipStream_t s) {
  hipLaunchKernelGGL(moments_kernel, dim3(1), dim3(MTREE), 0, s, in, k, out);
  return hipGetLastError();
}

hipError_t launch_normalize(const float* gae, float* adv, long long count, const double* mom, double total,
                            float eps, hipStream_t s) {
  const bool aligned = ((uintptr_t)gae % 16 == 0) && ((uintptr_t)adv % 16 == 0);
  long long work = aligned ? count / 4 : count;
  int blocks = (int)((work + 255) / 256);
  if (blocks > 2048) blocks = 2048; /* 256 CUs x 8 waves of 4 per CU: grid-stride the rest */
  if (blocks < 1) blocks = 1;
  /* unaligned views: the scalar tail loop handles everything */
  hipLaunchKernelGGL(normalize_kernel, dim3(blocks), dim3(256), 0, s, gae, adv, count, mom, total, eps, aligned);
  return hipGetLastError();
}

}  // namespace zb
