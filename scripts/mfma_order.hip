// Diagnostic: do v_mfma_f32_16x16x4_f32 / 32x32x2_f32 accumulate as a k-ordered fmaf chain?
//   hipcc --offload-arch=gfx950 -O2 -o /tmp/mfma_order scripts/mfma_order.hip && /tmp/mfma_order
// Does v_mfma_f32_16x16x4_f32 accumulate as a k-ordered fmaf chain (like 32x32x2)? Diagnostic.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));
constexpr int K = 128;
// A: [16][K] row-major, B: [K][16]; C[i][j] = sum_k A[i][k] B[k][j]
__global__ void k16(const float* A, const float* B, float* C) {
  const int l = threadIdx.x;
  const int i = l & 15, kk = l >> 4;
  v4f acc = {0, 0, 0, 0};
  for (int k0 = 0; k0 < K; k0 += 4) {
    float a = A[i * K + k0 + kk];
    float b = B[(k0 + kk) * 16 + i];
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
  }
  for (int v = 0; v < 4; v++) C[(4 * kk + v) * 16 + i] = acc[v];
}
// 32x32x2 on a 32x32 problem
__global__ void k32(const float* A, const float* B, float* C) {
  const int l = threadIdx.x;
  const int i = l & 31, kk = l >> 5;
  v16f acc = {};
  for (int k0 = 0; k0 < K; k0 += 2) {
    float a = A[i * K + k0 + kk];
    float b = B[(k0 + kk) * 32 + i];
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
  }
  for (int r = 0; r < 16; r++) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * kk;
    C[row * 32 + i] = acc[r];
  }
}
int main() {
  srand(1);
  const int N = 32;
  float *A = new float[N * K], *B = new float[K * N], *C = new float[N * N];
  for (int t = 0; t < N * K; t++) A[t] = (rand() / (float)RAND_MAX - 0.5f) * (t % 7 == 0 ? 1000.f : 1.f);
  for (int t = 0; t < K * N; t++) B[t] = (rand() / (float)RAND_MAX - 0.5f) * (t % 5 == 0 ? 0.001f : 1.f);
  float *dA, *dB, *dC;
  hipMalloc(&dA, N * K * 4); hipMalloc(&dB, K * N * 4); hipMalloc(&dC, N * N * 4);
  for (int shape = 16; shape <= 32; shape += 16) {
    // pack B as [K][shape]
    float* Bp = new float[K * shape];
    for (int k = 0; k < K; k++) for (int j = 0; j < shape; j++) Bp[k * shape + j] = B[k * N + j];
    hipMemcpy(dA, A, N * K * 4, hipMemcpyHostToDevice);
    hipMemcpy(dB, Bp, K * shape * 4, hipMemcpyHostToDevice);
    if (shape == 16) hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    else hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    hipMemcpy(C, dC, shape * shape * 4, hipMemcpyDeviceToHost);
    int same_fma = 0, same_pair = 0, tot = 0;
    for (int i = 0; i < shape; i++) for (int j = 0; j < shape; j++) {
      float acc = 0.f;
      for (int k = 0; k < K; k++) acc = fmaf(A[i * K + k], Bp[k * shape + j], acc);
      same_fma += (memcmp(&acc, &C[i * shape + j], 4) == 0);
      tot++;
    }
    printf("shape %dx%d: %d / %d bit-identical to the k-ordered fmaf chain\n", shape, shape, same_fma, tot);
    delete[] Bp;
  }
  return 0;
}
