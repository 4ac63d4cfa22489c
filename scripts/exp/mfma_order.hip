// Experiment: is v_mfma_f32_16x16x32_f16 (one 32-deep K-step from C) bitwise equal to two chained
// v_mfma_f32_32x32x16_f16 (k 0-15, then k 16-31)?  Every A row / B column is the same vector, so each output element
// is sum_k a[k] b[k] whatever the output layout.  Prints the number of mismatching trials.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

__global__ void k(const _Float16* a, const _Float16* b, const float* c, float* out, int trials) {
  const int lane = threadIdx.x;
  for (int t = blockIdx.x; t < trials; t += gridDim.x) {
    const _Float16* at = a + t * 32;
    const _Float16* bt = b + t * 32;
    h8 A, B;
    for (int j = 0; j < 8; ++j) {
      A[j] = at[8 * (lane / 16) + j];
      B[j] = bt[8 * (lane / 16) + j];
    }
    f4 acc = {c[t], c[t], c[t], c[t]};
    const f4 d16 = __builtin_amdgcn_mfma_f32_16x16x32_f16(A, B, acc, 0, 0, 0);
    h8 A0, B0, A1, B1;
    for (int j = 0; j < 8; ++j) {
      A0[j] = at[8 * (lane / 32) + j];
      B0[j] = bt[8 * (lane / 32) + j];
      A1[j] = at[16 + 8 * (lane / 32) + j];
      B1[j] = bt[16 + 8 * (lane / 32) + j];
    }
    f16v acc2;
    for (int j = 0; j < 16; ++j) acc2[j] = c[t];
    acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(A0, B0, acc2, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, B1, acc2, 0, 0, 0);
    // the same 16 products in the other order of the halves
    f16v acc3;
    for (int j = 0; j < 16; ++j) acc3[j] = c[t];
    acc3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, B1, acc3, 0, 0, 0);
    acc3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(A0, B0, acc3, 0, 0, 0);
    if (lane == 0) {
      out[t * 3 + 0] = d16[0];
      out[t * 3 + 1] = acc2[0];
      out[t * 3 + 2] = acc3[0];
    }
  }
}

int main() {
  const int trials = 200000;
  std::vector<_Float16> a(trials * 32), b(trials * 32);
  std::vector<float> c(trials);
  srand(1);
  for (int t = 0; t < trials; ++t) {
    const int mode = t % 4;
    for (int i = 0; i < 32; ++i) {
      float x = (rand() / (float)RAND_MAX - 0.5f) * 4.f, y = (rand() / (float)RAND_MAX - 0.5f) * 4.f;
      if (mode == 1) x *= powf(2.f, (float)(rand() % 20 - 10));
      if (mode == 2 && i % 7 == 0) y *= 1000.f;
      a[t * 32 + i] = (_Float16)x;
      b[t * 32 + i] = (_Float16)y;
    }
    c[t] = mode == 3 ? (rand() / (float)RAND_MAX - 0.5f) * 100.f : 0.f;
  }
  _Float16 *da, *db;
  float *dc, *dout;
  hipMalloc(&da, a.size() * 2);
  hipMalloc(&db, b.size() * 2);
  hipMalloc(&dc, c.size() * 4);
  hipMalloc(&dout, trials * 3 * 4);
  hipMemcpy(da, a.data(), a.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(db, b.data(), b.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dc, c.data(), c.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1024), dim3(64), 0, 0, da, db, dc, dout, trials);
  std::vector<float> out(trials * 3);
  hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost);
  int m01 = 0, m02 = 0, m12 = 0;
  for (int t = 0; t < trials; ++t) {
    unsigned u0, u1, u2;
    memcpy(&u0, &out[t * 3], 4);
    memcpy(&u1, &out[t * 3 + 1], 4);
    memcpy(&u2, &out[t * 3 + 2], 4);
    m01 += u0 != u1;
    m02 += u0 != u2;
    m12 += u1 != u2;
    if (t < 4) printf("t %d: 16x16x32 %.9g  32x32x16 lo,hi %.9g  hi,lo %.9g\n", t, out[t * 3], out[t * 3 + 1], out[t * 3 + 2]);
  }
  printf("trials %d: 16x16x32 != 32x32x16(lo,hi): %d   != (hi,lo): %d   (lo,hi) != (hi,lo): %d\n", trials, m01, m02, m12);
  return 0;
}
