// Experiment: issue cost per wave of v_fma_mix_f32 (fp16 x fp32 + fp32) against v_fma_f32 and v_pk_fma_f32, one wave
// per SIMD, 8 independent accumulator chains; cycles from s_memtime around an unrolled loop.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ void k(const float* in, float* out, int iters, unsigned long long* cyc) {
  float a[8], w = in[1];
  unsigned h = __float_as_uint(in[2]);
  f2 p[4], pw = {in[3], in[4]};
  for (int j = 0; j < 8; ++j) a[j] = in[0] + j;
  for (int j = 0; j < 4; ++j) p[j] = f2{a[2 * j], a[2 * j + 1]};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (MODE == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(a[j]) : "v"(h), "v"(w));
      } else if (MODE == 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[j]) : "v"(w), "v"(w));
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p[j]) : "v"(pw), "v"(pw));
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int j = 0; j < 8; ++j) s += a[j];
  for (int j = 0; j < 4; ++j) s += p[j][0] + p[j][1];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  float* in;
  float* out;
  unsigned long long* cyc;
  hipMalloc(&in, 64);
  hipMalloc(&out, 1 << 20);
  hipMalloc(&cyc, 8);
  float h_in[5] = {0.001f, 0.999f, 0.f, 0.5f, 0.25f};
  hipMemcpy(in, h_in, sizeof(h_in), hipMemcpyHostToDevice);
  const int iters = 1000;
  const char* names[3] = {"v_fma_mix_f32 (8 per round)", "v_fma_f32 (8 per round)", "v_pk_fma_f32 (4 per round = 8 fma)"};
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, in, out, iters, cyc);
      if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, in, out, iters, cyc);
      if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(1), dim3(64), 0, 0, in, out, iters, cyc);
      hipDeviceSynchronize();
    }
    unsigned long long c = 0;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    const double ninst = double(iters) * 16 * (mode == 2 ? 4 : 8);
    printf("%-36s %.2f cycles per instruction (one wave)\n", names[mode], c / ninst);
  }
  return 0;
}
