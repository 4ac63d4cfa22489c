// Shared helpers for the gfx950 kernels and the C-ABI glue.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/fce_yolo.h"

namespace fce {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------- error state (thread-local)
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

#define FCE_HIP_CHECK(expr)                                                                    \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess)                                                                      \
      return ::fce::fail(FCE_ERR_HIP, std::string(#expr " failed: ") + hipGetErrorString(_e)); \
  } while (0)

#define FCE_CHECK(cond, msg)                                           \
  do {                                                                 \
    if (!(cond)) return ::fce::fail(FCE_ERR_INVALID, std::string(msg)); \
  } while (0)

inline int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(FCE_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
  return FCE_OK;
}

// ---------------------------------------------------------------- per-kernel timing probe
// While fce_net_profile runs an op, g_probe points at a pool of timing events and every launch goes
// through hipExtLaunchKernelGGL with a (start, stop) pair attached to its own dispatch packet, so the
// measured interval is exactly the kernel's execution (no event packets between kernels).
struct LaunchProbe {
  hipEvent_t* ev;  // 2 * cap events
  int cap, n;      // pairs available / used
};
LaunchProbe*& probe_slot();  // thread-local slot (api.hip)

#define FCE_LAUNCH(K, G, B, SH, S, ...)                                                            \
  do {                                                                                             \
    ::fce::LaunchProbe* _p = ::fce::probe_slot();                                                       \
    if (_p && _p->n < _p->cap) {                                                                   \
      hipExtLaunchKernelGGL(K, G, B, SH, S, _p->ev[2 * _p->n], _p->ev[2 * _p->n + 1], 0, __VA_ARGS__); \
      ++_p->n;                                                                                     \
    } else {                                                                                       \
      hipLaunchKernelGGL(K, G, B, SH, S, __VA_ARGS__);                                             \
    }                                                                                              \
  } while (0)

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ---------------------------------------------------------------- device math
// x * sigmoid(x) with the hardware reciprocal (v_rcp_f32, 1 ulp) in place of IEEE division: the division
// expands to ~10 VALU ops (scale / rcp / 4 fma / fmas / fixup) and the conv epilogues are VALU-heavy
// (a 1x1 conv with cin 64 spends more SIMD cycles on its epilogue than on its MFMAs).  Every kernel
// uses this one definition, so the variants stay bitwise identical to each other.  The product is kept out of
// FMA contraction (the pragma): unlike a quotient, hipcc fuses it with a following add (a residual: one v_fma,
// one rounding) in some kernels and not in others.  (An fpin here would also do, but it cannot be speculated:
// every `act ? silu(t) : t` becomes a branch per element.)
__device__ __forceinline__ float silu(float x) {
#pragma clang fp contract(off)
  return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x));
}
// bias[co] for co < n, else 0, with the load unconditional (index clamped): a load under a branch makes hipcc wait
// for it with vmcnt(0), which on CDNA4 also waits for every store the epilogue has issued before it
__device__ __forceinline__ float bias_or0(const float* b, int co, int n) {
  const float v = b[co < n ? co : n - 1];
  return co < n ? v : 0.f;
}
// fmaf((float)h, w, acc) for the low / high fp16 half h of a packed pair as ONE v_fma_mix_f32: the f16 -> f32
// conversion is exact, so the result is bitwise the fmaf of the converted value (hipcc mixes this form with a
// separate conversion + v_fma_f32 for the high halves, two VALU ops).  Only for operands that come from loads or
// ordinary VALU ops: hipcc's hazard recognizer does not see inside inline asm, and the BiCoord gate fed a v_rcp_f32
// result straight into one of these and read wrong values (bicoord parity failed; reverted there)
__device__ __forceinline__ float fma_mix_lo(uint32_t hp, float w, float acc) {
  float r;
  asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(hp), "v"(w), "v"(acc));
  return r;
}
__device__ __forceinline__ float fma_mix_hi(uint32_t hp, float w, float acc) {
  float r;
  asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(hp), "v"(w), "v"(acc));
  return r;
}
// acc[j] = fmaf((float)v[j], w[j], acc[j]) for the 8 halves of v, as 8 v_fma_mix_f32
__device__ __forceinline__ void fma8_mix(const h8& v, const float* w, float* acc) {
  const u4 pk = __builtin_bit_cast(u4, v);
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    acc[2 * jj] = fma_mix_lo(pk[jj], w[2 * jj], acc[2 * jj]);
    acc[2 * jj + 1] = fma_mix_hi(pk[jj], w[2 * jj + 1], acc[2 * jj + 1]);
  }
}
// An fp32 value pinned in a register.  Without it hipcc fuses a multiply or add with the fp16
// conversion that follows (v_fma_mix*: one rounding instead of two) in some kernels and not in
// others, and conv variants that must be bitwise identical differ in the last fp16 bit.
__device__ __forceinline__ float fpin(float x) {
  asm volatile("" : "+v"(x));
  return x;
}
// Detect scores (the cls epilogue, detect_decode): v_exp_f32 and v_rcp_f32 instead of the libm expf and IEEE
// division (~40 VALU ops per score against 4); the score moves by ~1e-7, far inside CLS_TOL
__device__ __forceinline__ float sigmoidf_(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }

// BiFPN normalised weight (fce_block.py:57-58): relu(w_i) / (sum_j relu(w_j) + 1e-4)
__device__ __forceinline__ float fusion_alpha(const float* w, int n, int i) {
  float s = 0.f;
  for (int j = 0; j < n; ++j) s += fmaxf(w[j], 0.f);
  return fmaxf(w[i], 0.f) / (s + 1e-4f);
}

// NHWC element offset of pixel (n,y,x) channel c in a view
// A store that every lane of the wave issues (no branch around it): a lane with nothing to write stores to an
// offset past the buffer resource's end, which the hardware drops. Branched stores are counted as maybe-absent,
// so the compiler's wait for a load issued before them (the next tile's x prefetch) became vmcnt(0), i.e. a wait
// for the stores too (vmcnt retires in issue order); unconditional ones let it wait for the load alone.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t out_rsrc(void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(base, 0, int(bytes), 0x00020000);  // gfx9 dword3: raw, range-checked
}
__device__ __forceinline__ void store_h4_or_drop(__amdgpu_buffer_rsrc_t r, bool ok, uint32_t byte_off, h4 v) {
  typedef unsigned int u2 __attribute__((ext_vector_type(2)));
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, v), r, int(ok ? byte_off : 0x80000000u), 0, 0);
}

__device__ __forceinline__ void store_h1_or_drop(__amdgpu_buffer_rsrc_t r, bool ok, uint32_t byte_off, _Float16 v) {
  __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, v), r, int(ok ? byte_off : 0x80000000u), 0, 0);
}

__host__ __device__ __forceinline__ int64_t nhwc_off(int n, int y, int x, int H, int W, int cstride) {
  return ((int64_t(n) * H + y) * W + x) * cstride;
}

inline int64_t numel(const fce_tensor& t) { return int64_t(t.n) * t.c * t.h * t.w; }
inline int dtype_size(int dt) { return dt == FCE_F32 ? 4 : dt == FCE_U8 ? 1 : 2; }

int check_nhwc(const fce_tensor* t, const char* name, int dtype);

}  // namespace fce
