// SPPF max-pool chain, BiFPN identity-branch fusion and layout/dtype edge copies (NHWC fp16).
//
// maxpool_chain replaces block.py:228-232: y1 = mp5(x), y2 = mp5(y1), y3 = mp5(y2) with
// MaxPool2d(5, 1, 2) (-inf padding, Q13).  A chain of k x k stride-1 max pools with -inf padding
// equals one (2k-1) / (3k-2) window pool over the clamped window (max is associative and every
// in-range element of the larger window is reachable through an in-range intermediate), so all
// three outputs come from one read of x and are written straight into the concat buffer slices.
#include "common.h"

namespace fce {

struct MpArgs {
  const _Float16* x;
  int xcs;
  _Float16* y1;
  _Float16* y2;
  _Float16* y3;
  int y1cs, y2cs, y3cs;
  int N, H, W, C, r;  // r = k/2
};

__global__ __launch_bounds__(256) void maxpool_chain_kernel(MpArgs a) {
  const int cg = a.C / 8;
  const int64_t total = int64_t(a.N) * a.H * a.W * cg;
  const int R3 = 3 * a.r;
  for (int64_t t = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; t < total; t += int64_t(gridDim.x) * blockDim.x) {
    const int g = int(t % cg);
    const int64_t pix = t / cg;
    const int ox = int(pix % a.W), oy = int((pix / a.W) % a.H), n = int(pix / (int64_t(a.W) * a.H));
    float m1[8], m2[8], m3[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) m1[j] = m2[j] = m3[j] = -INFINITY;
    for (int dy = -R3; dy <= R3; ++dy) {
      const int iy = oy + dy;
      if (iy < 0 || iy >= a.H) continue;
      const int ady = dy < 0 ? -dy : dy;
      float r1[8], r2[8], r3[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) r1[j] = r2[j] = r3[j] = -INFINITY;
      for (int dx = -R3; dx <= R3; ++dx) {
        const int ix = ox + dx;
        if (ix < 0 || ix >= a.W) continue;
        const int adx = dx < 0 ? -dx : dx;
        const h8 v = *reinterpret_cast<const h8*>(a.x + nhwc_off(n, iy, ix, a.H, a.W, a.xcs) + g * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = (float)v[j];
          r3[j] = fmaxf(r3[j], f);
          if (adx <= 2 * a.r) r2[j] = fmaxf(r2[j], f);
          if (adx <= a.r) r1[j] = fmaxf(r1[j], f);
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        m3[j] = fmaxf(m3[j], r3[j]);
        if (ady <= 2 * a.r) m2[j] = fmaxf(m2[j], r2[j]);
        if (ady <= a.r) m1[j] = fmaxf(m1[j], r1[j]);
      }
    }
    h8 o1, o2, o3;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o1[j] = (_Float16)m1[j];
      o2[j] = (_Float16)m2[j];
      o3[j] = (_Float16)m3[j];
    }
    *reinterpret_cast<h8*>(a.y1 + pix * a.y1cs + g * 8) = o1;
    *reinterpret_cast<h8*>(a.y2 + pix * a.y2cs + g * 8) = o2;
    *reinterpret_cast<h8*>(a.y3 + pix * a.y3cs + g * 8) = o3;
  }
}

// LDS-plane variant (the SPPF map is the stride-32 one: 20x20 at 640): one block per (image,
// 8-channel group) holds the whole H x W plane in LDS, takes row maxima over radii r/2r/3r
// (13 LDS reads), then column maxima of those (5+9+13 reads).  fp16 max is exact, so the result
// equals the window max of the direct kernel bit for bit.
__device__ __forceinline__ h8 hmax8(h8 a, h8 b) { return __builtin_elementwise_max(a, b); }

__global__ __launch_bounds__(256) void maxpool_chain_lds_kernel(MpArgs a) {
  extern __shared__ __attribute__((aligned(16))) h8 pl[];
  const int HW = a.H * a.W, cg = a.C >> 3;
  // XCD-aware order: block b runs on XCD b % 8; give each XCD a contiguous range of (image, group)
  // pairs so an image's channel groups (16-byte pieces of the same 128-byte lines) share one L2
  int L;
  {
    const int total = int(gridDim.x), b = int(blockIdx.x), per = total >> 3, body = per << 3;
    L = b < body ? (b & 7) * per + (b >> 3) : b;
  }
  const int n = L / cg, g = L - n * cg;
  h8* xs = pl;
  h8* r1 = pl + HW;
  h8* r2 = pl + 2 * HW;
  h8* r3 = pl + 3 * HW;
  const _Float16* xb = a.x + int64_t(n) * HW * a.xcs + g * 8;
  // plane staging, 4 loads in flight per thread (clamped index; the LDS image is sized HW + 1 so the
  // out-of-range slot is a dummy and the stores are unconditional)
  for (int p0 = 0; p0 < HW; p0 += 4 * 256) {
    h8 v[4];
    int d[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = p0 + int(threadIdx.x) + 256 * u;
      v[u] = *reinterpret_cast<const h8*>(xb + int64_t(min(p, HW - 1)) * a.xcs);
      d[u] = p < HW ? p : 4 * HW;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) pl[d[u]] = v[u];
  }
  __syncthreads();
  const int r = a.r;
  for (int p = threadIdx.x; p < HW; p += 256) {
    const int y = p / a.W, x = p - y * a.W;
    const h8* row = xs + y * a.W;
    h8 m1 = row[x], m2, m3;
    for (int d = 1; d <= r; ++d) {
      if (x - d >= 0) m1 = hmax8(m1, row[x - d]);
      if (x + d < a.W) m1 = hmax8(m1, row[x + d]);
    }
    m2 = m1;
    for (int d = r + 1; d <= 2 * r; ++d) {
      if (x - d >= 0) m2 = hmax8(m2, row[x - d]);
      if (x + d < a.W) m2 = hmax8(m2, row[x + d]);
    }
    m3 = m2;
    for (int d = 2 * r + 1; d <= 3 * r; ++d) {
      if (x - d >= 0) m3 = hmax8(m3, row[x - d]);
      if (x + d < a.W) m3 = hmax8(m3, row[x + d]);
    }
    r1[p] = m1;
    r2[p] = m2;
    r3[p] = m3;
  }
  __syncthreads();
  const int64_t pix0 = int64_t(n) * HW;
  for (int p = threadIdx.x; p < HW; p += 256) {
    const int y = p / a.W, x = p - y * a.W;
    h8 m1 = r1[p], m2 = r2[p], m3 = r3[p];
    for (int d = 1; d <= 3 * r; ++d) {
      const int yu = y - d, yd = y + d;
      if (d <= r) {
        if (yu >= 0) m1 = hmax8(m1, r1[yu * a.W + x]);
        if (yd < a.H) m1 = hmax8(m1, r1[yd * a.W + x]);
      }
      if (d <= 2 * r) {
        if (yu >= 0) m2 = hmax8(m2, r2[yu * a.W + x]);
        if (yd < a.H) m2 = hmax8(m2, r2[yd * a.W + x]);
      }
      if (yu >= 0) m3 = hmax8(m3, r3[yu * a.W + x]);
      if (yd < a.H) m3 = hmax8(m3, r3[yd * a.W + x]);
    }
    const int64_t pix = pix0 + p;
    *reinterpret_cast<h8*>(a.y1 + pix * a.y1cs + g * 8) = m1;
    *reinterpret_cast<h8*>(a.y2 + pix * a.y2cs + g * 8) = m2;
    *reinterpret_cast<h8*>(a.y3 + pix * a.y3cs + g * 8) = m3;
  }
}

int maxpool_chain(const fce_tensor& x, const fce_tensor& y1, const fce_tensor& y2, const fce_tensor& y3, int k,
                  hipStream_t s) {
  for (const fce_tensor* t : {&x, &y1, &y2, &y3}) {
    FCE_CHECK(t->layout == FCE_NHWC && t->dtype == FCE_F16, "maxpool_chain: NHWC f16 views");
    FCE_CHECK(t->cstride % 8 == 0 && t->coff % 8 == 0, "maxpool_chain: 8-channel aligned slices");
    FCE_CHECK(t->n == x.n && t->c == x.c && t->h == x.h && t->w == x.w, "maxpool_chain: shape mismatch");
  }
  FCE_CHECK(x.c % 8 == 0 && (k & 1), "maxpool_chain: c % 8 == 0, odd k");
  MpArgs a{static_cast<const _Float16*>(x.data) + x.coff, x.cstride,
           static_cast<_Float16*>(y1.data) + y1.coff, static_cast<_Float16*>(y2.data) + y2.coff,
           static_cast<_Float16*>(y3.data) + y3.coff, y1.cstride, y2.cstride, y3.cstride,
           x.n, x.h, x.w, x.c, k / 2};
  const int64_t total = int64_t(x.n) * x.h * x.w * (x.c / 8);
  if (total == 0) return FCE_OK;
  const size_t lds = (size_t(4) * x.h * x.w + 1) * sizeof(h8);  // 4 planes + the staging dummy
  // > 64 KiB (the 40 x 40 SPPF map at imgsz 1280) needs the gfx950 LDS opt-in (up to 160 KiB)
  static const bool lds_big = hipFuncSetAttribute(reinterpret_cast<const void*>(&maxpool_chain_lds_kernel),
                                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
  if (lds <= (lds_big ? 160 : 64) * 1024 && int64_t(x.n) * (x.c / 8) < (int64_t(1) << 31)) {  // H*W <= 2560
    FCE_LAUNCH(maxpool_chain_lds_kernel, dim3(x.n * (x.c / 8)), dim3(256), lds, s, a);
    return launch_status("maxpool_chain_lds_kernel");
  }
  int blocks = int(std::min<int64_t>((total + 255) / 256, 65535 * 8));
  FCE_LAUNCH(maxpool_chain_kernel, dim3(blocks), dim3(256), 0, s, a);
  return launch_status("maxpool_chain_kernel");
}

// ---------------------------------------------------------------------------- BiFPN identity term
struct WaddArgs {
  const _Float16* x;
  int xcs, Hs, Ws, up;
  _Float16* y;
  int ycs, N, H, W, C;
  const float* fw;
  int fn, fi, accumulate;
};

__global__ __launch_bounds__(256) void weighted_add_kernel(WaddArgs a) {
  const float alpha = fusion_alpha(a.fw, a.fn, a.fi);
  const int cg = a.C / 8;
  const int64_t total = int64_t(a.N) * a.H * a.W * cg;
  for (int64_t t = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; t < total; t += int64_t(gridDim.x) * blockDim.x) {
    const int g = int(t % cg);
    const int64_t pix = t / cg;
    const int ox = int(pix % a.W), oy = int((pix / a.W) % a.H), n = int(pix / (int64_t(a.W) * a.H));
    const h8 v = *reinterpret_cast<const h8*>(a.x + nhwc_off(n, oy >> a.up, ox >> a.up, a.Hs, a.Ws, a.xcs) + g * 8);
    _Float16* yo = a.y + pix * a.ycs + g * 8;
    h8 prev = h8{0, 0, 0, 0, 0, 0, 0, 0};
    if (a.accumulate) prev = *reinterpret_cast<const h8*>(yo);
    h8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (_Float16)((a.accumulate ? (float)prev[j] : 0.f) + alpha * (float)v[j]);
    *reinterpret_cast<h8*>(yo) = o;
  }
}

int weighted_add(const fce_tensor& x, int up, const float* fw, int fn, int fi, int accumulate, const fce_tensor& y,
                 hipStream_t s) {
  FCE_CHECK(x.layout == FCE_NHWC && y.layout == FCE_NHWC && x.dtype == FCE_F16 && y.dtype == FCE_F16,
            "weighted_add: NHWC f16 views");
  FCE_CHECK(x.c == y.c && x.n == y.n && (x.h << up) == y.h && (x.w << up) == y.w, "weighted_add: shape mismatch");
  FCE_CHECK(x.c % 8 == 0 && x.cstride % 8 == 0 && x.coff % 8 == 0 && y.cstride % 8 == 0 && y.coff % 8 == 0,
            "weighted_add: 8-channel aligned slices");
  FCE_CHECK(fw && fn > fi && fi >= 0, "weighted_add: fusion weights");
  WaddArgs a{static_cast<const _Float16*>(x.data) + x.coff, x.cstride, x.h, x.w, up,
             static_cast<_Float16*>(y.data) + y.coff, y.cstride, y.n, y.h, y.w, y.c, fw, fn, fi, accumulate};
  const int64_t total = int64_t(y.n) * y.h * y.w * (y.c / 8);
  if (total == 0) return FCE_OK;
  FCE_LAUNCH(weighted_add_kernel, dim3(int(std::min<int64_t>((total + 255) / 256, 65535 * 8))), dim3(256),
                     0, s, a);
  return launch_status("weighted_add_kernel");
}

// ---------------------------------------------------------------------------- layout / dtype copies
struct CopyArgs {
  const void* src;
  int sdt, slay, scs, scoff;
  void* dst;
  int ddt, dlay, dcs, dcoff;
  int N, C, H, W;
};

__device__ __forceinline__ int64_t view_index(int lay, int cs, int coff, int n, int c, int y, int x, int C, int H,
                                              int W) {
  return lay == FCE_NCHW ? ((int64_t(n) * C + c) * H + y) * W + x : ((int64_t(n) * H + y) * W + x) * cs + coff + c;
}

__global__ __launch_bounds__(256) void copy_kernel(CopyArgs a) {
  const int64_t total = int64_t(a.N) * a.C * a.H * a.W;
  for (int64_t t = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; t < total; t += int64_t(gridDim.x) * blockDim.x) {
    // iterate in destination order for coalesced stores
    int n, c, y, x;
    if (a.dlay == FCE_NCHW) {
      x = int(t % a.W);
      y = int((t / a.W) % a.H);
      c = int((t / (int64_t(a.W) * a.H)) % a.C);
      n = int(t / (int64_t(a.W) * a.H * a.C));
    } else {
      c = int(t % a.C);
      x = int((t / a.C) % a.W);
      y = int((t / (int64_t(a.C) * a.W)) % a.H);
      n = int(t / (int64_t(a.C) * a.W * a.H));
    }
    const int64_t si = view_index(a.slay, a.scs, a.scoff, n, c, y, x, a.C, a.H, a.W);
    const int64_t di = view_index(a.dlay, a.dcs, a.dcoff, n, c, y, x, a.C, a.H, a.W);
    float v;
    if (a.sdt == FCE_F16)
      v = (float)static_cast<const _Float16*>(a.src)[si];
    else if (a.sdt == FCE_F32)
      v = static_cast<const float*>(a.src)[si];
    else
      v = (float)static_cast<const uint8_t*>(a.src)[si];
    if (a.ddt == FCE_F16)
      static_cast<_Float16*>(a.dst)[di] = (_Float16)v;
    else
      static_cast<float*>(a.dst)[di] = v;
  }
}

int copy(const fce_tensor& src, const fce_tensor& dst, hipStream_t s) {
  FCE_CHECK(src.n == dst.n && src.c == dst.c && src.h == dst.h && src.w == dst.w, "copy: shape mismatch");
  FCE_CHECK(dst.dtype == FCE_F16 || dst.dtype == FCE_F32, "copy: destination must be f16 or f32");
  const int64_t total = numel(src);
  if (total == 0) return FCE_OK;
  CopyArgs a{src.data, src.dtype, src.layout, src.cstride, src.coff, dst.data, dst.dtype,
             dst.layout, dst.cstride, dst.coff, src.n, src.c, src.h, src.w};
  FCE_LAUNCH(copy_kernel, dim3(int(std::min<int64_t>((total + 255) / 256, 65535 * 8))), dim3(256), 0, s, a);
  return launch_status("copy_kernel");
}

}  // namespace fce
