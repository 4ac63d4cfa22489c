// Convolutions for gfx950: MFMA implicit GEMM (dense 1x1 / 3x3), depthwise 3x3, and the
// Cin<=4 stem that reads the NCHW network input directly.
//
// Replaces (reference, ultralytics/): nn/modules/conv.py:39-89 Conv.forward_fuse with the BN
// folded by utils/torch_utils.py:237-267; conv.py:185-200 DWConv; the Detect 1x1 nn.Conv2d
// (head.py:86-107); Bottleneck's residual add (block.py:474-476); torch.cat / chunk of
// C2f / C3 / SPPF / C2PSA (block.py:303-307, 338-340, 228-232, 1453-1464) through channel-offset
// reads and writes; nn.Upsample(x2, nearest) feeding a 1x1 conv through `up`.
//
// Data layout: activations NHWC fp16, any view may be a channel slice of a wider buffer.
// Dense conv as GEMM  D[cout][pixel] = sum_k W[cout][k] * X[k][pixel],  k = (tap, cin):
//   v_mfma_f32_16x16x32_f16 with A = weights (16 couts x 32 k), B = activations (32 k x 16 px).
//   Lane l owns A[co = l&15][k = 8(l>>4)+j] and B[k = 8(l>>4)+j][px = l&15]: one 16-byte load
//   of 8 consecutive input channels of one pixel (coalesced along NHWC) per fragment; the
//   weight fragments are pre-packed in exactly this lane order (1 KiB per fragment).
//   D: lane l holds px = l&15, couts 4(l>>4)+0..3  -> 8-byte NHWC stores.
#include "common.h"

namespace fce {

// ============================================================================ packing (host)
struct DenseGeom {
  int cpt, taps, nchunk, nsteps, cotiles;
};
static DenseGeom dense_geom(const fce_conv_desc& d) {
  DenseGeom g;
  g.cpt = d.cin / 8;
  g.taps = d.k * d.k;
  g.nchunk = g.taps * g.cpt;
  g.nsteps = (g.nchunk + 3) / 4;
  g.cotiles = (d.cout + 15) / 16;
  return g;
}

static bool is_stem(const fce_conv_desc& d) { return d.groups == 1 && d.cin <= 4; }
static bool is_dw(const fce_conv_desc& d) { return d.groups > 1; }

size_t conv_weight_bytes(const fce_conv_desc& d) {
  if (is_stem(d)) return size_t(d.cin) * d.k * d.k * d.cout * sizeof(float);  // [cin*k*k][cout] fp32
  if (is_dw(d)) return size_t(d.k) * d.k * d.cin * sizeof(float);             // [k*k][c] fp32
  DenseGeom g = dense_geom(d);
  return size_t(g.cotiles) * g.nsteps * 64 * 8 * sizeof(_Float16);
}

int conv_pack(const fce_conv_desc& d, const float* w, void* out) {
  const int k = d.k, kk = k * k;
  if (is_stem(d)) {  // [ci][ky][kx][co]
    float* o = static_cast<float*>(out);
    for (int co = 0; co < d.cout; ++co)
      for (int ci = 0; ci < d.cin; ++ci)
        for (int t = 0; t < kk; ++t) o[(ci * kk + t) * d.cout + co] = w[(co * d.cin + ci) * kk + t];
    return FCE_OK;
  }
  if (is_dw(d)) {  // [t][c]
    float* o = static_cast<float*>(out);
    for (int c = 0; c < d.cin; ++c)
      for (int t = 0; t < kk; ++t) o[t * d.cin + c] = w[c * kk + t];
    return FCE_OK;
  }
  DenseGeom g = dense_geom(d);
  _Float16* o = static_cast<_Float16*>(out);
  for (int ct = 0; ct < g.cotiles; ++ct)
    for (int s = 0; s < g.nsteps; ++s)
      for (int l = 0; l < 64; ++l) {
        const int co = ct * 16 + (l & 15);
        const int c = s * 4 + (l >> 4);
        _Float16* dst = o + ((size_t(ct) * g.nsteps + s) * 64 + l) * 8;
        for (int j = 0; j < 8; ++j) {
          float v = 0.f;
          if (co < d.cout && c < g.nchunk) {
            const int tap = c / g.cpt, ci = (c % g.cpt) * 8 + j;
            v = w[(size_t(co) * d.cin + ci) * kk + tap];
          }
          dst[j] = (_Float16)v;
        }
      }
  return FCE_OK;
}

// ============================================================================ dense MFMA kernel
struct ConvArgs {
  const _Float16* x;  // input view base (already offset by coff)
  int N, Hs, Ws, xcs;  // source buffer spatial size, channel stride
  int Hin, Win;        // logical input size (Hs << up)
  int up;
  int cin, cout, stride;
  int Ho, Wo, P;  // output spatial, pixels total
  const _Float16* w;
  const float* bias;
  const _Float16* res;  // residual view base or null
  int rcs;
  void* y;  // output view base
  int ycs;
  int act;
  const float* fw;
  int fn, fi;
  int cpt, nchunk, nsteps;
  int vec_ok;
};

enum { OUT_F16 = 0, OUT_F32 = 1, OUT_WSTORE = 2, OUT_ACCUM = 3 };

template <int KS, int RC, int RP, int OUT>
__global__ __launch_bounds__(256) void conv_mfma_kernel(ConvArgs a) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int col = lane & 15;
  const int grp = lane >> 4;
  const int pix_base = (blockIdx.x * 4 + wave) * (RP * 16);
  const int cot0 = blockIdx.y * RC;
  const int cotiles = (a.cout + 15) >> 4;

  // per-rep pixel decode for this lane's B column
  int pn[RP], py[RP], px[RP];
  bool pv[RP];
#pragma unroll
  for (int p = 0; p < RP; ++p) {
    int pix = pix_base + p * 16 + col;
    pv[p] = pix < a.P;
    pix = pv[p] ? pix : 0;
    const int hw = a.Ho * a.Wo;
    pn[p] = pix / hw;
    const int r = pix - pn[p] * hw;
    py[p] = (r / a.Wo) * a.stride - (KS / 2);
    px[p] = (r % a.Wo) * a.stride - (KS / 2);
  }

  f4 acc[RC][RP];
#pragma unroll
  for (int r = 0; r < RC; ++r)
#pragma unroll
    for (int p = 0; p < RP; ++p) acc[r][p] = f4{0.f, 0.f, 0.f, 0.f};

  // per-lane K-chunk cursor: chunk c = 4*s + grp  ->  (tap, cc)
  int tap = 0, cc = grp;
  while (cc >= a.cpt) {
    cc -= a.cpt;
    ++tap;
  }
  const h8* wfrag[RC];
#pragma unroll
  for (int r = 0; r < RC; ++r) {
    const int ct = min(cot0 + r, cotiles - 1);
    wfrag[r] = reinterpret_cast<const h8*>(a.w) + (size_t(ct) * a.nsteps) * 64 + lane;
  }

  auto load_b = [&](int tap_, int cc_, h8 (&b)[RP]) {
    const int ky = KS == 1 ? 0 : tap_ / KS;
    const int kx = KS == 1 ? 0 : tap_ - ky * KS;
    const bool tap_ok = tap_ < KS * KS;
#pragma unroll
    for (int p = 0; p < RP; ++p) {
      const int iy = py[p] + ky, ix = px[p] + kx;
      const bool ok = tap_ok && pv[p] && iy >= 0 && iy < a.Hin && ix >= 0 && ix < a.Win;
      h8 v = h8{0, 0, 0, 0, 0, 0, 0, 0};
      if (ok) {
        const int64_t off = nhwc_off(pn[p], iy >> a.up, ix >> a.up, a.Hs, a.Ws, a.xcs) + cc_ * 8;
        v = *reinterpret_cast<const h8*>(a.x + off);
      }
      b[p] = v;
    }
  };

  h8 bcur[RP], bnext[RP];
  h8 acur[RC], anext[RC];
  load_b(tap, cc, bcur);
#pragma unroll
  for (int r = 0; r < RC; ++r) acur[r] = wfrag[r][0];

  for (int s = 0; s < a.nsteps; ++s) {
    // advance cursor and prefetch step s+1
    cc += 4;
    while (cc >= a.cpt) {
      cc -= a.cpt;
      ++tap;
    }
    const bool more = s + 1 < a.nsteps;
    if (more) {
      load_b(tap, cc, bnext);
#pragma unroll
      for (int r = 0; r < RC; ++r) anext[r] = wfrag[r][(s + 1) * 64];
    }
#pragma unroll
    for (int r = 0; r < RC; ++r)
#pragma unroll
      for (int p = 0; p < RP; ++p)
        acc[r][p] = __builtin_amdgcn_mfma_f32_16x16x32_f16(acur[r], bcur[p], acc[r][p], 0, 0, 0);
    if (more) {
#pragma unroll
      for (int p = 0; p < RP; ++p) bcur[p] = bnext[p];
#pragma unroll
      for (int r = 0; r < RC; ++r) acur[r] = anext[r];
    }
  }

  // ---------------------------------------------------------------- epilogue
  float alpha = 1.f;
  if (OUT == OUT_WSTORE || OUT == OUT_ACCUM) alpha = fusion_alpha(a.fw, a.fn, a.fi);
#pragma unroll
  for (int r = 0; r < RC; ++r) {
    const int co0 = (cot0 + r) * 16 + grp * 4;
    if (cot0 + r >= cotiles || co0 >= a.cout) continue;
    float bz[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bz[j] = (co0 + j < a.cout) ? a.bias[co0 + j] : 0.f;
#pragma unroll
    for (int p = 0; p < RP; ++p) {
      const int pix = pix_base + p * 16 + col;
      if (pix >= a.P) continue;
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float t = acc[r][p][j] + bz[j];
        v[j] = a.act ? silu(t) : t;
      }
      if (OUT == OUT_F32) {
        float* yo = static_cast<float*>(a.y) + int64_t(pix) * a.ycs + co0;
        if (a.vec_ok && co0 + 3 < a.cout) {
          *reinterpret_cast<f4*>(yo) = f4{v[0], v[1], v[2], v[3]};
        } else {
          for (int j = 0; j < 4; ++j)
            if (co0 + j < a.cout) yo[j] = v[j];
        }
        continue;
      }
      _Float16* yo = static_cast<_Float16*>(a.y) + int64_t(pix) * a.ycs + co0;
      if (a.res) {
        const _Float16* ro = a.res + int64_t(pix) * a.rcs + co0;
        if (a.vec_ok && co0 + 3 < a.cout) {
          h4 rv = *reinterpret_cast<const h4*>(ro);
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] += (float)rv[j];
        } else {
          for (int j = 0; j < 4; ++j)
            if (co0 + j < a.cout) v[j] += (float)ro[j];
        }
      }
      if (OUT == OUT_WSTORE) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] *= alpha;
      }
      if (a.vec_ok && co0 + 3 < a.cout) {
        if (OUT == OUT_ACCUM) {
          h4 pv4 = *reinterpret_cast<const h4*>(yo);
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = (float)pv4[j] + alpha * v[j];
        }
        *reinterpret_cast<h4*>(yo) = h4{(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
      } else {
        for (int j = 0; j < 4; ++j) {
          if (co0 + j >= a.cout) continue;
          float t = v[j];
          if (OUT == OUT_ACCUM) t = (float)yo[j] + alpha * t;
          yo[j] = (_Float16)t;
        }
      }
    }
  }
}

// ============================================================================ depthwise 3x3
struct DwArgs {
  const _Float16* x;
  int N, H, W, xcs;
  int C, stride, k;
  int Ho, Wo;
  const float* w;  // [k*k][C]
  const float* bias;
  _Float16* y;
  int ycs;
  int act;
};

__global__ __launch_bounds__(256) void dwconv_kernel(DwArgs a) {
  const int cg8 = a.C / 8;
  const int64_t total = int64_t(a.N) * a.Ho * a.Wo * cg8;
  for (int64_t t = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; t < total; t += int64_t(gridDim.x) * blockDim.x) {
    const int g = int(t % cg8);
    const int64_t pix = t / cg8;
    const int ox = int(pix % a.Wo);
    const int oy = int((pix / a.Wo) % a.Ho);
    const int n = int(pix / (int64_t(a.Wo) * a.Ho));
    const int c0 = g * 8;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = a.bias[c0 + j];
    const int pad = a.k / 2;
    for (int ky = 0; ky < a.k; ++ky) {
      const int iy = oy * a.stride - pad + ky;
      if (iy < 0 || iy >= a.H) continue;
      for (int kx = 0; kx < a.k; ++kx) {
        const int ix = ox * a.stride - pad + kx;
        if (ix < 0 || ix >= a.W) continue;
        const h8 v = *reinterpret_cast<const h8*>(a.x + nhwc_off(n, iy, ix, a.H, a.W, a.xcs) + c0);
        const float* wt = a.w + (ky * a.k + kx) * a.C + c0;
        const f4 w0 = *reinterpret_cast<const f4*>(wt);
        const f4 w1 = *reinterpret_cast<const f4*>(wt + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[j] += (float)v[j] * w0[j];
          acc[j + 4] += (float)v[j + 4] * w1[j];
        }
      }
    }
    h8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (_Float16)(a.act ? silu(acc[j]) : acc[j]);
    *reinterpret_cast<h8*>(a.y + pix * a.ycs + c0) = o;
  }
}

// ============================================================================ stem (NCHW input, cin <= 4)
struct StemArgs {
  const void* x;
  int dtype;
  int N, C, H, W;
  int stride, k;
  int Ho, Wo, cout;
  const float* w;  // [ci][ky][kx][co]
  const float* bias;
  _Float16* y;
  int ycs;
  int act;
};

template <typename T>
__device__ __forceinline__ float ld_in(const T* p, int64_t i);
template <>
__device__ __forceinline__ float ld_in<_Float16>(const _Float16* p, int64_t i) {
  return (float)p[i];
}
template <>
__device__ __forceinline__ float ld_in<float>(const float* p, int64_t i) {
  return p[i];
}
template <>
__device__ __forceinline__ float ld_in<uint8_t>(const uint8_t* p, int64_t i) {
  return (float)p[i] * (1.0f / 255.0f);
}

template <int COUT, typename T>
__global__ __launch_bounds__(256) void stem_kernel(StemArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int nw = a.C * a.k * a.k * COUT;
  for (int i = threadIdx.x; i < nw; i += blockDim.x) {
    const int co = i % COUT, r = i / COUT;
    smem[i] = co < a.cout ? a.w[r * a.cout + co] : 0.f;
  }
  __syncthreads();
  const T* x = static_cast<const T*>(a.x);
  const int64_t P = int64_t(a.N) * a.Ho * a.Wo;
  const int pad = a.k / 2;
  for (int64_t pix = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; pix < P; pix += int64_t(gridDim.x) * blockDim.x) {
    const int ox = int(pix % a.Wo);
    const int oy = int((pix / a.Wo) % a.Ho);
    const int n = int(pix / (int64_t(a.Wo) * a.Ho));
    float acc[COUT];
#pragma unroll
    for (int co = 0; co < COUT; ++co) acc[co] = 0.f;
    for (int ci = 0; ci < a.C; ++ci) {
      const int64_t plane = (int64_t(n) * a.C + ci) * a.H * a.W;
      for (int ky = 0; ky < a.k; ++ky) {
        const int iy = oy * a.stride - pad + ky;
        if (iy < 0 || iy >= a.H) continue;
        for (int kx = 0; kx < a.k; ++kx) {
          const int ix = ox * a.stride - pad + kx;
          if (ix < 0 || ix >= a.W) continue;
          const float v = ld_in<T>(x, plane + int64_t(iy) * a.W + ix);
          const float* wt = smem + ((ci * a.k + ky) * a.k + kx) * COUT;
#pragma unroll
          for (int co = 0; co < COUT; ++co) acc[co] += v * wt[co];
        }
      }
    }
    _Float16* yo = a.y + pix * a.ycs;
#pragma unroll
    for (int co0 = 0; co0 < COUT; co0 += 8) {
      if (co0 >= a.cout) break;
      h8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int co = co0 + j;
        const float t = acc[co] + (co < a.cout ? a.bias[co] : 0.f);
        o[j] = (_Float16)(a.act ? silu(t) : t);
      }
      *reinterpret_cast<h8*>(yo + co0) = o;
    }
  }
}

// ============================================================================ dispatch
static int grid_cap(int64_t blocks) { return int(blocks < 65535 * 16 ? blocks : 65535 * 16); }

template <int KS, int RC, int RP>
static void launch_dense(const ConvArgs& a, int out_kind, dim3 grid, hipStream_t s) {
  switch (out_kind) {
    case OUT_F16:
      hipLaunchKernelGGL((conv_mfma_kernel<KS, RC, RP, OUT_F16>), grid, dim3(256), 0, s, a);
      break;
    case OUT_F32:
      hipLaunchKernelGGL((conv_mfma_kernel<KS, RC, RP, OUT_F32>), grid, dim3(256), 0, s, a);
      break;
    case OUT_WSTORE:
      hipLaunchKernelGGL((conv_mfma_kernel<KS, RC, RP, OUT_WSTORE>), grid, dim3(256), 0, s, a);
      break;
    default:
      hipLaunchKernelGGL((conv_mfma_kernel<KS, RC, RP, OUT_ACCUM>), grid, dim3(256), 0, s, a);
      break;
  }
}

template <int KS>
static void launch_dense_rc(const ConvArgs& a, int out_kind, int rc, hipStream_t s) {
  constexpr int RP = 2;
  const int cotiles = (a.cout + 15) / 16;
  dim3 grid((a.P + 64 * RP - 1) / (64 * RP), (cotiles + rc - 1) / rc);
  if (rc == 1)
    launch_dense<KS, 1, RP>(a, out_kind, grid, s);
  else if (rc == 2)
    launch_dense<KS, 2, RP>(a, out_kind, grid, s);
  else
    launch_dense<KS, 4, RP>(a, out_kind, grid, s);
}

int conv2d(const fce_conv_desc& d, const fce_tensor& x, const void* w, const float* bias, const fce_tensor* res,
           const fce_tensor& y, hipStream_t s) {
  FCE_CHECK(d.k == 1 || d.k == 3 || (is_stem(d) && d.k <= 7), "conv: kernel size must be 1 or 3");
  FCE_CHECK(d.stride >= 1 && d.stride <= 2, "conv: stride must be 1 or 2");
  FCE_CHECK(x.n == y.n && x.c == d.cin && y.c == d.cout, "conv: channel/batch mismatch");
  const int Hin = x.h << d.up, Win = x.w << d.up;
  const int pad = d.k / 2;
  const int Ho = (Hin + 2 * pad - d.k) / d.stride + 1, Wo = (Win + 2 * pad - d.k) / d.stride + 1;
  FCE_CHECK(y.h == Ho && y.w == Wo, "conv: output spatial size mismatch");
  FCE_CHECK(y.layout == FCE_NHWC, "conv: output must be NHWC");
  if (int64_t(y.n) * Ho * Wo == 0) return FCE_OK;

  if (is_stem(d)) {
    FCE_CHECK(x.layout == FCE_NCHW && y.dtype == FCE_F16 && d.up == 0, "stem conv: NCHW input, f16 NHWC output");
    FCE_CHECK(d.epilogue == FCE_EPI_STORE && res == nullptr, "stem conv: plain store only");
    FCE_CHECK(y.cstride % 8 == 0 && y.coff % 8 == 0 && d.cout % 8 == 0, "stem conv: output slice must be 8-aligned");
    StemArgs a{x.data, x.dtype, x.n, x.c, x.h, x.w, d.stride, d.k, Ho, Wo, d.cout, static_cast<const float*>(w),
               bias, static_cast<_Float16*>(y.data) + y.coff, y.cstride, d.act};
    const int64_t P = int64_t(x.n) * Ho * Wo;
    const int blocks = grid_cap((P + 255) / 256);
    int coutT = d.cout <= 16 ? 16 : d.cout <= 32 ? 32 : d.cout <= 64 ? 64 : d.cout <= 96 ? 96 : 0;
    FCE_CHECK(coutT > 0, "stem conv: cout > 96 unsupported");
    const size_t shm = size_t(x.c) * d.k * d.k * coutT * sizeof(float);
#define STEM_LAUNCH(CT, T) hipLaunchKernelGGL((stem_kernel<CT, T>), dim3(blocks), dim3(256), shm, s, a)
#define STEM_DT(CT)                      \
  do {                                   \
    if (x.dtype == FCE_F16)              \
      STEM_LAUNCH(CT, _Float16);         \
    else if (x.dtype == FCE_F32)         \
      STEM_LAUNCH(CT, float);            \
    else                                 \
      STEM_LAUNCH(CT, uint8_t);          \
  } while (0)
    if (coutT == 16)
      STEM_DT(16);
    else if (coutT == 32)
      STEM_DT(32);
    else if (coutT == 64)
      STEM_DT(64);
    else
      STEM_DT(96);
#undef STEM_DT
#undef STEM_LAUNCH
    return launch_status("stem_kernel");
  }

  FCE_CHECK(x.layout == FCE_NHWC && x.dtype == FCE_F16, "conv: input must be NHWC f16");
  FCE_CHECK(x.cstride % 8 == 0 && x.coff % 8 == 0, "conv: input slice must be 8-channel aligned");

  if (is_dw(d)) {
    FCE_CHECK(d.groups == d.cin && d.cin == d.cout && d.cin % 8 == 0, "dwconv: groups == cin == cout, cin % 8 == 0");
    FCE_CHECK(y.dtype == FCE_F16 && d.up == 0 && res == nullptr && d.epilogue == FCE_EPI_STORE,
              "dwconv: plain f16 store only");
    FCE_CHECK(y.cstride % 8 == 0 && y.coff % 8 == 0, "dwconv: output slice must be 8-aligned");
    DwArgs a{static_cast<const _Float16*>(x.data) + x.coff, x.n, x.h, x.w, x.cstride, d.cin, d.stride, d.k, Ho, Wo,
             static_cast<const float*>(w), bias, static_cast<_Float16*>(y.data) + y.coff, y.cstride, d.act};
    const int64_t total = int64_t(x.n) * Ho * Wo * (d.cin / 8);
    hipLaunchKernelGGL(dwconv_kernel, dim3(grid_cap((total + 255) / 256)), dim3(256), 0, s, a);
    return launch_status("dwconv_kernel");
  }

  FCE_CHECK(d.cin % 8 == 0, "conv: cin must be a multiple of 8");
  int out_kind;
  if (y.dtype == FCE_F32) {
    FCE_CHECK(d.epilogue == FCE_EPI_STORE && res == nullptr, "conv: f32 output supports plain store only");
    out_kind = OUT_F32;
  } else {
    out_kind = d.epilogue == FCE_EPI_WSTORE ? OUT_WSTORE : d.epilogue == FCE_EPI_ACCUM ? OUT_ACCUM : OUT_F16;
  }
  if (res) {
    FCE_CHECK(res->layout == FCE_NHWC && res->dtype == FCE_F16 && res->c == d.cout && res->h == Ho && res->w == Wo,
              "conv: residual must match the output view");
  }
  DenseGeom g = dense_geom(d);
  ConvArgs a;
  a.x = static_cast<const _Float16*>(x.data) + x.coff;
  a.N = x.n;
  a.Hs = x.h;
  a.Ws = x.w;
  a.xcs = x.cstride;
  a.Hin = Hin;
  a.Win = Win;
  a.up = d.up;
  a.cin = d.cin;
  a.cout = d.cout;
  a.stride = d.stride;
  a.Ho = Ho;
  a.Wo = Wo;
  a.P = y.n * Ho * Wo;
  a.w = static_cast<const _Float16*>(w);
  a.bias = bias;
  a.res = res ? static_cast<const _Float16*>(res->data) + res->coff : nullptr;
  a.rcs = res ? res->cstride : 0;
  a.ycs = y.cstride;
  a.y = y.dtype == FCE_F32 ? static_cast<void*>(static_cast<float*>(y.data) + y.coff)
                           : static_cast<void*>(static_cast<_Float16*>(y.data) + y.coff);
  a.act = d.act;
  a.fw = d.fusion_w;
  a.fn = d.fusion_n;
  a.fi = d.fusion_i;
  a.cpt = g.cpt;
  a.nchunk = g.nchunk;
  a.nsteps = g.nsteps;
  a.vec_ok = (y.cstride % 4 == 0 && y.coff % 4 == 0 && (!res || (res->cstride % 4 == 0 && res->coff % 4 == 0))) ? 1 : 0;
  if (out_kind == OUT_WSTORE || out_kind == OUT_ACCUM) FCE_CHECK(d.fusion_w && d.fusion_n > d.fusion_i, "conv: fusion weights");
  const int rc = g.cotiles >= 4 ? 4 : g.cotiles >= 2 ? 2 : 1;
  if (d.k == 1)
    launch_dense_rc<1>(a, out_kind, rc, s);
  else
    launch_dense_rc<3>(a, out_kind, rc, s);
  return launch_status("conv_mfma_kernel");
}

}  // namespace fce
