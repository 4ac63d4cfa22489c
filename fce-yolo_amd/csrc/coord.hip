// FCE coordinate-attention operators (reference ultralytics/nn/modules/fce_block.py):
//   BiCoordCrossAtt  :183-284   CoordAtt :65-116   CoordCrossAtt :119-180
//
// All three are HBM-bound passes over x (NHWC fp16) around a tiny per-image computation:
//   1. pool:   xh[n][y][c] = mean_x x      (row kernel: one block per (n, y), LDS tree reduce)
//              xw[n][x][c] = mean_y x      (column kernel: per (n, y-chunk, x-chunk) partial sums,
//                                           reduced in fixed order by the compute kernel)
//   2. compute (per image): 1x1 projections, axial softmax attention, output projection -> gates
//      (fp32 throughout; deterministic, no atomics)
//   3. apply:  y = id(x) * gate  (vectorised 16-byte NHWC pass; id = optional 1x1 conv into y first)
#include "common.h"

namespace fce {

int conv2d(const fce_conv_desc& d, const fce_tensor& x, const void* w, const float* bias, const fce_tensor* res,
           const fce_tensor& y, hipStream_t s);

static constexpr int ROWS_PER_CHUNK = 16;

struct CoordWs {
  float* xh;       // N*H*C
  float* colpart;  // N*YC*W*C
  float* scratch;  // per op
  float* g1;       // N*H*oup (gate_h / a_h / y_att)
  float* g2;       // N*W*oup (gate_w / a_w)
  int YC;
};

static size_t align_f(size_t n) { return (n + 63) & ~size_t(63); }

static size_t scratch_floats(int kind, const fce_coord_desc& d, int h, int w) {
  const int L = h > w ? h : w;
  if (kind == 0) return size_t(2) * 4 * L * d.mid;  // per image: 2 branches x (q,k,v,y)
  return size_t(h + w) * d.mid * 4;                 // per image: y (+ q,k,v,z for CoordCross)
}

static size_t ws_floats(int kind, const fce_coord_desc& d, int n, int h, int w, CoordWs* out, float* base) {
  const int YC = (h + ROWS_PER_CHUNK - 1) / ROWS_PER_CHUNK;
  size_t off = 0;
  size_t xh = align_f(size_t(n) * h * d.inp), col = align_f(size_t(n) * YC * w * d.inp);
  size_t sc = align_f(size_t(n) * scratch_floats(kind, d, h, w));
  size_t g1 = align_f(size_t(n) * h * d.oup), g2 = align_f(size_t(n) * w * d.oup);
  if (out) {
    out->xh = base + off;
    out->colpart = base + off + xh;
    out->scratch = base + off + xh + col;
    out->g1 = base + off + xh + col + sc;
    out->g2 = base + off + xh + col + sc + g1;
    out->YC = YC;
  }
  return xh + col + sc + g1 + g2;
}

size_t coord_ws_bytes(const fce_coord_desc& d, int n, int h, int w) {
  size_t m = 0;
  for (int k = 0; k < 3; ++k) m = std::max(m, ws_floats(k, d, n, h, w, nullptr, nullptr));
  return m * sizeof(float);
}

// ---------------------------------------------------------------------------- 1. pooling
__global__ __launch_bounds__(256) void pool_rows_kernel(const _Float16* x, int xcs, int H, int W, int C, float* xh) {
  __shared__ float red[256 * 8];
  const int n = blockIdx.y, y = blockIdx.x;
  const int CG = C / 8;
  const int XT = 256 / CG;
  const int t = threadIdx.x;
  const int cg = t % CG, xt = t / CG;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (xt < XT) {
    for (int xx = xt; xx < W; xx += XT) {
      const h8 v = *reinterpret_cast<const h8*>(x + nhwc_off(n, y, xx, H, W, xcs) + cg * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += (float)v[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[t * 8 + j] = acc[j];
  __syncthreads();
  const float inv = 1.0f / (float)W;
  for (int c = t; c < C; c += 256) {
    const int g = c / 8, j = c % 8;
    float s = 0.f;
    for (int k = 0; k < XT; ++k) s += red[(k * CG + g) * 8 + j];
    xh[(int64_t(n) * H + y) * C + c] = s * inv;
  }
}

__global__ __launch_bounds__(256) void pool_cols_kernel(const _Float16* x, int xcs, int H, int W, int C,
                                                        float* colpart, int YC) {
  const int n = blockIdx.z, yc = blockIdx.y;
  const int CG = C / 8;
  const int XW = 256 / CG;
  const int t = threadIdx.x;
  const int cg = t % CG, xi = t / CG;
  const int xx = blockIdx.x * XW + xi;
  if (xi >= XW || xx >= W) return;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int y0 = yc * ROWS_PER_CHUNK, y1 = min(H, y0 + ROWS_PER_CHUNK);
  for (int y = y0; y < y1; ++y) {
    const h8 v = *reinterpret_cast<const h8*>(x + nhwc_off(n, y, xx, H, W, xcs) + cg * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += (float)v[j];
  }
  float* o = colpart + ((int64_t(n) * YC + yc) * W + xx) * C + cg * 8;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = acc[j];
}

// xw[x][c] for image n, reduced in fixed chunk order
__device__ __forceinline__ float xw_at(const float* colpart, int n, int YC, int W, int C, int xx, int c, float invH) {
  float s = 0.f;
  for (int k = 0; k < YC; ++k) s += colpart[((int64_t(n) * YC + k) * W + xx) * C + c];
  return s * invH;
}

// ---------------------------------------------------------------------------- 2. compute
struct CoordArgs {
  fce_coord_desc d;
  int H, W;
  CoordWs ws;
};

// out[i][m] = act(sum_c Wt[m][c] * src(i, c) + b[m]) for i < L, m < M; src given by a functor
template <typename Src>
__device__ void proj(const float* Wt, const float* b, int M, int K, int L, Src src, float* out, int act) {
  for (int e = threadIdx.x; e < L * M; e += blockDim.x) {
    const int i = e / M, m = e % M;
    const float* wr = Wt + int64_t(m) * K;
    float s = b ? b[m] : 0.f;
    for (int c = 0; c < K; ++c) s += wr[c] * src(i, c);
    out[int64_t(i) * M + m] = act == 1 ? silu(s) : s;
  }
}

// y[i][h*dh+d] = sum_j softmax_j(scale * q_i . k_j) v[j][h*dh+d]  (per head, axial)
__device__ void axial_attention(const float* q, const float* k, const float* v, int Lq, int Lk, int mid, int heads,
                                float scale, float* y) {
  const int dh = mid / heads;
  for (int e = threadIdx.x; e < Lq * heads; e += blockDim.x) {
    const int i = e / heads, hd = e % heads;
    const float* qi = q + int64_t(i) * mid + hd * dh;
    float mx = -INFINITY;
    for (int j = 0; j < Lk; ++j) {
      const float* kj = k + int64_t(j) * mid + hd * dh;
      float s = 0.f;
      for (int d = 0; d < dh; ++d) s += qi[d] * kj[d];
      mx = fmaxf(mx, s * scale);
    }
    float den = 0.f;
    for (int j = 0; j < Lk; ++j) {
      const float* kj = k + int64_t(j) * mid + hd * dh;
      float s = 0.f;
      for (int d = 0; d < dh; ++d) s += qi[d] * kj[d];
      den += expf(s * scale - mx);
    }
    const float inv = 1.0f / den;
    for (int d0 = 0; d0 < dh; d0 += 16) {
      float acc[16];
#pragma unroll
      for (int t = 0; t < 16; ++t) acc[t] = 0.f;
      for (int j = 0; j < Lk; ++j) {
        const float* kj = k + int64_t(j) * mid + hd * dh;
        float s = 0.f;
        for (int d = 0; d < dh; ++d) s += qi[d] * kj[d];
        const float p = expf(s * scale - mx) * inv;
        const float* vj = v + int64_t(j) * mid + hd * dh + d0;
#pragma unroll
        for (int t = 0; t < 16; ++t)
          if (d0 + t < dh) acc[t] += p * vj[t];
      }
      for (int t = 0; t < 16 && d0 + t < dh; ++t) y[int64_t(i) * mid + hd * dh + d0 + t] = acc[t];
    }
  }
}

__device__ __forceinline__ void block_sync_global() {
  __threadfence_block();
  __syncthreads();
}

// BiCoordCrossAtt: grid (N, 2): branch 0 = H branch (q from x_h, k/v from x_w) -> gate_h[H][oup]
//                                branch 1 = W branch (q from x_w, k/v from x_h) -> gate_w[W][oup]
__global__ __launch_bounds__(256) void bicoord_compute_kernel(CoordArgs a) {
  const int n = blockIdx.x, br = blockIdx.y;
  const int C = a.d.inp, H = a.H, W = a.W, mid = a.d.mid, YC = a.ws.YC;
  const int L = H > W ? H : W;
  float* base = a.ws.scratch + (int64_t(n) * 2 + br) * 4 * L * mid;
  float *q = base, *k = base + L * mid, *v = base + 2 * L * mid, *y = base + 3 * L * mid;
  const float* xh = a.ws.xh + int64_t(n) * H * C;
  const float* colp = a.ws.colpart;
  const float invH = 1.0f / (float)H;
  auto src_h = [&](int i, int c) { return xh[int64_t(i) * C + c]; };
  auto src_w = [&](int i, int c) { return xw_at(colp, n, YC, W, C, i, c, invH); };
  const int Lq = br == 0 ? H : W, Lk = br == 0 ? W : H;
  const int wq = br == 0 ? 0 : 3;  // weight index base: q,k,v
  if (br == 0) {
    proj(a.d.w[wq + 0], a.d.b[wq + 0], mid, C, Lq, src_h, q, 0);
    proj(a.d.w[wq + 1], a.d.b[wq + 1], mid, C, Lk, src_w, k, 0);
    proj(a.d.w[wq + 2], a.d.b[wq + 2], mid, C, Lk, src_w, v, 0);
  } else {
    proj(a.d.w[wq + 0], a.d.b[wq + 0], mid, C, Lq, src_w, q, 0);
    proj(a.d.w[wq + 1], a.d.b[wq + 1], mid, C, Lk, src_h, k, 0);
    proj(a.d.w[wq + 2], a.d.b[wq + 2], mid, C, Lk, src_h, v, 0);
  }
  block_sync_global();
  axial_attention(q, k, v, Lq, Lk, mid, a.d.heads, a.d.scale, y);
  block_sync_global();
  float* gate = (br == 0 ? a.ws.g1 + int64_t(n) * H * a.d.oup : a.ws.g2 + int64_t(n) * W * a.d.oup);
  auto src_y = [&](int i, int m) { return y[int64_t(i) * mid + m]; };
  proj(a.d.w[6 + br], a.d.b[6 + br], a.d.oup, mid, Lq, src_y, gate, 0);
}

// CoordAtt: one block per image.  y = SiLU(cv1(cat[x_h, x_w])) ; a_h = sigmoid(cv_h(y_h)) ; a_w = sigmoid(cv_w(y_w))
__global__ __launch_bounds__(256) void coordatt_compute_kernel(CoordArgs a) {
  const int n = blockIdx.x;
  const int C = a.d.inp, H = a.H, W = a.W, mid = a.d.mid, YC = a.ws.YC;
  float* y = a.ws.scratch + int64_t(n) * (H + W) * mid * 4;
  const float* xh = a.ws.xh + int64_t(n) * H * C;
  const float invH = 1.0f / (float)H;
  auto src_cat = [&](int i, int c) {
    return i < H ? xh[int64_t(i) * C + c] : xw_at(a.ws.colpart, n, YC, W, C, i - H, c, invH);
  };
  proj(a.d.w[0], a.d.b[0], mid, C, H + W, src_cat, y, 1);
  block_sync_global();
  auto src_yh = [&](int i, int m) { return y[int64_t(i) * mid + m]; };
  auto src_yw = [&](int i, int m) { return y[int64_t(H + i) * mid + m]; };
  float* ah = a.ws.g1 + int64_t(n) * H * a.d.oup;
  float* aw = a.ws.g2 + int64_t(n) * W * a.d.oup;
  proj(a.d.w[1], a.d.b[1], a.d.oup, mid, H, src_yh, ah, 0);
  proj(a.d.w[2], a.d.b[2], a.d.oup, mid, W, src_yw, aw, 0);
  block_sync_global();
  for (int e = threadIdx.x; e < H * a.d.oup; e += blockDim.x) ah[e] = 1.0f / (1.0f + expf(-ah[e]));
  for (int e = threadIdx.x; e < W * a.d.oup; e += blockDim.x) aw[e] = 1.0f / (1.0f + expf(-aw[e]));
}

// CoordCrossAtt: one block per image.  y = cv1(cat) (no act); q = q_conv(y_h), k/v = k/v_conv(y_w);
// z = softmax_W(q k^T * scale) v ; y_att = sigmoid(proj(z))  [H][oup]
__global__ __launch_bounds__(256) void coordcross_compute_kernel(CoordArgs a) {
  const int n = blockIdx.x;
  const int C = a.d.inp, H = a.H, W = a.W, mid = a.d.mid, YC = a.ws.YC;
  float* base = a.ws.scratch + int64_t(n) * (H + W) * mid * 4;
  float* y = base;                       // (H+W) x mid
  float* q = base + (H + W) * mid;       // H x mid
  float* k = q + H * mid;                // W x mid
  float* v = k + W * mid;                // W x mid
  float* z = v + W * mid;                // H x mid  (fits: (H+W)*mid*4 >= (H+W)+H+2W+H)
  const float* xh = a.ws.xh + int64_t(n) * H * C;
  const float invH = 1.0f / (float)H;
  auto src_cat = [&](int i, int c) {
    return i < H ? xh[int64_t(i) * C + c] : xw_at(a.ws.colpart, n, YC, W, C, i - H, c, invH);
  };
  proj(a.d.w[0], a.d.b[0], mid, C, H + W, src_cat, y, 0);
  block_sync_global();
  auto src_yh = [&](int i, int m) { return y[int64_t(i) * mid + m]; };
  auto src_yw = [&](int i, int m) { return y[int64_t(H + i) * mid + m]; };
  proj(a.d.w[1], a.d.b[1], mid, mid, H, src_yh, q, 0);
  proj(a.d.w[2], a.d.b[2], mid, mid, W, src_yw, k, 0);
  proj(a.d.w[3], a.d.b[3], mid, mid, W, src_yw, v, 0);
  block_sync_global();
  axial_attention(q, k, v, H, W, mid, a.d.heads, a.d.scale, z);
  block_sync_global();
  float* g = a.ws.g1 + int64_t(n) * H * a.d.oup;
  auto src_z = [&](int i, int m) { return z[int64_t(i) * mid + m]; };
  proj(a.d.w[4], a.d.b[4], a.d.oup, mid, H, src_z, g, 0);
  block_sync_global();
  for (int e = threadIdx.x; e < H * a.d.oup; e += blockDim.x) g[e] = 1.0f / (1.0f + expf(-g[e]));
}

// ---------------------------------------------------------------------------- 3. apply
enum { GATE_BICOORD = 0, GATE_COORD = 1, GATE_ROW = 2 };

template <int MODE>
__global__ __launch_bounds__(256) void gate_apply_kernel(const _Float16* x, int xcs, _Float16* y, int ycs, int N,
                                                         int H, int W, int C, const float* g1, const float* g2) {
  const int CG = C / 8;
  const int64_t total = int64_t(N) * H * W * CG;
  for (int64_t t = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; t < total; t += int64_t(gridDim.x) * blockDim.x) {
    const int g = int(t % CG);
    const int64_t pix = t / CG;
    const int xx = int(pix % W), yy = int((pix / W) % H), n = int(pix / (int64_t(W) * H));
    const h8 v = *reinterpret_cast<const h8*>(x + pix * xcs + g * 8);
    const float* gh = g1 + (int64_t(n) * H + yy) * C + g * 8;
    const f4 gh0 = *reinterpret_cast<const f4*>(gh), gh1 = *reinterpret_cast<const f4*>(gh + 4);
    float gv[8] = {gh0[0], gh0[1], gh0[2], gh0[3], gh1[0], gh1[1], gh1[2], gh1[3]};
    float wv[8] = {1, 1, 1, 1, 1, 1, 1, 1};
    if (MODE != GATE_ROW) {
      const float* gw = g2 + (int64_t(n) * W + xx) * C + g * 8;
      const f4 gw0 = *reinterpret_cast<const f4*>(gw), gw1 = *reinterpret_cast<const f4*>(gw + 4);
      wv[0] = gw0[0]; wv[1] = gw0[1]; wv[2] = gw0[2]; wv[3] = gw0[3];
      wv[4] = gw1[0]; wv[5] = gw1[1]; wv[6] = gw1[2]; wv[7] = gw1[3];
    }
    h8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float r;
      if (MODE == GATE_BICOORD)
        r = (float)v[j] * (1.0f / (1.0f + __expf(-(gv[j] + wv[j]))));
      else if (MODE == GATE_COORD)
        r = (float)v[j] * gv[j] * wv[j];
      else
        r = (float)v[j] * gv[j];
      o[j] = (_Float16)r;
    }
    *reinterpret_cast<h8*>(y + pix * ycs + g * 8) = o;
  }
}

// ---------------------------------------------------------------------------- host
static int coord_common(int kind, const fce_coord_desc& d, const fce_tensor& x, const fce_tensor& y, void* ws,
                        size_t ws_bytes, hipStream_t s) {
  FCE_CHECK(x.layout == FCE_NHWC && y.layout == FCE_NHWC && x.dtype == FCE_F16 && y.dtype == FCE_F16,
            "coord attention: NHWC f16 views");
  FCE_CHECK(x.c == d.inp && y.c == d.oup && x.n == y.n && x.h == y.h && x.w == y.w, "coord attention: shape mismatch");
  FCE_CHECK(d.inp % 8 == 0 && d.oup % 8 == 0 && d.inp <= 2048, "coord attention: channels % 8 == 0, <= 2048");
  FCE_CHECK(x.cstride % 8 == 0 && x.coff % 8 == 0 && y.cstride % 8 == 0 && y.coff % 8 == 0,
            "coord attention: 8-channel aligned slices");
  FCE_CHECK(d.mid > 0 && d.heads > 0 && d.mid % d.heads == 0, "coord attention: mid % heads == 0");
  FCE_CHECK(d.inp == d.oup || d.id_w, "coord attention: identity conv required when inp != oup");
  FCE_CHECK(!(kind == 2 && d.inp != d.oup), "CoordCrossAtt requires oup == inp (fce_block.py:180, Q3)");
  const int N = x.n, H = x.h, W = x.w;
  if (int64_t(N) * H * W == 0) return FCE_OK;
  FCE_CHECK(ws && ws_bytes >= coord_ws_bytes(d, N, H, W), "coord attention: workspace too small");
  CoordArgs a;
  a.d = d;
  a.H = H;
  a.W = W;
  ws_floats(kind, d, N, H, W, &a.ws, static_cast<float*>(ws));
  const _Float16* xp = static_cast<const _Float16*>(x.data) + x.coff;
  hipLaunchKernelGGL(pool_rows_kernel, dim3(H, N), dim3(256), 0, s, xp, x.cstride, H, W, d.inp, a.ws.xh);
  const int XW = 256 / (d.inp / 8);
  hipLaunchKernelGGL(pool_cols_kernel, dim3((W + XW - 1) / XW, a.ws.YC, N), dim3(256), 0, s, xp, x.cstride, H, W,
                     d.inp, a.ws.colpart, a.ws.YC);
  if (kind == 0)
    hipLaunchKernelGGL(bicoord_compute_kernel, dim3(N, 2), dim3(256), 0, s, a);
  else if (kind == 1)
    hipLaunchKernelGGL(coordatt_compute_kernel, dim3(N), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(coordcross_compute_kernel, dim3(N), dim3(256), 0, s, a);
  int st = launch_status("coord compute");
  if (st) return st;
  // identity branch (1x1 conv with bias, no act) written into y first, then gated in place
  const _Float16* src = xp;
  int scs = x.cstride;
  if (d.inp != d.oup) {
    fce_conv_desc cd{d.inp, d.oup, 1, 1, 1, FCE_ACT_NONE, 0, FCE_EPI_STORE, nullptr, 0, 0};
    st = conv2d(cd, x, d.id_w, d.id_b, nullptr, y, s);
    if (st) return st;
    src = static_cast<const _Float16*>(y.data) + y.coff;
    scs = y.cstride;
  }
  _Float16* yp = static_cast<_Float16*>(y.data) + y.coff;
  const int64_t total = int64_t(N) * H * W * (d.oup / 8);
  const int blocks = int(std::min<int64_t>((total + 255) / 256, 65535 * 8));
  if (kind == 0)
    hipLaunchKernelGGL(gate_apply_kernel<GATE_BICOORD>, dim3(blocks), dim3(256), 0, s, src, scs, yp, y.cstride, N, H,
                       W, d.oup, a.ws.g1, a.ws.g2);
  else if (kind == 1)
    hipLaunchKernelGGL(gate_apply_kernel<GATE_COORD>, dim3(blocks), dim3(256), 0, s, src, scs, yp, y.cstride, N, H,
                       W, d.oup, a.ws.g1, a.ws.g2);
  else
    hipLaunchKernelGGL(gate_apply_kernel<GATE_ROW>, dim3(blocks), dim3(256), 0, s, src, scs, yp, y.cstride, N, H, W,
                       d.oup, a.ws.g1, a.ws.g2);
  return launch_status("gate_apply_kernel");
}

int bicoordcrossatt(const fce_coord_desc& d, const fce_tensor& x, const fce_tensor& y, void* ws, size_t wsb,
                    hipStream_t s) {
  return coord_common(0, d, x, y, ws, wsb, s);
}
int coordatt(const fce_coord_desc& d, const fce_tensor& x, const fce_tensor& y, void* ws, size_t wsb, hipStream_t s) {
  return coord_common(1, d, x, y, ws, wsb, s);
}
int coordcrossatt(const fce_coord_desc& d, const fce_tensor& x, const fce_tensor& y, void* ws, size_t wsb,
                  hipStream_t s) {
  return coord_common(2, d, x, y, ws, wsb, s);
}

}  // namespace fce
