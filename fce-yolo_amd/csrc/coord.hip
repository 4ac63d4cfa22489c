// FCE coordinate-attention operators (reference ultralytics/nn/modules/fce_block.py):
//   BiCoordCrossAtt  :183-284   CoordAtt :65-116   CoordCrossAtt :119-180
//
// All three are HBM-bound passes over x (NHWC fp16) around a small per-image computation:
//   1. pool:    xh[n][y][c] = mean_x x   (one block per (n, y): 16-byte loads, LDS tree reduce)
//               xw[n][x][c] = mean_y x   (one block per (n, column strip): each thread owns 8 channels
//                                         of one column and walks all rows; no cross-thread reduce)
//   2. project: 1x1 convs on the pooled vectors as "jobs" (src rows staged in LDS, weights stored
//               transposed [in][out] so a wave reads one contiguous row per input channel)
//   3. attend:  axial softmax attention per (image, branch, query tile) with K/V in LDS, online
//               softmax in registers, then the output projection from LDS -> gates (fp32)
//   4. apply:   y = id(x) * gate, one vectorised 16-byte NHWC pass (id = optional 1x1 conv into y first)
// Everything is deterministic (fixed reduction orders, no atomics).
#include "common.h"

#include <algorithm>
#include <vector>

namespace fce {

int conv2d(const fce_conv_desc& d, const fce_tensor& x, const void* w, const float* bias, const fce_tensor* res,
           const fce_tensor& y, hipStream_t s, int tile = -1, const fce_tensor* dup = nullptr, int duplo = 0);

enum { ACT_NONE_ = 0, ACT_SILU_ = 1, ACT_SIGMOID_ = 2 };

struct CoordWs {
  float* xh;      // N*H*C
  float* xw;      // N*W*C
  float* part;    // N*bands*W*C: column sums of each row band (band pooling)
  float* buf[6];  // N*L*mid each
  float* g1;      // N*H*oup
  float* g2;      // N*W*oup
};

static size_t align_f(size_t n) { return (n + 63) & ~size_t(63); }

// Band pooling (one read of x) for C >= 256 (C % 64 == 0, W <= 256); rows per band so that the grid has >= 512
// blocks when it can.  At C = 128 (n scale) the two-pass kernel stays: its extra read hits L2 and the band path's
// second launch costs more (n L5 58.5 vs 62.0 us per call; l L5 256 -> 252, m L5 434.5 -> 422.6, r03r)
static constexpr int kBandMaxK = 8;  // columns per thread: W <= 32 * kBandMaxK
static bool band_pool_ok(int C, int W) { return C >= 256 && C % 64 == 0 && W <= 32 * kBandMaxK; }
// Rows per pooling band: fixed.  The column means add the bands' partial sums, so the band height sets the
// summation order; a height chosen by batch size (8 rows below 512 blocks, as before) made an image's pooled
// columns depend on its batch whenever the fp32 sums were inexact (test_batch_invariance, m-h8 1280 bs16).
// (Round 5: 32-row bands halve the fp32 partials the column pass reads back, but l32 / m16 BiCoord calls took
// 254.8 / 419.3 us against 249.7 / 415.3 us with 16: half the blocks.)
static int band_rows(int, int, int) { return 16; }

static size_t ws_layout(const fce_coord_desc& d, int n, int h, int w, CoordWs* out, float* base) {
  const int L = h > w ? h : w;
  const int mx = d.mid > d.oup ? d.mid : d.oup;
  size_t off = 0;
  auto take = [&](size_t cnt) {
    float* p = base ? base + off : nullptr;
    off += align_f(cnt);
    return p;
  };
  CoordWs ws;
  ws.xh = take(size_t(n) * h * d.inp);
  ws.xw = take(size_t(n) * w * d.inp);
  const int R = band_rows(n, h, d.inp);
  ws.part = band_pool_ok(d.inp, w) ? take(size_t(n) * ((h + R - 1) / R) * w * d.inp) : nullptr;
  for (int i = 0; i < 6; ++i) ws.buf[i] = take(size_t(n) * L * mx);
  ws.g1 = take(size_t(n) * h * d.oup);
  ws.g2 = take(size_t(n) * w * d.oup);
  if (out) *out = ws;
  return off;
}

size_t coord_ws_bytes(const fce_coord_desc& d, int n, int h, int w) {
  return ws_layout(d, n, h, w, nullptr, nullptr) * sizeof(float);
}

// ---------------------------------------------------------------------------- 1. pooling
// sums of fp16 values as v_fma_mix_f32 (acc + h * 1: one op, bitwise the add of the converted half)
static __device__ __constant__ float kOnes8[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
__device__ __forceinline__ void pool_rows(const _Float16* x, int xcs, int H, int W, int C, float* xh, int y, int n) {
  __shared__ float red[256 * 8];
  const int CG = C / 8;
  const int XT = 256 / CG;
  const int t = threadIdx.x;
  const int cg = t % CG, xt = t / CG;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (xt < XT) {
    for (int xx = xt; xx < W; xx += XT) {
      const h8 v = *reinterpret_cast<const h8*>(x + nhwc_off(n, y, xx, H, W, xcs) + cg * 8);
      fma8_mix(v, kOnes8, acc);
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

// column means: a block owns XW = 256 / (CG * RG) columns; thread (cg, column, row group) sums its RG-th
// share of the rows (contiguous row ranges, 8 loads in flight), the RG partials are added in row-group
// order through LDS (fixed order: deterministic)
__device__ __forceinline__ int pool_col_groups(int C, int H) {
  const int CG = C / 8;
  int RG = 1;
  while (RG < 8 && CG * RG * 2 <= 256 && H >= 16 * RG) RG *= 2;
  return RG;
}

__device__ __forceinline__ void pool_cols(const _Float16* x, int xcs, int H, int W, int C, float* xw, int bx, int n) {
  __shared__ float part[256 * 8];
  const int CG = C / 8;
  const int RG = pool_col_groups(C, H);
  const int XW = 256 / (CG * RG);
  const int t = threadIdx.x;
  const int cg = t % CG, xi = (t / CG) % XW, rg = t / (CG * XW);
  const int xx = bx * XW + xi;
  const bool live = rg < RG && xx < W;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (live) {
    const int rows = (H + RG - 1) / RG, y0 = rg * rows, y1 = min(H, y0 + rows);
    const _Float16* p = x + nhwc_off(n, 0, xx, H, W, xcs) + cg * 8;
    const int64_t rs = int64_t(W) * xcs;
    int y = y0;
    for (; y + 7 < y1; y += 8) {
      h8 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = *reinterpret_cast<const h8*>(p + (y + k) * rs);
#pragma unroll
      for (int k = 0; k < 8; ++k)
        fma8_mix(v[k], kOnes8, acc);
    }
    for (; y < y1; ++y) {
      const h8 v0 = *reinterpret_cast<const h8*>(p + y * rs);
      fma8_mix(v0, kOnes8, acc);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) part[t * 8 + j] = acc[j];
  __syncthreads();
  if (rg == 0 && live) {
    const float inv = 1.0f / (float)H;
    float* o = xw + (int64_t(n) * W + xx) * C + cg * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float sum = part[t * 8 + j];
      for (int r = 1; r < RG; ++r) sum += part[(t + r * CG * XW) * 8 + j];
      o[j] = sum * inv;
    }
  }
}

// both poolings in one launch: per image H row blocks (a row each) then the column-strip blocks (XW columns
// each).  The 1-D grid is XCD-aware: block b runs on XCD b % 8, and all blocks of image n sit on XCD n % 8 in
// that order, so an image's column strips re-read its rows from the L2 that the row blocks just filled
// instead of from another XCD's fabric path.  Blocks past the last image exit at once.  Below 8 images
// (aff = 0) the blocks of an image spread over every XCD instead, so a small batch still uses the whole chip.
__global__ __launch_bounds__(256) void pool_kernel(const _Float16* x, int xcs, int H, int W, int C, float* xh,
                                                   float* xw, int N, int BPI, int aff) {
  const int b = int(blockIdx.x);
  int n, j;
  if (aff) {
    const int xcd = b & 7, slot = b >> 3, il = slot / BPI;
    j = slot - il * BPI;
    n = il * 8 + xcd;
  } else {
    n = b / BPI;
    j = b - n * BPI;
  }
  if (n >= N) return;
  if (j < H)
    pool_rows(x, xcs, H, W, C, xh, j, n);
  else
    pool_cols(x, xcs, H, W, C, xw, j - H, n);
}

// Band pooling: x is read ONCE.  Block (image n, band of R rows, 64-channel slice): thread (cg = t & 7, xt = t >> 3)
// loads the 8 channels cg of its columns xx = xt + 32 k of every band row; per row it adds them into its column
// sums (registers) and its row sum, the 32 row sums of a channel group are added by an xor tree over the 8 lanes of
// the wave that share cg and then over the 4 waves in order (LDS), so the row means come out complete; the column
// sums of the band go to part[n][band][x][c] and pool_band_cols_kernel adds the bands in order.  Fixed orders
// throughout: deterministic.  (The two-pass pool_kernel above re-reads x for the columns: 1.19-1.45x the
// algorithmic bytes in PMC.)
template <int R, int KW>
__global__ __launch_bounds__(256) void pool_band_kernel(const _Float16* x, int xcs, int H, int W, int C, float* xh,
                                                        float* part, int NB) {
  __shared__ float red[R][4][64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int cg = t & 7, xt = t >> 3;
  const int ncs = C >> 6;
  int b = int(blockIdx.x);
  const int cs = b % ncs;
  b /= ncs;
  const int band = b % NB, n = b / NB;
  const int y0 = band * R, y1 = min(H, y0 + R);
  const int c0 = cs * 64 + cg * 8;
  const _Float16* xn = x + nhwc_off(n, 0, 0, H, W, xcs) + c0;
  float col[KW][8];
#pragma unroll
  for (int k = 0; k < KW; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) col[k][j] = 0.f;
  for (int y = y0; y < y1; ++y) {
    h8 v[KW];
#pragma unroll
    for (int k = 0; k < KW; ++k) {
      const int xx = xt + 32 * k;
      v[k] = xx < W ? *reinterpret_cast<const h8*>(xn + (int64_t(y) * W + xx) * xcs) : h8{};
    }
    float r[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < KW; ++k) {
      fma8_mix(v[k], kOnes8, col[k]);
      fma8_mix(v[k], kOnes8, r);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      r[j] += __shfl_xor(r[j], 8);
      r[j] += __shfl_xor(r[j], 16);
      r[j] += __shfl_xor(r[j], 32);
    }
    if (lane < 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) red[y - y0][wave][cg * 8 + j] = r[j];
    }
  }
  __syncthreads();
  const float inv = 1.0f / (float)W;
  for (int e = t; e < (y1 - y0) * 64; e += 256) {
    const int yy = e >> 6, c = e & 63;
    const float sum = ((red[yy][0][c] + red[yy][1][c]) + red[yy][2][c]) + red[yy][3][c];
    xh[(int64_t(n) * H + y0 + yy) * C + cs * 64 + c] = sum * inv;
  }
  float* pb = part + (int64_t(n) * NB + band) * W * C + c0;
#pragma unroll
  for (int k = 0; k < KW; ++k) {
    const int xx = xt + 32 * k;
    if (xx < W) {
      float* o = pb + int64_t(xx) * C;
      *reinterpret_cast<f4*>(o) = f4{col[k][0], col[k][1], col[k][2], col[k][3]};
      *reinterpret_cast<f4*>(o + 4) = f4{col[k][4], col[k][5], col[k][6], col[k][7]};
    }
  }
}

// xw[n][x][c] = (sum over bands, in order, of part[n][band][x][c]) / H; 4 channels per thread
__global__ __launch_bounds__(256) void pool_band_cols_kernel(const float* part, float* xw, int N, int NB, int H, int WC) {
  const int64_t e = (int64_t(blockIdx.x) * 256 + threadIdx.x) * 4;
  if (e >= int64_t(N) * WC) return;
  const int64_t n = e / WC, r = e - n * WC;
  const float* p = part + n * NB * WC + r;
  f4 s = *reinterpret_cast<const f4*>(p);
  for (int b = 1; b < NB; ++b) {
    const f4 v = *reinterpret_cast<const f4*>(p + int64_t(b) * WC);
    s = f4{s[0] + v[0], s[1] + v[1], s[2] + v[2], s[3] + v[3]};
  }
  const float inv = 1.0f / (float)H;
  *reinterpret_cast<f4*>(xw + e) = f4{s[0] * inv, s[1] * inv, s[2] * inv, s[3] * inv};
}

// ---------------------------------------------------------------------------- 2. projections
struct ProjJob {
  const float* src;  // [N][L][K]
  const float* wt;   // [K][M]  (transposed 1x1 weight)
  const float* b;    // [M]
  float* dst;        // [N][L][M]
  int L, K, M, act;
};
struct ProjArgs {
  ProjJob job[6];
};

__device__ __forceinline__ float act_f(float v, int act) {
  return act == ACT_SILU_ ? v / (1.0f + expf(-v)) : act == ACT_SIGMOID_ ? 1.0f / (1.0f + expf(-v)) : v;
}

// grid (position tiles, jobs, N): a block computes TP positions x all M outputs of one job.  K is
// walked in chunks of KC: the TP x KC source slice and the KC x M weight slice are staged in LDS with
// coalesced loads, then every thread accumulates its (position, output) pairs from LDS (consecutive
// threads = consecutive outputs: conflict-free weight reads, broadcast source reads).
__global__ __launch_bounds__(256) void coord_proj_kernel(ProjArgs pa, int TP, int KC) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const ProjJob& jb = pa.job[blockIdx.y];
  const int n = blockIdx.z;
  const int p0 = blockIdx.x * TP;
  if (p0 >= jb.L) return;
  const int np = min(TP, jb.L - p0), M = jb.M, K = jb.K;
  float* ss = sm;              // [TP][KC]
  float* ws = sm + TP * KC;    // [KC][M]
  constexpr int OPT = 16;      // outputs per thread (TP * M <= 256 * OPT)
  float acc[OPT];
#pragma unroll
  for (int i = 0; i < OPT; ++i) {
    const int e = threadIdx.x + i * 256;
    acc[i] = (e < np * M && jb.b) ? jb.b[e % M] : 0.f;
  }
  const float* src = jb.src + (int64_t(n) * jb.L + p0) * K;
  for (int k0 = 0; k0 < K; k0 += KC) {
    const int kc = min(KC, K - k0);
    __syncthreads();
    // staging in rounds of 8 loads per thread issued back to back (a load -> LDS-store loop otherwise
    // waits out one memory latency per element); loads use clamped indices and the stores of the
    // out-of-range slots go to one dummy float past the weights, so neither is conditional
    float* dummy = ws + KC * M;
    const int n1 = np * kc, n2 = kc * M;
    for (int e0 = 0; e0 < n1; e0 += 8 * 256) {
      float v[8];
      float* d[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + int(threadIdx.x) + 256 * u, ec = min(e, n1 - 1);
        const int i = ec / kc, c = ec - i * kc;
        v[u] = src[int64_t(i) * K + k0 + c];
        d[u] = e < n1 ? ss + i * KC + c : dummy;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) *d[u] = v[u];
    }
    for (int e0 = 0; e0 < n2; e0 += 8 * 256) {
      float v[8];
      float* d[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + int(threadIdx.x) + 256 * u;
        v[u] = jb.wt[int64_t(k0) * M + min(e, n2 - 1)];
        d[u] = e < n2 ? ws + e : dummy;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) *d[u] = v[u];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < OPT; ++i) {
      const int e = threadIdx.x + i * 256;
      if (e >= np * M) break;
      const int pi = e / M, m = e - pi * M;
      const float* sp = ss + pi * KC;
      float t = acc[i];
      for (int c = 0; c < kc; ++c) t += sp[c] * ws[c * M + m];
      acc[i] = t;
    }
  }
  float* dst = jb.dst + (int64_t(n) * jb.L + p0) * M;
#pragma unroll
  for (int i = 0; i < OPT; ++i) {
    const int e = threadIdx.x + i * 256;
    if (e < np * M) dst[e] = act_f(acc[i], jb.act);
  }
}

// Register-tiled form (every M % 4 == 0): a thread owns 4 positions x 4 consecutive outputs and reads,
// per k, one 16-byte weight quad (consecutive lanes = consecutive quads: conflict-free) and 4 source
// values (broadcast over the 16 lanes sharing the positions; source rows padded by 4 floats so the 4
// position groups of a wave land on distinct banks): 16 FMAs per 5 LDS reads instead of 1 per 2.  Each
// output still accumulates bias + sum over k in k order with FMAs: bitwise equal to coord_proj_kernel.
constexpr int PJ_TPT = 2;  // tasks (4 x 4 output tiles) per thread
__global__ __launch_bounds__(256) void coord_proj4_kernel(ProjArgs pa, int TP, int KC) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const ProjJob& jb = pa.job[blockIdx.y];
  const int n = blockIdx.z;
  const int p0 = blockIdx.x * TP;
  if (p0 >= jb.L) return;
  const int np = min(TP, jb.L - p0), M = jb.M, K = jb.K, KCP = KC + 4;
  float* ss = sm;              // [TP][KCP]
  float* ws = sm + TP * KCP;   // [KC][M]
  const int mq = M >> 2, ntask = ((np + 3) >> 2) * mq;
  f4 acc[PJ_TPT][4];
#pragma unroll
  for (int u = 0; u < PJ_TPT; ++u) {
    const int t = threadIdx.x + u * 256;
    const int m4 = (t % mq) * 4;
    const f4 b = (t < ntask && jb.b) ? *reinterpret_cast<const f4*>(jb.b + m4) : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[u][q] = b;
  }
  const float* src = jb.src + (int64_t(n) * jb.L + p0) * K;
  for (int k0 = 0; k0 < K; k0 += KC) {
    const int kc = min(KC, K - k0);
    __syncthreads();
    // 16-byte staging (K, kc, M multiples of 4), 8 quads per thread in flight per round: one round covers
    // 32 KiB, so a chunk usually stages in one memory round trip
    float* dummy = ws + KC * M;  // 4 floats past the weights
    const int kq = kc >> 2, n1 = np * kq, n2 = kc * M / 4, nt = n1 + n2;
    for (int e0 = 0; e0 < nt; e0 += 8 * 256) {
      f4 v[8];
      float* d[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + int(threadIdx.x) + 256 * u;
        const bool s1 = e < n1;  // address selects only: every load unconditional
        const int i = s1 ? e / kq : 0, c4 = s1 ? (e - i * kq) * 4 : 0;
        const int e2 = s1 ? 0 : min(e - n1, n2 - 1);
        const float* sp = s1 ? src + int64_t(i) * K + k0 + c4 : jb.wt + int64_t(k0) * M + 4 * e2;
        d[u] = s1 ? ss + i * KCP + c4 : (e < nt ? ws + 4 * e2 : dummy);
        v[u] = *reinterpret_cast<const f4*>(sp);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) *reinterpret_cast<f4*>(d[u]) = v[u];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < PJ_TPT; ++u) {
      const int t = threadIdx.x + u * 256;
      if (t >= ntask) break;
      const int pi = (t / mq) * 4, m4 = (t % mq) * 4;
      // rows past np read unstaged LDS: computed, never stored
      const float* sr[4] = {ss + min(pi + 0, TP - 1) * KCP, ss + min(pi + 1, TP - 1) * KCP,
                            ss + min(pi + 2, TP - 1) * KCP, ss + min(pi + 3, TP - 1) * KCP};
      for (int c = 0; c < kc; ++c) {
        const f4 w = *reinterpret_cast<const f4*>(ws + c * M + m4);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float sv = sr[q][c];
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[u][q][j] += sv * w[j];
        }
      }
    }
  }
  float* dst = jb.dst + (int64_t(n) * jb.L + p0) * M;
#pragma unroll
  for (int u = 0; u < PJ_TPT; ++u) {
    const int t = threadIdx.x + u * 256;
    if (t >= ntask) break;
    const int pi = (t / mq) * 4, m4 = (t % mq) * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (pi + q >= np) break;
      f4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = act_f(acc[u][q][j], jb.act);
      *reinterpret_cast<f4*>(dst + (pi + q) * M + m4) = o;
    }
  }
}

// ---------------------------------------------------------------------------- 3. attention + out proj
struct AttJob {
  const float* q;   // [N][Lq][mid]
  const float* k;   // [N][Lk][mid]
  const float* v;   // [N][Lk][mid]
  const float* wt;  // [mid][oup]
  const float* b;   // [oup]
  float* dst;       // [N][Lq][oup]
  int Lq, Lk, act;
};
struct AttArgs {
  AttJob job[2];
  int mid, heads, oup, QT;
  float scale;
  int wlds;  // output-projection weights staged in LDS
};

template <int DH>
__global__ __launch_bounds__(256) void coord_attend_kernel(AttArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const AttJob& jb = a.job[blockIdx.y];
  const int n = blockIdx.z;
  const int i0 = blockIdx.x * a.QT;
  if (i0 >= jb.Lq) return;
  const int mid = a.mid, Lk = jb.Lk;
  float* ks = sm;                 // Lk*mid
  float* vs = ks + Lk * mid;      // Lk*mid
  float* ys = vs + Lk * mid;      // QT*mid
  float* wo = ys + a.QT * mid;    // [mid][oup] output projection (when a.wlds)
  const float* kg = jb.k + int64_t(n) * Lk * mid;
  const float* vg = jb.v + int64_t(n) * Lk * mid;
  for (int e = threadIdx.x; e < Lk * mid; e += blockDim.x) {
    ks[e] = kg[e];
    vs[e] = vg[e];
  }
  const float* wt = jb.wt;
  if (a.wlds) {
    for (int e = threadIdx.x; e < mid * a.oup; e += blockDim.x) wo[e] = jb.wt[e];
    wt = wo;
  }
  __syncthreads();
  const int nq = min(a.QT, jb.Lq - i0);
  for (int e = threadIdx.x; e < nq * a.heads; e += blockDim.x) {
    const int il = e / a.heads, hd = e - il * a.heads;
    const float* qg = jb.q + (int64_t(n) * jb.Lq + i0 + il) * mid + hd * DH;
    float q[DH], acc[DH];
#pragma unroll
    for (int d = 0; d < DH; ++d) {
      q[d] = qg[d];
      acc[d] = 0.f;
    }
    float m = -INFINITY, l = 0.f;
    for (int j = 0; j < Lk; ++j) {
      const float* kj = ks + j * mid + hd * DH;
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < DH; ++d) s += q[d] * kj[d];
      s *= a.scale;
      const float mn = fmaxf(m, s);
      const float corr = expf(m - mn), p = expf(s - mn);
      l = l * corr + p;
      const float* vj = vs + j * mid + hd * DH;
#pragma unroll
      for (int d = 0; d < DH; ++d) acc[d] = acc[d] * corr + p * vj[d];
      m = mn;
    }
    const float inv = 1.0f / l;
#pragma unroll
    for (int d = 0; d < DH; ++d) ys[il * mid + hd * DH + d] = acc[d] * inv;
  }
  __syncthreads();
  float* dst = jb.dst + (int64_t(n) * jb.Lq + i0) * a.oup;
  for (int e = threadIdx.x; e < nq * a.oup; e += blockDim.x) {
    const int il = e / a.oup, c = e - il * a.oup;
    const float* y = ys + il * mid;
    float acc = jb.b ? jb.b[c] : 0.f;
    for (int m2 = 0; m2 < mid; ++m2) acc += y[m2] * wt[m2 * a.oup + c];
    dst[e] = act_f(acc, jb.act);
  }
}

// Lane-group version: a group of KG = 16 lanes owns one (query, head) and splits the keys (lane g takes
// keys g, g + 16, ...), each lane an online softmax over its keys; the 16 partial (max, sum, acc) states
// are merged with 4 xor-shuffle rounds.  Blocks loop over query tiles of QT = 16 / heads queries (x
// heads = 16 groups = 256 threads); K/V of the (image, branch) are staged in LDS once per block.  The
// serial chain per lane is Lk / 16 keys instead of Lk.
constexpr int KG = 16;

template <int DH>
__global__ __launch_bounds__(256) void coord_attend_groups_kernel(AttArgs a, int qper) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const AttJob& jb = a.job[blockIdx.y];
  const int n = blockIdx.z;
  const int mid = a.mid, Lk = jb.Lk, heads = a.heads;
  const int QT = KG / heads;  // queries per tile (16 groups per block)
  const int q0 = blockIdx.x * qper;
  if (q0 >= jb.Lq) return;
  const int q1 = min(jb.Lq, q0 + qper), nq = q1 - q0;
  // K / V rows at an odd float stride: the 16 lanes of a group read 16 different keys at once, and an
  // even stride (mid = 16 / 64) would put them in 4..16 of the same LDS banks
  const int ld = mid | 1;
  float* ks = sm;              // Lk*ld
  float* vs = ks + Lk * ld;    // Lk*ld
  float* ys = vs + Lk * ld;    // qper*mid: attention outputs of all the block's queries
  float* qs = ys + qper * mid;  // qper*mid: the block's queries
  const float* kg = jb.k + int64_t(n) * Lk * mid;
  const float* vg = jb.v + int64_t(n) * Lk * mid;
  // K / V staging in rounds of 4 elements per thread (8 loads in flight; clamped loads, out-of-range
  // stores to a dummy float past the queries, so nothing is conditional)
  {
    float* dummy = qs + qper * mid;
    const int nkv = Lk * mid;
    for (int e0 = 0; e0 < nkv; e0 += 4 * int(blockDim.x)) {
      float kv[4], vv[4];
      int dj[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + int(threadIdx.x) + u * int(blockDim.x), ec = min(e, nkv - 1);
        const int j = ec / mid, c = ec - j * mid;
        kv[u] = kg[ec];
        vv[u] = vg[ec];
        dj[u] = e < nkv ? j * ld + c : -1;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        *(dj[u] >= 0 ? ks + dj[u] : dummy) = kv[u];
        *(dj[u] >= 0 ? vs + dj[u] : dummy) = vv[u];
      }
    }
  }
  const float* qg0 = jb.q + (int64_t(n) * jb.Lq + q0) * mid;
  for (int e = threadIdx.x; e < nq * mid; e += blockDim.x) qs[e] = qg0[e];
  __syncthreads();
  const int grp = threadIdx.x / KG, gl = threadIdx.x % KG;
  const int qi = grp / heads, hd = grp - qi * heads;  // group -> (query in tile, head)
  for (int t0 = 0; t0 < nq; t0 += QT) {
    const int il = t0 + qi;
    if (qi < QT && il < nq) {
      const float* qg = qs + il * mid + hd * DH;
      float q[DH], acc[DH];
#pragma unroll
      for (int d = 0; d < DH; ++d) {
        q[d] = qg[d];
        acc[d] = 0.f;
      }
      float m = -INFINITY, l = 0.f;
      for (int j = gl; j < Lk; j += KG) {
        const float* kj = ks + j * ld + hd * DH;
        float sc = 0.f;
#pragma unroll
        for (int d = 0; d < DH; ++d) sc += q[d] * kj[d];
        sc *= a.scale;
        const float mn = fmaxf(m, sc);
        const float corr = expf(m - mn), pj = expf(sc - mn);
        l = l * corr + pj;
        const float* vj = vs + j * ld + hd * DH;
#pragma unroll
        for (int d = 0; d < DH; ++d) acc[d] = acc[d] * corr + pj * vj[d];
        m = mn;
      }
#pragma unroll
      for (int off = 1; off < KG; off <<= 1) {  // merge the 16 partial softmax states of the group
        const float mo = __shfl_xor(m, off), lo = __shfl_xor(l, off);
        const float mn = fmaxf(m, mo);
        const float ca = m == -INFINITY ? 0.f : expf(m - mn), cb = mo == -INFINITY ? 0.f : expf(mo - mn);
        l = l * ca + lo * cb;
#pragma unroll
        for (int d = 0; d < DH; ++d) acc[d] = acc[d] * ca + __shfl_xor(acc[d], off) * cb;
        m = mn;
      }
      if (gl == 0) {
        const float inv = 1.0f / l;
#pragma unroll
        for (int d = 0; d < DH; ++d) ys[il * mid + hd * DH + d] = acc[d] * inv;
      }
    }
  }
  __syncthreads();
  // attention outputs [Lq][mid] (the output projection runs as a coord_proj job)
  float* dst = jb.dst + (int64_t(n) * jb.Lq + q0) * mid;
  for (int e = threadIdx.x; e < nq * mid; e += blockDim.x) dst[e] = ys[e];
}

// ---------------------------------------------------------------------------- 2+3 fused (small problems)
// BiCoordCrossAtt's whole per-image middle in one workgroup per (image, branch): the branch's q / k / v
// projections of the pooled vectors (staged in LDS), the axial multi-head attention and the output
// projection to the gate logits -- one launch instead of projection + attention + projection, for the
// n / s scales where a branch is ~0.5-2 M MACs.  Branch 0 (h): q <- x_h, k, v <- x_w; branch 1 (w):
// q <- x_w, k, v <- x_h (fce_block.py:235-284).
struct CoreArgs {
  const float* xh;  // [N][H][C]
  const float* xw;  // [N][W][C]
  const float* wq[2];
  const float* bq[2];
  const float* wk[2];
  const float* bk[2];
  const float* wv[2];
  const float* bv[2];
  const float* wo[2];  // [mid][oup]
  const float* bo[2];
  float* g[2];         // [N][L][oup] gate logits
  int H, W, C, mid, heads, oup;
  int qsplit;  // query chunks per (image, branch): blockIdx.z takes rows [z * qc, z * qc + qc) of the queries
  float scale;
  unsigned long long* tm;  // diagnostics (FCE_COORD_TIMING): per-workgroup phase clocks, else null
};

static constexpr int CORE_THREADS = 1024;

// LDS floats of the fused middle: pooled rows of both axes (odd stride), the three projection weights
// and the output projection, q / k / v / attention outputs
static size_t core_lds_floats(int H, int W, int C, int mid, int oup) {
  const int L = H > W ? H : W;
  return size_t(2) * L * (C + 4) + size_t(3) * C * mid + size_t(mid) * oup + size_t(4) * L * (mid + 4) + 4;
}

template <int DH>
__global__ __launch_bounds__(CORE_THREADS) void coord_core_kernel(CoreArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int n = blockIdx.x, br = blockIdx.y;
  // row strides: lc = C + 4 floats (16-byte rows; a wave's 16 positions land on distinct bank quads),
  // lm = mid + 4
  const int C = a.C, mid = a.mid, oup = a.oup, lc = C + 4, lm = mid + 4;
  const int Lq0 = br == 0 ? a.H : a.W, Lk = br == 0 ? a.W : a.H;
  // query chunk of this workgroup: every chunk projects all keys / values (cheap at these sizes) and
  // only its own queries, so the attention and the output projection spread over qsplit CUs
  const int qc = (Lq0 + a.qsplit - 1) / a.qsplit, q0 = min(Lq0, int(blockIdx.z) * qc);
  const int Lq = min(Lq0, q0 + qc) - q0;
  const float* gq = (br == 0 ? a.xh + int64_t(n) * a.H * C : a.xw + int64_t(n) * a.W * C) + int64_t(q0) * C;
  const float* gk = (br == 0 ? a.xw + int64_t(n) * a.W * C : a.xh + int64_t(n) * a.H * C);
  const int L = a.H > a.W ? a.H : a.W;
  float* wq = sm;                // [C][mid]
  float* wk = wq + C * mid;      // [C][mid]
  float* wv = wk + C * mid;      // [C][mid]
  float* wo = wv + C * mid;      // [mid][oup]
  float* q = wo + mid * oup;     // [Lq][lm]
  float* k = q + L * lm;         // [Lk][lm]
  float* v = k + L * lm;         // [Lk][lm]
  float* ys = v + L * lm;        // [Lq][lm]
  float* sq = ys + L * lm;       // [Lq][lc]
  float* skv = sq + L * lc;      // [Lk][lc]
  unsigned long long t0 = a.tm ? __builtin_amdgcn_s_memtime() : 0;
  {
    // all staging (weights, output weights, both pooled axes) as one flat space of 16-byte pieces, 8 loads
    // per thread in flight before their LDS stores (one memory round trip instead of six)
    const int C4 = C / 4, nw = C * mid / 4, no4 = mid * oup / 4, nq4 = Lq * C4, nk4 = Lk * C4;
    const int total = 3 * nw + no4 + nq4 + nk4;
    float* dummy = skv + L * lc;
    for (int e0 = 0; e0 < total; e0 += 8 * CORE_THREADS) {
      f4 val[8];
      float* dst[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        int e = e0 + int(threadIdx.x) + u * CORE_THREADS;
        const bool ok = e < total;
        e = ok ? e : total - 1;
        const float* sp;
        float* dp;
        if (e < 3 * nw) {
          const int m = e / nw, r = 4 * (e - m * nw);
          sp = (m == 0 ? a.wq[br] : m == 1 ? a.wk[br] : a.wv[br]) + r;
          dp = wq + m * C * mid + r;
        } else if ((e -= 3 * nw) < no4) {
          sp = a.wo[br] + 4 * e;
          dp = wo + 4 * e;
        } else if ((e -= no4) < nq4) {
          const int p = e / C4, c = (e - p * C4) * 4;
          sp = gq + p * C + c;
          dp = sq + p * lc + c;
        } else {
          e -= nq4;
          const int p = e / C4, c = (e - p * C4) * 4;
          sp = gk + p * C + c;
          dp = skv + p * lc + c;
        }
        val[u] = *reinterpret_cast<const f4*>(sp);
        dst[u] = ok ? dp : dummy;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) *reinterpret_cast<f4*>(dst[u]) = val[u];
    }
  }
  __syncthreads();
  unsigned long long t1 = a.tm ? __builtin_amdgcn_s_memtime() : 0;
  // projections, task = (matrix, position, 4 consecutive outputs): one broadcast source read and one
  // 16-byte weight read per 4 FMAs
  const int mq = mid / 4, tq = Lq * mq, tk = Lk * mq;
  for (int e = threadIdx.x; e < tq + 2 * tk; e += CORE_THREADS) {
    int t = e, mat = 0;
    if (t >= tq) {
      t -= tq;
      mat = 1 + (t >= tk);
      if (t >= tk) t -= tk;
    }
    const int p = t / mq, m4 = (t - p * mq) * 4;
    const float* src = (mat == 0 ? sq : skv) + p * lc;
    const float* w = (mat == 0 ? wq : mat == 1 ? wk : wv) + m4;
    const float* b = mat == 0 ? a.bq[br] : mat == 1 ? a.bk[br] : a.bv[br];
    f4 acc0 = b ? *reinterpret_cast<const f4*>(b + m4) : f4{0.f, 0.f, 0.f, 0.f};
    f4 acc1 = {0.f, 0.f, 0.f, 0.f}, acc2 = acc1, acc3 = acc1;
#pragma unroll 4
    for (int c = 0; c < C; c += 4) {  // C % 8 == 0
      const f4 sv = *reinterpret_cast<const f4*>(src + c);
      const f4 w0 = *reinterpret_cast<const f4*>(w + c * mid), w1 = *reinterpret_cast<const f4*>(w + (c + 1) * mid);
      const f4 w2 = *reinterpret_cast<const f4*>(w + (c + 2) * mid), w3 = *reinterpret_cast<const f4*>(w + (c + 3) * mid);
      acc0 += sv[0] * w0;
      acc1 += sv[1] * w1;
      acc2 += sv[2] * w2;
      acc3 += sv[3] * w3;
    }
    *reinterpret_cast<f4*>((mat == 0 ? q : mat == 1 ? k : v) + p * lm + m4) = (acc0 + acc1) + (acc2 + acc3);
  }
  __syncthreads();
  unsigned long long t2 = a.tm ? __builtin_amdgcn_s_memtime() : 0;
  // attention: G lanes per (query, head) split the keys (lane g takes keys g, g + G, ..); two passes
  // (row max, then exp-sum and P.V) so each key costs one exp, the G partial states merged by xor-shuffles
  const int pairs = Lq * a.heads;
  int G = 1;
  while (G < 16 && pairs * G * 2 <= CORE_THREADS) G *= 2;
  for (int e0 = 0; e0 < pairs * G; e0 += CORE_THREADS) {
    const int e = e0 + int(threadIdx.x);
    const bool live = e < pairs * G;
    const int pr = live ? e / G : 0, gl = e % G;
    const int i = pr / a.heads, hd = pr - i * a.heads;
    float qq[DH], acc[DH];
#pragma unroll
    for (int d = 0; d < DH; ++d) {
      qq[d] = q[i * lm + hd * DH + d] * a.scale;
      acc[d] = 0.f;
    }
    float m = -INFINITY;
    float l = 0.f;
    constexpr int KR = DH <= 4 ? 12 : 1;  // keys per lane held in registers (small heads)
    if (DH <= 4 && (Lk + G - 1) / G <= KR) {
      // all of this lane's keys and values loaded up front (one LDS round trip instead of one per key);
      // the same per-key arithmetic and order as the loop below, so the result is bitwise the same
      float kr[KR][DH], vr[KR][DH];
#pragma unroll
      for (int u = 0; u < KR; ++u) {
        const int j = min(gl + u * G, Lk - 1);
#pragma unroll
        for (int d = 0; d < DH; ++d) {
          kr[u][d] = k[j * lm + hd * DH + d];
          vr[u][d] = v[j * lm + hd * DH + d];
        }
      }
      float sc[KR];
#pragma unroll
      for (int u = 0; u < KR; ++u) {
        sc[u] = 0.f;
#pragma unroll
        for (int d = 0; d < DH; ++d) sc[u] += qq[d] * kr[u][d];
        if (gl + u * G < Lk) m = fmaxf(m, sc[u]);
      }
      for (int off = 1; off < G; off <<= 1) m = fmaxf(m, __shfl_xor(m, off));
#pragma unroll
      for (int u = 0; u < KR; ++u) {
        if (gl + u * G >= Lk) break;
        const float pj = __expf(sc[u] - m);
        l += pj;
#pragma unroll
        for (int d = 0; d < DH; ++d) acc[d] += pj * vr[u][d];
      }
    } else {
#pragma unroll 4
      for (int j = gl; j < Lk; j += G) {
        const float* kj = k + j * lm + hd * DH;
        float sc = 0.f;
#pragma unroll
        for (int d = 0; d < DH; ++d) sc += qq[d] * kj[d];
        m = fmaxf(m, sc);
      }
      for (int off = 1; off < G; off <<= 1) m = fmaxf(m, __shfl_xor(m, off));
#pragma unroll 4
      for (int j = gl; j < Lk; j += G) {
        const float* kj = k + j * lm + hd * DH;
        float sc = 0.f;
#pragma unroll
        for (int d = 0; d < DH; ++d) sc += qq[d] * kj[d];
        const float pj = __expf(sc - m);
        l += pj;
        const float* vj = v + j * lm + hd * DH;
#pragma unroll
        for (int d = 0; d < DH; ++d) acc[d] += pj * vj[d];
      }
    }
    for (int off = 1; off < G; off <<= 1) {
      l += __shfl_xor(l, off);
#pragma unroll
      for (int d = 0; d < DH; ++d) acc[d] += __shfl_xor(acc[d], off);
    }
    if (live && gl == 0) {
      const float inv = 1.0f / l;
#pragma unroll
      for (int d = 0; d < DH; ++d) ys[i * lm + hd * DH + d] = acc[d] * inv;
    }
  }
  __syncthreads();
  unsigned long long t3 = a.tm ? __builtin_amdgcn_s_memtime() : 0;
  // output projection to the gate logits, task = (position, 4 consecutive outputs), 16-byte stores
  float* g = a.g[br] + (int64_t(n) * Lq0 + q0) * oup;
  const float* bo = a.bo[br];
  const int o4n = oup / 4;
  for (int e = threadIdx.x; e < Lq * o4n; e += CORE_THREADS) {
    const int i = e / o4n, o4 = (e - i * o4n) * 4;
    const float* y = ys + i * lm;
    f4 acc0 = bo ? *reinterpret_cast<const f4*>(bo + o4) : f4{0.f, 0.f, 0.f, 0.f};
    f4 acc1 = {0.f, 0.f, 0.f, 0.f}, acc2 = acc1, acc3 = acc1;
    for (int m2 = 0; m2 < mid; m2 += 4) {  // mid % 4 == 0
      const f4 yv = *reinterpret_cast<const f4*>(y + m2);
      acc0 += yv[0] * *reinterpret_cast<const f4*>(wo + m2 * oup + o4);
      acc1 += yv[1] * *reinterpret_cast<const f4*>(wo + (m2 + 1) * oup + o4);
      acc2 += yv[2] * *reinterpret_cast<const f4*>(wo + (m2 + 2) * oup + o4);
      acc3 += yv[3] * *reinterpret_cast<const f4*>(wo + (m2 + 3) * oup + o4);
    }
    *reinterpret_cast<f4*>(g + i * oup + o4) = (acc0 + acc1) + (acc2 + acc3);
  }
  if (a.tm) {
    __syncthreads();
    const unsigned long long t4 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
      unsigned long long* o = a.tm + ((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 5;
      o[0] = t0;
      o[1] = t1 - t0;
      o[2] = t2 - t1;
      o[3] = t3 - t2;
      o[4] = t4 - t3;
    }
  }
}

// ---------------------------------------------------------------------------- 4. apply
enum { GATE_BICOORD = 0, GATE_COORD = 1, GATE_ROW = 2 };

// grid (row chunks of GPX * 256 elements, N*H): element = (column, 8-channel group) of one row, 32-bit
// index math.  A thread takes GPX elements 256 apart and issues all their x and gate loads before any
// math (GPX x more bytes in flight per wave: the kernel streams x once and y once at ~HBM rate).
template <int MODE, int GPX>
__global__ __launch_bounds__(256) void gate_apply_kernel(const _Float16* x, int xcs, _Float16* y, int ycs, int N,
                                                         int H, int W, int C, const float* g1, const float* g2) {
  const int CG = C / 8;
  // 1-D grid, XCD-aware: block b runs on XCD b % 8 and takes logical block (b % 8) * per + b / 8, so each XCD walks
  // a contiguous range of rows (whole images): an image's column gates g2 (W x C fp32) enter one L2, not eight
  const int gx = (W * CG + 256 * GPX - 1) / (256 * GPX);
  const int total = int(gridDim.x), b = int(blockIdx.x), per = total >> 3, body = per << 3;
  const int L = b < body ? (b & 7) * per + (b >> 3) : b;
  const int row = L / gx, bx = L - row * gx, n = row / H, yy = row - n * H;
  h8 v[GPX];
  f4 ga[GPX][2], gb[GPX][2];
  int xx[GPX], gg[GPX];
  bool live[GPX];
#pragma unroll
  for (int k = 0; k < GPX; ++k) {
    const int e = (bx * GPX + k) * 256 + threadIdx.x;
    live[k] = e < W * CG;
    const int ec = live[k] ? e : 0;
    xx[k] = ec / CG;
    gg[k] = ec - xx[k] * CG;
    const int64_t pix = int64_t(row) * W + xx[k];
    v[k] = *reinterpret_cast<const h8*>(x + pix * xcs + gg[k] * 8);
    const float* gh = g1 + (int64_t(n) * H + yy) * C + gg[k] * 8;
    ga[k][0] = *reinterpret_cast<const f4*>(gh);
    ga[k][1] = *reinterpret_cast<const f4*>(gh + 4);
    if (MODE != GATE_ROW) {
      const float* gw = g2 + (int64_t(n) * W + xx[k]) * C + gg[k] * 8;
      gb[k][0] = *reinterpret_cast<const f4*>(gw);
      gb[k][1] = *reinterpret_cast<const f4*>(gw + 4);
    }
  }
#pragma unroll
  for (int k = 0; k < GPX; ++k) {
    if (!live[k]) continue;
    float gv[8] = {ga[k][0][0], ga[k][0][1], ga[k][0][2], ga[k][0][3], ga[k][1][0], ga[k][1][1], ga[k][1][2], ga[k][1][3]};
    float wv[8] = {1, 1, 1, 1, 1, 1, 1, 1};
    if (MODE != GATE_ROW) {
      wv[0] = gb[k][0][0]; wv[1] = gb[k][0][1]; wv[2] = gb[k][0][2]; wv[3] = gb[k][0][3];
      wv[4] = gb[k][1][0]; wv[5] = gb[k][1][1]; wv[6] = gb[k][1][2]; wv[7] = gb[k][1][3];
    }
    h8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float r;
      if (MODE == GATE_BICOORD)
        r = (float)v[k][j] * sigmoidf_(gv[j] + wv[j]);  // v_exp + v_rcp (the gate is VALU-bound)
      else if (MODE == GATE_COORD)
        r = (float)v[k][j] * gv[j] * wv[j];
      else
        r = (float)v[k][j] * gv[j];
      o[j] = (_Float16)r;
    }
    const int64_t pix = int64_t(row) * W + xx[k];
    *reinterpret_cast<h8*>(y + pix * ycs + gg[k] * 8) = o;
  }
}


// ---------------------------------------------------------------------------- host
static int launch_proj(ProjJob* jobs, int nj, int N, hipStream_t s) {
  ProjArgs pa;
  int maxL = 1, maxM = 1, maxK = 1;
  for (int i = 0; i < nj; ++i) {
    pa.job[i] = jobs[i];
    maxL = std::max(maxL, jobs[i].L);
    maxM = std::max(maxM, jobs[i].M);
    maxK = std::max(maxK, jobs[i].K);
  }
  FCE_CHECK(maxM <= 256 * 16, "coord projection: too many outputs");
  bool m4 = true;
  for (int i = 0; i < nj; ++i) m4 = m4 && jobs[i].M % 4 == 0 && jobs[i].K % 4 == 0;
  const char* pe = getenv("FCE_COORD_PROJ1");  // diagnostics: the scalar projection kernel
  if (m4 && maxM <= 1024 && !(pe && atoi(pe))) {
    // 4 x 4 tiles, <= PJ_TPT per thread: TP positions with (TP / 4) (M / 4) <= 256 PJ_TPT
    int TP = 4 * std::max(1, std::min(16, 256 * PJ_TPT / (maxM / 4)));
    // fewer positions per block while the grid is short of ~1.5 blocks per CU (m 160^2, M 64: 288 -> 480
    // blocks, 55 -> 47 us); below 32 the idle task slots cost more than the extra blocks gain
    while (TP > 32 && int64_t((maxL + TP - 1) / TP) * nj * N < 384) TP /= 2;
    const char* te = getenv("FCE_COORD_PJTP");  // diagnostics: positions per block
    if (te && atoi(te) >= 4) TP = std::min(TP, atoi(te) & ~3);
    const int KC = std::max(4, std::min({maxK, 128, (12288 - TP * 68) / maxM}) & ~3);  // <= 48 KiB
    const size_t shm = (size_t(TP) * (KC + 4) + size_t(KC) * maxM + 4) * sizeof(float);
    dim3 grid((maxL + TP - 1) / TP, nj, N);
    FCE_LAUNCH(coord_proj4_kernel, grid, dim3(256), shm, s, pa, TP, KC);
    return launch_status("coord_proj4_kernel");
  }
  const int TP = std::max(1, std::min(16, 256 * 16 / maxM));                       // positions per block
  const int KC = std::max(1, std::min({maxK, 256, (8192 - TP * 64) / maxM}));      // <= 32 KiB of weights
  const size_t shm = (size_t(TP) * KC + size_t(KC) * maxM + 1) * sizeof(float);  // + the staging dummy
  dim3 grid((maxL + TP - 1) / TP, nj, N);
  FCE_LAUNCH(coord_proj_kernel, grid, dim3(256), shm, s, pa, TP, KC);
  return launch_status("coord_proj_kernel");
}

// heads dividing 16: lane-group kernel writing the attention outputs (the caller then runs the output
// projection as a coord_proj job); otherwise the per-thread kernel with the projection fused
static bool attend_grouped(const fce_coord_desc& d) { return d.heads <= KG && KG % d.heads == 0; }

static int launch_attend(AttJob* jobs, int nj, int N, const fce_coord_desc& d, hipStream_t s) {
  AttArgs a;
  a.mid = d.mid;
  a.heads = d.heads;
  a.oup = d.oup;
  a.scale = d.scale;
  int maxLq = 1, maxLk = 1;
  for (int i = 0; i < nj; ++i) {
    a.job[i] = jobs[i];
    maxLq = std::max(maxLq, jobs[i].Lq);
    maxLk = std::max(maxLk, jobs[i].Lk);
  }
  constexpr size_t kMaxLds = 160 * 1024;  // gfx950 LDS per workgroup (opted in below)
  const bool groups = attend_grouped(d);
  a.QT = groups ? KG / d.heads : std::max(1, 256 / d.heads);
  // group kernel: ~8 blocks per (image, branch), each looping over its query tiles (K/V staged once
  // per block) and projecting all of its <= 32 queries at the end
  const int tiles = (maxLq + a.QT - 1) / a.QT;
  const int per = std::max(1, std::min((tiles + 7) / 8, 32 / std::max(1, a.QT)));
  const int qper = per * a.QT;
  size_t shm = (size_t(2) * maxLk * (groups ? (d.mid | 1) : d.mid) + size_t(groups ? 2 * qper : a.QT) * d.mid +
                (groups ? 1 : 0)) *  // + the staging dummy of the grouped kernel
               sizeof(float);
  if (shm > kMaxLds) return fail(FCE_ERR_UNSUPPORTED, "coord attention: K/V do not fit in LDS");
  a.wlds = !groups && shm + size_t(d.mid) * d.oup * sizeof(float) <= kMaxLds;
  if (a.wlds) shm += size_t(d.mid) * d.oup * sizeof(float);
  dim3 grid = groups ? dim3((maxLq + qper - 1) / qper, nj, N) : dim3((maxLq + a.QT - 1) / a.QT, nj, N);
  const int dh = d.mid / d.heads;
  switch (dh) {
#define ATT(DH)                                                                                          \
  case DH: {                                                                                             \
    if (groups) {                                                                                        \
      static const bool lds_ok = hipFuncSetAttribute(                                                    \
          reinterpret_cast<const void*>(&coord_attend_groups_kernel<DH>),                                \
          hipFuncAttributeMaxDynamicSharedMemorySize, int(kMaxLds)) == hipSuccess;                       \
      if (!lds_ok && shm > 64 * 1024) return fail(FCE_ERR_HIP, "coord attention: cannot opt in to >64 KiB LDS"); \
      FCE_LAUNCH(coord_attend_groups_kernel<DH>, grid, dim3(256), shm, s, a, qper);                      \
    } else {                                                                                             \
      static const bool lds_ok = hipFuncSetAttribute(reinterpret_cast<const void*>(&coord_attend_kernel<DH>), \
                                                      hipFuncAttributeMaxDynamicSharedMemorySize,        \
                                                      int(kMaxLds)) == hipSuccess;                       \
      if (!lds_ok && shm > 64 * 1024) return fail(FCE_ERR_HIP, "coord attention: cannot opt in to >64 KiB LDS"); \
      FCE_LAUNCH(coord_attend_kernel<DH>, grid, dim3(256), shm, s, a);                                   \
    }                                                                                                    \
    break;                                                                                               \
  }
    ATT(1) ATT(2) ATT(3) ATT(4) ATT(5) ATT(6) ATT(7) ATT(8) ATT(10) ATT(12) ATT(16) ATT(20) ATT(24) ATT(32)
    ATT(48) ATT(64)
#undef ATT
    default:
      return fail(FCE_ERR_UNSUPPORTED, "coord attention: unsupported head dim " + std::to_string(dh));
  }
  return launch_status("coord_attend_kernel");
}

// the fused middle for problems of <= ~2 M MACs per (image, branch) whose staging fits in LDS
static constexpr size_t kCoreMaxMacs = size_t(2) << 20;
static bool use_core(const fce_coord_desc& d, int H, int W) {
  const size_t L = size_t(H > W ? H : W);
  const int dh = d.mid / d.heads;
  return (dh == 1 || dh == 2 || dh == 4 || dh == 8 || dh == 16) && d.mid % 4 == 0 && d.oup % 4 == 0 &&
         3 * L * d.mid * d.inp <= kCoreMaxMacs && core_lds_floats(H, W, d.inp, d.mid, d.oup) * sizeof(float) <= 160 * 1024;
}

static int launch_core(const fce_coord_desc& d, const CoordWs& w, int N, int H, int W, hipStream_t s) {
  CoreArgs a;
  a.xh = w.xh;
  a.xw = w.xw;
  for (int br = 0; br < 2; ++br) {
    a.wq[br] = d.w[3 * br + 0];
    a.bq[br] = d.b[3 * br + 0];
    a.wk[br] = d.w[3 * br + 1];
    a.bk[br] = d.b[3 * br + 1];
    a.wv[br] = d.w[3 * br + 2];
    a.bv[br] = d.b[3 * br + 2];
    a.wo[br] = d.w[6 + br];
    a.bo[br] = d.b[6 + br];
  }
  a.g[0] = w.g1;
  a.g[1] = w.g2;
  a.H = H;
  a.W = W;
  a.C = d.inp;
  a.mid = d.mid;
  a.heads = d.heads;
  a.oup = d.oup;
  a.scale = d.scale;
  // query chunks: 2 N (image, branch) workgroups alone leave most CUs idle; up to 2 chunks of at least
  // 8 queries.  The split depends on the map size only, never on N: the chunk size sets the attention's
  // key split, so a batch-dependent split would break batch invariance (test_batch_invariance_640).
  {
    const int L = H < W ? H : W;
    int qs = 1;
    // each chunk's workgroup stages and projects the whole axis again, so with several batches in flight fewer
    // chunks are cheaper overall: n32 (4 lanes) 36.5k images/s with 4 chunks, 36.8-37.0k with 2, 37.0k with 1
    // (profiles/r04ai_qsplit*, FCE_COORD_QSPLIT); 2 keeps part of the split for one-batch latency
    while (qs < 2 && L / (2 * qs) >= 8) qs *= 2;
    const char* qe = getenv("FCE_COORD_QSPLIT");  // diagnostics: force the query split
    if (qe && atoi(qe) > 0) qs = atoi(qe);
    a.qsplit = qs;
  }
  a.tm = nullptr;
  static unsigned long long* tm_buf = nullptr;
  const char* tenv = getenv("FCE_COORD_TIMING");
  if (tenv && atoi(tenv)) {
    if (!tm_buf) FCE_HIP_CHECK(hipMalloc(&tm_buf, size_t(2) * 4096 * 5 * 8));
    a.tm = N * a.qsplit <= 4096 ? tm_buf : nullptr;
  }
  const size_t shm = core_lds_floats(H, W, d.inp, d.mid, d.oup) * sizeof(float);
  switch (d.mid / d.heads) {
#define CORE(DH)                                                                                              \
  case DH: {                                                                                                  \
    static const bool lds_ok = hipFuncSetAttribute(reinterpret_cast<const void*>(&coord_core_kernel<DH>),     \
                                                    hipFuncAttributeMaxDynamicSharedMemorySize,               \
                                                    160 * 1024) == hipSuccess;                                \
    if (!lds_ok && shm > 64 * 1024) return fail(FCE_ERR_HIP, "coord core: cannot opt in to >64 KiB LDS");     \
    FCE_LAUNCH(coord_core_kernel<DH>, dim3(N, 2, a.qsplit), dim3(CORE_THREADS), shm, s, a);                            \
    break;                                                                                                    \
  }
    CORE(1) CORE(2) CORE(4) CORE(8) CORE(16)
#undef CORE
    default:
      return fail(FCE_ERR_UNSUPPORTED, "coord core: head dim");
  }
  int st = launch_status("coord_core_kernel");
  if (!st && a.tm) {  // diagnostics: print the phase clocks of this launch
    const int nb = 2 * N * a.qsplit;
    std::vector<unsigned long long> h(size_t(nb) * 5);
    FCE_HIP_CHECK(hipStreamSynchronize(s));
    FCE_HIP_CHECK(hipMemcpy(h.data(), a.tm, h.size() * 8, hipMemcpyDeviceToHost));
    unsigned long long mn = ~0ull, mx = 0, ph[4] = {0, 0, 0, 0};
    for (int b = 0; b < nb; ++b) {
      mn = std::min(mn, h[b * 5]);
      mx = std::max(mx, h[b * 5]);
      for (int k = 0; k < 4; ++k) ph[k] += h[b * 5 + 1 + k];
    }
    fprintf(stderr, "coord_core N%d H%d W%d qsplit %d: start spread %llu, mean phase clocks stage %llu proj %llu attend %llu out %llu\n",
            N, H, W, a.qsplit, mx - mn, ph[0] / nb, ph[1] / nb, ph[2] / nb, ph[3] / nb);
  }
  return st;
}

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
  CoordWs w;
  ws_layout(d, N, H, W, &w, static_cast<float*>(ws));
  const _Float16* xp = static_cast<const _Float16*>(x.data) + x.coff;
  const int C = d.inp, mid = d.mid;
  const char* tp = getenv("FCE_COORD_TWO_PASS");  // diagnostics: the two-pass row / column pooling
  if (w.part && !(tp && atoi(tp))) {  // band pooling: one read of x
    const int R = band_rows(N, H, C), NB = (H + R - 1) / R;
    const int64_t nblk = int64_t(N) * NB * (C / 64);
    FCE_CHECK(nblk < (int64_t(1) << 31), "coord pooling: grid too large");
#define FCE_BAND(RR, KK) \
  FCE_LAUNCH((pool_band_kernel<RR, KK>), dim3(unsigned(nblk)), dim3(256), 0, s, xp, x.cstride, H, W, C, w.xh, w.part, NB)
    const int kw = (W + 31) / 32;  // columns per thread: 3 (W <= 96), 5 (<= 160) or 8 registers' worth
    if (R == 16) {
      if (kw <= 3) FCE_BAND(16, 3); else if (kw <= 5) FCE_BAND(16, 5); else FCE_BAND(16, 8);
    } else {
      if (kw <= 3) FCE_BAND(8, 3); else if (kw <= 5) FCE_BAND(8, 5); else FCE_BAND(8, 8);
    }
#undef FCE_BAND
    const int64_t ncol = (int64_t(N) * W * C / 4 + 255) / 256;
    FCE_LAUNCH(pool_band_cols_kernel, dim3(unsigned(ncol)), dim3(256), 0, s, w.part, w.xw, N, NB, H, W * C);
  } else {
    int RG = 1;  // pool_col_groups on the host
    while (RG < 8 && (C / 8) * RG * 2 <= 256 && H >= 16 * RG) RG *= 2;
    const int XW = 256 / ((C / 8) * RG);
    const int BPI = H + (W + XW - 1) / XW;
    const int aff = N >= 8;
    const int64_t nblk = int64_t(aff ? 8 * ((N + 7) / 8) : N) * BPI;
    FCE_CHECK(nblk < (int64_t(1) << 31), "coord pooling: grid too large");
    FCE_LAUNCH(pool_kernel, dim3(unsigned(nblk)), dim3(256), 0, s, xp, x.cstride, H, W, C, w.xh, w.xw, N, BPI, aff);
  }
  int st = launch_status("coord pooling");
  if (st) return st;
  const char* nc = getenv("FCE_COORD_NO_CORE");  // diagnostics: force the split projection / attention path
  if (kind == 0 && !(nc && atoi(nc)) && use_core(d, H, W)) {
    if ((st = launch_core(d, w, N, H, W, s))) return st;
  } else if (kind == 0) {  // BiCoordCrossAtt
    ProjJob pj[6] = {
        {w.xh, d.w[0], d.b[0], w.buf[0], H, C, mid, ACT_NONE_},  // q_h  <- x_h
        {w.xw, d.w[1], d.b[1], w.buf[1], W, C, mid, ACT_NONE_},  // k_h  <- x_w
        {w.xw, d.w[2], d.b[2], w.buf[2], W, C, mid, ACT_NONE_},  // v_h  <- x_w
        {w.xw, d.w[3], d.b[3], w.buf[3], W, C, mid, ACT_NONE_},  // q_w  <- x_w
        {w.xh, d.w[4], d.b[4], w.buf[4], H, C, mid, ACT_NONE_},  // k_w  <- x_h
        {w.xh, d.w[5], d.b[5], w.buf[5], H, C, mid, ACT_NONE_},  // v_w  <- x_h
    };
    if ((st = launch_proj(pj, 6, N, s))) return st;
    const bool grp = attend_grouped(d);  // grouped: attention outputs overwrite the queries (each block
                                         // writes exactly the rows it read), then out_h / out_w jobs
    AttJob aj[2] = {{w.buf[0], w.buf[1], w.buf[2], d.w[6], d.b[6], grp ? w.buf[0] : w.g1, H, W, ACT_NONE_},
                    {w.buf[3], w.buf[4], w.buf[5], d.w[7], d.b[7], grp ? w.buf[3] : w.g2, W, H, ACT_NONE_}};
    if ((st = launch_attend(aj, 2, N, d, s))) return st;
    if (grp) {
      ProjJob po[2] = {{w.buf[0], d.w[6], d.b[6], w.g1, H, mid, d.oup, ACT_NONE_},
                       {w.buf[3], d.w[7], d.b[7], w.g2, W, mid, d.oup, ACT_NONE_}};
      if ((st = launch_proj(po, 2, N, s))) return st;
    }
  } else if (kind == 1) {  // CoordAtt: y = SiLU(cv1 [x_h; x_w]); a_h / a_w = sigmoid(cv_h / cv_w)
    ProjJob p1[2] = {{w.xh, d.w[0], d.b[0], w.buf[0], H, C, mid, ACT_SILU_},
                     {w.xw, d.w[0], d.b[0], w.buf[1], W, C, mid, ACT_SILU_}};
    if ((st = launch_proj(p1, 2, N, s))) return st;
    ProjJob p2[2] = {{w.buf[0], d.w[1], d.b[1], w.g1, H, mid, d.oup, ACT_SIGMOID_},
                     {w.buf[1], d.w[2], d.b[2], w.g2, W, mid, d.oup, ACT_SIGMOID_}};
    if ((st = launch_proj(p2, 2, N, s))) return st;
  } else {  // CoordCrossAtt: y = cv1 [x_h; x_w]; q <- y_h, k,v <- y_w; y_att = sigmoid(proj(attn))
    ProjJob p1[2] = {{w.xh, d.w[0], d.b[0], w.buf[0], H, C, mid, ACT_NONE_},
                     {w.xw, d.w[0], d.b[0], w.buf[1], W, C, mid, ACT_NONE_}};
    if ((st = launch_proj(p1, 2, N, s))) return st;
    ProjJob p2[3] = {{w.buf[0], d.w[1], d.b[1], w.buf[2], H, mid, mid, ACT_NONE_},
                     {w.buf[1], d.w[2], d.b[2], w.buf[3], W, mid, mid, ACT_NONE_},
                     {w.buf[1], d.w[3], d.b[3], w.buf[4], W, mid, mid, ACT_NONE_}};
    if ((st = launch_proj(p2, 3, N, s))) return st;
    const bool grp = attend_grouped(d);
    AttJob aj[1] = {{w.buf[2], w.buf[3], w.buf[4], d.w[4], d.b[4], grp ? w.buf[2] : w.g1, H, W, ACT_SIGMOID_}};
    if ((st = launch_attend(aj, 1, N, d, s))) return st;
    if (grp) {
      ProjJob po[1] = {{w.buf[2], d.w[4], d.b[4], w.g1, H, mid, d.oup, ACT_SIGMOID_}};
      if ((st = launch_proj(po, 1, N, s))) return st;
    }
  }
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
  // 4 elements per thread on wide rows (m/l 160^2 x 512: 208 -> 183 us); 1 on narrow rows, where the
  // 4-wide blocks leave too few of them (n 80^2 x 128: 22.5 vs 29 us)
  const int gpx = W * (d.oup / 8) >= 4096 ? 4 : 1;
  const int64_t gblocks = int64_t((W * (d.oup / 8) + 256 * gpx - 1) / (256 * gpx)) * N * H;
  FCE_CHECK(gblocks < (int64_t(1) << 31), "coord attention: gate grid too large");
  const dim3 grid{unsigned(gblocks)};
  if (kind == 0)
    FCE_LAUNCH((gpx == 4 ? gate_apply_kernel<GATE_BICOORD, 4> : gate_apply_kernel<GATE_BICOORD, 1>), grid, dim3(256), 0, s, src, scs, yp, y.cstride, N, H, W,
                       d.oup, w.g1, w.g2);
  else if (kind == 1)
    FCE_LAUNCH((gpx == 4 ? gate_apply_kernel<GATE_COORD, 4> : gate_apply_kernel<GATE_COORD, 1>), grid, dim3(256), 0, s, src, scs, yp, y.cstride, N, H, W, d.oup,
                       w.g1, w.g2);
  else
    FCE_LAUNCH((gpx == 4 ? gate_apply_kernel<GATE_ROW, 4> : gate_apply_kernel<GATE_ROW, 1>), grid, dim3(256), 0, s, src, scs, yp, y.cstride, N, H, W, d.oup,
                       w.g1, w.g2);
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
