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

namespace fce {

int conv2d(const fce_conv_desc& d, const fce_tensor& x, const void* w, const float* bias, const fce_tensor* res,
           const fce_tensor& y, hipStream_t s, int tile = -1);

enum { ACT_NONE_ = 0, ACT_SILU_ = 1, ACT_SIGMOID_ = 2 };

struct CoordWs {
  float* xh;      // N*H*C
  float* xw;      // N*W*C
  float* buf[6];  // N*L*mid each
  float* g1;      // N*H*oup
  float* g2;      // N*W*oup
};

static size_t align_f(size_t n) { return (n + 63) & ~size_t(63); }

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

__global__ __launch_bounds__(256) void pool_cols_kernel(const _Float16* x, int xcs, int H, int W, int C, float* xw) {
  const int n = blockIdx.y;
  const int CG = C / 8;
  const int XW = 256 / CG;
  const int t = threadIdx.x;
  const int cg = t % CG, xi = t / CG;
  const int xx = blockIdx.x * XW + xi;
  if (xi >= XW || xx >= W) return;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const _Float16* p = x + nhwc_off(n, 0, xx, H, W, xcs) + cg * 8;
  const int64_t rs = int64_t(W) * xcs;
  // 8 rows in flight per step (the walk down a column is latency-bound otherwise); rows are still
  // added in order, so the sum is the sequential one
  int y = 0;
  for (; y + 7 < H; y += 8) {
    h8 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = *reinterpret_cast<const h8*>(p + (y + k) * rs);
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += (float)v[k][j];
  }
  for (; y < H; ++y) {
    const h8 v0 = *reinterpret_cast<const h8*>(p + y * rs);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += (float)v0[j];
  }
  const float inv = 1.0f / (float)H;
  float* o = xw + (int64_t(n) * W + xx) * C + cg * 8;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = acc[j] * inv;
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

// ---------------------------------------------------------------------------- 4. apply
enum { GATE_BICOORD = 0, GATE_COORD = 1, GATE_ROW = 2 };

// grid (row chunks, N*H): thread = (column, 8-channel group) of one row, 32-bit index math
template <int MODE>
__global__ __launch_bounds__(256) void gate_apply_kernel(const _Float16* x, int xcs, _Float16* y, int ycs, int N,
                                                         int H, int W, int C, const float* g1, const float* g2) {
  const int CG = C / 8;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= W * CG) return;
  {
    const int xx = e / CG, g = e - xx * CG;
    const int row = blockIdx.y, n = row / H, yy = row - n * H;
    const int64_t pix = int64_t(row) * W + xx;
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
  FCE_LAUNCH(pool_rows_kernel, dim3(H, N), dim3(256), 0, s, xp, x.cstride, H, W, C, w.xh);
  const int XW = 256 / (C / 8);
  FCE_LAUNCH(pool_cols_kernel, dim3((W + XW - 1) / XW, N), dim3(256), 0, s, xp, x.cstride, H, W, C, w.xw);
  int st = launch_status("coord pooling");
  if (st) return st;
  if (kind == 0) {  // BiCoordCrossAtt
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
  FCE_CHECK(int64_t(N) * H < 65536 * 1024, "coord attention: too many rows");
  const dim3 grid((W * (d.oup / 8) + 255) / 256, N * H);
  if (kind == 0)
    FCE_LAUNCH(gate_apply_kernel<GATE_BICOORD>, grid, dim3(256), 0, s, src, scs, yp, y.cstride, N, H, W,
                       d.oup, w.g1, w.g2);
  else if (kind == 1)
    FCE_LAUNCH(gate_apply_kernel<GATE_COORD>, grid, dim3(256), 0, s, src, scs, yp, y.cstride, N, H, W, d.oup,
                       w.g1, w.g2);
  else
    FCE_LAUNCH(gate_apply_kernel<GATE_ROW>, grid, dim3(256), 0, s, src, scs, yp, y.cstride, N, H, W, d.oup,
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
