// C2PSA attention (reference ultralytics/nn/modules/block.py:1247-1304, Attention.forward):
//   q,k,v = qkv.view(B, heads, 2*kd+hd, N).split([kd,kd,hd]) ;  out = v @ softmax(q^T k * kd^-0.5)^T + pe(v)
// with pe = depthwise 3x3 (BN folded, no act) over v viewed as (B, heads*hd, H, W).
// qkv is the NHWC fp16 output of the qkv 1x1 conv: channel (head*(2kd+hd) + r) is row r of that head.
//
// pe(v) is computed in the attention kernel's epilogue for each query pixel, with the depthwise kernel's exact
// arithmetic (the diagnostic per-64-key-tile kernel still takes it from a depthwise pass per head).
//
// Attention = flash-style on MFMA (v_mfma_f32_16x16x32_f16), one block = (image, head, 64 queries),
// one wave = 16 queries, K/V streamed in 64-key tiles:
//   S^T[key][q] = K . Q^T     A = K rows (16 keys x 32 d, 16-byte loads), B = Q^T (one per wave)
//                             -> each lane owns ONE query column (q = lane&15) and 4 keys per tile,
//                                so the online softmax needs only two xor-shuffles (lanes ^16, ^32)
//   O^T[d][q] += V^T . P^T     B = P^T straight from the S^T registers (cvt to f16): the MFMA's k
//                             index is relabelled (slot j<4 -> key 4g+j, j>=4 -> key 16+4g+j-4) and
//                             the A operand V^T is read from an LDS transpose of the V tile in that
//                             same key order (two 8-byte LDS reads per fragment)
#include "common.h"

namespace fce {

int dwconv3x3(const fce_tensor& x, int stride, const float* w, int wcs, const float* bias, int act,
              const fce_tensor& y, hipStream_t s, int variant = -1);

// XCD-aware block order: the grid is 1-D, block b runs on XCD b % 8, and all QT query tiles of one (image, head)
// pair get blocks on the same XCD (pair p on XCD p % 8), so that pair's K / V lines are fetched into one L2
// instead of up to QT of them.  Blocks past the last pair exit at once.
__device__ __forceinline__ bool psa_block(int QT, int P, int heads, int& qt, int& n, int& hd) {
  const int b = int(blockIdx.x), xcd = b & 7, slot = b >> 3;
  const int pl = slot / QT;
  qt = slot - pl * QT;
  const int pair = pl * 8 + xcd;
  if (pair >= P) return false;
  n = pair / heads;
  hd = pair - n * heads;
  return true;
}

template <int KD, int HD>
__global__ __launch_bounds__(256) void psa_attention_mfma_kernel(const _Float16* qkv, int qcs, int N, _Float16* y,
                                                                 int ycs, float scale_log2, int QT, int P, int heads) {
  static_assert(KD == 32 && HD == 64, "C2PSA geometry");
  constexpr int KT = 64, VTS = KT + 4;  // key tile, padded LDS row (conflict-free 8-byte reads)
  __shared__ __attribute__((aligned(16))) _Float16 vt[HD * VTS];
  int qt, n, hd;
  if (!psa_block(QT, P, heads, qt, n, hd)) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 15, g = lane >> 4;
  const int q = qt * 64 + wave * 16 + col;
  const _Float16* base = qkv + int64_t(n) * N * qcs + hd * (2 * KD + HD);
  // B operand Q^T: lane holds Q[q][8g..8g+7]
  h8 qf = h8{0, 0, 0, 0, 0, 0, 0, 0};
  if (q < N) qf = *reinterpret_cast<const h8*>(base + int64_t(q) * qcs + 8 * g);
  float m = -INFINITY, l = 0.f;
  f4 acc[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) acc[dt] = f4{0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < N; k0 += KT) {
    __syncthreads();
    // stage V tile transposed: vt[d][key]
    for (int e = threadIdx.x; e < KT * (HD / 8); e += 256) {
      const int key = e / (HD / 8), dc = (e % (HD / 8)) * 8;
      h8 v = h8{0, 0, 0, 0, 0, 0, 0, 0};
      if (k0 + key < N) v = *reinterpret_cast<const h8*>(base + int64_t(k0 + key) * qcs + 2 * KD + dc);
#pragma unroll
      for (int j = 0; j < 8; ++j) vt[(dc + j) * VTS + key] = v[j];
    }
    // S^T tiles (16 keys each): A = K[key][8g..8g+7]
    f4 s[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int key = k0 + 16 * t + col;
      h8 kf = h8{0, 0, 0, 0, 0, 0, 0, 0};
      if (key < N) kf = *reinterpret_cast<const h8*>(base + int64_t(key) * qcs + KD + 8 * g);
      s[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf, qf, f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    }
    // online softmax over the 64 keys of this tile for query column q (log2 domain)
    float mt = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int key = k0 + 16 * t + 4 * g + j;
        const float v = key < N ? s[t][j] * scale_log2 : -INFINITY;
        s[t][j] = v;
        mt = fmaxf(mt, v);
      }
    mt = fmaxf(mt, __shfl_xor(mt, 16));
    mt = fmaxf(mt, __shfl_xor(mt, 32));
    const float mn = fmaxf(m, mt);
    const float corr = exp2f(m - mn);
    float rs = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float p = exp2f(s[t][j] - mn);
        s[t][j] = p;
        rs += p;
      }
    rs += __shfl_xor(rs, 16);
    rs += __shfl_xor(rs, 32);
    l = l * corr + rs;
    m = mn;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[dt][j] *= corr;
    __syncthreads();
    // O^T += V^T P^T over two 32-key steps
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      h8 pf;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pf[j] = (_Float16)s[2 * u][j];
        pf[j + 4] = (_Float16)s[2 * u + 1][j];
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const _Float16* row = vt + (16 * dt + col) * VTS + 32 * u + 4 * g;
        const h4 lo = *reinterpret_cast<const h4*>(row);
        const h4 hi = *reinterpret_cast<const h4*>(row + 16);
        const h8 vf = h8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        acc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vf, pf, acc[dt], 0, 0, 0);
      }
    }
  }
  if (q >= N) return;
  const float inv = 1.0f / l;
  _Float16* yo = y + (int64_t(n) * N + q) * ycs + hd * HD;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    _Float16* p = yo + 16 * dt + 4 * g;
    const h4 pe = *reinterpret_cast<const h4*>(p);  // pe(v) written by the depthwise pass
    h4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = (_Float16)((float)pe[j] + acc[dt][j] * inv);
    *reinterpret_cast<h4*>(p) = o;
  }
}

// Chunked variant: K (swizzled [key][32], conflict-free fragment reads) and V^T for KC = 256 keys are
// staged in LDS once per chunk with one barrier pair, and the four 64-key tiles of the chunk run back
// to back from LDS (the per-tile kernel above has two barriers and a V transpose per 64 keys, and
// reads K straight from L2 inside the dependency chain).  Same MFMA operands, the same online-softmax
// order over 64-key tiles: bitwise-identical results.
template <int KD, int HD>
__global__ __launch_bounds__(256) void psa_attention_chunk_kernel(const _Float16* qkv, int qcs, int N, _Float16* y,
                                                                  int ycs, float scale_log2, int QT, int P,
                                                                  int heads, int H, int W, const float* pe_w,
                                                                  const float* pe_b) {
  static_assert(KD == 32 && HD == 64, "C2PSA geometry");
  constexpr int KT = 64, KC = 256, VTS = KC + 4;
  __shared__ __attribute__((aligned(16))) _Float16 vt[HD * VTS];
  __shared__ __attribute__((aligned(16))) h8 kl[KC * 4];  // [key][4 x 8 dims], piece g at g ^ ((key >> 1) & 3)
  int qt, n, hd;
  if (!psa_block(QT, P, heads, qt, n, hd)) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 15, g = lane >> 4;
  const int q = qt * 64 + wave * 16 + col;
  const _Float16* base = qkv + int64_t(n) * N * qcs + hd * (2 * KD + HD);
  h8 qf = h8{0, 0, 0, 0, 0, 0, 0, 0};
  if (q < N) qf = *reinterpret_cast<const h8*>(base + int64_t(q) * qcs + 8 * g);
  float m = -INFINITY, l = 0.f;
  f4 acc[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) acc[dt] = f4{0.f, 0.f, 0.f, 0.f};
  for (int c0 = 0; c0 < N; c0 += KC) {
    __syncthreads();
    // stage K rows and V^T of keys c0 .. c0 + KC - 1 (zeros past N)
    // all loads unconditional (clamped key, zero-selected past N) and issued before the LDS stores
    constexpr int NK = KC * 4 / 256, NV = KC * (HD / 8) / 256;
    h8 kv[NK], vv[NV];
    const h8 z8 = h8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < NK; ++i) {
      const int e = threadIdx.x + 256 * i, key = e >> 2, pc = e & 3;
      const h8 v = *reinterpret_cast<const h8*>(base + int64_t(min(c0 + key, N - 1)) * qcs + KD + 8 * pc);
      kv[i] = c0 + key < N ? v : z8;
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int e = threadIdx.x + 256 * i, key = e / (HD / 8), dc = (e % (HD / 8)) * 8;
      const h8 v = *reinterpret_cast<const h8*>(base + int64_t(min(c0 + key, N - 1)) * qcs + 2 * KD + dc);
      vv[i] = c0 + key < N ? v : z8;
    }
#pragma unroll
    for (int i = 0; i < NK; ++i) {
      const int e = threadIdx.x + 256 * i, key = e >> 2, pc = e & 3;
      kl[key * 4 + (pc ^ ((key >> 1) & 3))] = kv[i];
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int e = threadIdx.x + 256 * i, key = e / (HD / 8), dc = (e % (HD / 8)) * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) vt[(dc + j) * VTS + key] = vv[i][j];
    }
    __syncthreads();
    const int nt = min(KC, N - c0);
    for (int k1 = 0; k1 < nt; k1 += KT) {
      const int k0 = c0 + k1;
      f4 s[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int key = k1 + 16 * t + col;
        const h8 kf = kl[key * 4 + (g ^ ((key >> 1) & 3))];
        s[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf, qf, f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      }
      float mt = -INFINITY;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int key = k0 + 16 * t + 4 * g + j;
          const float v = key < N ? s[t][j] * scale_log2 : -INFINITY;
          s[t][j] = v;
          mt = fmaxf(mt, v);
        }
      mt = fmaxf(mt, __shfl_xor(mt, 16));
      mt = fmaxf(mt, __shfl_xor(mt, 32));
      const float mn = fmaxf(m, mt);
      const float corr = exp2f(m - mn);
      float rs = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float p = exp2f(s[t][j] - mn);
          s[t][j] = p;
          rs += p;
        }
      rs += __shfl_xor(rs, 16);
      rs += __shfl_xor(rs, 32);
      l = l * corr + rs;
      m = mn;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[dt][j] *= corr;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        h8 pf;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pf[j] = (_Float16)s[2 * u][j];
          pf[j + 4] = (_Float16)s[2 * u + 1][j];
        }
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const _Float16* row = vt + (16 * dt + col) * VTS + k1 + 32 * u + 4 * g;
          const h4 lo = *reinterpret_cast<const h4*>(row);
          const h4 hi = *reinterpret_cast<const h4*>(row + 16);
          const h8 vf = h8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          acc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vf, pf, acc[dt], 0, 0, 0);
        }
      }
    }
  }
  if (q >= N) return;
  const float inv = 1.0f / l;
  _Float16* yo = y + (int64_t(n) * N + q) * ycs + hd * HD;
  // pe(v) of this query's pixel, computed here exactly as the depthwise kernel does it (bias, then the taps in
  // (ky, kx) order with fmaf, rows outside the image skipped, columns outside read as zero, fp16 rounding): the
  // separate per-head depthwise launches and the y round trip they needed are gone, results unchanged
  const int py = q / W, px = q - py * W;
  const int wcs = heads * HD;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    const int d0 = 16 * dt + 4 * g;
    const f4 bb = *reinterpret_cast<const f4*>(pe_b + hd * HD + d0);
    float pa[4] = {bb[0], bb[1], bb[2], bb[3]};
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int iy = py - 1 + ky;
      if (iy < 0 || iy >= H) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int ix = px - 1 + kx;
        const h4 v = (ix >= 0 && ix < W)
                         ? *reinterpret_cast<const h4*>(base + int64_t(iy * W + ix) * qcs + 2 * KD + d0)
                         : h4{0, 0, 0, 0};
        const f4 wk = *reinterpret_cast<const f4*>(pe_w + (ky * 3 + kx) * wcs + hd * HD + d0);
#pragma unroll
        for (int j = 0; j < 4; ++j) pa[j] = __builtin_fmaf((float)v[j], wk[j], pa[j]);
      }
    }
    _Float16* p = yo + d0;
    h4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const _Float16 pe = (_Float16)fpin(pa[j]);
      o[j] = (_Float16)((float)pe + acc[dt][j] * inv);
    }
    *reinterpret_cast<h4*>(p) = o;
  }
}

int psa_attention(const fce_tensor& qkv, int heads, int key_dim, int head_dim, const float* pe_w, const float* pe_b,
                  const fce_tensor& y, hipStream_t s) {
  FCE_CHECK(qkv.layout == FCE_NHWC && y.layout == FCE_NHWC && qkv.dtype == FCE_F16 && y.dtype == FCE_F16,
            "psa_attention: NHWC f16 views");
  FCE_CHECK(qkv.c == heads * (2 * key_dim + head_dim) && y.c == heads * head_dim, "psa_attention: channel mismatch");
  FCE_CHECK(qkv.n == y.n && qkv.h == y.h && qkv.w == y.w, "psa_attention: shape mismatch");
  FCE_CHECK(y.cstride % 8 == 0 && y.coff % 8 == 0 && qkv.cstride % 8 == 0 && qkv.coff % 8 == 0,
            "psa_attention: 8-aligned slices");
  if (!(key_dim == 32 && head_dim == 64))
    return fail(FCE_ERR_UNSUPPORTED, "psa_attention: only key_dim 32 / head_dim 64 (C2PSA, num_heads = c // 64)");
  const int N = qkv.h * qkv.w;
  if (N == 0 || qkv.n == 0) return FCE_OK;
  static const bool tiled = [] {  // diagnostics: FCE_PSA_TILED=1 runs the per-64-key-tile kernel
    const char* e = getenv("FCE_PSA_TILED");
    return e && atoi(e) != 0;
  }();
  // pe(v) for the diagnostic tiled kernel: depthwise 3x3 on each head's v slice -> y slice (the kernel adds on
  // top); the default chunk kernel computes pe itself in its epilogue
  for (int h = 0; tiled && h < heads; ++h) {
    fce_tensor vx = qkv;
    vx.c = head_dim;
    vx.coff = qkv.coff + h * (2 * key_dim + head_dim) + 2 * key_dim;
    fce_tensor vy = y;
    vy.c = head_dim;
    vy.coff = y.coff + h * head_dim;
    const int st = dwconv3x3(vx, 1, pe_w + h * head_dim, heads * head_dim, pe_b + h * head_dim, 0, vy, s);
    if (st) return st;
  }
  const int QT = (N + 63) / 64, P = heads * qkv.n;
  FCE_CHECK(int64_t(8) * ((P + 7) / 8) * QT < (int64_t(1) << 31), "psa_attention: grid too large");
  const dim3 grid(unsigned(8 * ((P + 7) / 8) * QT));
  const float scale_log2 = 1.4426950408889634f / sqrtf((float)key_dim);
  if (tiled) {
    FCE_LAUNCH((psa_attention_mfma_kernel<32, 64>), grid, dim3(256), 0, s,
               static_cast<const _Float16*>(qkv.data) + qkv.coff, qkv.cstride, N,
               static_cast<_Float16*>(y.data) + y.coff, y.cstride, scale_log2, QT, P, heads);
    return launch_status("psa_attention_mfma_kernel");
  }
  FCE_LAUNCH((psa_attention_chunk_kernel<32, 64>), grid, dim3(256), 0, s,
             static_cast<const _Float16*>(qkv.data) + qkv.coff, qkv.cstride, N,
             static_cast<_Float16*>(y.data) + y.coff, y.cstride, scale_log2, QT, P, heads, qkv.h, qkv.w, pe_w, pe_b);
  return launch_status("psa_attention_chunk_kernel");
}

}  // namespace fce
