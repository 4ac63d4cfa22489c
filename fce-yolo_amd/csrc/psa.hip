// C2PSA attention (reference ultralytics/nn/modules/block.py:1247-1304, Attention.forward):
//   q,k,v = qkv.view(B, heads, 2*kd+hd, N).split([kd,kd,hd]) ;  out = v @ softmax(q^T k * kd^-0.5)^T + pe(v)
// with pe = depthwise 3x3 (BN folded, no act) over v viewed as (B, heads*hd, H, W).
// qkv is the NHWC fp16 output of the qkv 1x1 conv: channel (head*(2kd+hd) + r) is row r of that head.
// One block = (image, head, 64 queries); K/V streamed through LDS in 64-key tiles with an online
// (running max / sum) softmax in fp32; the pe term is added in the epilogue from the same v.
#include "common.h"

namespace fce {

template <int KD, int HD>
__global__ __launch_bounds__(256) void psa_attention_kernel(const _Float16* qkv, int qcs, int H, int W, int heads,
                                                            const float* pe_w, const float* pe_b, _Float16* y,
                                                            int ycs, float scale) {
  constexpr int QT = 64, KT = 64, DG = 4, DPT = HD / DG;
  __shared__ float ks[KT][KD + 1];
  __shared__ float vs[KT][HD + 4];
  const int N = H * W;
  const int n = blockIdx.z, hd = blockIdx.y;
  const int t = threadIdx.x;
  const int qi = t / DG, dg = t % DG;
  const int tok = blockIdx.x * QT + qi;
  const int hstride = 2 * KD + HD;
  const _Float16* base = qkv + int64_t(n) * N * qcs + hd * hstride;
  float q[KD];
  const bool qok = tok < N;
#pragma unroll
  for (int d = 0; d < KD; ++d) q[d] = qok ? (float)base[int64_t(tok) * qcs + d] : 0.f;
  float m = -INFINITY, l = 0.f, acc[DPT];
#pragma unroll
  for (int d = 0; d < DPT; ++d) acc[d] = 0.f;
  for (int k0 = 0; k0 < N; k0 += KT) {
    __syncthreads();
    for (int e = t; e < KT * KD; e += 256) {
      const int j = e / KD, d = e % KD;
      ks[j][d] = (k0 + j < N) ? (float)base[int64_t(k0 + j) * qcs + KD + d] : 0.f;
    }
    for (int e = t; e < KT * HD; e += 256) {
      const int j = e / HD, d = e % HD;
      vs[j][d] = (k0 + j < N) ? (float)base[int64_t(k0 + j) * qcs + 2 * KD + d] : 0.f;
    }
    __syncthreads();
    const int kn = min(KT, N - k0);
    for (int j = 0; j < kn; ++j) {
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < KD; ++d) s += q[d] * ks[j][d];
      s *= scale;
      const float mn = fmaxf(m, s);
      const float corr = __expf(m - mn);
      const float p = __expf(s - mn);
      l = l * corr + p;
#pragma unroll
      for (int d = 0; d < DPT; ++d) acc[d] = acc[d] * corr + p * vs[j][dg * DPT + d];
      m = mn;
    }
  }
  if (!qok) return;
  const float inv = 1.0f / l;
  const int ty = tok / W, tx = tok % W;
  const int c0 = hd * HD + dg * DPT;  // channel in the (B, heads*hd, H, W) view
  float o[DPT];
#pragma unroll
  for (int d = 0; d < DPT; ++d) o[d] = acc[d] * inv + pe_b[c0 + d];
  for (int ky = -1; ky <= 1; ++ky) {
    const int iy = ty + ky;
    if (iy < 0 || iy >= H) continue;
    for (int kx = -1; kx <= 1; ++kx) {
      const int ix = tx + kx;
      if (ix < 0 || ix >= W) continue;
      const _Float16* vp = base + int64_t(iy * W + ix) * qcs + 2 * KD + dg * DPT;
      const int tap = (ky + 1) * 3 + (kx + 1);
#pragma unroll
      for (int d = 0; d < DPT; ++d) o[d] += (float)vp[d] * pe_w[(c0 + d) * 9 + tap];
    }
  }
  _Float16* yo = y + (int64_t(n) * N + tok) * ycs + c0;
#pragma unroll
  for (int d = 0; d < DPT; d += 8) {
    h8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (_Float16)o[d + j];
    *reinterpret_cast<h8*>(yo + d) = v;
  }
}

int psa_attention(const fce_tensor& qkv, int heads, int key_dim, int head_dim, const float* pe_w, const float* pe_b,
                  const fce_tensor& y, hipStream_t s) {
  FCE_CHECK(qkv.layout == FCE_NHWC && y.layout == FCE_NHWC && qkv.dtype == FCE_F16 && y.dtype == FCE_F16,
            "psa_attention: NHWC f16 views");
  FCE_CHECK(qkv.c == heads * (2 * key_dim + head_dim) && y.c == heads * head_dim, "psa_attention: channel mismatch");
  FCE_CHECK(qkv.n == y.n && qkv.h == y.h && qkv.w == y.w, "psa_attention: shape mismatch");
  FCE_CHECK(y.cstride % 8 == 0 && y.coff % 8 == 0, "psa_attention: 8-aligned output slice");
  if (!(key_dim == 32 && head_dim == 64))
    return fail(FCE_ERR_UNSUPPORTED, "psa_attention: only key_dim 32 / head_dim 64 (C2PSA, num_heads = c // 64)");
  const int N = qkv.h * qkv.w;
  if (N == 0 || qkv.n == 0) return FCE_OK;
  dim3 grid((N + 63) / 64, heads, qkv.n);
  hipLaunchKernelGGL((psa_attention_kernel<32, 64>), grid, dim3(256), 0, s,
                     static_cast<const _Float16*>(qkv.data) + qkv.coff, qkv.cstride, qkv.h, qkv.w, heads, pe_w, pe_b,
                     static_cast<_Float16*>(y.data) + y.coff, y.cstride, 1.0f / sqrtf((float)key_dim));
  return launch_status("psa_attention_kernel");
}

}  // namespace fce
