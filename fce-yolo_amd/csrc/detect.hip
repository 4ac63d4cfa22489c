// Detect tail (reference ultralytics/nn/modules/head.py:149-167 Detect._inference):
//   DFL (block.py:58-80): per side, softmax over reg_max bins, expectation sum_i i * p_i
//   make_anchors (utils/tal.py:352-364): anchor = (x + 0.5, y + 0.5) per level, stride per level
//   dist2bbox(xywh) (tal.py:367-376): x1y1 = a - lt, x2y2 = a + rb, c = (x1y1+x2y2)/2, wh = x2y2-x1y1, * stride
//   cls = sigmoid(logits)
// All in fp32 from fp32 logits (Q11: an fp16 decode cannot meet the 1e-3 tolerance).
// Output (N, 4+nc, A) fp32, anchors ordered level-major then row-major, like torch.cat in _inference.
#include "common.h"

namespace fce {

struct Level {
  const float* box;
  const float* cls;
  int bcs, ccs, h, w, a0;
  float stride;
};
struct DecodeArgs {
  Level lv[4];
  int nl, N, A, nc, reg_max;
  float* out;
};

__global__ __launch_bounds__(256) void detect_decode_kernel(DecodeArgs a) {
  const int64_t total = int64_t(a.N) * a.A;
  for (int64_t t = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; t < total; t += int64_t(gridDim.x) * blockDim.x) {
    const int n = int(t / a.A), an = int(t % a.A);
    int li = 0;
    while (li + 1 < a.nl && an >= a.lv[li + 1].a0) ++li;
    const Level& L = a.lv[li];
    const int p = an - L.a0;
    const int py = p / L.w, px = p % L.w;
    const float* bx = L.box + (int64_t(n) * L.h * L.w + p) * L.bcs;
    float dist[4];
    for (int s = 0; s < 4; ++s) {
      // same reduction tree as the fused conv epilogue (conv.hip OUT_DFL): four partial sums of
      // 4 consecutive bins, combined as (g0 + g1) + (g2 + g3), so both paths agree bit for bit
      const float* b = bx + s * a.reg_max;
      float mx = -INFINITY;
      for (int i = 0; i < a.reg_max; ++i) mx = fmaxf(mx, b[i]);
      float den = 0.f, num = 0.f;
      if (a.reg_max == 16) {
        float sd[4], sn[4];
        for (int g = 0; g < 4; ++g) {
          sd[g] = 0.f;
          sn[g] = 0.f;
          for (int j = 0; j < 4; ++j) {
            const float e = __expf(b[g * 4 + j] - mx);
            sd[g] += e;
            sn[g] = __fadd_rn(sn[g], __fmul_rn(e, (float)(g * 4 + j)));  // no FMA: match the fused path
          }
        }
        den = (sd[0] + sd[1]) + (sd[2] + sd[3]);
        num = (sn[0] + sn[1]) + (sn[2] + sn[3]);
      } else {
        for (int i = 0; i < a.reg_max; ++i) {
          const float e = __expf(b[i] - mx);
          den += e;
          num += e * (float)i;
        }
      }
      dist[s] = num / den;
    }
    const float ax = (float)px + 0.5f, ay = (float)py + 0.5f;
    const float x1 = ax - dist[0], y1 = ay - dist[1], x2 = ax + dist[2], y2 = ay + dist[3];
    float* o = a.out + int64_t(n) * (4 + a.nc) * a.A + an;
    o[0] = (x1 + x2) / 2.0f * L.stride;
    o[int64_t(1) * a.A] = (y1 + y2) / 2.0f * L.stride;
    o[int64_t(2) * a.A] = (x2 - x1) * L.stride;
    o[int64_t(3) * a.A] = (y2 - y1) * L.stride;
    const float* cl = L.cls + (int64_t(n) * L.h * L.w + p) * L.ccs;
    for (int c = 0; c < a.nc; ++c) o[int64_t(4 + c) * a.A] = sigmoidf_(cl[c]);
  }
}

int detect_decode(const fce_tensor* box, const fce_tensor* cls, int nl, const float* strides, int reg_max,
                  float* out, hipStream_t s) {
  FCE_CHECK(nl >= 1 && nl <= 4, "detect_decode: 1..4 levels");
  DecodeArgs a;
  a.nl = nl;
  a.N = box[0].n;
  a.nc = cls[0].c;
  a.reg_max = reg_max;
  a.out = out;
  int A = 0;
  for (int i = 0; i < nl; ++i) {
    FCE_CHECK(box[i].dtype == FCE_F32 && cls[i].dtype == FCE_F32 && box[i].layout == FCE_NHWC &&
                  cls[i].layout == FCE_NHWC,
              "detect_decode: NHWC f32 maps");
    FCE_CHECK(box[i].c == 4 * reg_max && cls[i].c == a.nc && box[i].n == a.N && cls[i].n == a.N &&
                  box[i].h == cls[i].h && box[i].w == cls[i].w,
              "detect_decode: map shape mismatch");
    a.lv[i] = Level{static_cast<const float*>(box[i].data) + box[i].coff, static_cast<const float*>(cls[i].data) + cls[i].coff,
                    box[i].cstride, cls[i].cstride, box[i].h, box[i].w, A, strides[i]};
    A += box[i].h * box[i].w;
  }
  a.A = A;
  const int64_t total = int64_t(a.N) * A;
  if (total == 0) return FCE_OK;
  FCE_LAUNCH(detect_decode_kernel, dim3(int(std::min<int64_t>((total + 255) / 256, 65535 * 8))), dim3(256),
                     0, s, a);
  return launch_status("detect_decode_kernel");
}

}  // namespace fce
