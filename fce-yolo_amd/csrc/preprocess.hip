// Device pre- and post-processing around the detection forward.
//
// letterbox_kernel replaces the reference's host-side preprocessing of a batch of decoded images
// (ultralytics/engine/predictor.py:151-173 preprocess + :184-201 pre_transform, i.e.
// data/augment.py:1555-1610 LetterBox.__call__ with auto=False, center=True, scaleup=True, pad 114):
// every uint8 HWC BGR source image is resized to its new_unpad size with OpenCV's INTER_LINEAR u8
// arithmetic (cv2.resize, restated below), placed at (top, left) of the (H, W) canvas, padded with 114,
// and written as uint8 NCHW RGB — the network input the stem reads (it divides by 255 exactly as
// `im.half() / 255` does).  scale_boxes_kernel replaces utils/ops.py:102-150 scale_boxes (+ clip_boxes
// :153-176) applied per image in models/yolo/detect/predict.py construct_result: kept boxes back to the
// original image's pixel frame.
//
// cv2.resize INTER_LINEAR for 8-bit images (OpenCV imgproc resize.cpp, fixed point, restated):
//   scale = src / dst (double); fx = float((d + 0.5) * scale - 0.5); s = floor(fx); fx -= s;
//   s < 0 -> (s, fx) = (0, 0);  s >= src - 1 -> (s, fx) = (src - 1, 0);
//   coefficients c0 = round(float(1 - fx) * 2048), c1 = round(fx * 2048)   (11 fractional bits)
//   horizontal: h = S[s] * c0 + S[s+1] * c1                                (int)
//   vertical, per element e of the resized row (new_w * 3 bytes): the 16-lane SIMD body (SSE / NEON
//   builds; e < 16 * floor(new_w * 3 / 16)) computes
//     dst = (((b0 * (h0 >> 4)) >> 16) + ((b1 * (h1 >> 4)) >> 16) + 2) >> 2, saturated to [0, 255],
//   and the scalar tail (FixedPtCast<int, uchar, 22>)  dst = (b0 * h0 + b1 * h1 + 2^21) >> 22.
// cv2 is not importable here, so this restatement is pinned only by its identity / pure-padding cases
// (DESIGN.md "Preprocessing"); the letterbox geometry is pinned by the reference's own LetterBox.
#include "common.h"

namespace fce {

struct LbAxis {
  int s0, s1;  // source samples
  int c0, c1;  // 11-bit coefficients
};

__device__ __forceinline__ LbAxis lb_axis(int d, int src, int dst) {
  const double scale = double(src) / double(dst);
  float f = float((d + 0.5) * scale - 0.5);
  int s = int(floorf(f));
  f -= float(s);
  if (s < 0) {
    s = 0;
    f = 0.f;
  }
  if (s >= src - 1) {
    s = src - 1;
    f = 0.f;
  }
  LbAxis a;
  a.s0 = s;
  a.s1 = min(s + 1, src - 1);
  a.c0 = int(rintf((1.f - f) * 2048.f));
  a.c1 = int(rintf(f * 2048.f));
  return a;
}

// one thread per output pixel (all 3 channels): grid (ceil(W/256), H, n)
__global__ __launch_bounds__(256) void letterbox_kernel(const fce_letterbox_img* imgs, uint8_t* dst, int H, int W,
                                                        int pad) {
  const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, n = blockIdx.z;
  if (x >= W) return;
  const fce_letterbox_img im = imgs[n];
  const int64_t plane = int64_t(H) * W;
  uint8_t* o = dst + int64_t(n) * 3 * plane + int64_t(y) * W + x;
  const int ux = x - im.left, uy = y - im.top;
  if (ux < 0 || uy < 0 || ux >= im.new_w || uy >= im.new_h) {
    o[0] = o[plane] = o[2 * plane] = uint8_t(pad);
    return;
  }
  const LbAxis ax = lb_axis(ux, im.w0, im.new_w), ay = lb_axis(uy, im.h0, im.new_h);
  const uint8_t* r0 = im.src + int64_t(ay.s0) * im.row_stride;
  const uint8_t* r1 = im.src + int64_t(ay.s1) * im.row_stride;
  const int simd_end = (im.new_w * 3 / 16) * 16;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int h0 = int(r0[ax.s0 * 3 + c]) * ax.c0 + int(r0[ax.s1 * 3 + c]) * ax.c1;
    const int h1 = int(r1[ax.s0 * 3 + c]) * ax.c0 + int(r1[ax.s1 * 3 + c]) * ax.c1;
    int v;
    if (ux * 3 + c < simd_end)
      v = (((ay.c0 * (h0 >> 4)) >> 16) + ((ay.c1 * (h1 >> 4)) >> 16) + 2) >> 2;
    else
      v = int((int64_t(ay.c0) * h0 + int64_t(ay.c1) * h1 + (1 << 21)) >> 22);
    v = min(max(v, 0), 255);
    o[int64_t(2 - c) * plane] = uint8_t(v);  // BGR source -> RGB planes
  }
}

// one thread per (image, kept slot): boxes -= pad, /= gain, clamp to the original image
__global__ __launch_bounds__(256) void scale_boxes_kernel(float* dets, const int32_t* counts, int n, int max_det,
                                                          const fce_box_scale* sc) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n * max_det) return;
  const int b = i / max_det, k = i - b * max_det;
  if (k >= counts[b]) return;
  const fce_box_scale s = sc[b];
  float* d = dets + int64_t(i) * 6;
  const float px = float(s.pad_x), py = float(s.pad_y);
  // ops.py:133-143: boxes[..., 0] -= pad_x ... ; boxes[..., :4] /= gain; clip_boxes :165-168
  const float x1 = (d[0] - px) / s.gain, y1 = (d[1] - py) / s.gain;
  const float x2 = (d[2] - px) / s.gain, y2 = (d[3] - py) / s.gain;
  const float w0 = float(s.w0), h0 = float(s.h0);
  d[0] = fminf(fmaxf(x1, 0.f), w0);
  d[1] = fminf(fmaxf(y1, 0.f), h0);
  d[2] = fminf(fmaxf(x2, 0.f), w0);
  d[3] = fminf(fmaxf(y2, 0.f), h0);
}

int letterbox(const fce_letterbox_img* imgs, int n, uint8_t* dst, int H, int W, int pad, hipStream_t s) {
  FCE_CHECK(n >= 0 && H > 0 && W > 0 && pad >= 0 && pad <= 255, "letterbox: bad arguments");
  FCE_CHECK(n <= 65535 && H <= 65535, "letterbox: batch / height too large for the grid");
  if (n == 0) return FCE_OK;
  FCE_CHECK(imgs && dst, "letterbox: null pointer");
  FCE_LAUNCH(letterbox_kernel, dim3((W + 255) / 256, H, n), dim3(256), 0, s, imgs, dst, H, W, pad);
  return launch_status("letterbox_kernel");
}

int scale_boxes(float* dets, const int32_t* counts, int n, int max_det, const fce_box_scale* sc, hipStream_t s) {
  FCE_CHECK(n >= 0 && max_det >= 1, "scale_boxes: bad sizes");
  if (n == 0) return FCE_OK;
  FCE_CHECK(dets && counts && sc, "scale_boxes: null pointer");
  FCE_LAUNCH(scale_boxes_kernel, dim3((n * max_det + 255) / 256), dim3(256), 0, s, dets, counts, n, max_det, sc);
  return launch_status("scale_boxes_kernel");
}

}  // namespace fce
